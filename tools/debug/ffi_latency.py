"""Debug: per-call latency of the torch-free binding (integration/mano_hip_ffi.py)
at batch 1, zero copy (pinned host block, the default) vs the copy form
(device buffers + mano_memcpy); same inputs, same process, no torch.

    python tools/debug/ffi_latency.py [--calls 300]
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "integration"), os.path.join(REPO, "mano-hand_amd"), REPO]


def main():
    calls = int(sys.argv[sys.argv.index("--calls") + 1]) if "--calls" in sys.argv else 300
    import mano_hip_ffi
    from mano_amd.model_io import synthetic_params
    params = synthetic_params(0)
    rng = np.random.default_rng(3)
    betas, pose = rng.normal(0, 1, (calls, 1, 10)), rng.normal(0, 0.5, (calls, 1, 16, 3))
    res = {}
    for name, zc in (("zero_copy", True), ("copy", False), ("zero_copy_again", True)):
        e = mano_hip_ffi.Engine(type("M", (), params), device=0, capacity=1, zero_copy=zc)
        for i in range(30):
            e.forward(betas[i], pose[i])
        ts, dig = [], 0.0
        for i in range(calls):
            t0 = time.perf_counter()
            o = e.forward(betas[i], pose[i])
            ts.append(time.perf_counter() - t0)
            dig += float(o["verts"][0, ::97].sum())
        res[name] = {"median_us": float(np.median(ts) * 1e6), "p90_us": float(np.percentile(ts, 90) * 1e6),
                     "digest": dig}
        e.close()
    res["same_results"] = len({res[k]["digest"] for k in res}) == 1
    res["torch_loaded"] = "torch" in sys.modules
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
