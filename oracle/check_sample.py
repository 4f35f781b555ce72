"""bench.py's correctness leg: sampled hands of a timed step vs the oracle.

TEST INFRASTRUCTURE (like the rest of oracle/): bench.py writes the sampled
hands' inputs and the GPU outputs of its last timed step to an .npz and runs
this file as a child process, so the GPU process never imports oracle/.

    python oracle/check_sample.py sample.npz

The .npz holds `index` (global hand indices), `betas` (n,10), `pose` (n,16,3),
optional `trans` (n,3), the GPU's `verts` (n,V,3) and `joints` (n,16,3), and
`model` ("synthetic:<seed>" or a dump_model.py pickle path).  Prints one JSON
line: the max |GPU - oracle| over the sample (metres) and the hand where it
occurs.  The oracle (mano_oracle.forward, float64) restates mano_np.py:79-115
and is pinned to the reference's own outputs (tests/test_oracle_golden.py).
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "mano-hand_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

from mano_amd.model_io import load_dump, synthetic_params  # noqa: E402  (numpy only)
from oracle import mano_oracle  # noqa: E402


def check(path):
    with np.load(path, allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    model = str(d["model"])
    params = synthetic_params(int(model.split(":")[1])) if model.startswith("synthetic:") else load_dump(model)
    trans = d.get("trans")
    ref = mano_oracle.forward(params, d["betas"].astype(np.float64), d["pose"].astype(np.float64),
                              None if trans is None else trans.astype(np.float64))
    ev = np.abs(d["verts"].astype(np.float64) - ref["verts"]).max(axis=(1, 2))
    ej = np.abs(d["joints"].astype(np.float64) - ref["joints"]).max(axis=(1, 2))
    idx = d["index"]
    return {"max_abs_err_verts": float(ev.max()), "max_abs_err_joints": float(ej.max()),
            "worst_hand_verts": int(idx[int(ev.argmax())]), "worst_hand_joints": int(idx[int(ej.argmax())]),
            "n_sampled": int(len(idx)), "finite": bool(np.isfinite(d["verts"]).all() and np.isfinite(d["joints"]).all())}


if __name__ == "__main__":
    print(json.dumps(check(sys.argv[1])), flush=True)
