"""Debug: does row alignment matter to the standalone LBS?  (a bound, no new kernel)

    python tools/debug/skin_align_probe.py [--reps 2]

skin_pair streams 4-hand x 64-vertex units: four 768-B row segments that for
V = 778 start at the rows' sector phase (rows are 9,336 B apart: 3 hands in 4
are off a 32-B boundary, half of them 8 B off a 16-B one).  A mesh of V = 776
vertices (the synthetic model cut to its first 776) has rows of 9,312 B =
291 sectors: every segment of every hand starts on a sector.  Same kernel,
same unit count (12 full spans + a tail group per hand quad), 0.26 % fewer
bytes.  Per run (own process), 65,536 hands: skin_pair back to back and the
unfused blend GEMM, event-timed over 100 launches after 300 warm-up ones, and
the time per algorithmic byte."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r'''
import json, os, sys
sys.path[:0] = [os.path.join(sys.argv[1], "mano-hand_amd"), sys.argv[1]]
import numpy as np, torch
from mano_amd import ManoHip, synthetic_params
V = int(sys.argv[2])
B = 65536
p = synthetic_params(0)
if V != 778:
    p = dict(p)
    for k in ("mesh_template", "mesh_shape_basis", "mesh_pose_basis", "skinning_weights"):
        p[k] = np.ascontiguousarray(np.asarray(p[k])[:V])
    jr = np.asarray(p["J_regressor"])[:, :V]
    p["J_regressor"] = jr / jr.sum(1, keepdims=True)
    p["faces"] = np.asarray(p["faces"])[np.all(np.asarray(p["faces"]) < V, axis=1)]
m = ManoHip(p, device=0)
inp = m.synthetic_inputs(1001, 0, B)
v = torch.empty((B, V, 3), device="cuda:0")
m.workspace(B)
m.stage_articulate(inp["betas"], inp["pose"])
m.stage_blend(B)
E = lambda: torch.cuda.Event(enable_timing=True)
def t(fn, warm=300, reps=100):
    for _ in range(warm): fn()
    ev = [(E(), E()) for _ in range(reps)]
    for a, b in ev:
        a.record(); fn(); b.record()
    torch.cuda.synchronize()
    return float(np.mean([a.elapsed_time(b) for a, b in ev]))
skin = t(lambda: m.stage_skin(B, v))
blend = t(lambda: m.stage_blend(B))
skin_bytes = B * (V * 3 * 4 * 2 + 768)
print("RESULT " + json.dumps({"V": V, "row_bytes": 12 * V, "skin_ms": skin, "blend_ms": blend,
      "skin_GBs": skin_bytes / skin / 1e6, "skin_ns_per_kB": skin * 1e6 / (skin_bytes / 1e3),
      "status": m.device_status()}), flush=True)
'''


def main():
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 2
    for rep in range(reps):
        for V in (778, 776):
            r = subprocess.run([sys.executable, "-c", CHILD, REPO, str(V)], capture_output=True, text=True,
                               timeout=300)
            lines = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
            if r.returncode != 0 or not lines:
                print(json.dumps({"V": V, "rc": r.returncode, "err": r.stderr[-1500:]}), flush=True)
                sys.exit(1)
            d = json.loads(lines[-1][7:])
            d["rep"] = rep
            print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
