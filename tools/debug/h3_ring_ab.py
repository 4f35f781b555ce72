"""Debug: A/B blend_skin_h3 (f16x3 fused, verts only) across library builds.

    python tools/debug/h3_ring_ab.py libmano_hip.so libmano_hip_h3r3.so ... [--reps 3]

Each library runs in its own child process, the list `--reps` times in
alternation (same box).  Per run, at 65,536 hands (C2 inputs, seed 1001, with
and without translation): blend_skin_h3 back to back, mean ms over 100
launches after 300 warm-up launches (one event pair around the 100), the
articulate + blend_skin_h3 step with per-kernel events, and a digest of verts
so builds can be compared bit for bit (the ring depth / wave shape must not
change a bit)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r'''
import json, os, sys
sys.path[:0] = [os.path.join(sys.argv[1], "mano-hand_amd"), sys.argv[1]]
from mano_amd import _abi
_abi.LIB_PATH = os.path.join(os.path.dirname(_abi.LIB_PATH), sys.argv[2])
import numpy as np, torch
from mano_amd import ManoHip, synthetic_params
B = int(os.environ.get("B", 65536))
m = ManoHip(synthetic_params(0), device=0, precision="f16x3")
inp = m.synthetic_inputs(1001, 0, B, trans=True)
betas, pose, trans = inp["betas"], inp["pose"], inp["trans"]
v = torch.empty((B, 778, 3), device="cuda:0")
m.workspace(B)
E = lambda: torch.cuda.Event(enable_timing=True)

def b2b(k, warm=300, reps=100):
    for _ in range(warm):
        k()
    e0, e1 = E(), E()
    e0.record()
    for _ in range(reps):
        k()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps

def digest(t):
    return int(t.contiguous().view(torch.int32).to(torch.int64).sum().item()) & 0xFFFFFFFF

res = {"lib": sys.argv[2]}
for tr_name, tr in (("no_trans", None), ("trans", trans)):
    m.stage_articulate(betas, pose, tr)
    res[tr_name] = b2b(lambda: m.stage_blend_skin(B, v, trans=tr))
    res[tr_name + "_digest"] = digest(v)
    ev = [[E() for _ in range(3)] for _ in range(50)]
    for _ in range(100):
        m.stage_articulate(betas, pose, tr); m.stage_blend_skin(B, v, trans=tr)
    for e in ev:
        e[0].record(); m.stage_articulate(betas, pose, tr); e[1].record()
        m.stage_blend_skin(B, v, trans=tr); e[2].record()
    torch.cuda.synchronize()
    res[tr_name + "_step"] = {"articulate": float(np.mean([e[0].elapsed_time(e[1]) for e in ev])),
                              "blend_skin_h3": float(np.mean([e[1].elapsed_time(e[2]) for e in ev]))}
res["check_device"] = m.device_status()
print("RESULT " + json.dumps(res), flush=True)
'''


def main():
    args = sys.argv[1:]
    reps = 3
    if "--reps" in args:
        i = args.index("--reps")
        reps = int(args[i + 1])
        del args[i:i + 2]
    for r in range(reps):
        for lib in args:
            p = subprocess.run([sys.executable, "-c", CHILD, REPO, lib], capture_output=True, text=True,
                               timeout=300)
            line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")]
            if p.returncode != 0 or not line:
                print(json.dumps({"lib": lib, "rep": r, "error": p.stderr[-1500:]}), flush=True)
                sys.exit(1)
            out = json.loads(line[0][7:])
            out["rep"] = r
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
