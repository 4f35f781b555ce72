"""Debug: the unfused step with the LBS in place vs out of place (round 6).

    python tools/debug/time_inplace.py [libmano_hip.so [libmano_hip_<variant>.so ...]] [--reps 3]

Each library runs in its own child process, the list `--reps` times in
alternation.  Per run, at 65,536 hands (C2 inputs, seed 1001, trans): the
unfused step in two forms, alternating inside the process --
  separate: articulate -> blend (v_posed in the workspace) -> skin into verts
  in_place: articulate -> blend (v_posed into verts) -> skin over verts
(mano_stage_skin with rest_verts == verts, ABI 7) -- each kernel
event-bracketed, mean ms over 100 steps after 300 warm ones, and the verts
digest of each form (they must be equal: the same MFMA chains and fmaf apply).
DESIGN.md §4 round 6 holds the prediction and the result."""
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
m = ManoHip(synthetic_params(0), device=0)
inp = m.synthetic_inputs(1001, 0, B, trans=True)
betas, pose, tr = inp["betas"], inp["pose"], inp["trans"]
v_sep = torch.empty((B, 778, 3), device="cuda:0")
v_ip = torch.empty((B, 778, 3), device="cuda:0")
m.workspace(B)
E = lambda: torch.cuda.Event(enable_timing=True)

def steps(kernels, warm=300, reps=100):
    for _ in range(warm):
        for k in kernels: k()
    ev = [[E() for _ in range(len(kernels) + 1)] for _ in range(reps)]
    for e in ev:
        e[0].record()
        for i, k in enumerate(kernels):
            k(); e[i + 1].record()
    torch.cuda.synchronize()
    return [float(np.mean([e[i].elapsed_time(e[i + 1]) for e in ev])) for i in range(len(kernels))]

def digest(t):
    return int(t.contiguous().view(torch.int32).to(torch.int64).sum().item()) & 0xFFFFFFFF

art = lambda: m.stage_articulate(betas, pose, tr)
forms = {
    "separate": [art, lambda: m.stage_blend(B), lambda: m.stage_skin(B, v_sep, trans=tr)],
    "in_place": [art, lambda: m.stage_blend(B, rest_verts=v_ip), lambda: m.stage_skin(B, v_ip, rest_verts=v_ip, trans=tr)],
}
res = {"lib": sys.argv[2], "B": B}
for rnd in range(int(os.environ.get("ROUNDS", 2))):
    for name, ks in forms.items():
        a, b, s = steps(ks)
        res.setdefault(name, []).append({"articulate": a, "blend": b, "skin": s, "step": a + b + s,
                                         "skin_frac": 19440 * B / (s * 1e-3) / 8e12})
res["digest_separate"], res["digest_in_place"] = digest(v_sep), digest(v_ip)
res["bit_identical"] = bool(torch.equal(v_sep, v_ip))
res["skin_b2b"] = steps([lambda: m.stage_skin(B, v_sep, trans=tr)])[0]
print(json.dumps(res))
'''


def main():
    args = sys.argv[1:]
    reps = 1
    if "--reps" in args:
        i = args.index("--reps")
        reps = int(args[i + 1])
        del args[i:i + 2]
    libs = args or ["libmano_hip.so"]
    for _ in range(reps):
        for lib in libs:
            r = subprocess.run([sys.executable, "-c", CHILD, REPO, lib], capture_output=True, text=True,
                               timeout=300)
            if r.returncode != 0:
                print(json.dumps({"lib": lib, "error": r.stderr[-1500:]}), flush=True)
                sys.exit(1)
            print(r.stdout.strip().splitlines()[-1], flush=True)


if __name__ == "__main__":
    main()
