"""Debug: A/B the forward's kernels across library builds (same box, alternating).

    python tools/debug/time_path.py libmano_hip.so libmano_hip_<variant>.so ... [--reps 2]

Each library runs in its own child process (one library per process), the
list `--reps` times in alternation.  Per run, at 65,536 hands (C2 inputs,
seed 1001, no trans): the unfused step (articulate -> blend -> skin, each
kernel event-bracketed, as bench.py --path unfused), skin back to back, the
fused step (articulate -> blend_skin), blend_skin with rest_verts back to back;
mean ms over 100 steps after 300 warm-up steps, and a digest of verts so
builds can be compared bit for bit."""
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
inp = m.synthetic_inputs(1001, 0, B)
betas, pose = inp["betas"], inp["pose"]
v = torch.empty((B, 778, 3), device="cuda:0")
vp = torch.empty((B, 778, 3), device="cuda:0")
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

art = lambda: m.stage_articulate(betas, pose)
res = {"lib": sys.argv[2]}
a, b, s = steps([art, lambda: m.stage_blend(B), lambda: m.stage_skin(B, v)])
res["unfused"] = {"articulate": a, "blend": b, "skin": s}
res["unfused_digest"] = digest(v)
res["skin_b2b"] = steps([lambda: m.stage_skin(B, v)])[0]
# the same step with 1 GiB of unrelated copies between the blend GEMM and the
# LBS: if the LBS's in-path penalty is the blend's dirty v_posed lines in the
# caches, the flush moves it into the copy
fa = torch.empty(1 << 28, device="cuda:0"); fb = torch.empty_like(fa)
a, b, c, s2 = steps([art, lambda: m.stage_blend(B), lambda: fb.copy_(fa), lambda: m.stage_skin(B, v)], reps=50)
res["unfused_flushed"] = {"blend": b, "copy": c, "skin": s2}
del fa, fb
a, f = steps([art, lambda: m.stage_blend_skin(B, v)])
res["fused"] = {"articulate": a, "blend_skin": f, "step": a + f}
res["fused_digest"] = digest(v)
res["blend_skin_rest_verts"] = steps([lambda: m.stage_blend_skin(B, v, rest_verts=vp)])[0]
jo = torch.empty((B, 16, 3), device="cuda:0")
# bench.py's forward step: the articulation also writes the posed joints
a, f = steps([lambda: m.stage_articulate(betas, pose, joints=jo), lambda: m.stage_blend_skin(B, v)])
res["fused_joints"] = {"articulate": a, "blend_skin": f, "step": a + f}
outd = {"verts": v, "joints": jo}
res["single_launch"] = steps([lambda: m.forward(betas, pose, None, joints=True, out=outd)])[0]
res["single_digest"] = [digest(v), digest(jo)]
res["rest_digest"] = [digest(v), digest(vp)]
res["status"] = m.device_status()
print("RESULT " + json.dumps(res), flush=True)
'''


def main():
    args = sys.argv[1:]
    reps = 2
    if "--reps" in args:
        i = args.index("--reps")
        reps = int(args[i + 1])
        del args[i:i + 2]
    libs = args or ["libmano_hip.so"]
    # MANO_BS_ABLATE=4 builds write verts in a larger scratch layout
    # (n x n_groups x 256 B, tools/debug/align_bound.py): this tool's
    # reference-layout buffers are too small for them (out-of-bounds writes)
    bad = [l for l in libs if "abl4" in l]
    if bad:
        raise SystemExit(f"time_path.py cannot run scratch-layout builds {bad}: use align_bound.py")
    for rep in range(reps):
        for lib in libs:
            r = subprocess.run([sys.executable, "-c", CHILD, REPO, lib], capture_output=True, text=True,
                               timeout=300)
            lines = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
            if r.returncode != 0 or not lines:
                print(json.dumps({"lib": lib, "rc": r.returncode, "err": r.stderr[-1500:]}), flush=True)
                if r.returncode < 0 or r.returncode in (124, 134, 137, 139) or "HIP error" in r.stderr:
                    sys.exit(1)
                continue
            d = json.loads(lines[-1][7:])
            d["rep"] = rep
            print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
