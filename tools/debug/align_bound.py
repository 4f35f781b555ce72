"""Debug: the upper bound of any 32-B-aligned store design for blend_skin16.

    python tools/debug/align_bound.py libmano_hip.so libmano_hip_abl4.so [--reps 3]
    python tools/debug/align_bound.py --loop <lib> <verts|rest> [K]     (for rocprofv3 --pmc)

The product kernel stores each 16-vertex group of a hand row as 16 12-B
points: a 192-B segment that, for 3 hands in 4 (rows are 9,336 B apart),
starts and ends inside a 32-B sector the neighbouring group fills later
(WRITE_SIZE 1.15x of the verts bytes).  The MANO_BS_ABLATE=4 build issues the
SAME store instructions (same bytes, cache policy, deferral and order) into a
layout with every segment at a 256-B boundary (n x n_groups x 64 floats), so
no sector is ever partially written.  No aligned-store design that keeps the
reference layout can write fewer partial sectors or issue fewer instructions,
so its time is the bound of what such a design can gain.

Each library runs in its own child process, alternating; per run at 65,536
hands (C2 inputs): the fused step (articulate -> blend_skin16, verts only) and
blend_skin16 with rest_verts back to back, event-timed over 100 launches after
300 warm-up ones, and a digest of verts / rest_verts read back in the
reference layout (the ablation's scratch segments un-permuted), so both builds
are shown to produce the same bits."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r'''
import json, os, sys
sys.path[:0] = [os.path.join(sys.argv[1], "mano-hand_amd"), sys.argv[1]]
from mano_amd import _abi
lib = sys.argv[2]
_abi.LIB_PATH = os.path.join(os.path.dirname(_abi.LIB_PATH), lib)
import numpy as np, torch
from mano_amd import ManoHip, synthetic_params
B = int(os.environ.get("B", 65536))
V, G = 778, 49
scratch = "abl4" in lib
m = ManoHip(synthetic_params(0), device=0)
inp = m.synthetic_inputs(1001, 0, B)
betas, pose = inp["betas"], inp["pose"]
nfl = B * G * 64 if scratch else B * V * 3
v = torch.empty(nfl, device="cuda:0")
vp = torch.empty(nfl, device="cuda:0")
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

def ref_layout(t):
    """(B, V, 3) in the reference layout: the scratch segments un-permuted
    (group g of row h at floats (h * G + g) * 64 .. + 48, vertices vb .. vb + 15,
    vb = min(16 g, V - 16))."""
    if not scratch:
        return t.view(B, V, 3)
    s = t.view(B, G, 64)[:, :, :48].reshape(B, G, 16, 3)
    out = torch.empty((B, V, 3), device=t.device)
    for g in range(G):
        vb = min(16 * g, V - 16)
        out[:, vb:vb + 16] = s[:, g]
    return out

def digest(t):
    return int(t.contiguous().view(torch.int32).to(torch.int64).sum().item()) & 0xFFFFFFFF

if len(sys.argv) > 3:   # --loop: K launches of one kernel form (rocprofv3 --pmc)
    what, K = sys.argv[3], int(sys.argv[4])
    m.stage_articulate(betas, pose)
    for _ in range(K):
        if what == "verts":
            m.stage_blend_skin(B, v)
        else:
            m.stage_blend_skin(B, v, rest_verts=vp)
    torch.cuda.synchronize()
    print("done", lib, what, K)
    sys.exit(0)

res = {"lib": lib}
art = lambda: m.stage_articulate(betas, pose)
a, f = steps([art, lambda: m.stage_blend_skin(B, v)])
res["fused"] = {"articulate": a, "blend_skin": f, "step": a + f}
res["verts_digest"] = digest(ref_layout(v))
res["blend_skin_b2b"] = steps([lambda: m.stage_blend_skin(B, v)])[0]
res["blend_skin_rest_verts"] = steps([lambda: m.stage_blend_skin(B, v, rest_verts=vp)])[0]
res["rest_digest"] = [digest(ref_layout(v)), digest(ref_layout(vp))]
if not scratch:   # the f16x3 fused kernel (blend_skin_h3) the same way
    m.set_precision("f16x3")
    a, f = steps([art, lambda: m.stage_blend_skin(B, v)])
    res["h3_fused"] = {"articulate": a, "blend_skin": f, "step": a + f}
    res["h3_verts_digest"] = digest(ref_layout(v))
    res["h3_rest_verts"] = steps([lambda: m.stage_blend_skin(B, v, rest_verts=vp)])[0]
    res["h3_rest_digest"] = [digest(ref_layout(v)), digest(ref_layout(vp))]
    m.set_precision("fp32")
res["status"] = m.device_status()
print("RESULT " + json.dumps(res), flush=True)
'''


def main():
    args = sys.argv[1:]
    if args and args[0] == "--loop":
        lib, what = args[1], args[2]
        K = args[3] if len(args) > 3 else "20"
        sys.argv = [sys.argv[0], REPO, lib, what, K]   # in this process (the profiler's)
        exec(CHILD, {"__name__": "__align_child__"})
        return
    reps = 3
    if "--reps" in args:
        i = args.index("--reps")
        reps = int(args[i + 1])
        del args[i:i + 2]
    libs = args or ["libmano_hip.so"]
    for rep in range(reps):
        for lib in libs:
            r = subprocess.run([sys.executable, "-c", CHILD, REPO, lib], capture_output=True, text=True,
                               timeout=300)
            lines = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
            if r.returncode != 0 or not lines:
                print(json.dumps({"lib": lib, "rc": r.returncode, "err": r.stderr[-1500:]}), flush=True)
                sys.exit(1)
            d = json.loads(lines[-1][7:])
            d["rep"] = rep
            print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
