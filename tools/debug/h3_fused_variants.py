"""Debug: fused f16x3 verts vs the standalone skin on the exact v_posed, per kernel variant."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mano-hand_amd"), REPO]
import numpy as np, torch
from mano_amd import _abi
if len(sys.argv) > 1:
    _abi.LIB_PATH = os.path.join(os.path.dirname(_abi.LIB_PATH), sys.argv[1])
print("library", _abi.LIB_PATH)
from mano_amd import ManoHip, synthetic_params
params = synthetic_params(0)
m = ManoHip(params, device=0, precision="f16x3")
dev = torch.device("cuda", 0)
for B in (65536,):
    rng = np.random.default_rng(7)
    f = lambda a: torch.tensor(a, dtype=torch.float32, device=dev)
    betas = f(rng.normal(0, 1, (B, 10))); pose = f(rng.normal(0, 0.6, (B, 16, 3)))
    trans = f(rng.uniform(-1, 1, (B, 3)))
    # reference: exact-fp32 v_posed (unfused blend) + standalone skin_h3
    m.stage_articulate(betas, pose, trans)
    vp = torch.empty((B, 778, 3), device=dev); ref = torch.empty((B, 778, 3), device=dev)
    m.stage_blend(B, rest_verts=vp)
    for with_trans in (False, True):
        t = trans if with_trans else None
        m.stage_skin(B, ref, rest_verts=vp, trans=t)
        for with_vp in (False, True):
            for rep in range(3):
                out = m.forward(betas, pose, t, rest_verts=with_vp)
                torch.cuda.synchronize()
                d = (out["verts"] - ref).abs()
                bad = (d > 1e-5).nonzero()
                msg = f"B={B} trans={with_trans} vposed={with_vp} rep={rep}: max {d.max().item():.3e} n_bad {bad.shape[0]}"
                if bad.shape[0]:
                    rows = torch.bincount(bad[:, 0] % 16, minlength=16).tolist()
                    coords = torch.bincount(bad[:, 2], minlength=3).tolist()
                    msg += f" rows%16 {rows} coords {coords}"
                print(msg, flush=True)
