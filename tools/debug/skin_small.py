"""Debug: standalone LBS of one library build vs the fused kernel on small batches.

    python tools/debug/skin_small.py libmano_hip_<variant>.so [n ...]"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mano-hand_amd"), REPO]
import torch
from mano_amd import _abi
_abi.LIB_PATH = os.path.join(os.path.dirname(_abi.LIB_PATH), sys.argv[1])
from mano_amd import ManoHip, synthetic_params
dev = torch.device("cuda", 0)
m = ManoHip(synthetic_params(0), device=0)
for n in [int(a) for a in sys.argv[2:]] or [1, 4, 5, 64, 1000]:
    g = torch.Generator(device=dev).manual_seed(3)
    betas = torch.randn((n, 10), generator=g, device=dev)
    pose = 0.5 * torch.randn((n, 16, 3), generator=g, device=dev)
    fused = m.forward(betas, pose, rest_verts=True)
    v = torch.full_like(fused["verts"], float("nan"))
    m.stage_articulate(betas, pose)
    torch.cuda.synchronize()
    t0 = time.time()
    m.stage_skin(n, v, rest_verts=fused["rest_verts"])
    torch.cuda.synchronize()
    dt = time.time() - t0
    d = (v - fused["verts"]).abs()
    bad = torch.nonzero(~(d == 0).all(-1))
    print(f"n={n:6d} {dt*1e3:8.2f} ms  max diff {d.nan_to_num(1e9).max().item():.3e}  "
          f"wrong (hand, vertex) {bad.shape[0]}  first {bad[:6].tolist()}", flush=True)
