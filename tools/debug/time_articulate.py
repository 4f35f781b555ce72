"""Debug: articulate_kernel's duration by what runs before it (the bench step
runs it right after blend_skin16, which leaves ~0.6 GB of freshly written verts
behind it).

    python tools/debug/time_articulate.py"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mano-hand_amd"), REPO]
import numpy as np, torch
from mano_amd import ManoHip, synthetic_params
B = 65536
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
betas = torch.randn((B, 10), generator=g, device=dev)
pose = 0.5 * torch.randn((B, 16, 3), generator=g, device=dev)
joints = torch.empty((B, 16, 3), device=dev)
m = ManoHip(synthetic_params(0), device=0)
v = torch.empty((B, 778, 3), device=dev)
m.workspace(B)


def timed(before, jt, n=200):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        before()
        a.record(); m.stage_articulate(betas, pose, joints=jt); b.record()
    torch.cuda.synchronize()
    return float(np.mean([a.elapsed_time(b) for a, b in ev]))


m.stage_articulate(betas, pose)
for _ in range(300):
    m.stage_blend_skin(B, v)
cases = {
    "after articulate, no joints": (lambda: None, None),
    "after articulate, joints": (lambda: None, joints),
    "after blend_skin16, joints": (lambda: m.stage_blend_skin(B, v), joints),
    "after blend_skin16, no joints": (lambda: m.stage_blend_skin(B, v), None),
    "after 64 MB copy, joints": (lambda: v.view(-1)[: 1 << 24].copy_(v.view(-1)[1 << 24: 2 << 24]), joints),
}
for r in range(2):
    for name, (before, jt) in cases.items():
        print(f"{name:32s} {timed(before, jt):.4f} ms", flush=True)
m.close()
