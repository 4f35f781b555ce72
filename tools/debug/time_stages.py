"""Debug: time every stage kernel of one library build at 65,536 hands.

    python tools/debug/time_stages.py [libmano_hip_<variant>.so]

Per precision: articulate, blend (unfused, v_posed out), skin (standalone
LBS), blend_skin (fused, verts out) and blend_skin with rest_verts -- mean
event-timed duration of 200 launches after 300 warm-up launches, plus a
checksum of each output so builds can be compared for identical bits."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mano-hand_amd"), REPO]
import numpy as np, torch
from mano_amd import _abi
if len(sys.argv) > 1:
    _abi.LIB_PATH = os.path.join(os.path.dirname(_abi.LIB_PATH), sys.argv[1])
from mano_amd import ManoHip, synthetic_params
B = 65536
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
betas = torch.randn((B, 10), generator=g, device=dev)
pose = 0.5 * torch.randn((B, 16, 3), generator=g, device=dev)


def timed(fn, warm=300, reps=200):
    for _ in range(warm):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(); fn(); b.record()
    torch.cuda.synchronize()
    return float(np.mean([a.elapsed_time(b) for a, b in ev]))


def digest(t):
    return int(t.contiguous().view(torch.int32).to(torch.int64).sum().item()) & 0xFFFFFFFF


name = os.path.basename(_abi.LIB_PATH)
for prec in ("fp32", "f16x3"):
    m = ManoHip(synthetic_params(0), device=0, precision=prec)
    v = torch.empty((B, 778, 3), device=dev)
    vp = torch.empty((B, 778, 3), device=dev)
    m.stage_articulate(betas, pose)
    t_art = timed(lambda: m.stage_articulate(betas, pose))
    t_blend = timed(lambda: m.stage_blend(B, rest_verts=vp))
    d_vp = digest(vp)
    t_skin = timed(lambda: m.stage_skin(B, v, rest_verts=vp))
    d_skin = digest(v)
    t_bs = timed(lambda: m.stage_blend_skin(B, v))
    d_bs = digest(v)
    t_bsr = timed(lambda: m.stage_blend_skin(B, v, rest_verts=vp))
    print(f"{name:24s} {prec:6s} articulate {t_art:.4f}  blend {t_blend:.4f}  skin {t_skin:.4f}  "
          f"blend_skin {t_bs:.4f}  +rest {t_bsr:.4f} ms  digests {d_vp:08x} {d_skin:08x} {d_bs:08x}",
          flush=True)
