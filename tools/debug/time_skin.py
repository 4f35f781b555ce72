"""Debug: time the standalone LBS (stage_skin) of one library build, both precisions.

    python tools/debug/time_skin.py [libmano_hip_<variant>.so]

Prints the mean event-timed duration over 200 launches (after 300 warm-up
launches) at 65,536 hands and checks the result against the fused kernel's
verts for the same v_posed (bit for bit)."""
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
trans = torch.rand((B, 3), generator=g, device=dev)
for prec in os.environ.get("PRECS", "fp32,f16x3").split(","):
    m = ManoHip(synthetic_params(0), device=0, precision=prec)
    fused = m.forward(betas, pose, trans, rest_verts=True)
    vp = fused["rest_verts"].clone()
    v = torch.empty_like(vp)
    m.stage_articulate(betas, pose, trans)
    for _ in range(300):
        m.stage_skin(B, v, rest_verts=vp, trans=trans)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
    for a, b in ev:
        a.record(); m.stage_skin(B, v, rest_verts=vp, trans=trans); b.record()
    torch.cuda.synchronize()
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    ok = torch.equal(v, fused["verts"])
    print(f"{os.path.basename(_abi.LIB_PATH):24s} {prec:6s} skin {ms:.4f} ms  {19440 * B / ms / 1e6:7.1f} GB/s  "
          f"equal_fused={ok}", flush=True)
    m.close()
