"""Debug: time mano_forward's fused kernel (stage_blend_skin) of one library build, both precisions.

    python tools/debug/time_forward.py [libmano_hip_<variant>.so]"""
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
ref = None
for prec in ("fp32", "f16x3"):
    m = ManoHip(synthetic_params(0), device=0, precision=prec)
    v = torch.empty((B, int(os.environ.get("VERTS_ROW", 778)), 3), device=dev)
    m.stage_articulate(betas, pose)
    for _ in range(300):
        m.stage_blend_skin(B, v)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
    for a, b in ev:
        a.record(); m.stage_blend_skin(B, v); b.record()
    torch.cuda.synchronize()
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    for _ in range(300):
        m.stage_articulate(betas, pose)
    ev2 = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
    for a, b in ev2:
        a.record(); m.stage_articulate(betas, pose); b.record()
    torch.cuda.synchronize()
    ms_art = float(np.mean([a.elapsed_time(b) for a, b in ev2]))
    if ref is None:
        ref = v.clone()
        # the default library's fp32 result, for the other builds' "vs default"
        refp = "/tmp/time_forward_ref.pt"
        if os.path.basename(_abi.LIB_PATH) == "libmano_hip.so":
            torch.save(ref[:, :778].cpu(), refp)
        if os.path.exists(refp):
            d = (ref[:, :778].cpu() - torch.load(refp, weights_only=True)).abs().max().item()
            print(f"{os.path.basename(_abi.LIB_PATH):24s} fp32 vs default build max {d:.2e}", flush=True)
    err = (v[:, :778] - ref[:, :778]).abs().max().item()
    print(f"{os.path.basename(_abi.LIB_PATH):24s} {prec:6s} blend_skin {ms:.4f} ms  articulate {ms_art:.4f} ms  "
          f"vs fp32 max {err:.2e}", flush=True)
    m.close()
