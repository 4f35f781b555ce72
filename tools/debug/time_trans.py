"""Debug: time blend_skin16 with per-hand translation (the C5 path) of one library build.

    python tools/debug/time_trans.py [libmano_hip_<variant>.so]

65,536 hands, 300 warm-up + 200 event-bracketed launches; prints the mean and a
digest of verts so builds can be compared bit for bit."""
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
m = ManoHip(synthetic_params(0), device=0)
inp = m.synthetic_inputs(1004, 0, B, trans=True)
betas, pose, trans = inp["betas"], inp["pose"], inp["trans"]
v = torch.empty((B, 778, 3), device=dev)
m.stage_articulate(betas, pose, trans)
for _ in range(300):
    m.stage_blend_skin(B, v, trans=trans)
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
for a, b in ev:
    a.record(); m.stage_blend_skin(B, v, trans=trans); b.record()
torch.cuda.synchronize()
ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
dig = int(v.contiguous().view(torch.int32).to(torch.int64).sum().item()) & 0xFFFFFFFF
print(f"{os.path.basename(_abi.LIB_PATH):24s} blend_skin (trans) {ms:.4f} ms  digest {dig}", flush=True)
m.close()
