"""Debug: run one forward path K times (no timing) for rocprofv3 --pmc passes.

    python tools/debug/run_path.py <path> [K] [B]

path: unfused (articulate, blend, skin), skin_b2b (the LBS alone, back to
back), staged (articulate, blend_skin16), rest_verts (blend_skin16 with
rest_verts).  65,536 hands of C2 inputs by default; MANO_LIB=<name> loads
mano_amd/<name> instead of libmano_hip.so."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mano-hand_amd"), REPO]
import torch  # noqa: E402
from mano_amd import _abi  # noqa: E402
if os.environ.get("MANO_LIB"):  # another build of the library (A/B), in mano_amd/
    _abi.LIB_PATH = os.path.join(os.path.dirname(_abi.LIB_PATH), os.environ["MANO_LIB"])
from mano_amd import ManoHip, synthetic_params  # noqa: E402

path = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
B = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
m = ManoHip(synthetic_params(0), device=0)
inp = m.synthetic_inputs(1001, 0, B)
betas, pose = inp["betas"], inp["pose"]
v = torch.empty((B, 778, 3), device="cuda:0")
vp = torch.empty((B, 778, 3), device="cuda:0")
m.workspace(B)
m.stage_articulate(betas, pose)
m.stage_blend(B)
for _ in range(K):
    if path == "unfused":
        m.stage_articulate(betas, pose)
        m.stage_blend(B)
        m.stage_skin(B, v)
    elif path == "skin_b2b":
        m.stage_skin(B, v)
    elif path == "staged":
        m.stage_articulate(betas, pose)
        m.stage_blend_skin(B, v)
    elif path == "rest_verts":
        m.stage_blend_skin(B, v, rest_verts=vp)
    else:
        raise SystemExit(f"unknown path {path}")
torch.cuda.synchronize()
m.check_device()
print("done", path, K, B)
