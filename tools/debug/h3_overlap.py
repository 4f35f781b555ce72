"""Debug (f16x3 fault): what value lands in a wrong vertex of the packed build?

verts and v_posed are views into one NaN-filled buffer with NaN guard bands
around them; after one fused blend_skin_h3 launch (rest_verts requested),
each wrong x coordinate is classified: NaN (never written), equal to a v_posed
value (which one), equal to another verts entry, or other.  Guard bands must
stay NaN (no stray writes).

    python tools/debug/h3_overlap.py libmano_hip_pack.so
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mano-hand_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mano_amd import _abi  # noqa: E402
if len(sys.argv) > 1:
    _abi.LIB_PATH = os.path.join(os.path.dirname(_abi.LIB_PATH), sys.argv[1])
print("library", _abi.LIB_PATH)
from mano_amd import ManoHip, synthetic_params  # noqa: E402

m = ManoHip(synthetic_params(0), device=0, precision="f16x3")
dev = torch.device("cuda", 0)
B, V = 65536, 778
rng = np.random.default_rng(7)
f = lambda a: torch.tensor(a, dtype=torch.float32, device=dev)  # noqa: E731
betas = f(rng.normal(0, 1, (B, 10)))
pose = f(rng.normal(0, 0.6, (B, 16, 3)))
m.stage_articulate(betas, pose)
vp_exact = torch.empty((B, V, 3), device=dev)
m.stage_blend(B, rest_verts=vp_exact)
ref = torch.empty((B, V, 3), device=dev)
m.stage_skin(B, ref, rest_verts=vp_exact)
N, G = B * V * 3, 1 << 20
for rep in range(3):
    big = torch.full((2 * N + 3 * G,), float("nan"), device=dev)
    verts = big[G:G + N].view(B, V, 3)
    vposed = big[2 * G + N:2 * G + 2 * N].view(B, V, 3)
    m.stage_blend_skin(B, verts, rest_verts=vposed)
    torch.cuda.synchronize()
    guards = torch.cat([big[:G], big[G + N:2 * G + N], big[2 * G + 2 * N:]])
    bad = ((verts - ref).abs() > 1e-5).nonzero()
    msg = f"rep {rep}: wrong verts entries {bad.shape[0]}, guard writes {int((~torch.isnan(guards)).sum())}, " \
          f"NaN left in verts {int(torch.isnan(verts).sum())}, v_posed vs exact max {float((vposed - vp_exact).abs().max()):.2e}"
    print(msg)
    if bad.shape[0] == 0:
        continue
    h, v, c = bad[:, 0], bad[:, 1], bad[:, 2]
    got = verts[h, v, c]
    cls = {"nan": int(torch.isnan(got).sum()),
           "= own v_posed": int((got == vposed[h, v, c]).sum()),
           "= own ref y": int((got == ref[h, v, 1]).sum()),
           "= own ref z": int((got == ref[h, v, 2]).sum()),
           "= 0": int((got == 0).sum())}
    # the same coordinate of the same vertex in the other hands of the tile
    tile0 = (h // 16) * 16
    same_tile = 0
    for k in range(16):
        same_tile += int((got == ref[tile0 + k, v, c]).sum())
    cls["= ref of a tile-mate"] = same_tile
    other_v = 0
    for dv in (-16, 16, -48, 48):
        vv = (v + dv).clamp(0, V - 1)
        other_v += int((got == ref[h, vv, c]).sum())
    cls["= ref of vertex +-16/48"] = other_v
    print("   rows%16", torch.bincount(h % 16, minlength=16).tolist(), "coords",
          torch.bincount(c, minlength=3).tolist(), "vert%16", torch.bincount(v % 16, minlength=16).tolist())
    print("   classes", cls)
    i = 0
    print("   example: hand", int(h[i]), "vert", int(v[i]), "coord", int(c[i]), "got", float(got[i]),
          "ref", float(ref[h[i], v[i], c[i]]), "vposed", float(vposed[h[i], v[i], c[i]]))
