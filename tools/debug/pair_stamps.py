"""Debug: where skin_pair's waves spend their cycles (a MANO_PAIR_STAMP=1 build).

    python tools/debug/pair_stamps.py libmano_hip_pstamp.so

After 300 warm-up launches at 65,536 hands (with trans), one launch: per
role (memory wave, compute waves) the cycles from entry to exit and the
share spent polling the LDS hand-over counters."""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mano-hand_amd"), REPO]
import numpy as np, torch
from mano_amd import _abi
_abi.LIB_PATH = os.path.join(os.path.dirname(_abi.LIB_PATH), sys.argv[1] if len(sys.argv) > 1 else "libmano_hip_pstamp.so")
from mano_amd import ManoHip, synthetic_params
B = 65536
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
betas = torch.randn((B, 10), generator=g, device=dev)
pose = 0.5 * torch.randn((B, 16, 3), generator=g, device=dev)
trans = torch.rand((B, 3), generator=g, device=dev)
m = ManoHip(synthetic_params(0), device=0)
vp = m.forward(betas, pose, trans, rest_verts=True)["rest_verts"].clone()
v = torch.empty_like(vp)
m.stage_articulate(betas, pose, trans)
for _ in range(300):
    m.stage_skin(B, v, rest_verts=vp, trans=trans)
torch.cuda.synchronize()
lib = ctypes.CDLL(_abi.LIB_PATH)
W = 256 * 12
buf = (ctypes.c_ulonglong * (W * 8))()
for rep in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    m.stage_skin(B, v, rest_verts=vp, trans=trans)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    assert lib.mano_debug_pair_stamps(buf, W * 8) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(256, 12, 8).astype(np.int64)
    mem, cmp_ = a[:, :4], a[:, 4:]
    for name, r in (("memory", mem), ("compute", cmp_)):
        r = r[r[..., 3] == 1]
        tot, wait, units = r[:, 0], r[:, 1], r[:, 2]
        print(f"rep {rep} ({ms:.4f} ms)  {name:7s} waves {len(r)}: cycles median {np.median(tot):.0f} "
              f"(min {tot.min()} max {tot.max()}), polling {np.median(wait / tot) * 100:.1f} % "
              f"(p10 {np.percentile(wait / tot, 10) * 100:.1f}, p90 {np.percentile(wait / tot, 90) * 100:.1f}), "
              f"units median {np.median(units):.0f}, cycles/unit {np.median(tot / np.maximum(units, 1)):.0f}, "
              f"non-poll cycles/unit {np.median((tot - wait) / np.maximum(units, 1)):.0f}", flush=True)
        if name == "memory":
            u = np.maximum(units, 1)
            print(f"      memory phases per unit: stage / DMA wait {np.median(r[:, 4] / u):.0f}, "
                  f"store {np.median(r[:, 5] / u):.0f}, fetch / DMA issue {np.median(r[:, 6] / u):.0f} cycles", flush=True)
    a[:] = 0
m.close()
