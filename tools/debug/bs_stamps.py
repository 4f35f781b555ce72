"""Debug: per-wave entry/exit clocks of blend_skin16 (a MANO_BS_STAMP=1 build).

    python tools/debug/bs_stamps.py libmano_hip_stamp.so

After 300 warm-up launches at 65,536 hands, one launch's waves: start skew,
exit spread (the tail the slowest SIMDs leave), work per wave vs exit time."""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mano-hand_amd"), REPO]
import numpy as np, torch
from mano_amd import _abi
_abi.LIB_PATH = os.path.join(os.path.dirname(_abi.LIB_PATH), sys.argv[1] if len(sys.argv) > 1 else "libmano_hip_stamp.so")
from mano_amd import ManoHip, synthetic_params
B = int(os.environ.get("HANDS", 65536))
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
betas = torch.randn((B, 10), generator=g, device=dev)
pose = 0.5 * torch.randn((B, 16, 3), generator=g, device=dev)
m = ManoHip(synthetic_params(0), device=0)
v = torch.empty((B, 778, 3), device=dev)
m.stage_articulate(betas, pose)
for _ in range(int(os.environ.get("WARM", 300))):
    m.stage_blend_skin(B, v)
torch.cuda.synchronize()
lib = ctypes.CDLL(_abi.LIB_PATH)
W = 4096
buf = (ctypes.c_ulonglong * (W * 8))()
for rep in range(3):
    m.stage_blend_skin(B, v)
    torch.cuda.synchronize()
    assert lib.mano_debug_bs_stamps(buf, W * 8) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(W, 8).astype(np.int64)
    a = a[a[:, 2] > 0]
    t0 = a[:, 2].min()
    start = (a[:, 2] - t0) / 100.0  # us (100 MHz)
    end = (a[:, 3] - t0) / 100.0
    clk = (a[:, 1] - a[:, 0]) / ((a[:, 3] - a[:, 2]) / 100.0)  # MHz
    units = a[:, 5]
    ranges = a[:, 6]
    hwid = a[:, 4] & 0xFFFFFFFF
    xcc = (a[:, 4] >> 32) & 0xF
    simd = (hwid >> 4) & 3
    cu = (hwid >> 8) & 15
    se = (hwid >> 13) & 7
    print(f"rep {rep}: waves {len(a)}  span {end.max():.1f} us  clock median {np.median(clk):.0f} MHz")
    print(f"  start: median {np.median(start):.2f}  p99 {np.percentile(start, 99):.2f}  max {start.max():.2f} us")
    print(f"  end:   min {end.min():.1f}  p10 {np.percentile(end, 10):.1f}  median {np.median(end):.1f}  "
          f"p90 {np.percentile(end, 90):.1f}  max {end.max():.1f} us")
    for uu in sorted(set(units.tolist())):
        s = units == uu
        print(f"  units {uu}: {s.sum()} waves, end median {np.median(end[s]):.1f} max {end[s].max():.1f}")
    for rr in sorted(set(ranges.tolist())):
        s = ranges == rr
        print(f"  quads {rr}: {s.sum()} waves, end median {np.median(end[s]):.1f} max {end[s].max():.1f}")
    t_first = (a[:, 7] & 0xFFFFFFFF) / clk  # us (cycles / MHz)
    t_pro = (a[:, 7] >> 32) / clk
    print(f"  first-range prologue (entry -> first barrier): median {np.median(t_first):.2f}  p90 "
          f"{np.percentile(t_first, 90):.2f}  max {t_first.max():.2f} us; all range prologues per wave: median "
          f"{np.median(t_pro):.2f} us ({np.median(t_pro / (end - start)) * 100:.1f} % of the wave's time)")
    ex = [np.median(end[xcc == x]) for x in range(8)]
    print("  end median per XCC:", " ".join(f"{e:.1f}" for e in ex))
    # per SIMD (xcc, se, cu, simd): the last exit of its waves
    key = xcc * 1000 + se * 100 + cu * 4 + simd
    last = {}
    for k, e in zip(key.tolist(), end.tolist()):
        last[k] = max(last.get(k, 0), e)
    lv = np.array(list(last.values()))
    print(f"  SIMDs {len(lv)}: last exit min {lv.min():.1f} median {np.median(lv):.1f} max {lv.max():.1f}; "
          f"idle tail = mean(max - last) {np.mean(lv.max() - lv):.1f} us ({np.mean(lv.max() - lv) / lv.max() * 100:.1f} %)")
m.close()
