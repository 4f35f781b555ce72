"""Debug: per-step blend_skin16 / articulate durations of the bench's timed
region at the driver's flags (1-s clock ramp, 5 warmup steps, sync, 20 timed
steps each bracketed by events) -- is the first step after the sync slower?

    python tools/debug/time_first_steps.py"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mano-hand_amd"), REPO]
import numpy as np, torch
from mano_amd import ManoHip, synthetic_params
B = 65536
dev = torch.device("cuda", 0)
m = ManoHip(synthetic_params(0), device=0)
inp = m.synthetic_inputs(1001, 0, B)
betas, pose = inp["betas"], inp["pose"]
v = torch.empty((B, 778, 3), device=dev)
j = torch.empty((B, 16, 3), device=dev)
m.workspace(B)
st = torch.cuda.current_stream(dev)


def step(e=None):
    if e: e[0].record(st)
    m.stage_articulate(betas, pose, joints=j)
    if e: e[1].record(st)
    m.stage_blend_skin(B, v)
    if e: e[2].record(st)


for rep in range(3):
    t = time.perf_counter()
    while time.perf_counter() - t < 1.0:
        for _ in range(10):
            step()
        torch.cuda.synchronize()
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(20)]
    torch.cuda.synchronize()
    for e in ev:
        step(e)
    torch.cuda.synchronize()
    bs = [e[1].elapsed_time(e[2]) for e in ev]
    ar = [e[0].elapsed_time(e[1]) for e in ev]
    print(f"rep {rep}: blend_skin16 per step (ms): " + " ".join(f"{x:.3f}" for x in bs), flush=True)
    print(f"        articulate per step (ms):   " + " ".join(f"{x:.3f}" for x in ar), flush=True)
    print(f"        mean all {np.mean(bs):.4f}  steps 0,4,..: {np.mean(bs[0::4]):.4f}  steps 3,7,..: {np.mean(bs[3::4]):.4f}", flush=True)
m.close()
