"""Debug: what per-kernel timing events cost the bench's forward step.

    python tools/debug/time_events.py

The bench's "forward" step (articulate, blend_skin16) at 65,536 hands, K steps
between two syncs, wall time per step, with: no events; the bench's three
events per step (start, between, end); two per step (each step's start is the
previous step's end event); events on every 8th step only; 8 steps captured
in one HIP graph."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mano-hand_amd"), REPO]
import numpy as np, torch
from mano_amd import ManoHip, synthetic_params
B, K = 65536, 400
dev = torch.device("cuda", 0)
m = ManoHip(synthetic_params(0), device=0)
inp = m.synthetic_inputs(1001, 0, B)
betas, pose = inp["betas"], inp["pose"]
v = torch.empty((B, 778, 3), device=dev)
j = torch.empty((B, 16, 3), device=dev)
m.workspace(B)
st = torch.cuda.current_stream(dev)


def run(mode, k):
    evs = []
    prev = None
    for i in range(k):
        e = None
        if mode == "three" or (mode == "sparse8" and i % 8 == 0):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record(st)
        elif mode == "two":
            e = [prev or torch.cuda.Event(enable_timing=True)] + [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            if prev is None:
                e[0].record(st)
        m.stage_articulate(betas, pose, joints=j)
        if e:
            e[1].record(st)
        m.stage_blend_skin(B, v)
        if e:
            e[2].record(st)
            evs.append(e)
            prev = e[2]
    return evs


g = torch.cuda.CUDAGraph()
cs = torch.cuda.Stream(dev)
m.workspace(B, stream=cs)
try:
    with torch.cuda.stream(cs):
        with torch.cuda.graph(g, stream=cs):
            for _ in range(8):
                m.stage_articulate(betas, pose, joints=j, stream=cs)
                m.stage_blend_skin(B, v, stream=cs)
except Exception as exc:  # noqa: BLE001
    print("graph capture failed:", exc, flush=True)
    g = None


def run_graph(k):
    for _ in range(k // 8):
        g.replay()


for mode in ("none", "three", "two", "sparse8", "graph8", "none", "three", "two", "sparse8", "graph8"):
    if mode == "graph8":
        if g is None:
            continue
        run_graph(300)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run_graph(K)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K * 1e3
        print(f"{mode:8s} {dt:.4f} ms/step  {B / dt * 1e3 / 1e6:.1f} M hands/s", flush=True)
        continue
    run(mode, 300)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs = run(mode, K)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K * 1e3
    ks = ""
    if evs:
        a = np.mean([e[0].elapsed_time(e[1]) for e in evs])
        b = np.mean([e[1].elapsed_time(e[2]) for e in evs])
        ks = f"  articulate {a:.4f}  blend_skin16 {b:.4f} ms"
    print(f"{mode:8s} {dt:.4f} ms/step  {B / dt * 1e3 / 1e6:.1f} M hands/s{ks}", flush=True)
m.close()
