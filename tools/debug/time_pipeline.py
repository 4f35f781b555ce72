"""Debug: back-to-back forward steps on one stream vs batches alternating over S streams.

    python tools/debug/time_pipeline.py [libmano_hip_<variant>.so]

Each step is mano_forward's two launches (articulate, blend_skin16) over the
65,536-hand batch; with S streams step i runs on stream i % S with that
stream's own workspace and output buffers, so step i + 1's articulate can
fill step i's blend_skin16 tail.  Wall time of K steps between two syncs."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mano-hand_amd"), REPO]
import numpy as np, torch
from mano_amd import _abi
if len(sys.argv) > 1:
    _abi.LIB_PATH = os.path.join(os.path.dirname(_abi.LIB_PATH), sys.argv[1])
from mano_amd import ManoHip, synthetic_params
B = 65536
K = 400
dev = torch.device("cuda", 0)
m = ManoHip(synthetic_params(0), device=0)
inp = m.synthetic_inputs(1001, 0, B)
betas, pose = inp["betas"], inp["pose"]
streams = [torch.cuda.Stream(dev) for _ in range(4)]
bufs = [(torch.empty((B, 778, 3), device=dev), torch.empty((B, 16, 3), device=dev)) for _ in range(4)]
main = torch.cuda.current_stream(dev)


def run(S, k):
    if S == 0:  # the bench's order: one stream
        for _ in range(k):
            m.stage_articulate(betas, pose, joints=bufs[0][1])
            m.stage_blend_skin(B, bufs[0][0])
        return
    for s in streams[:S]:
        s.wait_stream(main)
    for i in range(k):
        s = streams[i % S]
        v, j = bufs[i % S]
        m.stage_articulate(betas, pose, joints=j, stream=s)
        m.stage_blend_skin(B, v, stream=s)
    for s in streams[:S]:
        main.wait_stream(s)


for S in (0, 1, 2, 3, 0, 2, 3):
    for s in streams:
        m.workspace(B, stream=s)
    run(S, 300)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(S, K)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K * 1e3
    ok = all(torch.equal(bufs[i][0], bufs[0][0]) for i in range(1, max(S, 1)))
    print(f"{os.path.basename(_abi.LIB_PATH):20s} streams {S}  {dt:.4f} ms/step  {B / dt * 1e3 / 1e6:.1f} M hands/s  "
          f"outputs equal {ok}", flush=True)
m.close()
