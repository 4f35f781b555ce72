"""The data-parallel path with the HIP kernels: 2 ranks (gloo, sharing cuda:0)
each run the forward on their `shard_range` shard of one global batch and
gather verts + joints to rank 0, which must equal the single-process forward
of the whole batch bit for bit (hands are independent, mano_np.py:79-115;
bench.py's N > 1 layout).  The RCCL variant of the same gather runs only on a
multi-GPU node (the driver's N > 1 bench)."""
import os
import socket
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_TOTAL = 1003  # ragged: the shards end mid-tile


def _inputs():
    rng = np.random.default_rng(11)
    betas = rng.normal(0, 1, (N_TOTAL, 10)).astype(np.float32)
    pose = rng.normal(0, 0.5, (N_TOTAL, 16, 3)).astype(np.float32)
    trans = rng.uniform(-1, 1, (N_TOTAL, 3)).astype(np.float32)
    return betas, pose, trans


def _forward(betas, pose, trans):
    from mano_amd import ManoHip, synthetic_params
    dev = torch.device("cuda", 0)
    m = ManoHip(synthetic_params(0), device=0)
    f = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    out = m.forward(f(betas), f(pose), f(trans), joints=True)
    torch.cuda.synchronize()
    res = out["verts"].cpu(), out["joints"].cpu()
    m.close()
    return res


def _worker(rank, world, port, q):
    for p in (os.path.join(REPO, "mano-hand_amd"), REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from mano_amd.distributed import gather_to_root, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a, b = shard_range(N_TOTAL, rank, world)
        betas, pose, trans = _inputs()
        verts, joints = _forward(betas[a:b], pose[a:b], trans[a:b])
        fv = gather_to_root(verts, N_TOTAL, root=0)
        fj = gather_to_root(joints, N_TOTAL, root=0)
        q.put((rank, None if fv is None else (fv.numpy(), fj.numpy())))
    finally:
        dist.destroy_process_group()


def test_dp2_shards_gather_equal_single_process():
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert got[1] is None
    verts, joints = got[0]
    ref_v, ref_j = _forward(*_inputs())
    assert verts.shape == (N_TOTAL, 778, 3) and joints.shape == (N_TOTAL, 16, 3)
    assert np.array_equal(verts, ref_v.numpy())
    assert np.array_equal(joints, ref_j.numpy())


def test_bench_c4_gather_rehearsal_layout(tmp_path):
    """bench.py's C4 path with 2 ranks (gloo rehearsal, sharing cuda:0):
    GPU 0's gathered verts + joints -- the contiguous per-rank layout
    mano_gather produces -- equal a single-process forward of the global
    batch bit for bit, and the bench line's own gather_check and
    correctness leg report it."""
    import json
    import subprocess
    B, world = 300, 2
    dump = tmp_path / "gather.npz"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(world), "--backend", "gloo",
                        "--workload", "C4", "--batch", str(B), "--steps", "3", "--warmup", "1",
                        "--ramp-seconds", "0", "--no-cpu", "--no-extra", "--no-live-pmc",
                        "--dump-gather", str(dump)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == world and line["config"]["gather_to_gpu0"]
    assert line["gather_check"]["bit_exact"] and line["gather_check"]["hands_checked"] > 0
    assert line["correctness"]["pass"], line["correctness"]
    with np.load(dump) as z:
        gv, gj = z["verts"], z["joints"]
    from mano_amd import ManoHip, synthetic_params
    m = ManoHip(synthetic_params(0), device=0)
    inp = m.synthetic_inputs(1003, 0, B * world)   # C4's seed, global indices 0 .. 599
    out = m.forward(inp["betas"], inp["pose"], None, joints=True)
    torch.cuda.synchronize()
    assert gv.shape == (B * world, 778, 3) and gj.shape == (B * world, 16, 3)
    assert np.array_equal(gv, out["verts"].cpu().numpy())
    assert np.array_equal(gj, out["joints"].cpu().numpy())
    m.close()
