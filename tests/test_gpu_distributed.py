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
                        "--workload", "C4", "--batch", str(B), "--steps", "5", "--warmup", "1",
                        "--ramp-seconds", "0", "--cpu-seconds", "1", "--cpu-procs", "2", "--no-extra",
                        "--no-dropin", "--dump-gather", str(dump), "--legs", "off"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == world and line["config"]["gather_to_gpu0"]
    assert line["gather_check"]["bit_exact"] and line["gather_check"]["hands_checked"] > 0
    assert line["correctness"]["pass"], line["correctness"]
    assert line["correctness"]["ranks_checked"] == world
    # the N > 1 line's own measurements: the gather timed on GPU 0, the CPU
    # baseline on rank 0 while rank 1 waits, live HBM traffic of rank 0's kernel
    g = line["gather"]
    assert g["ms"] > 0 and g["sampled_steps"] >= 5 and g["bytes_to_gpu0"] == B * 9528
    assert g["GBs_to_gpu0"] > 0 and g["link_frac"] is not None
    assert line["cpu_baseline"]["value"] > 0 and line["cpu_baseline"]["cores"] == 2
    assert "note" in line["cpu_baseline"]
    assert line["roofline"]["traffic"] > 0, line["roofline"].get("traffic_source")
    assert line["roofline"]["traffic_source"].startswith("measured in this run")
    assert line["process_group"]["backend"] == "gloo" and line["process_group"]["world"] == world
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


@pytest.mark.parametrize("impl", ["sendrecv", "allgather"])
def test_bench_one_rank_nccl_process_group(impl):
    """The RCCL form of the N > 1 code, on one GPU: bench.py under torchrun
    with one rank on the nccl backend and --force-pg runs
    init_process_group("nccl", device_id), AbiGather's id broadcast
    (broadcast_object_list) -> mano_comm_create, the timed gather
    (mano_gather or mano_allgather) with its events, the on-device all_reduce
    of the step time, all_gather_object of the correctness legs, the other
    gather form as the comparison leg (RCCL's ring all-gather runs even at one
    rank), and gather_check on GPU 0's assembled buffers."""
    import json
    import subprocess
    B = 4096
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--force-pg", "--backend", "nccl",
           "--workload", "C4", "--batch", str(B), "--steps", "10", "--warmup", "2", "--ramp-seconds", "0",
           "--gather-impl", impl, "--no-extra", "--no-dropin"]
    if impl == "sendrecv":   # the rank-0 legs of an N > 1 line, through the process-group path
        cmd += ["--cpu-seconds", "1", "--cpu-procs", "2"]
    else:
        cmd += ["--no-cpu", "--no-live-pmc"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["process_group"] == {"backend": "nccl", "world": 1, "forced_at_one_rank": True}
    assert line["config"]["gather_to_gpu0"] and line["n_gpus"] == 1
    assert line["config"]["gather_impl"].startswith({"sendrecv": "mano_gather", "allgather": "mano_allgather"}[impl])
    assert line["gather_check"]["bit_exact"], line["gather_check"]
    assert line["correctness"]["pass"] and line["correctness"]["ranks_checked"] == 1, line["correctness"]
    g = line["gather"]
    # one rank: its shard is computed in place, the timed gather moves nothing
    assert g["impl"] == impl and g["ms"] >= 0 and g["bytes_to_gpu0"] == 0
    c = g["compare"]
    assert c["impl"] == ("allgather" if impl == "sendrecv" else "sendrecv")
    assert c["ms"] > 0 and c["reps"] >= 1 and c["bit_exact"]
    if impl == "sendrecv":
        assert line["cpu_baseline"]["value"] > 0
        assert line["roofline"]["traffic"] > 0
        assert line["roofline"]["traffic_source"].startswith("measured in this run")


def _nccl_worker(rank, world, port, q):
    """Rank `rank` on GPU `rank`: its ragged shard of N_TOTAL hands, gathered
    to rank 0 through the C-ABI's RCCL gather (AbiGather -> mano_gather)."""
    for p in (os.path.join(REPO, "mano-hand_amd"), REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from mano_amd import ManoHip, synthetic_params
    from mano_amd.distributed import AbiGather, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(rank)
    dev = torch.device("cuda", rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    try:
        a, b = shard_range(N_TOTAL, rank, world)
        betas, pose, trans = _inputs()
        m = ManoHip(synthetic_params(0), device=rank)
        f = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
        out = m.forward(f(betas[a:b]), f(pose[a:b]), f(trans[a:b]), joints=True)
        g = AbiGather(rank)
        fv = g.gather(out["verts"], N_TOTAL, root=0)
        fj = g.gather(out["joints"], N_TOTAL, root=0)
        torch.cuda.synchronize()
        q.put((rank, None if fv is None else (fv.cpu().numpy(), fj.cpu().numpy())))
        dist.barrier()
        m.close()
    finally:
        dist.destroy_process_group()


def _visible_gpus():
    # counting devices does not initialise the GPU in this process
    return torch.cuda.device_count()


@pytest.mark.skipif(_visible_gpus() < 2, reason="the RCCL gather across ranks needs 2 GPUs (RCCL refuses two ranks on one)")
@pytest.mark.parametrize("impl", ["sendrecv", "allgather"])
def test_bench_two_gpus_nccl_gather(impl):
    """On a node with 2+ GPUs: bench.py --gpus 2 on the nccl backend with the
    C4 gather -- mano_gather's grouped ncclSend / ncclRecv (or RCCL's ring
    all-gather) between two ranks for real, GPU 0's assembled verts / joints
    checked bit for bit against hands regenerated by global index over both
    ranks' ranges, both ranks' sampled hands against the oracle, and the
    gather's bytes and link figures in the line."""
    import json
    import subprocess
    B = 16384
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "nccl",
           "--workload", "C4", "--batch", str(B), "--steps", "5", "--warmup", "2", "--ramp-seconds", "0",
           "--gather-impl", impl, "--no-extra", "--no-dropin", "--no-cpu", "--no-live-pmc",
           "--leg-global", "C3=131072,C4=65536"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["process_group"]["backend"] == "nccl"
    assert line["gather_check"]["bit_exact"] and line["gather_check"]["ranks"] == 2, line["gather_check"]
    assert line["correctness"]["pass"] and line["correctness"]["ranks_checked"] == 2, line["correctness"]
    g = line["gather"]
    assert g["impl"] == impl and g["ms"] > 0 and g["comm_ranks"] == 2   # RCCL saw both ranks
    assert g["bytes_to_gpu0"] == B * (778 * 3 + 16 * 3) * 4
    assert g["GBs_to_gpu0"] > 0 and g["link_frac"] is not None
    c = g["compare"]
    assert c["bit_exact"] and c["ms"] > 0
    # the multi-GPU legs ran too (smaller than BASELINE's: --leg-global)
    legs = line["legs"]
    assert legs["C3"]["correctness"]["pass"] and legs["C3"]["correctness"]["ranks_checked"] == 2
    lg = legs["C4"]["gather"]
    assert lg["backend"] == "nccl" and lg["comm_ranks"] == 2 and lg["GBs_to_gpu0"] > 0
    assert legs["C4"]["gather_check"]["bit_exact"] and lg["compare"]["bit_exact"]


@pytest.mark.skipif(_visible_gpus() < 2, reason="the RCCL gather across ranks needs 2 GPUs")
def test_abi_gather_ragged_two_gpus():
    """mano_gather between two GPUs with ragged shards (1,003 hands: 502 +
    501): GPU 0's assembled verts / joints equal the single-process forward
    of the whole batch bit for bit."""
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_nccl_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=200) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[1] is None
    verts, joints = got[0]
    ref_v, ref_j = _forward(*_inputs())
    assert np.array_equal(verts, ref_v.numpy())
    assert np.array_equal(joints, ref_j.numpy())


def test_bench_c4_ramp_ends_together():
    """With the C4 gather every step is a collective, so the ranks must run
    the same number of clock-ramp steps: a 1-s ramp of short steps (many
    10-step chunks, each rank reading its own clock) completes on 2 gloo
    ranks with GPU 0's gathered rows intact (ranks that disagreed would
    leave a gather unmatched: a hang, ended by the 200-s watchdog)."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--workload", "C4", "--batch", "256", "--steps", "5", "--warmup", "2",
                        "--ramp-seconds", "1", "--no-cpu", "--no-extra", "--no-dropin", "--no-live-pmc",
                        "--watchdog-seconds", "200", "--legs", "off"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["ramp"]["steps"] > 10, line["ramp"]
    assert line["gather_check"]["bit_exact"]


def test_bench_watchdog_in_a_gpu_run():
    """The watchdog inside a real GPU run: 2 gloo ranks sharing the GPU, rank 1
    stalls outside the clock ramp's all_reduce (--inject-hang 1): rank 0
    prints the status line naming the phase ("ramp") with its phase history,
    both ranks' Python stacks reach stderr, the launcher exits non-zero, all
    well inside the watchdog budget given."""
    import json
    import subprocess
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--batch", "1024", "--steps", "5", "--warmup", "1", "--ramp-seconds", "0.2",
                        "--no-cpu", "--no-extra", "--no-dropin", "--no-live-pmc",
                        "--inject-hang", "1", "--watchdog-seconds", "30", "--pg-timeout-seconds", "200",
                        "--legs", "off"],
                       capture_output=True, text=True, timeout=170, env=env)
    wall = time.monotonic() - t0
    assert r.returncode != 0
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["status"] == "watchdog" and line["phase"] == "ramp" and line["value"] is None
    assert [p[0] for p in line["phases"]][:3] == ["init_process_group", "model_create", "ramp"]
    assert "rank 0/2: watchdog" in r.stderr and r.stderr.count("in run") >= 2
    assert wall < 150


def test_bench_deadline_skips_rank0_legs():
    """--deadline-seconds too short for rank 0's host legs: the line still
    lands (status ok) with every leg it could not fit listed in
    run.skipped_legs, and the timed numbers intact."""
    import json
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--batch", "4096", "--steps", "10",
                        "--warmup", "2", "--ramp-seconds", "0.2", "--no-extra", "--deadline-seconds", "35"],
                       capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["status"] == "ok" and line["value"] > 0 and line["correctness"]["pass"]
    sk = line["run"]["skipped_legs"]
    assert set(sk) == {"live_pmc", "dropin", "cpu_baseline"}, sk
    assert "cpu_baseline" not in line and "dropin" not in line
    assert line["roofline"]["traffic"] is not None            # the committed PMC summary stands in
    assert "skipped" in line["roofline"]["traffic_source"]
    assert line["run"]["wall_s"] < 60


def _legs_run(extra, timeout=400):
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--batch", "4096", "--steps", "5",
                        "--warmup", "1", "--ramp-seconds", "0", "--no-cpu", "--no-extra", "--no-dropin",
                        "--no-live-pmc", *extra], capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


def _check_legs(legs, world, sizes):
    assert set(legs) == {"C3", "C4"}
    for name, n in sizes.items():
        leg = legs[name]
        assert leg["global_batch"] == n and not leg["baseline_size"] and leg["scaling"] == "strong"
        assert sum(leg["hands_per_rank"]) == n and leg["ranks"] == world
        assert leg["value"] > 0 and leg["ms_per_step"] > 0 and leg["forward_ms_rank0"] > 0
        c = leg["correctness"]
        assert c["pass"] and c["ranks_checked"] == world and c["max_abs_err_verts"] <= 1e-5, c
    assert "gather" not in legs["C3"]
    g = legs["C4"]["gather"]
    assert legs["C4"]["gather_check"]["bit_exact"], legs["C4"]["gather_check"]
    assert legs["C4"]["gather_check"]["ranks"] == world
    return g


def test_bench_legs_gloo_two_ranks():
    """The legs of an N > 1 run, rehearsed with 2 gloo ranks sharing the GPU:
    C3 and C4 at ragged sizes (1,003-hand-odd splits), every rank's sampled
    hands vs the oracle, and C4's gather of both ranks' verts + joints into
    GPU 0's contiguous buffers through host memory in pieces -- bit-exact
    against hands regenerated by global index."""
    line = _legs_run(["--gpus", "2", "--backend", "gloo", "--leg-global", "C3=40003,C4=20001"])
    assert line["status"] == "ok" and line["n_gpus"] == 2
    g = _check_legs(line["legs"], 2, {"C3": 40003, "C4": 20001})
    assert g["backend"] == "gloo" and g["ms"] > 0 and g["bytes_to_gpu0"] > 0


def test_bench_legs_one_rank_nccl():
    """The RCCL form of the legs at one rank (--force-pg): C4's mano_gather
    (GPU 0's shard in place), the communicator reporting 1 rank, and the ring
    all-gather comparison bit-exact."""
    line = _legs_run(["--force-pg", "--backend", "nccl", "--legs", "on", "--leg-global", "C3=131072,C4=65536"])
    assert line["process_group"]["backend"] == "nccl"
    g = _check_legs(line["legs"], 1, {"C3": 131072, "C4": 65536})
    assert g["backend"] == "nccl" and g["comm_ranks"] == 1 and g["bytes_to_gpu0"] == 0
    assert g["compare"]["bit_exact"] and g["compare"]["ms"] > 0


def test_bench_leg_hang_keeps_the_headline():
    """A multi-GPU leg that hangs (rank 1 stalls at the start of C4) must not
    cost the run its headline: the watchdog fires inside the leg, rank 0
    prints the line with the measured value, the finished C3 leg and the
    hung one named, and every rank exits 0 (the legs are not part of
    `value`)."""
    import json
    import subprocess
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--batch", "2048", "--steps", "5", "--warmup", "1", "--ramp-seconds", "0",
                        "--no-cpu", "--no-extra", "--no-dropin", "--no-live-pmc",
                        "--leg-global", "C3=8192,C4=4096", "--leg-min-seconds", "5",
                        "--inject-hang-leg", "1", "--watchdog-seconds", "45", "--pg-timeout-seconds", "200"],
                       capture_output=True, text=True, timeout=170, env=env)
    wall = time.monotonic() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["status"] == "ok" and line["value"] > 0 and line["correctness"]["pass"]
    assert line["legs"]["C3"]["correctness"]["pass"]
    assert line["legs"]["hung"]["phase"].startswith("leg_C4")
    assert "C4" not in line["legs"]
    assert wall < 150
