"""bench.py's launcher and bookkeeping, on CPU (no GPU work).

`bench.py --gpus N` with no WORLD_SIZE must start N ranks itself (the
driver's 1/2/4/8 scaling command); `--launch-check` runs the real launch path
-- torch.distributed.run, one process per rank, gloo barrier -- and exits
before any GPU call."""
import json
import os
import subprocess
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def _last_json(out):
    return json.loads([l for l in out.splitlines() if l.startswith("{")][-1])


@pytest.mark.parametrize("n", [1, 2])
def test_gpus_flag_launches_n_ranks(n):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n),
                        "--backend", "gloo", "--launch-check"], capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == n and line["local_ranks_ok"]


@pytest.mark.parametrize("n", [2, 8])
def test_launch_check_plans_the_multi_gpu_legs(n):
    """Every N > 1 run measures BASELINE's multi-GPU configs after the C2
    headline: the launch path (torchrun, gloo, no GPU) reports the legs each
    rank will run -- C3's 2^24 hands and C4's 2^22 hands split over the N
    ranks (strong scaling, the BASELINE sizes), C4 with the gather to GPU 0."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n),
                        "--backend", "gloo", "--launch-check"], capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    legs = _last_json(r.stdout)["legs"]
    assert set(legs) == {"C3", "C4"}
    c3, c4 = legs["C3"], legs["C4"]
    assert c3["global_batch"] == 2 ** 24 and c3["seed"] == 1002 and not c3["gather_to_gpu0"]
    assert c4["global_batch"] == 2 ** 22 and c4["seed"] == 1003 and c4["gather_to_gpu0"]
    for leg in (c3, c4):
        assert leg["baseline_size"] and leg["scaling"] == "strong"
        assert leg["hands_per_rank"] == [leg["global_batch"] // n] * n
    if n == 8:   # SURVEY.md §8 per-GPU sizes
        assert c3["hands_per_rank"][0] == 2097152 and c4["hands_per_rank"][0] == 524288


def test_legs_plan_flags():
    """One rank: no legs unless asked; --leg-global resizes a leg (and says
    so); ragged splits keep every hand."""
    assert bench.plan_legs(bench.parse([]), 1) == {}
    assert bench.plan_legs(bench.parse(["--legs", "off"]), 8) == {}
    p = bench.plan_legs(bench.parse(["--legs", "on", "--leg-global", "C3=1003,C4=64"]), 3)
    assert p["C3"]["global_batch"] == 1003 and not p["C3"]["baseline_size"]
    assert sum(p["C3"]["hands_per_rank"]) == 1003 and sum(p["C4"]["hands_per_rank"]) == 64
    with pytest.raises(SystemExit):
        bench.parse_leg_global("C9=4")
    a = bench.parse([])
    assert a.leg_min_seconds < a.watchdog_seconds and a.leg_steps >= 1


def test_failure_budgets_inside_driver_lease():
    """The driver kills a bench run at 600 s: a stalled collective must raise
    (process-group timeout) before the watchdog fires, the watchdog before the
    lease ends, and rank 0's host legs end by the deadline (the re-armed
    watchdog at deadline + 30 s still inside 600 s)."""
    a = bench.parse([])
    assert 0 < a.pg_timeout_seconds < a.watchdog_seconds < 600
    assert a.watchdog_seconds <= a.deadline_seconds and a.deadline_seconds + 30 < 600
    # a shard's oracle check (the collective that merges them waits for it) is
    # bounded well inside the process-group timeout: bench.check_sample uses 120 s
    assert 120 < a.pg_timeout_seconds


def _hang_run(extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--launch-check", "--inject-hang", "1", *extra],
                       capture_output=True, text=True, timeout=240, env=env)
    return r, time.monotonic() - t0


def test_hang_path_watchdog_names_phase_and_dumps_both_ranks():
    """Rank 1 stalls outside the all_reduce rank 0 waits in (longer PG timeout):
    both watchdogs fire, rank 0 prints the status line with the phase, both
    ranks' Python stacks reach stderr, the launcher exits non-zero -- well
    inside the default watchdog."""
    r, wall = _hang_run(["--watchdog-seconds", "12", "--pg-timeout-seconds", "200"])
    assert r.returncode != 0
    line = _last_json(r.stdout)
    assert line["status"] == "watchdog" and line["value"] is None and line["rank"] == 0
    assert line["phase"] == "launch_check:all_reduce"
    # rank 0 fires first (the others allow it a grace period); rank 1's stack
    # comes from its own watchdog or from torchrun's SIGTERM after rank 0 exits
    assert "rank 0/2: watchdog" in r.stderr
    assert r.stderr.count("in launch_check") >= 2          # both main threads' stacks
    assert "in all_reduce" in r.stderr                      # rank 0 was inside the collective
    assert wall < bench.parse([]).watchdog_seconds


def test_hang_path_pg_timeout_raises_and_peer_stack_dumped():
    """Process-group timeout shorter than the watchdog: rank 0's collective
    raises, its status line says "error" in the phase, and torchrun's SIGTERM
    to the stalled rank dumps that rank's stack."""
    r, wall = _hang_run(["--watchdog-seconds", "100", "--pg-timeout-seconds", "5"])
    assert r.returncode != 0
    line = _last_json(r.stdout)
    assert line["status"] == "error" and line["phase"] == "launch_check:all_reduce"
    assert "Timed out" in line["error"] or "timeout" in line["error"].lower()
    assert r.stderr.count("in launch_check") >= 2           # rank 0's traceback + rank 1's SIGTERM dump
    assert "bench: rank 1/2 pid" in r.stderr
    assert wall < 100


def test_launch_command_is_torchrun():
    cmd = bench.launch_command(["--gpus", "4", "--steps", "3"], 4)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-3:] == ["--gpus", "4", "--steps", "3"] or cmd[-4:-1] == ["--gpus", "4", "--steps"]


def test_workloads_match_baseline_configs():
    w = bench.WORKLOADS
    assert w["C2"]["hands"] == 65536 and not w["C2"]["trans"]
    assert w["C3"]["hands"] * 8 == 2 ** 24
    assert w["C4"]["hands"] * 8 == 2 ** 22 and w["C4"]["gather"]
    assert w["C5"]["hands"] == 2 ** 20 and w["C5"]["trans"]
    assert bench.parse([]).workload == "C2"          # the metric's config (BASELINE configs[1])
    assert bench.parse([]).gpus == 1


def test_algorithmic_work_constants():
    assert bench.BLEND_FLOP_PER_HAND == 676860
    assert bench.FUSED_MFMA_FLOP_PER_HAND == 975612
    # GEMM 676,860 + LBS 778 x 405 = 315,090 (the roofline's numerator)
    assert bench.LBS_FLOP_PER_HAND == 315090 and bench.FUSED_FLOP_PER_HAND == 991950
    assert bench.SKIN_BYTES_PER_HAND == 19440
    assert bench.FUSED_BYTES_PER_HAND == 10744


def test_traffic_lookup(tmp_path):
    p = tmp_path / "t.json"
    p.write_text(json.dumps({"kernels": {"blend_skin": [
        {"batch": 65536, "hbm_bytes_per_launch": 6.5536e8},
        {"batch": 1048576, "hbm_bytes_per_launch": 2.0 * 1048576 * 1e4}]}}))
    t, src = bench.load_traffic(str(p), "blend_skin", 65536)
    assert t == 6.5536e8 and "65536" in src
    t, src = bench.load_traffic(str(p), "blend_skin", 2097152)   # per-hand bytes of the largest x B
    assert t == pytest.approx(2.0 * 2097152 * 1e4) and "per-hand" in src
    assert bench.load_traffic(str(p), "skin", 65536) == (None, None)
    # round-1 single-batch form
    p.write_text(json.dumps({"batch": 65536, "kernels": {"skin": {"hbm_bytes_per_launch": 5.0}}}))
    assert bench.load_traffic(str(p), "skin", 65536)[0] == 5.0


def test_cpu_share_bounded():
    assert 1 <= bench.cpu_share() <= 16
    assert bench.cpu_share() <= bench.cpu_share(8) <= 128


def test_gather_stats():
    """The C4 line's gather figures: bytes into GPU 0 and per-link rates of the
    two forms (send/recv: one shard per peer link; ring: world - 1 shards per
    link)."""
    B, w = 524288, 8
    shard = B * 9528
    g = bench.gather_stats("sendrecv", w, B, 40.0)
    assert g["shard_bytes"] == shard and g["bytes_to_gpu0"] == 7 * shard and g["links"] == 7
    assert g["GBs_to_gpu0"] == pytest.approx(7 * shard / 0.040 / 1e9)
    assert g["link_GBs"] == pytest.approx(shard / 0.040 / 1e9)
    assert g["link_frac"] == pytest.approx(g["link_GBs"] / 153.0)
    a = bench.gather_stats("allgather", w, B, 200.0)
    assert a["links"] == 8 and a["bytes_landed_total"] == 8 * 7 * shard
    assert a["link_GBs"] == pytest.approx(7 * shard / 0.2 / 1e9)
    one = bench.gather_stats("sendrecv", 1, 4096, 0.1)
    assert one["bytes_to_gpu0"] == 0 and one["link_frac"] is None


def test_child_device_env():
    """The --pmc child at N > 1 sees only rank 0's GPU."""
    assert bench.child_device_env({}, 3)["HIP_VISIBLE_DEVICES"] == "3"
    assert bench.child_device_env({"HIP_VISIBLE_DEVICES": "4,5,6"}, 1)["HIP_VISIBLE_DEVICES"] == "5"
    e = bench.child_device_env({"CUDA_VISIBLE_DEVICES": "2,7"}, 1)
    assert e["CUDA_VISIBLE_DEVICES"] == "7" and "HIP_VISIBLE_DEVICES" not in e


def test_force_pg_and_gather_flags():
    a = bench.parse(["--force-pg", "--gather-impl", "allgather", "--workload", "C4"])
    assert a.force_pg and a.gather_impl == "allgather" and a.gather_compare_reps > 0
    assert bench.parse([]).gather_impl == "sendrecv" and not bench.parse([]).force_pg


def test_pmc_values_parse(tmp_path):
    """bench.py's live roofline.traffic reads rocprofv3's counter CSV: per-dispatch
    values of one counter for the dominant kernel only."""
    import bench
    sub = tmp_path / "host" / "123"
    sub.mkdir(parents=True)
    hdr = "Correlation_Id,Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value\n"
    rows = [
        '1,1,"void mano::(anonymous namespace)::blend_skin16_kernel<false, false>(float const*)",FETCH_SIZE,100\n',
        '2,2,"void mano::(anonymous namespace)::articulate_kernel<false>(float const*)",FETCH_SIZE,7\n',
        '3,3,"void mano::(anonymous namespace)::blend_skin16_kernel<false, false>(float const*)",FETCH_SIZE,300\n',
        '4,3,"void mano::(anonymous namespace)::blend_skin16_kernel<false, false>(float const*)",WRITE_SIZE,9\n',
    ]
    (sub / "p_counter_collection.csv").write_text(hdr + "".join(rows))
    frag = bench.PMC_KERNEL_NAME["blend_skin"]
    assert bench.pmc_values(str(tmp_path), "FETCH_SIZE", frag) == [100.0, 300.0]
    assert bench.pmc_values(str(tmp_path), "WRITE_SIZE", frag) == [9.0]
    assert bench.pmc_values(str(tmp_path), "FETCH_SIZE", bench.PMC_KERNEL_NAME["blend_skin_h3"]) == []


def test_merge_checks_takes_the_worst_rank():
    """bench.py's per-rank correctness legs merge into one rank-0 summary."""
    a = {"max_abs_err_verts": 1e-7, "max_abs_err_joints": 5e-8, "n_sampled": 60, "pass": True,
         "finite": True, "device_status": 0, "worst_hand_verts": 3}
    b = {"max_abs_err_verts": 2e-7, "max_abs_err_joints": 1e-8, "n_sampled": 62, "pass": True,
         "finite": True, "device_status": 0, "worst_hand_verts": 70000}
    m = bench.merge_checks([a, b])
    assert m["max_abs_err_verts"] == 2e-7 and m["max_abs_err_joints"] == 5e-8
    assert m["n_sampled"] == 122 and m["ranks_checked"] == 2 and m["pass"]
    assert m["worst_hand_verts"] == 70000
    bad = dict(b, **{"pass": False, "device_status": 1})
    m = bench.merge_checks([a, bad])
    assert not m["pass"] and m["device_status"] == 1
    assert "error" in bench.merge_checks([a, {"error": "x"}])


def test_sample_indices_cover_edges():
    idx = bench.sample_indices(65536)
    for h in (0, 15, 16, 63, 64, 32767, 32768, 65535):
        assert h in idx
    assert bench.sample_indices(3).tolist() == [0, 1, 2]


def test_pmc_child_measures_the_timed_path_only():
    """The --pmc child must not run the drop-in leg: its batch-1 launches of
    the same kernel would dilute roofline.traffic's per-launch average (round
    3 lines r03g-r03i read 36 MB for 857 MB launches)."""
    args = bench.parse(["--workload", "C2"])
    child = bench.pmc_child_args(args, 65536)
    assert "--no-dropin" in child and "--no-check" in child and "--no-live-pmc" in child
    parsed = bench.parse(child)
    assert parsed.no_dropin and parsed.batch == 65536 and parsed.path == args.path


def test_event_plan_skips_step_zero():
    """The sampled timed steps: at least 5, never step 0 when there is a
    choice (its bracket holds the host's first launch latency)."""
    for steps, ev in [(20, 8), (200, 8), (10, 8), (7, 8), (5, 8), (1, 8), (20, 1)]:
        every, first = bench.event_plan(steps, ev)
        picked = [i for i in range(steps) if i % every == first]
        assert len(picked) >= min(5, steps - (1 if every > 1 else 0)) and len(picked) >= 1
        if every > 1:
            assert 0 not in picked
    assert bench.event_plan(20, 8) == (4, 1)                 # the driver's 20 steps: 1, 5, 9, 13, 17
