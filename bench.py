"""Throughput benchmark of the MI355X MANO forward pass (driver contract).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload C2|C3|C4|C5]

One step = one forward pass (mano_forward: articulate, then the fused blend
GEMM + LBS kernel) over the workload's hands per GPU, inputs resident in HBM
before the timed region.  Workloads (BASELINE.json configs; per-GPU shard
fixed as N grows, so `scaling` is "weak"):

  C2  65,536 hands per GPU, full pose + per-hand betas, verts + joints (default:
      BASELINE.json configs[1], the metric's config)
  C3  2,097,152 hands per GPU (16M over 8 GPUs), per-shard outputs
  C4  524,288 hands per GPU (4M over 8 GPUs) + gather of verts + joints to GPU 0
      (RCCL, C-ABI mano_gather) inside every timed step
  C5  1,048,576 hands per GPU, per-hand betas + global rotation + translation,
      verts + joints

`--gpus N` with no WORLD_SIZE in the environment launches N ranks itself
(`python -m torch.distributed.run`, one process per GPU, started before this
process touches a GPU); under torchrun each rank reads RANK / LOCAL_RANK /
WORLD_SIZE.  Hand inputs come from the counter-based generator keyed by
(seed, global hand index), so rank r's shard is exactly hands r*B..(r+1)*B-1
of the same global batch at any N.  Shards are independent (no collective on
the hot path).

Before the untimed warmup the bench runs the step for `--ramp-seconds`
(reported as `ramp`): the chip needs ~50 back-to-back launches to reach its
steady clock (profiles/r01_kernel_trace_warmup.txt), so a short `--warmup`
does not leave the timed steps on the ramp; the ramp's length is fixed up
front (agreed by the ranks), and the ramp, the warmup and the opening
barrier run with no idle GPU in between.  `timed_region_rank0` splits the
timed region's host time (issue, sync, closing barrier) and gives the GPU
time per step.

Rank 0 prints ONE JSON line with the whole-node hands/s, the roofline of the
dominant kernel (per-kernel durations from HIP events recorded on the launch
stream around every E-th timed step, E = min(--event-every, steps // 5): every
4th at the driver's 20 steps; its HBM bytes per launch measured in the same run
by two rocprofv3 --pmc passes, FETCH_SIZE and WRITE_SIZE, over a short child
run of this bench on rank 0's GPU after the timed region) and the CPU baseline:
the float64 restatement of mano_np.py (oracle/, "port") timed on this host's
cores by rank 0 at every N (the other ranks wait with idle GPUs).

Every N > 1 run then measures BASELINE's multi-GPU configs as legs, after
the headline and not part of `value` (`legs` in the line; --legs auto|on|off):
C3 = 2^24 hands strong-scaled over the ranks, C4 = 2^22 hands + the gather of
verts + joints to GPU 0 (RCCL mano_gather; the ring all-gather beside it),
each with its own oracle / bit-exact checks.  A failing leg is recorded; a
hung one ends in the watchdog's line, which keeps the headline.

Failure handling with a process group (every N > 1 run): a collective that
stalls raises after --pg-timeout-seconds (240); a rank still inside the
collective phases after --watchdog-seconds (420, from process start) prints a
`"status": "watchdog"` JSON line naming its phase (rank 0 on stdout) and every
thread's Python stack, then exits; a rank that torchrun terminates dumps its
stacks too (SIGTERM).  Rank 0's host legs (PMC passes, drop-in, CPU baseline)
are fitted into --deadline-seconds (540, from process start; the driver's
bench lease is 600 s), a leg that no longer fits is skipped and says so.
"""
import argparse
import datetime
import faulthandler
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time

T_START = time.monotonic()   # process start: the watchdog and the deadline count from here
REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mano-hand_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

# Algorithmic work per hand.
V, NCOL, K = 778, 2334, 145
BLEND_FLOP_PER_HAND = 2 * NCOL * K                 # 676,860
SKIN_BYTES_PER_HAND = NCOL * 4 * 2 + 16 * 12 * 4   # v_posed in + verts out + transforms = 19,440
LBS_T_FLOP_PER_HAND = V * 16 * 12 * 2              # the transform blend (on MFMA when fused) = 298,752
FUSED_MFMA_FLOP_PER_HAND = BLEND_FLOP_PER_HAND + LBS_T_FLOP_PER_HAND  # 975,612
# SURVEY.md §8(d)'s per-hand figure for the fused kernel, the roofline's
# numerator: GEMM 676,860 + LBS 778 x 405 = 315,090 (the transform blend's
# 384 flop per vertex plus the apply's 21, which run on the VALU -- the same
# fp32 datapath and peak as the MFMAs on gfx950).
LBS_FLOP_PER_HAND = V * 405                        # 315,090
FUSED_FLOP_PER_HAND = BLEND_FLOP_PER_HAND + LBS_FLOP_PER_HAND  # 991,950
FUSED_BYTES_PER_HAND = 160 * 4 + 16 * 12 * 4 + NCOL * 4     # X row + transforms in, verts out = 10,744
ARTICULATE_BYTES_PER_HAND = (10 + 48) * 4 + 16 * 12 * 4 + 16 * 3 * 4 + 160 * 4  # in + A + joints + X row = 1,832
PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (= vector) peak, spec
PEAK_HBM_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

WORKLOADS = {
    "C2": {"hands": 65536, "trans": False, "gather": False, "seed": 1001,
           "desc": "C2: full-pose fp32 MANO forward, 65,536 hands per GPU, verts + joints"},
    "C3": {"hands": 2097152, "trans": False, "gather": False, "seed": 1002,
           "desc": "C3: 2,097,152 hands per GPU (16M over 8 GPUs), per-shard verts + joints"},
    "C4": {"hands": 524288, "trans": False, "gather": True, "seed": 1003,
           "desc": "C4: 524,288 hands per GPU (4M over 8 GPUs), RCCL gather of verts + joints to GPU 0"},
    "C5": {"hands": 1048576, "trans": True, "gather": False, "seed": 1004,
           "desc": "C5: 1,048,576 hands per GPU, per-hand betas + global rot + trans, verts + joints"},
}


# The BASELINE configs that need a multi-GPU node (configs[2] and [3]), run at
# every N > 1 as legs after the C2 headline: the GLOBAL batch is fixed and
# split over the ranks (strong scaling), keyed by global hand index.
LEGS = {
    "C3": {"global": 2 ** 24, "seed": 1002, "gather": False,
           "desc": "C3: 16,777,216 hands (2^24) data-parallel over the ranks, per-shard verts + joints "
                   "(no collective)"},
    "C4": {"global": 2 ** 22, "seed": 1003, "gather": True,
           "desc": "C4: 4,194,304 hands (2^22) over the ranks + gather of every rank's verts + joints to GPU 0"},
}


def parse_leg_global(text):
    """'C3=8192,C4=4096' -> {"C3": 8192, "C4": 4096} (--leg-global)."""
    out = {}
    for item in filter(None, (x.strip() for x in (text or "").split(","))):
        name, _, val = item.partition("=")
        if name not in LEGS or not val.isdigit() or int(val) < 1:
            raise SystemExit(f"--leg-global: bad item {item!r} (want C3=N or C4=N, N >= 1)")
        out[name] = int(val)
    return out


def plan_legs(args, world):
    """The legs this run takes and each rank's shard of them (empty at one
    rank unless --legs on)."""
    if args.legs == "off" or (args.legs == "auto" and world <= 1):
        return {}
    from mano_amd.distributed import shard_range
    over = parse_leg_global(args.leg_global)
    plan = {}
    for name, spec in LEGS.items():
        n = over.get(name, spec["global"])
        plan[name] = {"desc": spec["desc"], "global_batch": n, "baseline_size": n == spec["global"],
                      "seed": spec["seed"], "gather_to_gpu0": spec["gather"], "scaling": "strong",
                      "hands_per_rank": [b - a for a, b in (shard_range(n, r, world) for r in range(world))]}
    return plan


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--ramp-seconds", type=float, default=1.0,
                    help="run the step this long before the warmup (clock ramp)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="C2")
    ap.add_argument("--batch", type=int, default=None, help="override hands per GPU per step")
    ap.add_argument("--gather", action="store_true", default=None,
                    help="gather verts+joints to GPU 0 each step (default: the workload's)")
    ap.add_argument("--event-every", type=int, default=8,
                    help="bracket the kernels of every E-th timed step with HIP events (1 = every step; "
                         "each timing event costs the step ~4 us, tools/debug/time_events.py)")
    ap.add_argument("--path", choices=("forward", "api", "unfused", "unfused_separate"), default="forward",
                    help="forward: mano_forward's two kernels, each bracketed by events (default); "
                         "api: one mano_forward call per step; unfused: articulate + blend (v_posed into "
                         "verts) + the LBS in place over verts (ABI 7); unfused_separate: the same with "
                         "v_posed in the workspace and the LBS out of place")
    ap.add_argument("--precision", choices=("fp32", "f16x3"), default="fp32",
                    help="fp32: exact fp32 MFMA (default); f16x3: split-half MFMA "
                         "(include/mano_hip.h MANO_PRECISION_F16X3)")
    ap.add_argument("--model", default=None, help="dump_model.py pickle (default: synthetic seed 0)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline sample per form")
    ap.add_argument("--cpu-procs", type=int, default=None,
                    help="CPU-baseline processes (default: this box's CPU share, at most 16)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--dump-gather", default=None,
                    help="(tests) rank 0 saves GPU 0's gathered verts / joints to this .npz after timing")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the correctness leg (sampled hands of the timed step vs the oracle)")
    ap.add_argument("--no-extra", action="store_true", help="skip the untimed other-path kernel table")
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip the drop-in latency leg (MANOModel.set_params, batch 1, after timing)")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_traffic.json"),
                    help="committed rocprofv3 --pmc summary: roofline.traffic when the live passes fail")
    ap.add_argument("--no-live-pmc", action="store_true",
                    help="skip the two rocprofv3 --pmc passes that measure roofline.traffic in this run")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="process-group backend for N > 1 (gloo: rehearsal, ranks may share a GPU)")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the N ranks, meet in a barrier, print the world and exit (no GPU)")
    ap.add_argument("--force-pg", action="store_true",
                    help="take the process-group path even at one rank (init_process_group with "
                         "device_id, AbiGather's id broadcast, the gather, the on-device all_reduce, "
                         "all_gather_object): a 1-GPU rehearsal of the N > 1 code, under torchrun")
    ap.add_argument("--gather-impl", choices=("sendrecv", "allgather"), default="sendrecv",
                    help="the timed gather: sendrecv = mano_gather (grouped RCCL send/recv, every peer "
                         "straight to GPU 0); allgather = mano_allgather (RCCL ring all-gather)")
    ap.add_argument("--gather-compare-reps", type=int, default=4,
                    help="after timing, run the other gather form this many times and report it "
                         "beside the timed one (0 = skip; RCCL only)")
    ap.add_argument("--watchdog-seconds", type=float, default=420.0,
                    help="with a process group: a rank still in the collective phases this many "
                         "seconds after process start prints a status line and its Python stacks and "
                         "exits (a hang becomes a diagnosed failure inside the driver's 600-s lease; 0 = off)")
    ap.add_argument("--pg-timeout-seconds", type=float, default=240.0,
                    help="init_process_group timeout: a collective that stalls this long raises")
    ap.add_argument("--deadline-seconds", type=float, default=540.0,
                    help="wall-time budget from process start: rank 0's host legs (PMC passes, "
                         "drop-in, CPU baseline) are shortened or skipped to end inside it")
    ap.add_argument("--inject-hang", type=int, default=None,
                    help="(tests) this rank skips a collective and stalls: the launch check's all_reduce, "
                         "or with a process group the clock ramp's")
    ap.add_argument("--inject-hang-leg", type=int, default=None,
                    help="(tests) this rank stalls at the start of leg C4: the watchdog's leg path (the line "
                         "keeps the headline and names the hung leg, every rank exits 0)")
    ap.add_argument("--single-process", action="store_true",
                    help="ONE process and host thread drive --gpus N devices (mano_amd.ManoMultiDevice; "
                         "the gather is one RCCL group from that thread, ABI 6) instead of N torchrun ranks")
    ap.add_argument("--legs", choices=("auto", "on", "off"), default="auto",
                    help="the multi-GPU configs as untimed legs after the headline (BASELINE configs[2..3]: "
                         "C3 = 2^24 hands strong-scaled over the ranks, C4 = 2^22 hands + the gather to GPU 0); "
                         "auto = on when WORLD_SIZE > 1.  Not part of `value`")
    ap.add_argument("--leg-global", default="",
                    help="(tests) override a leg's global batch, e.g. C3=8192,C4=4096 (the line then says "
                         "baseline_size false)")
    ap.add_argument("--leg-steps", type=int, default=5,
                    help="timed steps per leg (after one untimed step); the gloo form of C4 runs its "
                         "host-memory gather once")
    ap.add_argument("--leg-min-seconds", type=float, default=90.0,
                    help="a leg starts only with this many seconds left before --watchdog-seconds "
                         "(rank-agreed); otherwise it is named in run.skipped_legs")
    ap.add_argument("--devices", default=None,
                    help="(--single-process) comma-separated device list (default 0..N-1; repeats allowed "
                         "for a 1-GPU rehearsal, which assembles with peer copies instead of RCCL)")
    return ap.parse_args(argv)


METRIC = "posed hand meshes/sec (whole node)"
WATCHDOG_EXIT = 3


def status_line(status, phase, rank, world, **extra):
    """The JSON line of a run that did not finish (watchdog / error): the
    metric with value null, the phase it was in and how long it had run."""
    line = {"metric": METRIC, "value": None, "unit": "hands/s", "n_gpus": world, "status": status,
            "phase": phase, "rank": rank, "elapsed_s": round(time.monotonic() - T_START, 3)}
    line.update(extra)
    return line


class Watchdog:
    """Per-rank guard of the collective phases of a process-group run.

    `enter(phase)` names what the rank is doing; once armed, a rank still
    running at the deadline prints `status_line("watchdog", phase)` (rank 0 on
    stdout, the others on stderr) and every thread's Python stack, then exits
    with WATCHDOG_EXIT -- so a first multi-GPU run that hangs ends as a
    diagnosed failure before the driver's lease kills it.  The check runs on
    a Python thread (every blocking call of the run -- torch collectives,
    torch.cuda.synchronize, the ctypes RCCL calls -- releases the GIL);
    faulthandler's C timer, 30 s later, is the backstop for a call that does
    not."""

    def __init__(self, rank, world):
        self.rank, self.world = rank, world
        self.phase = "start"
        self.phases = []
        self.deadline = None
        self._thread = None
        # Set once the headline is measured (rank 0: its finished line; the
        # other ranks: {}), with `legs` the dict the legs fill: a watchdog
        # firing inside a leg then prints that line -- the headline intact,
        # the finished legs, the hung one named -- and every rank exits 0.
        self.partial = None
        self.legs = None

    def enter(self, phase):
        self.phase = phase
        self.phases.append([phase, round(time.monotonic() - T_START, 3)])

    def arm(self, at):
        """Fire at monotonic time `at` (None or <= T_START: off).  Ranks other
        than 0 wait 5 s longer, so on a whole-job hang rank 0 reports first:
        its status line is the one on stdout, and torchrun's SIGTERM then
        dumps the others' stacks."""
        if at is None or at <= T_START:
            return
        if self.rank != 0:
            at += 5.0
        self.deadline = at
        faulthandler.dump_traceback_later(max(1.0, at - time.monotonic()) + 30.0, exit=True)
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, name="bench-watchdog", daemon=True)
            self._thread.start()

    def cancel(self):
        self.deadline = None
        faulthandler.cancel_dump_traceback_later()

    def _run(self):
        while True:
            time.sleep(0.25)
            d = self.deadline
            if d is not None and time.monotonic() >= d:
                self.fire()

    def fire(self):
        if self.partial is not None and self.phase.startswith("leg_"):
            # a multi-GPU leg hung (not part of `value`): keep the headline
            if self.rank == 0:
                line = dict(self.partial)
                line["legs"] = dict(self.legs or {})
                line["legs"]["hung"] = {"phase": self.phase, "elapsed_s": round(time.monotonic() - T_START, 3),
                                        "note": "watchdog inside a leg; the headline above is complete"}
                line["status"] = "ok"
                line["run"] = {"wall_s": round(time.monotonic() - T_START, 3), "phases": self.phases,
                               "skipped_legs": {"rank0_legs": "a multi-GPU leg hung (watchdog)"}}
                print(json.dumps(line), flush=True)
            sys.stderr.write(f"bench: rank {self.rank}/{self.world}: watchdog inside {self.phase!r} after "
                             f"{time.monotonic() - T_START:.1f} s; Python stacks of every thread:\n")
            sys.stderr.flush()
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
            sys.stderr.flush()
            os._exit(0)
        line = status_line("watchdog", self.phase, self.rank, self.world, phases=self.phases)
        print(json.dumps(line), file=sys.stdout if self.rank == 0 else sys.stderr, flush=True)
        sys.stderr.write(f"bench: rank {self.rank}/{self.world}: watchdog after {line['elapsed_s']} s "
                         f"in phase {self.phase!r}; Python stacks of every thread:\n")
        sys.stderr.flush()
        faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        sys.stderr.flush()
        os._exit(WATCHDOG_EXIT)


def install_stack_dumps():
    """Fatal signals and torchrun's SIGTERM (sent to the surviving ranks when
    one fails) print every thread's Python stack before the process ends."""
    faulthandler.enable(all_threads=True)
    try:
        faulthandler.register(signal.SIGTERM, all_threads=True, chain=True)
    except (AttributeError, ValueError, RuntimeError):  # pragma: no cover - not on this platform
        pass


def pg_timeout(args):
    return datetime.timedelta(seconds=max(1.0, args.pg_timeout_seconds))


def remaining(args):
    """Seconds left of --deadline-seconds."""
    return T_START + args.deadline_seconds - time.monotonic()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_command(argv, n):
    """torchrun command that re-runs this script as n ranks on one node."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
            os.path.abspath(__file__), *argv]


def cpu_share(n_gpus=1):
    """CPUs this process may use, at most 16 per GPU of the run (the GPU box's
    share per GPU)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(n, 16 * max(1, n_gpus)))


def child_device_env(env, local_dev):
    """`env` for a child process that must see only this rank's GPU: the
    visible-devices variable narrowed to entry `local_dev` (or set to it)."""
    env = dict(env)
    for var in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        if env.get(var):
            ids = [x for x in env[var].split(",") if x.strip()]
            if local_dev < len(ids):
                env[var] = ids[local_dev].strip()
            return env
    env["HIP_VISIBLE_DEVICES"] = str(local_dev)
    return env


XGMI_LINK_GBS = 153.0   # one xGMI link, GB/s per direction (7 links per MI355X)
HAND_OUT_BYTES = (V * 3 + 16 * 3) * 4   # verts + posed joints of one hand = 9,528 B


def gather_stats(impl, world, B, ms):
    """Bandwidth figures of one gather of every rank's verts + joints (B hands
    per rank) that took `ms` on GPU 0.  sendrecv: world - 1 peers each send
    their shard over their own link into GPU 0 (per-link bytes = one shard);
    allgather: RCCL's ring, every link carries world - 1 shards."""
    shard = B * HAND_OUT_BYTES
    to_gpu0 = (world - 1) * shard
    if impl == "allgather":
        links, link_bytes = world, (world - 1) * shard
    else:
        links, link_bytes = world - 1, shard
    out = {"impl": impl, "ms": ms, "shard_bytes": shard, "bytes_to_gpu0": to_gpu0,
           "bytes_landed_total": (world - 1) * shard * (world if impl == "allgather" else 1),
           "links": links, "link_GBs_spec": XGMI_LINK_GBS}
    if ms and ms > 0 and world > 1:
        out["GBs_to_gpu0"] = to_gpu0 / (ms * 1e-3) / 1e9
        out["link_GBs"] = link_bytes / (ms * 1e-3) / 1e9
        out["link_frac"] = out["link_GBs"] / XGMI_LINK_GBS
    else:
        out["GBs_to_gpu0"] = out["link_GBs"] = out["link_frac"] = None
    return out


def cpu_baseline(procs, seconds, timeout=None):
    """float64 restatement of mano_np.py:81-115 on `procs` host cores (oracle/cpu_baseline.py,
    run as a child process so its workers share nothing with the GPU process)."""
    try:
        r = subprocess.run([sys.executable, os.path.join(REPO, "oracle", "cpu_baseline.py"),
                            "--procs", str(procs), "--seconds", str(seconds)],
                           capture_output=True, text=True,
                           timeout=timeout if timeout is not None else 120 + 4 * seconds)
    except subprocess.TimeoutExpired:
        return {"value": None, "error": f"timed out after {timeout} s"}
    if r.returncode != 0:
        return {"value": None, "error": r.stderr[-500:]}
    res = json.loads(r.stdout.strip().splitlines()[-1])
    ph, bt = res["per_hand"], res["batched"]
    return {"value": ph["value"], "unit": "hands/s", "cores": procs, "kind": "port",
            "sample": f"{ph['hands']} hands one at a time (oracle.forward_one: the reference's "
                      f"batch-1 op sequence of mano_np.py:81-115 in float64 numpy) in {procs} "
                      f"processes x {ph['seconds']:.1f} s, OMP_NUM_THREADS=1; "
                      "beta ~ N(0,1), pose ~ N(0,0.5^2)",
            "batched": {"value": bt["value"], "unit": "hands/s", "cores": procs,
                        "sample": f"{bt['hands']} hands in 256-hand float64 BLAS-GEMM batches "
                                  f"(oracle/cpu_baseline.py forward_gemm) in {procs} processes x "
                                  f"{bt['seconds']:.1f} s, OMP_NUM_THREADS=1"}}


def dropin_latency(params, device, calls=300, warmup=30, seed=7):
    """The drop-in's batch-1 call (MANOModel.set_params(pose_abs, shape): host
    float64 in, the two forward kernels on the pinned host blocks (or, when
    they are not device-mapped, H2D + kernels + D2H), float64 attributes
    out) -- config C1's operation on the GPU, timed per call on the host
    clock."""
    from mano_amd import MANOModel
    m = MANOModel.from_params(params, device=device)
    rng = np.random.default_rng(seed)
    poses = rng.normal(0.0, 0.5, (calls + warmup, 16, 3))
    shapes = rng.normal(0.0, 1.0, (calls + warmup, 10))
    for i in range(warmup):
        m.set_params(pose_abs=poses[i], shape=shapes[i])
    ts = []
    for i in range(warmup, warmup + calls):
        t0 = time.perf_counter()
        m.set_params(pose_abs=poses[i], shape=shapes[i])
        ts.append(time.perf_counter() - t0)
    m.engine.close()
    ts = np.sort(np.asarray(ts)) * 1e6
    return {"op": "MANOModel.set_params(pose_abs=(16,3), shape=(10,)) -> verts (778,3) float64, "
                  "with J, R, rest_verts, joints updated (mano_np.py:48-115)",
            "io": "zero_copy" if m._zc.get(False) is not None else ("graph" if m.use_graphs else "eager"),
            "us_per_call_median": float(np.median(ts)), "us_per_call_p90": float(ts[int(0.9 * len(ts))]),
            "us_per_call_mean": float(ts.mean()), "calls": calls}


def sample_indices(B, n_random=48, seed=0):
    """First, last, tile-boundary (16-hand tiles, 64-hand quads), middle and
    random hands of a B-hand shard."""
    edges = [0, 1, 15, 16, 63, 64, B // 2 - 1, B // 2, B - 65, B - 64, B - 17, B - 16, B - 2, B - 1]
    rnd = np.random.default_rng(seed).integers(0, B, n_random)
    return np.unique(np.clip(np.concatenate([edges, rnd]), 0, B - 1))


def event_plan(steps, event_every):
    """(E, first): the timed steps whose kernels get HIP events are
    first, first + E, ... -- at least 5 of them (E = min(--event-every,
    steps // 5)), and not step 0 when there is a choice: the first timed
    step's opening event is reached by an idle GPU right after the sync,
    before the host has issued the kernel behind it, so its bracket would
    hold the host's launch latency (0.035-0.054 ms by events vs 23.6 us by
    rocprof's trace for the articulation, r06f / r06g)."""
    every = max(1, min(event_every, steps // 5))
    return every, (1 % every if steps > 1 else 0)


def check_sample(model, seed, first, B, betas, pose, trans, verts, joints, model_path, with_trans,
                 tol=1e-5):
    """Max |GPU - oracle| over sampled hands of the timed step's outputs: the
    hands' inputs and outputs go to an .npz, the float64 oracle runs in a child
    process (oracle/check_sample.py), so this process never imports oracle/."""
    import tempfile
    import torch
    idx = sample_indices(B)
    ti = torch.as_tensor(idx, device=verts.device)
    f = lambda t: t.index_select(0, ti).cpu().numpy()  # noqa: E731
    arrays = {"index": idx + first, "betas": f(betas), "pose": f(pose), "verts": f(verts),
              "joints": f(joints),
              "model": np.array(os.path.abspath(model_path) if model_path else "synthetic:0")}
    if with_trans and trans is not None:
        arrays["trans"] = f(trans)
    fd, path = tempfile.mkstemp(prefix="mano_check_", suffix=".npz", dir="/tmp")
    os.close(fd)
    try:
        np.savez(path, **arrays)
        # well inside --pg-timeout-seconds: the other ranks wait for this
        # leg in the collective that merges the checks
        try:
            r = subprocess.run([sys.executable, os.path.join(REPO, "oracle", "check_sample.py"), path],
                               capture_output=True, text=True, timeout=120)
        except subprocess.TimeoutExpired:
            return {"error": "oracle/check_sample.py timed out after 120 s"}
        if r.returncode != 0:
            return {"error": r.stderr[-500:]}
        res = json.loads(r.stdout.strip().splitlines()[-1])
    finally:
        os.unlink(path)
    res["tolerance_m"] = tol
    res["pass"] = bool(res["finite"] and res["max_abs_err_verts"] <= tol and res["max_abs_err_joints"] <= tol)
    res["reference"] = ("oracle/mano_oracle.py float64 (mano_np.py:79-115, pinned to the reference's "
                        "outputs by tests/test_oracle_golden.py), the last timed step's outputs")
    return res


def merge_checks(per_rank):
    """Rank 0's summary of every rank's check_sample result: the max errors
    over all shards, pass only if every rank passed."""
    ok = [r for r in per_rank if r and "max_abs_err_verts" in r]
    if len(ok) != len(per_rank):
        return {"error": "a rank's correctness leg failed", "per_rank": per_rank}
    out = dict(max(ok, key=lambda r: r["max_abs_err_verts"]))
    out["max_abs_err_joints"] = max(r["max_abs_err_joints"] for r in ok)
    out["n_sampled"] = sum(r["n_sampled"] for r in ok)
    out["ranks_checked"] = len(ok)
    out["pass"] = all(r["pass"] for r in ok)
    out["finite"] = all(r["finite"] for r in ok)
    out["device_status"] = max(r.get("device_status", 0) for r in ok)
    return out


def check_gather(model, seed, B, world, gv, gj, with_trans, per_rank=64, ranges=None):
    """GPU 0's gathered buffers vs a local forward: from every rank's range
    [r B, (r + 1) B) (or `ranges[r]`) the first 16, last 16 and a random run
    of 32 hands are regenerated by global index and forwarded on this GPU; the
    rows must equal gv / gj bit for bit (hands are independent,
    mano_np.py:79-115)."""
    import torch
    rng = np.random.default_rng(1)
    bad, n, ranks_bad = 0, 0, []
    if ranges is None:
        ranges = [(r * B, (r + 1) * B) for r in range(world)]
    for r, (first, stop) in enumerate(ranges):
        B = stop - first
        if B <= 0:
            continue
        k = min(16, B)
        runs = [(0, k), (max(0, B - k), k)]
        if B > 32:
            runs.append((int(rng.integers(0, B - 32)), 32))
        wrong = 0
        for off, cnt in runs:
            g0 = first + off
            inp = model.synthetic_inputs(seed, g0, cnt, trans=with_trans)
            out = model.forward(inp["betas"], inp["pose"], inp.get("trans"), joints=True)
            dv = (out["verts"] != gv[g0:g0 + cnt]).flatten(1).any(1)
            dj = (out["joints"] != gj[g0:g0 + cnt]).flatten(1).any(1)
            wrong += int((dv | dj).sum())
            n += cnt
        bad += wrong
        if wrong:
            ranks_bad.append(r)
    torch.cuda.synchronize()
    return {"ranks": world, "hands_checked": n, "hands_wrong": bad, "ranks_wrong": ranks_bad,
            "bit_exact": bad == 0,
            "method": "rank 0 regenerates each rank's first 16, last 16 and 32 random consecutive hands "
                      "by global index, forwards them locally, compares with GPU 0's gathered verts / joints"}


def run_legs(args, plan, model, rank, world, dev, local_dev, wd, skipped, out=None):
    """BASELINE's multi-GPU configs, after the headline (not part of `value`).

    C3: the 2^24-hand global batch split over the ranks (rank r: hands
    shard_range(2^24, r, N), Philox seed 1002 by global index), the forward
    (mano_forward: articulate + blend_skin16) timed over --leg-steps between a
    barrier + device sync on both sides, max over ranks -> whole-node hands/s
    at fixed total work; every rank's sampled hands vs the float64 oracle.
    C4: the 2^22-hand batch the same way, each step = forward + the gather of
    every rank's verts + joints to GPU 0 (nccl: mano_gather, one RCCL group of
    peer -> GPU 0 sends over xGMI, GPU 0's shard computed in place; the ring
    mano_allgather timed after it as the comparison; gloo rehearsal: the same
    layout through host memory in bounded pieces, once); GPU 0's rows of every
    rank's range checked bit for bit against hands regenerated by global index.
    Every rank runs this (collectives); returns rank 0's report."""
    import torch
    import torch.distributed as dist
    from mano_amd.distributed import AbiGather, gather_rows_to_root, shard_range
    nccl = args.backend == "nccl"
    red_dev = dev if nccl else "cpu"
    out = {} if out is None else out
    gatherer = None
    last_note = [0.0]

    def note(done, total):
        # a progress line on stderr at most every 20 s (rank 0): a long host
        # gather is not mistaken for a hang
        if rank == 0 and time.monotonic() - last_note[0] > 20.0:
            last_note[0] = time.monotonic()
            print(f"bench: {wd.phase}: gathered {done} of {total} rows per rank "
                  f"({time.monotonic() - T_START:.0f} s)", file=sys.stderr, flush=True)
    def one_leg(name, p):
        nonlocal gatherer
        wd.enter(f"leg_{name}")
        if rank == 0:
            print(f"bench: leg {name}: {p['global_batch']} hands over {world} ranks "
                  f"({time.monotonic() - T_START:.0f} s)", file=sys.stderr, flush=True)
        t_leg = time.monotonic()
        n_total, seed, gather = p["global_batch"], p["seed"], p["gather_to_gpu0"]
        a, b = shard_range(n_total, rank, world)
        Bl = b - a
        inp = model.synthetic_inputs(seed, a, Bl)
        # the forward's own workspace (1,408 B per hand), freed after the leg
        ws = torch.empty(model.forward_workspace_bytes(max(Bl, 1)) + 256, dtype=torch.uint8, device=dev)
        gv = gj = None
        if gather and rank == 0:
            gv = torch.empty((n_total, V, 3), device=dev)
            gj = torch.empty((n_total, 16, 3), device=dev)
            verts, joints = gv[a:b], gj[a:b]          # GPU 0's shard computed in place
        else:
            verts = torch.empty((Bl, V, 3), device=dev)
            joints = torch.empty((Bl, 16, 3), device=dev)
        if gather and nccl and gatherer is None:
            wd.enter(f"leg_{name}:comm_create")
            gatherer = AbiGather(local_dev)
            wd.enter(f"leg_{name}")

        def fwd():
            if Bl:
                model.forward(inp["betas"], inp["pose"], None, joints=True,
                              out={"verts": verts, "joints": joints}, workspace=ws)

        def gath():
            if nccl:
                gatherer.gather(verts, n_total, root=0, out=gv)
                gatherer.gather(joints, n_total, root=0, out=gj)
            else:
                gather_rows_to_root(verts, n_total, out=gv, root=0, progress=note)
                gather_rows_to_root(joints, n_total, out=gj, root=0)

        host_gather = gather and not nccl
        steps = 1 if host_gather else max(1, args.leg_steps)
        stream = torch.cuda.current_stream(dev)
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
        gather_host_s = []
        if not host_gather:       # one untimed step (C4 on RCCL: RCCL sets up its channels)
            fwd()
            if gather:
                gath()
        # no sync before the barrier: the GPU works through the rendezvous (the
        # untimed step warms the clock; an idle gap would cool it again)
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for e in evs:
            e[0].record(stream)
            fwd()
            e[1].record(stream)
            if gather:
                if host_gather:
                    torch.cuda.synchronize()
                    tg = time.perf_counter()
                    gath()
                    torch.cuda.synchronize()
                    gather_host_s.append(time.perf_counter() - tg)
                else:
                    gath()
            e[2].record(stream)
        torch.cuda.synchronize()
        dist.barrier()
        dt = time.perf_counter() - t0
        t = torch.tensor([dt], device=red_dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        fwd_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
        res = {"desc": p["desc"], "global_batch": n_total, "baseline_size": p["baseline_size"], "seed": seed,
               "ranks": world, "hands_per_rank": p["hands_per_rank"], "scaling": "strong",
               "value": n_total * steps / dt, "unit": "hands/s", "per_gpu_hands_s": n_total * steps / dt / world,
               "steps": steps, "ms_per_step": dt / steps * 1e3, "forward_ms_rank0": fwd_ms,
               "forward_hands_s_rank0": Bl / (fwd_ms * 1e-3) if Bl and fwd_ms > 0 else None,
               "path": "mano_forward (articulate + blend_skin16)" + (" + gather to GPU 0" if gather else ""),
               "timing": "barrier + device sync on both sides of the timed steps, max over ranks; the leg is "
                         "not part of the headline value"}
        if gather:
            per = -(-n_total // world)
            if host_gather:
                g = gather_stats("sendrecv", world, per, float(np.mean(gather_host_s)) * 1e3)
                g.update({"backend": "gloo", "form": "gloo rehearsal: gather_rows_to_root through host memory "
                                                     "in 32,768-row pieces (the mano_gather layout)",
                          "timing": "host clock around the gather with device syncs (not an xGMI figure)"})
            else:
                gms = [e[1].elapsed_time(e[2]) for e in evs]
                g = gather_stats("sendrecv", world, per, float(np.mean(gms)))
                g.update({"backend": "nccl", "ms_min": float(np.min(gms)), "ms_max": float(np.max(gms)),
                          "form": "mano_gather: one RCCL group of ncclSend (peers) / ncclRecv (GPU 0), each "
                                  "peer over its own xGMI link; GPU 0's shard in place",
                          "comm_ranks": gatherer.info()[0],
                          "timing": "HIP events on rank 0's stream around the gather of each timed step"})
            res["gather"] = g
        # every rank's sampled hands of its shard vs the float64 oracle
        wd.enter(f"leg_{name}:correctness")
        chk = (check_sample(model, seed, a, Bl, inp["betas"], inp["pose"], None, verts, joints,
                            args.model, False) if Bl else {"max_abs_err_verts": 0.0, "max_abs_err_joints": 0.0,
                                                          "n_sampled": 0, "pass": True, "finite": True})
        chk["device_status"] = model.device_status(clear=True)
        chk["pass"] = bool(chk.get("pass")) and chk["device_status"] == 0
        per_rank = [None] * world
        dist.all_gather_object(per_rank, chk)
        res["correctness"] = merge_checks(per_rank)
        if gather and rank == 0:
            ranges = [shard_range(n_total, r, world) for r in range(world)]
            res["gather_check"] = check_gather(model, seed, None, world, gv, gj, False, ranges=ranges)
        if gather and nccl and args.gather_compare_reps > 0 and n_total % world == 0:
            # the ring all-gather of the same shards (report both)
            wd.enter(f"leg_{name}:allgather_compare")
            av = torch.empty((n_total, V, 3), device=dev)
            aj = torch.empty((n_total, 16, 3), device=dev)
            gatherer.allgather(verts, out=av)
            gatherer.allgather(joints, out=aj)
            torch.cuda.synchronize()
            dist.barrier()
            cev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.gather_compare_reps)]
            for e in cev:
                e[0].record(stream)
                gatherer.allgather(verts, out=av)
                gatherer.allgather(joints, out=aj)
                e[1].record(stream)
            torch.cuda.synchronize()
            cms = [e[0].elapsed_time(e[1]) for e in cev]
            cmp_info = gather_stats("allgather", world, n_total // world, float(np.mean(cms)))
            cmp_info.update({"ms_min": float(np.min(cms)), "ms_max": float(np.max(cms)), "reps": len(cms),
                             "form": "mano_allgather: RCCL ring ncclAllGather, every rank receives the batch"})
            if rank == 0:
                ranges = [shard_range(n_total, r, world) for r in range(world)]
                c = check_gather(model, seed, None, world, av, aj, False, ranges=ranges)
                cmp_info["bit_exact"], cmp_info["hands_checked"] = c["bit_exact"], c["hands_checked"]
            res["gather"]["compare"] = cmp_info
            del av, aj
            dist.barrier()
        res["wall_s"] = round(time.monotonic() - t_leg, 3)
        return res

    for name, p in plan.items():
        # the ranks agree to start a leg (it must end before the watchdog)
        left = (T_START + args.watchdog_seconds - time.monotonic()) if args.watchdog_seconds > 0 else 1e9
        go = torch.tensor([1 if left >= args.leg_min_seconds else 0], device=red_dev, dtype=torch.int32)
        dist.all_reduce(go, op=dist.ReduceOp.MIN)
        if not int(go.item()):
            skipped[f"leg_{name}"] = (f"{left:.0f} s left before --watchdog-seconds on rank {rank} "
                                      f"(a leg needs --leg-min-seconds {args.leg_min_seconds:.0f})")
            continue
        if args.inject_hang_leg == rank and name == "C4":
            wd.enter("leg_C4")
            while True:       # (tests) this rank stalls outside the leg's first collective
                time.sleep(0.5)
        try:
            out[name] = one_leg(name, p)
        except Exception as e:   # a symmetric failure (e.g. RCCL refused): the headline stands
            out[name] = {"error": f"{type(e).__name__}: {e}"[:500], "phase": wd.phase,
                         "wall_s": round(time.monotonic() - T_START, 3)}
            print(f"bench: rank {rank}: leg {name} failed in {wd.phase}: {type(e).__name__}: {e}",
                  file=sys.stderr, flush=True)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()     # the leg's buffers are gone with one_leg's frame
    if gatherer is not None:
        gatherer.close()
    return out


def load_traffic(path, kernel, batch):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc summary
    (profiles/pmc_traffic.json, tools/pmc_traffic.py): the entry measured at this
    batch, else the per-hand bytes of the largest measured batch x batch."""
    try:
        with open(path) as f:
            data = json.load(f)
        ents = data["kernels"][kernel]
    except (OSError, KeyError, ValueError, TypeError):
        return None, None
    if isinstance(ents, dict) and "batch" in data:  # round-1 single-batch form
        ents = [dict(ents, batch=data["batch"])]
    for e in ents:
        if int(e["batch"]) == batch:
            return float(e["hbm_bytes_per_launch"]), f"rocprofv3 --pmc at {batch} hands"
    if not ents:
        return None, None
    e = max(ents, key=lambda x: int(x["batch"]))
    return (float(e["hbm_bytes_per_launch"]) / int(e["batch"]) * batch,
            f"rocprofv3 --pmc per-hand bytes at {e['batch']} hands x {batch}")


# Demangled-name fragment of each dominant kernel (rocprofv3 Kernel_Name).
PMC_KERNEL_NAME = {"blend_skin": "::blend_skin16_kernel<", "blend_skin_h3": "::blend_skin_h3_kernel<",
                   "blend": "::blend_kernel(", "skin": "::skin_pair_kernel<", "mano_forward": "::blend_skin16_kernel<",
                   "blend_separate": "::blend_kernel(", "skin_separate": "::skin_pair_kernel<"}


def pmc_values(d, counter, name_fragment):
    """Per-dispatch values of `counter` for kernels whose demangled name holds
    `name_fragment`, from the rocprofv3 --output-format csv tree under `d`."""
    import csv
    vals = []
    for root, _, files in os.walk(d):
        for fn in files:
            if fn.endswith("counter_collection.csv"):
                with open(os.path.join(root, fn)) as f:
                    vals += [float(row["Counter_Value"]) for row in csv.DictReader(f)
                             if name_fragment in row["Kernel_Name"] and row["Counter_Name"] == counter]
    return vals


def pmc_child_args(args, batch):
    """bench.py arguments of the --pmc child: the timed path's launches only
    (no drop-in leg, whose batch-1 launches of the same kernel would dilute
    the per-launch average; no correctness, CPU or extra-table legs)."""
    return ["--workload", args.workload, "--batch", str(batch), "--precision", args.precision,
            "--path", args.path, "--steps", "3", "--warmup", "1", "--ramp-seconds", "0",
            "--no-cpu", "--no-extra", "--no-live-pmc", "--no-check", "--no-dropin"]


def live_traffic(args, batch, name_fragment, timeout=120, local_dev=0):
    """HBM bytes per launch of the dominant kernel measured in this run: rocprofv3
    --pmc FETCH_SIZE and --pmc WRITE_SIZE as two separate passes (the counter
    budget of one pass, MI355X_MICROARCH.md) over a short child run of this bench
    at the same workload, batch, path and precision, started after the timed
    region.  hbm_read = 2 x FETCH_SIZE x 1 KB (gfx950 counts half of a wide
    coalesced read, same guide), hbm_write = WRITE_SIZE x 1 KB, averaged over the
    kernel's dispatches.  Returns (bytes, detail) or (None, reason)."""
    import shutil
    import tempfile
    if "ROCP_TOOL_LIBRARIES" in os.environ or "ROCPROF_OUTPUT_PATH" in os.environ:
        return None, "already running under rocprofv3 (no nested profiler)"
    rp = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(rp):
        return None, "rocprofv3 not found"
    child = [sys.executable, os.path.abspath(__file__), *pmc_child_args(args, batch)]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK",
                        "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    env = child_device_env(env, local_dev)   # at N > 1: only rank 0's GPU
    env["TMPDIR"] = "/tmp"
    kb = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="mano_pmc_", dir="/tmp")
        try:
            r = subprocess.run([rp, "--pmc", counter, "-d", d, "-o", "p", "--output-format", "csv", "--", *child],
                               capture_output=True, text=True, timeout=timeout, env=env, cwd="/tmp")
            if r.returncode != 0:
                return None, f"rocprofv3 --pmc {counter} rc {r.returncode}: {r.stderr[-300:]}"
            vals = pmc_values(d, counter, name_fragment)
            if not vals:
                return None, f"no {counter} rows for {name_fragment}"
            kb[counter] = sum(vals) / len(vals)
        except subprocess.TimeoutExpired:
            return None, f"rocprofv3 --pmc {counter} timed out"
        finally:
            shutil.rmtree(d, ignore_errors=True)
    rd, wr = 2.0 * kb["FETCH_SIZE"] * 1024, kb["WRITE_SIZE"] * 1024
    return rd + wr, {"read": rd, "write": wr, "fetch_size_kb": kb["FETCH_SIZE"],
                     "write_size_kb": kb["WRITE_SIZE"]}


def launch_check(args, wd):
    """--launch-check: the N ranks meet over gloo and rank 0 prints the world
    (no GPU).  With --inject-hang R, rank R skips the all_reduce and stalls:
    the hang path of the watchdog / process-group timeout, tested on CPU."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        wd.enter("launch_check:init_process_group")
        dist.init_process_group("gloo", timeout=pg_timeout(args))
        t = torch.tensor([rank], dtype=torch.int64)
        wd.enter("launch_check:all_reduce")
        if args.inject_hang == rank:
            while True:       # a rank stuck outside the collective (e.g. in a kernel)
                time.sleep(0.5)
        dist.all_reduce(t)
        total = int(t.item())
        wd.enter("launch_check:barrier")
        dist.barrier()
        dist.destroy_process_group()
    else:
        total = 0
    wd.cancel()
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "rank_sum": total,
                          "local_ranks_ok": total == world * (world - 1) // 2,
                          "legs": plan_legs(args, world)}), flush=True)


def main(argv=None):
    raw = sys.argv[1:] if argv is None else argv
    args = parse(raw)
    if args.single_process:
        return run_single_process(args)
    if "WORLD_SIZE" not in os.environ and (args.gpus > 1 or args.force_pg):
        # Launch N ranks; this process never touches a GPU (it only waits).
        sys.exit(subprocess.run(launch_command(raw, args.gpus)).returncode)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    wd = Watchdog(rank, world)
    guarded = world > 1 or args.force_pg
    if guarded:
        # A rank stuck in a collective (RCCL init, the gather, a barrier)
        # prints its phase and every thread's Python stack and exits, so a
        # first multi-GPU run that hangs leaves a diagnosis instead of a
        # silent kill at the driver's limit.
        install_stack_dumps()
        # ties a SIGTERM stack dump (no rank in it) to torchrun's pid table
        print(f"bench: rank {rank}/{world} pid {os.getpid()} local_rank "
              f"{os.environ.get('LOCAL_RANK', '0')}", file=sys.stderr, flush=True)
        if args.watchdog_seconds > 0:
            wd.arm(T_START + args.watchdog_seconds)
    try:
        if args.launch_check:
            return launch_check(args, wd)
        return run(args, wd)
    except Exception as e:
        if guarded or rank == 0:
            line = status_line("error", wd.phase, rank, world, error=f"{type(e).__name__}: {e}"[:500],
                               phases=wd.phases)
            print(json.dumps(line), file=sys.stdout if rank == 0 else sys.stderr, flush=True)
        raise


def run_single_process(args):
    """--single-process: one process and ONE host thread drive N devices
    (mano_amd.multi_device.ManoMultiDevice).  A step = every device's forward
    (articulate + blend_skin16 on its own stream, its contiguous shard of
    hands r*B .. (r+1)*B - 1 of the counter-based batch) and, with the
    workload's gather, the assembly of all verts + joints on device 0 by ONE
    RCCL group issued from this thread (mano_group_start / mano_gather x N /
    mano_group_end; peer copies when a device is listed twice).  Timed like
    the process-per-GPU form: K steps between device-wide syncs of every GPU."""
    import torch
    from mano_amd import ManoMultiDevice, load_dump, synthetic_params
    wl = WORKLOADS[args.workload]
    B = args.batch if args.batch else wl["hands"]
    n = args.gpus
    devices = ([int(x) for x in args.devices.split(",")] if args.devices else list(range(n)))
    if len(devices) != n:
        raise SystemExit(f"--devices lists {len(devices)} devices for --gpus {n}")
    gather = wl["gather"] if args.gather is None else args.gather
    impl = "rccl" if len(set(devices)) == len(devices) else "copy"
    with_trans = wl["trans"]
    params = load_dump(args.model) if args.model else synthetic_params(0)
    md = ManoMultiDevice(params, devices=devices, precision=args.precision)
    n_total = B * n
    ranges = md.shard_ranges(n_total)
    inps = [e.synthetic_inputs(wl["seed"], a, b - a, trans=with_trans, stream=s)
            for e, s, (a, b) in zip(md.engines, md.streams, ranges)]
    outs, assembled = None, None
    if gather:
        _, outs, assembled = md._alloc_outputs(n_total, True, impl)
    else:
        outs = [{"verts": torch.empty((b - a, V, 3), device=torch.device("cuda", d)),
                 "joints": torch.empty((b - a, 16, 3), device=torch.device("cuda", d))}
                for d, (a, b) in zip(devices, ranges)]
    for e, (a, b) in zip(md.engines, ranges):
        e.workspace(b - a)
    if gather and impl == "rccl":
        md.comms()
    keys = ["verts", "joints"]

    def step(marks=None):
        s0 = md.streams[0]
        if marks is not None:
            marks[0].record(s0)
        for i, (e, s) in enumerate(zip(md.engines, md.streams)):
            inp, o = inps[i], outs[i]
            e.stage_articulate(inp["betas"], inp["pose"], inp.get("trans"), joints=o["joints"], stream=s)
            if marks is not None and i == 0:
                marks[1].record(s0)
            e.stage_blend_skin(b_of(i), o["verts"], trans=inp.get("trans"), stream=s)
            if marks is not None and i == 0:
                marks[2].record(s0)
        if gather:
            if impl == "rccl":
                md.comms().gather([[outs[i][k] for k in keys] for i in range(n)],
                                  [assembled[k] for k in keys], 0, md.streams)
            else:
                for i in range(1, n):
                    a, b = ranges[i]
                    s0.wait_stream(md.streams[i])
                    with torch.cuda.stream(s0):
                        for k in keys:
                            assembled[k][a:b].copy_(outs[i][k], non_blocking=True)
                for i in range(1, n):
                    md.streams[i].wait_stream(s0)   # the next step's writes follow the copies
            if marks is not None:
                marks[3].record(s0)

    def b_of(i):
        return ranges[i][1] - ranges[i][0]

    def sync_all():
        for d in sorted(set(devices)):
            torch.cuda.synchronize(d)

    t_ramp = time.perf_counter()
    n_ramp = 0
    while time.perf_counter() - t_ramp < args.ramp_seconds or n_ramp == 0:
        for _ in range(10):
            step()
        n_ramp += 10
        sync_all()
    t_ramp = time.perf_counter() - t_ramp
    for _ in range(args.warmup):
        step()
    sync_all()
    every, first = event_plan(args.steps, args.event_every)
    n_marks = 4 if gather else 3
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(n_marks)] if i % every == first else None
              for i in range(args.steps)]
    sync_all()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(events[i])
    sync_all()
    dt = time.perf_counter() - t0
    sampled = [e for e in events if e is not None]
    ms = {"articulate": float(np.mean([e[0].elapsed_time(e[1]) for e in sampled])),
          "blend_skin": float(np.mean([e[1].elapsed_time(e[2]) for e in sampled]))}
    if gather:
        ms["gather"] = float(np.mean([e[2].elapsed_time(e[3]) for e in sampled]))
    device_status = max(e.device_status(clear=True) for e in md.engines)
    checks = []
    if not args.no_check:
        for i, e in enumerate(md.engines):
            a, b = ranges[i]
            src = ({k: assembled[k][a:b] for k in keys} if gather else outs[i])
            checks.append(check_sample(e, wl["seed"], a, b - a, inps[i]["betas"], inps[i]["pose"],
                                       inps[i].get("trans"), src["verts"], src["joints"], args.model,
                                       with_trans))
        correctness = merge_checks(checks)
        correctness["pass"] = bool(correctness.get("pass")) and device_status == 0
    else:
        correctness = None
    a_fl = FUSED_FLOP_PER_HAND * B / (ms["blend_skin"] * 1e-3) / 1e12 if args.precision == "fp32" else None
    line = {
        "metric": METRIC, "value": n_total * args.steps / dt, "unit": "hands/s", "n_gpus": n,
        "steps": args.steps, "warmup": args.warmup, "ramp": {"seconds": t_ramp, "steps": n_ramp},
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.precision,
        "data": "synthetic (random-init MANO arrays of the official shapes, seed 0; Philox inputs keyed by "
                "(seed, global hand index), generated on each device)",
        "config": {"workload": wl["desc"] if B == wl["hands"] else f"{args.workload} at {B} hands per GPU",
                   "hands_per_gpu": B, "global_batch": n_total, "outputs": "verts+joints", "trans": with_trans,
                   "path": "forward", "gather_to_gpu0": bool(gather),
                   "gather_impl": (None if not gather else
                                   "one RCCL group of mano_gather from this thread" if impl == "rccl"
                                   else "peer copies (a device listed twice)"),
                   "parallelism": f"dp{n}"},
        "process_model": {"single_process": True, "host_threads": 1, "devices": devices,
                          "streams": "one per device", "comm": "mano_comm_create_all" if gather and impl == "rccl"
                          else None},
        "kernels_device0": {k: {"ms": v} for k, v in ms.items()},
        "roofline": ({"kernel": "blend_skin16_kernel", "bound": "mfma", "achieved": a_fl,
                      "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": a_fl / PEAK_FP32_TFLOPS,
                      "algorithmic_per_hand": FUSED_FLOP_PER_HAND, "device": devices[0]} if a_fl else None),
        "correctness": correctness, "device_status": device_status, "status": "ok",
        "run": {"wall_s": round(time.monotonic() - T_START, 3)},
    }
    if gather and n > 1:
        line["gather"] = gather_stats("sendrecv", n, B, ms["gather"])
        line["gather"]["form"] = line["config"]["gather_impl"]
    print(json.dumps(line), flush=True)
    md.close()


def run(args, wd):
    """One benchmark run of this rank (main() holds the watchdog around it)."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus not in (1, world):
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}", file=sys.stderr)
    wl = WORKLOADS[args.workload]
    B = args.batch if args.batch else wl["hands"]
    gather = wl["gather"] if args.gather is None else args.gather
    with_trans = wl["trans"]
    # The process-group path: every N > 1 run, and with --force-pg a 1-rank
    # rehearsal of the same code (RCCL communicator, id broadcast, gather,
    # device all_reduce, all_gather_object) on one GPU.
    dist_on = world > 1 or args.force_pg
    # One process per GPU.  `--backend gloo` is a control-flow rehearsal mode
    # (several ranks may share one GPU); the real multi-GPU run uses RCCL.
    ndev = torch.cuda.device_count()
    local_dev = local if args.backend == "nccl" else local % max(ndev, 1)
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    end_group = None
    if dist_on:
        wd.enter("init_process_group")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=pg_timeout(args))
        else:
            dist.init_process_group("gloo", timeout=pg_timeout(args))
        # The last meeting of the run waits for rank 0's host legs (minutes of
        # CPU work, no GPU): a gloo group whose timeout covers the deadline,
        # so the RCCL group's short timeout never fires on a healthy run.
        try:
            end_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(
                seconds=max(60.0, args.deadline_seconds + 60.0)))
        except Exception as e:  # pragma: no cover - gloo unavailable on this node
            # the run goes on; the end barrier then uses the default group (its
            # timeout may be shorter than rank 0's host legs: they are fitted
            # into --deadline-seconds, and a timeout there ends a finished run)
            print(f"bench: rank {rank}: no gloo end group ({type(e).__name__}: {e}); "
                  "the end barrier uses the default group", file=sys.stderr, flush=True)
            end_group = None

    wd.enter("model_create")
    from mano_amd import ManoHip, load_dump, synthetic_params
    from mano_amd.distributed import AbiGather, all_gather, gather_to_root
    params = load_dump(args.model) if args.model else synthetic_params(0)
    model = ManoHip(params, device=local_dev, precision=args.precision)

    # Shard r = global hands r*B .. (r+1)*B - 1 of one counter-based batch.
    inp = model.synthetic_inputs(wl["seed"], rank * B, B, trans=with_trans)
    betas, pose, trans = inp["betas"], inp["pose"], inp.get("trans")
    verts = torch.empty((B, V, 3), device=dev)
    joints = torch.empty((B, 16, 3), device=dev)
    stream = torch.cuda.current_stream(dev)
    model.workspace(B)  # allocated before timing (covers every path)
    gatherer, gv, gj = None, None, None
    gather_on = bool(gather and dist_on)
    impl = args.gather_impl
    if gather_on:
        if args.backend == "nccl":
            wd.enter("comm_create")
            gatherer = AbiGather(local_dev)
        if rank == 0 or impl == "allgather":
            # the assembled buffers (rank r's rows at r*B), allocated once: GPU 0's
            # (mano_gather), or every GPU's (mano_allgather)
            gv = torch.empty((B * world, V, 3), device=dev)
            gj = torch.empty((B * world, 16, 3), device=dev)
            # this rank's shard is computed in place, in its rows of the
            # assembled buffers: the gather moves only the peers' shards
            verts = gv[rank * B:(rank + 1) * B]
            joints = gj[rank * B:(rank + 1) * B]

    def do_gather(which):
        if gatherer is not None:
            if which == "allgather":   # RCCL ring, every rank gets the batch
                gatherer.allgather(verts, out=gv)
                gatherer.allgather(joints, out=gj)
            else:                      # RCCL over xGMI, peer -> GPU 0 sends
                gatherer.gather(verts, B * world, root=0, out=gv)
                gatherer.gather(joints, B * world, root=0, out=gj)
        else:  # gloo rehearsal: verts + joints through the host into the same gv / gj layout
            if which == "allgather":
                fv = all_gather(verts.cpu(), B * world)
                fj = all_gather(joints.cpu(), B * world)
            else:
                fv = gather_to_root(verts.cpu(), B * world, root=0)
                fj = gather_to_root(joints.cpu(), B * world, root=0)
            if gv is not None:
                gv.copy_(fv)
                gj.copy_(fj)

    # Launch sequence of one step; `marks` get an event after each kernel.
    # "forward" issues exactly mano_forward's two launches (articulate, then
    # the fused blend GEMM + LBS) through the stage calls so that each kernel
    # is bracketed by events on its stream; "api" is one mano_forward call.
    # `dst` = (verts, joints) to write: the timed outputs, or the scratch
    # pair of the untimed kernel table (so the timed step's outputs are what
    # the correctness leg and the gathers read).
    def run_path(path, marks=None, dst=None):
        vo, jo = dst if dst is not None else (verts, joints)

        def mark(i):
            if marks is not None:
                marks[i].record(stream)
        mark(0)
        if path == "forward":
            model.stage_articulate(betas, pose, trans, joints=jo)
            mark(1)
            model.stage_blend_skin(B, vo, trans=trans)
            mark(2)
        elif path == "api":
            model.forward(betas, pose, trans, joints=True, out={"verts": vo, "joints": jo})
            mark(1)
        elif path == "unfused" and model.precision == "fp32":
            # articulate, blend GEMM (v_posed into verts), the LBS in place (f16x3
            # has no in-place kernel: it would stage the rows first, so it takes
            # the separate form below)
            model.stage_articulate(betas, pose, trans, joints=jo)
            mark(1)
            model.stage_blend(B, rest_verts=vo)
            mark(2)
            model.stage_skin(B, vo, rest_verts=vo, trans=trans)
            mark(3)
        else:  # unfused_separate (and f16x3's unfused): v_posed in the workspace, the LBS into verts
            model.stage_articulate(betas, pose, trans, joints=jo)
            mark(1)
            model.stage_blend(B)
            mark(2)
            model.stage_skin(B, vo, trans=trans)
            mark(3)

    n_marks = {"forward": 3, "api": 2, "unfused": 4, "unfused_separate": 4}

    def step(marks=None, gmarks=None):
        run_path(args.path, marks)
        if gather_on:
            if gmarks is not None:
                gmarks[0].record(stream)
            do_gather(impl)
            if gmarks is not None:
                gmarks[1].record(stream)

    # Clock ramp, then the untimed warmup, with no idle GPU before the timed
    # region: the chip needs ~50 back-to-back launches to reach its steady
    # clock and loses it in a ~millisecond idle gap (blend_skin16 545-555 vs
    # 485 us, §4 round 4; round 6: a process-group run that paused for a
    # collective every 10 ramp steps and for the pre-timing barrier timed its
    # 20 steps at 0.551 ms, `profiles/r06/r06e_legs1_bench.json`).  So the
    # ramp's length is fixed up front -- 10 steps, then 10 more on the host
    # clock give the step time -- and, with a process group, agreed once by
    # the ranks (MAX: with the C4 gather every step is a collective, so every
    # rank must run the same number); the rest of the ramp, the warmup and
    # the barrier then follow with no sync: the barrier's collective is
    # ordered after the warmup on the stream (nccl), or waits on the host
    # while the GPU works (gloo).
    wd.enter("ramp")
    t_ramp = time.perf_counter()
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    t_cal = time.perf_counter()
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    per_step = max(1e-6, (time.perf_counter() - t_cal) / 10)
    n_more = max(0, int(np.ceil((args.ramp_seconds - (time.perf_counter() - t_ramp)) / per_step)))
    if args.inject_hang == rank and dist_on:
        while True:       # (tests) this rank stalls outside the ramp's collective
            time.sleep(0.5)
    if dist_on:
        agreed = torch.tensor([n_more], device=dev if args.backend == "nccl" else "cpu", dtype=torch.int64)
        dist.all_reduce(agreed, op=dist.ReduceOp.MAX)
        n_more = int(agreed.item())
    t_agreed = time.perf_counter() - t_ramp
    for _ in range(n_more):
        step()
    n_ramp = 20 + n_more
    t_ramp = t_agreed + n_more * per_step    # the ramp's GPU time (its tail is still running here)
    wd.enter("warmup")
    for _ in range(args.warmup):
        step()

    # Per-kernel durations come from HIP events on the launch stream around
    # the kernels of every E-th timed step (E = --event-every): a timing event
    # is a release point on the stream, which costs the step ~4 us per event
    # (0.530 vs 0.518 ms with three per step, tools/debug/time_events.py), so
    # bracketing every step would bill the instrumentation to `value`.
    # Steps first, first + E, ... (event_plan: at least 5, not step 0).
    every, first = event_plan(args.steps, args.event_every)
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(n_marks[args.path])]
              if i % every == first else None for i in range(args.steps)]
    # the gather of the same sampled steps, bracketed on the same stream
    gevents = [[torch.cuda.Event(enable_timing=True) for _ in range(2)]
               if gather_on and i % every == first else None for i in range(args.steps)]
    wd.enter("timed")
    t_open = time.perf_counter()
    if dist_on and args.backend == "gloo":
        # the rehearsal backend: ranks share one GPU, and gloo's barrier is
        # host-only -- without this sync each rank would start its timed steps
        # when its own queue drained, beside the others' ramps
        torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()   # the ramp and warmup end here: the GPU has not idled since the ramp began
    t0 = time.perf_counter()
    span0 = torch.cuda.Event(enable_timing=True)
    span1 = torch.cuda.Event(enable_timing=True)
    span0.record(stream)
    for i in range(args.steps):
        step(events[i], gevents[i])
    span1.record(stream)
    t_issued = time.perf_counter()
    torch.cuda.synchronize()
    t_synced = time.perf_counter()
    if dist_on:
        # Every rank's GPU work is done (the sync above): the closing barrier
        # only has to meet the ranks, so it runs on the host-side gloo group
        # -- the default group's RCCL barrier (a kernel, a stream sync and
        # torch's bookkeeping) cost ~0.3 ms inside the timed region, 3 % of
        # the driver's 20 steps.  The opening barrier stays on the
        # default group: its collective is ordered after the warmup on the
        # stream, so the ranks start together once every GPU is ready.
        dist.barrier(group=end_group)
    dt = time.perf_counter() - t0
    # where the timed region's host time went (this rank): issuing the K
    # steps, waiting for the GPU to finish them, the closing barrier; and the
    # opening barrier + sync before t0 (outside the region)
    region = {"issue_s": t_issued - t0, "sync_s": t_synced - t_issued, "closing_barrier_s": t0 + dt - t_synced,
              "opening_barrier_and_sync_s": t0 - t_open,
              "gpu_ms_per_step": span0.elapsed_time(span1) / args.steps}
    if dist_on:
        t = torch.tensor([dt], device=dev if args.backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    gather_info = None
    if gather_on:
        gms = [e[0].elapsed_time(e[1]) for e in gevents if e is not None]
        gather_info = gather_stats(impl, world, B, float(np.mean(gms)))
        gather_info["ms_min"] = float(np.min(gms))
        gather_info["ms_max"] = float(np.max(gms))
        gather_info["sampled_steps"] = len(gms)
        gather_info["backend"] = args.backend
        # the rank count RCCL's communicator holds (mano_comm_info), not the launcher's
        gather_info["comm_ranks"] = gatherer.info()[0] if gatherer is not None else None
        gather_info["form"] = ({"sendrecv": "mano_gather: one RCCL group of ncclSend (peers) / ncclRecv "
                                            "(GPU 0), each peer over its own xGMI link",
                                "allgather": "mano_allgather: RCCL ring ncclAllGather"}[impl]
                               if gatherer is not None else "gloo rehearsal through the host")
        gather_info["timing"] = ("HIP events on rank 0's launch stream around the gather (verts + "
                                 "joints) of every sampled timed step, after that step's kernels; "
                                 "each rank's own shard is computed in place in its rows of the "
                                 "assembled buffers, so only the peers' shards move")

    def span(a, b, evs):
        return float(np.mean([e[a].elapsed_time(e[b]) for e in evs]))

    # Per-kernel table.  The timed path's kernels come from the timed steps;
    # the other paths' kernels are timed on the same stream afterwards (rank 0,
    # not part of `value`), so every kernel's roofline is reported each run.
    timed = {"forward": {"articulate": (0, 1), "blend_skin": (1, 2)},
             "api": {"mano_forward": (0, 1)},
             "unfused": {"articulate": (0, 1), "blend": (1, 2), "skin": (2, 3)},
             "unfused_separate": {"blend_separate": (1, 2), "skin_separate": (2, 3)}}
    sampled = [e for e in events if e is not None]
    ms = {k: span(a, b, sampled) for k, (a, b) in timed[args.path].items()}
    other = {"fp32": "f16x3", "f16x3": "fp32"}[args.precision]
    ms_other = {}
    wd.enter("kernel_table")
    if rank == 0 and not args.no_extra:
        scratch = (torch.empty_like(verts), torch.empty_like(joints))

        def time_path(path, into, reps=50):
            evs = [[torch.cuda.Event(enable_timing=True) for _ in range(n_marks[path])]
                   for _ in range(reps)]
            for _ in range(reps):
                run_path(path, dst=scratch)
            for e in evs:
                run_path(path, e, dst=scratch)
            torch.cuda.synchronize()
            for k, (a, b) in timed[path].items():
                into.setdefault(k, span(a, b, evs))
        for path in ("forward", "api", "unfused", "unfused_separate"):
            if path != args.path:
                time_path(path, ms)
        # The standalone LBS back to back (each launch after another LBS
        # launch, as rocprof's kernel trace sees it); in the unfused path it
        # follows the blend GEMM's 612 MB of freshly written v_posed.  One
        # event pair around 50 launches (a timing event between launches
        # adds its own few microseconds to each; §4, "Timing events cost").
        for _ in range(50):
            model.stage_skin(B, scratch[0], trans=trans)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(50):
            model.stage_skin(B, scratch[0], trans=trans)
        e1.record(stream)
        torch.cuda.synchronize()
        ms["skin_back_to_back"] = e0.elapsed_time(e1) / 50
        model.set_precision(other)
        for path in ("forward", "unfused"):
            time_path(path, ms_other)
        model.set_precision(args.precision)
        del scratch

    # The other gather form (report both), timed after the
    # timed region on every rank the same way; its buffers are freed after.
    if gather_on and gatherer is not None and args.gather_compare_reps > 0:
        wd.enter("gather_compare")
        other_impl = "allgather" if impl == "sendrecv" else "sendrecv"
        keep = (gv, gj)
        if other_impl == "allgather" or rank == 0:
            gv = torch.empty((B * world, V, 3), device=dev)
            gj = torch.empty((B * world, 16, 3), device=dev)
        else:
            gv = gj = None
        do_gather(other_impl)   # untimed first call (RCCL sets up its channels)
        torch.cuda.synchronize()
        dist.barrier()
        cev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)]
               for _ in range(args.gather_compare_reps)]
        for e in cev:
            e[0].record(stream)
            do_gather(other_impl)
            e[1].record(stream)
        torch.cuda.synchronize()
        cms = [e[0].elapsed_time(e[1]) for e in cev]
        cmp_info = gather_stats(other_impl, world, B, float(np.mean(cms)))
        cmp_info.update({"ms_min": float(np.min(cms)), "ms_max": float(np.max(cms)), "reps": len(cms),
                         "timing": "after the timed region, the gather alone back to back (no forward "
                                   "in between), HIP events on rank 0's stream; out of place (each rank's "
                                   "own shard is copied too, unlike the timed form's in-place shard)"})
        if rank == 0:
            chk = check_gather(model, wl["seed"], B, world, gv, gj, with_trans)
            cmp_info["bit_exact"] = chk["bit_exact"]
            cmp_info["hands_checked"] = chk["hands_checked"]
        gather_info["compare"] = cmp_info
        gv, gj = keep
        torch.cuda.synchronize()
        dist.barrier()

    def tflops(flop, t):
        return flop * B / (t * 1e-3) / 1e12

    def gbs(nbytes, t):
        return nbytes * B / (t * 1e-3) / 1e9

    in_path = {"forward": ("articulate", "blend_skin"), "api": ("mano_forward",),
               "unfused": ("articulate", "blend", "skin"),
               "unfused_separate": ("articulate", "blend_separate", "skin_separate")}[args.path]
    kernels = {}
    if "mano_forward" in ms:
        kernels["mano_forward"] = {"kernel": "articulate_kernel + blend_skin16_kernel (one ABI call)",
                                   "ms": ms["mano_forward"]}
    if "articulate" in ms:
        a = gbs(ARTICULATE_BYTES_PER_HAND, ms["articulate"])
        kernels["articulate"] = {"kernel": "articulate_kernel", "ms": ms["articulate"],
                                 "bound": "latency", "achieved_GBs": a,
                                 "bytes_per_hand": ARTICULATE_BYTES_PER_HAND}
    if "blend_skin" in ms and args.precision == "fp32":
        a = tflops(FUSED_FLOP_PER_HAND, ms["blend_skin"])
        a_mfma = tflops(FUSED_MFMA_FLOP_PER_HAND, ms["blend_skin"])
        kernels["blend_skin"] = {"kernel": "blend_skin16_kernel", "ms": ms["blend_skin"],
                                 "bound": "mfma", "achieved_TFLOPs": a,
                                 "frac": a / PEAK_FP32_TFLOPS,
                                 "flop_per_hand": FUSED_FLOP_PER_HAND,
                                 "flop_basis": ("SURVEY.md §8(d): blend GEMM 2x2334x145 + LBS 778x405 "
                                                "(transform blend on MFMA + the 21-flop apply on the VALU, "
                                                "the same fp32 datapath and peak on gfx950)"),
                                 "mfma_only": {"flop_per_hand": FUSED_MFMA_FLOP_PER_HAND, "achieved_TFLOPs": a_mfma,
                                               "frac": a_mfma / PEAK_FP32_TFLOPS,
                                               "flop_basis": "MFMA flops only: GEMM + the 16-joint transform "
                                                             "blend (rounds 1-3's numerator; compare rounds on this)"},
                                 "blend_gemm_TFLOPs": tflops(BLEND_FLOP_PER_HAND, ms["blend_skin"])}
    elif "blend_skin" in ms:  # f16x3: the split GEMM runs at 16/3 x the fp32 rate; HBM stores bound it
        a = gbs(FUSED_BYTES_PER_HAND, ms["blend_skin"])
        kernels["blend_skin"] = {"kernel": "blend_skin_h3_kernel", "ms": ms["blend_skin"],
                                 "bound": "hbm", "achieved_GBs": a, "frac": a / PEAK_HBM_GBS,
                                 "bytes_per_hand": FUSED_BYTES_PER_HAND,
                                 "fp32_equiv_TFLOPs": tflops(FUSED_MFMA_FLOP_PER_HAND, ms["blend_skin"])}
    if "blend" in ms:
        a = tflops(BLEND_FLOP_PER_HAND, ms["blend"])
        kernels["blend"] = {"kernel": "blend_kernel", "ms": ms["blend"], "bound": "mfma",
                            "achieved_TFLOPs": a, "frac": a / PEAK_FP32_TFLOPS,
                            "flop_per_hand": BLEND_FLOP_PER_HAND}
    if "skin" in ms:
        a = gbs(SKIN_BYTES_PER_HAND, ms["skin"])
        kernels["skin"] = {"kernel": "skin_pair_kernel" if args.precision == "fp32" else "skin_pair_kernel (f16x3)",
                           "ms": ms["skin"], "bound": "hbm",
                           "achieved_GBs": a, "frac": a / PEAK_HBM_GBS,
                           "bytes_per_hand": SKIN_BYTES_PER_HAND}
        if "skin_back_to_back" in ms:
            b2b = ms["skin_back_to_back"]
            kernels["skin"].update({"ms_back_to_back": b2b, "achieved_GBs_back_to_back": gbs(SKIN_BYTES_PER_HAND, b2b),
                                    "frac_back_to_back": gbs(SKIN_BYTES_PER_HAND, b2b) / PEAK_HBM_GBS,
                                    "timing_back_to_back": "one HIP event pair around 50 launches after 50 warm ones"})
    if "skin" in kernels:
        kernels["skin"]["form"] = ("in place over verts (mano_stage_skin rest_verts == verts, ABI 7), after the "
                                   "blend GEMM wrote v_posed into verts" if args.precision == "fp32" else
                                   "out of place (f16x3 has no in-place kernel)")
    if "blend_separate" in ms:
        a = tflops(BLEND_FLOP_PER_HAND, ms["blend_separate"])
        kernels["blend_separate"] = {"kernel": "blend_kernel (v_posed into the workspace)",
                                     "ms": ms["blend_separate"], "bound": "mfma", "achieved_TFLOPs": a,
                                     "frac": a / PEAK_FP32_TFLOPS, "flop_per_hand": BLEND_FLOP_PER_HAND}
    if "skin_separate" in ms:
        a = gbs(SKIN_BYTES_PER_HAND, ms["skin_separate"])
        kernels["skin_separate"] = {"kernel": "skin_pair_kernel (out of place, workspace v_posed -> verts)",
                                    "ms": ms["skin_separate"], "bound": "hbm", "achieved_GBs": a,
                                    "frac": a / PEAK_HBM_GBS, "bytes_per_hand": SKIN_BYTES_PER_HAND}
    for k, v in kernels.items():
        v["in_timed_path"] = k in in_path
        v["precision"] = args.precision
    # The other precision mode's kernels (timed after the timed region, not in `value`).
    if "blend_skin" in ms_other:
        t = ms_other["blend_skin"]
        kernels[f"blend_skin_{other}"] = {
            "kernel": "blend_skin_h3_kernel" if other == "f16x3" else "blend_skin16_kernel",
            "ms": t, "precision": other, "in_timed_path": False,
            "forward_hands_per_s": B / ((t + ms_other["articulate"]) * 1e-3),
            "achieved_GBs": gbs(FUSED_BYTES_PER_HAND, t), "bytes_per_hand": FUSED_BYTES_PER_HAND,
            "hbm_frac": gbs(FUSED_BYTES_PER_HAND, t) / PEAK_HBM_GBS,
            "fp32_equiv_TFLOPs": tflops(FUSED_MFMA_FLOP_PER_HAND, t)}
    if "skin" in ms_other:
        t = ms_other["skin"]
        kernels[f"skin_{other}"] = {
            "kernel": "skin_pair_kernel (f16x3)" if other == "f16x3" else "skin_pair_kernel",
            "ms": t, "precision": other, "in_timed_path": False, "bound": "hbm",
            "achieved_GBs": gbs(SKIN_BYTES_PER_HAND, t),
            "frac": gbs(SKIN_BYTES_PER_HAND, t) / PEAK_HBM_GBS, "bytes_per_hand": SKIN_BYTES_PER_HAND}

    # Roofline of the dominant kernel of the timed path.
    if args.path == "unfused":
        dominant = "blend" if ms["blend"] >= ms["skin"] else "skin"
    elif args.path == "unfused_separate":
        dominant = "blend_separate" if ms["blend_separate"] >= ms["skin_separate"] else "skin_separate"
    elif args.path == "api":
        dominant = "blend_skin" if "blend_skin" in kernels else None
    else:
        dominant = "blend_skin"
    roof = None
    if dominant is not None:
        kd = kernels[dominant]
        if kd["bound"] == "mfma":
            roof = {"kernel": kd["kernel"], "bound": "mfma", "achieved": kd["achieved_TFLOPs"],
                    "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": kd["frac"]}
        else:
            roof = {"kernel": kd["kernel"], "bound": "hbm", "achieved": kd["achieved_GBs"],
                    "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": kd["frac"]}
        roof["algorithmic_per_hand"] = kd.get("flop_per_hand", kd.get("bytes_per_hand"))
        if "flop_basis" in kd:
            roof["flop_basis"] = kd["flop_basis"]
        if "mfma_only" in kd:  # the same launches counted with the MFMA flops alone (rounds 1-3's numerator)
            roof["mfma_only"] = kd["mfma_only"]
        roof["hands_per_launch"] = B
        roof["timed_in_region"] = dominant in in_path

    # Correctness of the timed outputs (the last timed step's verts / joints):
    # on every rank, sampled hands of its shard vs the float64 oracle in a
    # child process (rank 0 reports the max over ranks), and at N > 1 with a
    # gather, GPU 0's assembled buffers vs a local forward of hands
    # regenerated by global index from every rank's range.
    correctness, gather_check = None, None
    skipped = {}
    wd.enter("correctness")
    device_status = model.device_status(clear=True)  # MANO_DEVICE_* bits raised by any launch (0 = none)
    if not args.no_check:
        correctness = check_sample(model, wl["seed"], rank * B, B, betas, pose, trans, verts, joints,
                                   args.model, with_trans)
        correctness["device_status"] = device_status
        correctness["pass"] = bool(correctness.get("pass")) and device_status == 0
        if dist_on:
            per_rank = [None] * world
            dist.all_gather_object(per_rank, correctness)
            correctness = merge_checks(per_rank)
    elif dist_on:
        st = [None] * world
        dist.all_gather_object(st, device_status)
        device_status = max(st)
    if correctness is not None:
        device_status = correctness.get("device_status", device_status)
    if rank == 0 and gv is not None:
        gather_check = check_gather(model, wl["seed"], B, world, gv, gj, with_trans)
        if args.dump_gather:
            np.savez(args.dump_gather, verts=gv.cpu().numpy(), joints=gj.cpu().numpy())

    # The headline is measured and checked: rank 0's line, before anything
    # that could hang (the roofline's traffic and the host legs fill it in
    # later).
    line = None
    if rank == 0:
        total = B * world * args.steps
        line = {
            "metric": METRIC,
            "value": total / dt,
            "unit": "hands/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ramp": {"seconds": t_ramp, "steps": n_ramp, "step_ms": per_step * 1e3},
            "kernel_events": {"every": every, "sampled_steps": len(sampled)},
            "timed_region_rank0": region,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (random-init MANO arrays of the official shapes, seed 0; "
                    "Philox inputs keyed by (seed, global hand index): beta ~ N(0,1), "
                    "pose ~ N(0,0.5^2) rad" + (", trans ~ U(-1,1) m" if with_trans else "") +
                    ", generated on device)",
            "config": {"workload": wl["desc"] if B == wl["hands"] else f"{args.workload} at {B} hands per GPU",
                       "hands_per_gpu": B, "global_batch": B * world,
                       "outputs": "verts+joints", "trans": with_trans, "path": args.path,
                       "gather_to_gpu0": gather_on,
                       "gather_impl": None if not gather_on else
                       ({"sendrecv": "mano_gather (RCCL send/recv)", "allgather": "mano_allgather (RCCL ring)"}[impl]
                        if gatherer is not None else "gloo rehearsal"),
                       "parallelism": f"dp{world}"},
            "process_group": ({"backend": args.backend, "world": world, "forced_at_one_rank": world == 1}
                              if dist_on else None),
            "roofline": roof,
            "kernels": kernels,
            "correctness": correctness,
            "device_status": device_status,
        }
        if gather_info is not None:
            line["gather"] = gather_info
        if gather_check is not None:
            line["gather_check"] = gather_check

    # BASELINE's multi-GPU configs (C3, C4) as legs after the headline: every
    # N > 1 run measures them (not part of `value`), inside the watchdog --
    # which, if a leg hangs, prints the line above with the finished legs
    # instead of a bare status line (Watchdog.partial).
    legs_plan = plan_legs(args, world) if dist_on else {}
    legs = None
    if legs_plan:
        legs = {}
        wd.partial, wd.legs = (line if rank == 0 else {}), legs
        run_legs(args, legs_plan, model, rank, world, dev, local_dev, wd, skipped, out=legs)
        wd.partial = None

    # The collective phases are over.  Rank 0's host legs hold no collective
    # and each is bounded by its own child timeout, fitted into the deadline;
    # the other ranks wait for them at the gloo end barrier.  From here the
    # watchdog fires only past the deadline (+30 s, inside the driver's lease).
    wd.enter("rank0_legs" if rank == 0 else "end_barrier")
    if dist_on and args.watchdog_seconds > 0:
        wd.arm(T_START + args.deadline_seconds + 30.0)

    # Rank 0's host-side legs, at every N (the other ranks wait at a barrier,
    # their GPUs idle): roofline.traffic by two rocprofv3 --pmc passes over a
    # child run on rank 0's GPU only, the drop-in latency, the CPU baseline.
    extra = {}
    if rank == 0:
        if roof is not None:
            traffic, src, live = None, None, None
            if not args.no_live_pmc:
                frag = PMC_KERNEL_NAME.get(dominant + ("_h3" if args.precision == "f16x3" else ""))
                left = remaining(args)
                if left < 100:
                    live = f"skipped: {left:.0f} s left of --deadline-seconds"
                    skipped["live_pmc"] = live
                elif frag is not None:
                    wd.enter("rank0_legs:live_pmc")
                    traffic, live = live_traffic(args, B, frag, local_dev=local_dev,
                                                 timeout=min(120.0, (left - 60.0) / 2.0))
                    if traffic is not None:
                        src = (f"measured in this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over "
                               f"a 3-step 1-rank child run at {B} hands on rank 0's GPU (read = 2 x FETCH_SIZE)"
                               + (" -- the kernel's per-launch bytes at this shard size; every rank's "
                                  "launch is the same shape" if world > 1 else ""))
            if traffic is None:
                traffic, src = load_traffic(args.pmc, dominant + ("_h3" if args.precision == "f16x3" else ""), B)
                if live is not None:
                    src = f"{src} (live passes failed: {live})"
            roof["traffic"] = traffic
            roof["traffic_source"] = src
            if isinstance(live, dict):
                roof["traffic_detail"] = live
            if traffic is not None and kernels.get(dominant, {}).get("ms"):
                # the HBM side of the same launches (north_star: "MFMA and HBM rooflines")
                hbm = traffic / (kernels[dominant]["ms"] * 1e-3) / 1e9
                roof["hbm_GBs"] = hbm
                roof["hbm_frac"] = hbm / PEAK_HBM_GBS
        if not args.no_dropin:
            if remaining(args) < 40:
                skipped["dropin"] = f"{remaining(args):.0f} s left of --deadline-seconds"
            else:
                wd.enter("rank0_legs:dropin")
                extra["dropin"] = dropin_latency(params, local_dev)
        if not args.no_cpu:
            # two forms of `secs` each plus process start-up must end 20 s
            # before the deadline
            secs = min(args.cpu_seconds, (remaining(args) - 50.0) / 2.5)
            if secs < 1.0:
                skipped["cpu_baseline"] = f"{remaining(args):.0f} s left of --deadline-seconds"
            else:
                wd.enter("rank0_legs:cpu_baseline")
                procs = args.cpu_procs or cpu_share(world)
                cb = cpu_baseline(procs, round(secs, 1), timeout=max(10.0, remaining(args) - 20.0))
                if secs < args.cpu_seconds:
                    cb["shortened"] = f"{secs:.1f} s per form (of {args.cpu_seconds}) to fit --deadline-seconds"
                if world > 1:
                    cb["note"] = (f"rank 0 after the timed region while the other {world - 1} ranks wait at a "
                                  f"barrier; {procs} of this node's cores")
                extra["cpu_baseline"] = cb
                if "dropin" in extra and cb.get("value"):
                    # the per-hand port's time per hand on ONE core (the reference's
                    # own loop runs at 1/1.055 of it: profiles/cpu_calibration.json)
                    extra["dropin"]["cpu_port_us_per_hand_one_core"] = cb["cores"] / cb["value"] * 1e6
    if dist_on:
        wd.enter("end_barrier")
        dist.barrier(group=end_group)
    wd.cancel()

    if rank == 0:
        if legs is not None:
            line["legs"] = legs
        line.update(extra)
        line["status"] = "ok"
        line["run"] = {"wall_s": round(time.monotonic() - T_START, 3), "phases": wd.phases,
                       "deadline_s": args.deadline_seconds,
                       "watchdog_s": args.watchdog_seconds if dist_on else None,
                       "pg_timeout_s": args.pg_timeout_seconds if dist_on else None,
                       "skipped_legs": skipped}
        print(json.dumps(line), flush=True)
    if gatherer is not None:
        gatherer.close()
    model.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
