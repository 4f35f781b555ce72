"""Throughput benchmark of the MI355X MANO forward pass (driver contract).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--gather]

One step = one forward pass (mano_forward: articulate, then the fused blend
GEMM + LBS kernel) over B hands per GPU
(BASELINE.json configs[1]: 65,536 hands, fp32 full pose, random betas), inputs
resident in HBM before the timed region.  N > 1 runs one process per GPU
(torch.distributed.run); shards are independent (no collective on the hot
path), `--gather` adds the RCCL gather of verts + joints to GPU 0 (config C4).

Rank 0 prints ONE JSON line with the whole-node hands/s, the roofline of the
dominant kernel (per-kernel durations from HIP events recorded on the launch
stream inside the timed steps) and, at N = 1, the CPU baseline: the float64
per-hand restatement of mano_np.py (oracle/, "port") timed on this host.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mano-hand_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# Algorithmic work per hand (DESIGN.md "Rooflines").
V, NCOL, K = 778, 2334, 145
BLEND_FLOP_PER_HAND = 2 * NCOL * K                 # 676,860
SKIN_BYTES_PER_HAND = NCOL * 4 * 2 + 16 * 12 * 4   # v_posed in + verts out + transforms = 19,440
SKIN_FLOP_PER_HAND = V * (16 * 12 * 2 + 9 * 2)     # blend 16 transforms + apply = 312,312
LBS_T_FLOP_PER_HAND = V * 16 * 12 * 2              # the transform blend (on MFMA when fused) = 298,752
FUSED_MFMA_FLOP_PER_HAND = BLEND_FLOP_PER_HAND + LBS_T_FLOP_PER_HAND  # 975,612
FUSED_BYTES_PER_HAND = 160 * 4 + 16 * 12 * 4 + NCOL * 4     # X row + transforms in, verts out = 10,744
ARTICULATE_BYTES_PER_HAND = (10 + 48) * 4 + 16 * 12 * 4 + 16 * 3 * 4 + 160 * 4  # in + A + joints + X row = 1,832
PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (= vector) peak, spec
PEAK_HBM_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # The chip takes ~50 back-to-back launches (~30 ms) to reach its steady
    # clock: blend_skin16 ran 0.73 ms -> 0.52 ms across the first 50 launches of
    # a cold box (profiles/r01_kernel_trace_warmup.txt), so the default warmup
    # is well past that.
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--batch", type=int, default=65536, help="hands per GPU per step")
    ap.add_argument("--gather", action="store_true", help="RCCL gather of verts+joints to GPU 0")
    ap.add_argument("--path", choices=("forward", "api", "unfused"), default="forward",
                    help="forward: mano_forward's two kernels, each bracketed by events (default); "
                         "api: one mano_forward call per step; unfused: articulate + blend + skin")
    ap.add_argument("--precision", choices=("fp32", "f16x3"), default="fp32",
                    help="fp32: exact fp32 MFMA (default); f16x3: split-half MFMA "
                         "(include/mano_hip.h MANO_PRECISION_F16X3)")
    ap.add_argument("--model", default=None, help="dump_model.py pickle (default: synthetic seed 0)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline sample length")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="process-group backend for N > 1 (gloo: CPU rehearsal, ranks may share a GPU)")
    return ap.parse_args()


def cpu_baseline(params, seconds):
    """float64 per-hand restatement (oracle.forward_one), one core, bounded sample."""
    from oracle import mano_oracle
    p = {k: (np.asarray(v, dtype=np.float64) if k not in ("parents", "faces") else v)
         for k, v in params.items()}
    rng = np.random.default_rng(1000)
    betas = rng.normal(0, 1, (256, 10))
    pose = rng.normal(0, 0.5, (256, 16, 3))
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        mano_oracle.forward_one(p, betas[n % 256], pose[n % 256])
        n += 1
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "hands/s", "cores": 1, "kind": "port",
            "sample": f"{n} hands, one at a time, float64 numpy restatement of mano_np.py:81-115 "
                      f"(oracle/mano_oracle.py forward_one), {dt:.1f} s on 1 host core"}


def load_traffic(path, kernel, batch):
    """HBM bytes per launch from a committed rocprofv3 --pmc summary, if it covers this batch."""
    try:
        with open(path) as f:
            data = json.load(f)
        ent = data["kernels"][kernel]
        if int(data["batch"]) != batch:
            return None
        return float(ent["hbm_bytes_per_launch"])
    except (OSError, KeyError, ValueError, TypeError):
        return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # One process per GPU.  `--backend gloo` is a control-flow rehearsal mode
    # (several ranks may share one GPU); the real multi-GPU run uses RCCL.
    ndev = torch.cuda.device_count()
    local_dev = local if args.backend == "nccl" else local % max(ndev, 1)
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    from mano_amd import ManoHip, load_dump, synthetic_params
    from mano_amd.distributed import gather_to_root
    params = load_dump(args.model) if args.model else synthetic_params(0)
    model = ManoHip(params, device=local_dev, precision=args.precision)

    B = args.batch
    g = torch.Generator(device=dev).manual_seed(1001 + rank)
    betas = torch.randn((B, 10), generator=g, device=dev)
    pose = 0.5 * torch.randn((B, 16, 3), generator=g, device=dev)
    verts = torch.empty((B, V, 3), device=dev)
    joints = torch.empty((B, 16, 3), device=dev)
    stream = torch.cuda.current_stream(dev)
    out = {"verts": verts, "joints": joints}
    model.workspace(B)  # allocated before timing (covers every path)

    # Launch sequence of one step; `marks` get an event after each kernel.
    # "forward" issues exactly mano_forward's two launches (articulate, then
    # the fused blend GEMM + LBS) through the stage calls so that each kernel
    # is bracketed by events on its stream; "api" is one mano_forward call.
    def run_path(path, marks=None):
        def mark(i):
            if marks is not None:
                marks[i].record(stream)
        mark(0)
        if path == "forward":
            model.stage_articulate(betas, pose, joints=joints)
            mark(1)
            model.stage_blend_skin(B, verts)
            mark(2)
        elif path == "api":
            model.forward(betas, pose, joints=True, out=out)
            mark(1)
        else:  # unfused: articulate, blend GEMM (v_posed to HBM), LBS
            model.stage_articulate(betas, pose, joints=joints)
            mark(1)
            model.stage_blend(B)
            mark(2)
            model.stage_skin(B, verts)
            mark(3)

    n_marks = {"forward": 3, "api": 2, "unfused": 4}

    def step(marks=None):
        run_path(args.path, marks)
        if args.gather and world > 1:
            if args.backend == "nccl":  # RCCL over xGMI, device to device
                gather_to_root(verts, B * world, root=0)
                gather_to_root(joints, B * world, root=0)
            else:
                gather_to_root(joints.cpu(), B * world, root=0)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    events = [[torch.cuda.Event(enable_timing=True) for _ in range(n_marks[args.path])]
              for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(events[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev if args.backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    def span(a, b, evs):
        return float(np.mean([e[a].elapsed_time(e[b]) for e in evs]))

    # Per-kernel table.  The timed path's kernels come from the timed steps;
    # the other paths' kernels are timed on the same stream afterwards (rank 0,
    # not part of `value`), so every kernel's roofline is reported each run.
    timed = {"forward": {"articulate": (0, 1), "blend_skin": (1, 2)},
             "api": {"mano_forward": (0, 1)},
             "unfused": {"articulate": (0, 1), "blend": (1, 2), "skin": (2, 3)}}
    ms = {k: span(a, b, events) for k, (a, b) in timed[args.path].items()}
    other = {"fp32": "f16x3", "f16x3": "fp32"}[args.precision]
    ms_other = {}
    if rank == 0:
        def time_path(path, into, reps=50):
            evs = [[torch.cuda.Event(enable_timing=True) for _ in range(n_marks[path])]
                   for _ in range(reps)]
            for _ in range(reps):
                run_path(path)
            for e in evs:
                run_path(path, e)
            torch.cuda.synchronize()
            for k, (a, b) in timed[path].items():
                into.setdefault(k, span(a, b, evs))
        for path in ("forward", "api", "unfused"):
            if path != args.path:
                time_path(path, ms)
        model.set_precision(other)
        for path in ("forward", "unfused"):
            time_path(path, ms_other)
        model.set_precision(args.precision)

    def tflops(flop, t):
        return flop * B / (t * 1e-3) / 1e12

    def gbs(nbytes, t):
        return nbytes * B / (t * 1e-3) / 1e9

    in_path = {"forward": ("articulate", "blend_skin"), "api": ("mano_forward",),
               "unfused": ("articulate", "blend", "skin")}[args.path]
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
        a = tflops(FUSED_MFMA_FLOP_PER_HAND, ms["blend_skin"])
        kernels["blend_skin"] = {"kernel": "blend_skin16_kernel", "ms": ms["blend_skin"],
                                 "bound": "mfma", "achieved_TFLOPs": a,
                                 "frac": a / PEAK_FP32_TFLOPS,
                                 "flop_per_hand": FUSED_MFMA_FLOP_PER_HAND,
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
        kernels["skin"] = {"kernel": "skin_span_kernel" if args.precision == "fp32" else "skin_span_h3_kernel",
                           "ms": ms["skin"], "bound": "hbm",
                           "achieved_GBs": a, "frac": a / PEAK_HBM_GBS,
                           "bytes_per_hand": SKIN_BYTES_PER_HAND}
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
            "kernel": "skin_span_h3_kernel" if other == "f16x3" else "skin_span_kernel",
            "ms": t, "precision": other, "in_timed_path": False, "bound": "hbm",
            "achieved_GBs": gbs(SKIN_BYTES_PER_HAND, t),
            "frac": gbs(SKIN_BYTES_PER_HAND, t) / PEAK_HBM_GBS, "bytes_per_hand": SKIN_BYTES_PER_HAND}

    # Roofline of the dominant kernel of the timed path.
    if args.path == "unfused":
        dominant = "blend" if ms["blend"] >= ms["skin"] else "skin"
    else:
        dominant = "blend_skin"
    kd = kernels[dominant]
    if kd["bound"] == "mfma":
        roof = {"kernel": kd["kernel"], "bound": "mfma", "achieved": kd["achieved_TFLOPs"],
                "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": kd["frac"]}
    else:
        roof = {"kernel": kd["kernel"], "bound": "hbm", "achieved": kd["achieved_GBs"],
                "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": kd["frac"]}
    roof["traffic"] = load_traffic(args.pmc, dominant + ("_h3" if args.precision == "f16x3" else ""), B)
    roof["algorithmic_per_hand"] = kd.get("flop_per_hand", kd.get("bytes_per_hand"))
    roof["timed_in_region"] = dominant in in_path

    if rank == 0:
        total = B * world * args.steps
        line = {
            "metric": "posed hand meshes/sec (whole node)",
            "value": total / dt,
            "unit": "hands/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (random-init MANO arrays of the official shapes, seed 0; "
                    "beta ~ N(0,1), pose ~ N(0,0.5^2) rad, generated on device)",
            "config": {"workload": "C2: full-pose fp32 MANO forward, 65,536 hands per GPU"
                       if B == 65536 else f"{B} hands per GPU",
                       "hands_per_gpu": B, "global_batch": B * world, "outputs": "verts+joints",
                       "path": args.path,
                       "gather_to_gpu0": bool(args.gather and world > 1),
                       "parallelism": f"dp{world}"},
            "roofline": roof,
            "kernels": kernels,
        }
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(params, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    model.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
