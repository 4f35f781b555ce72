"""Calibrate bench.py's CPU baseline "port" against the reference (build container only).

bench.py cannot run the reference on the GPU box (it does not travel), so its
CPU line times the float64 restatement `oracle.mano_oracle.forward_one`.  This
script runs both here, one process each with OMP_NUM_THREADS=1, on the same
hands: the reference `MANOModel.set_params(pose_abs=..., shape=...)` loop
(/root/reference/mano_np.py:48-115) and forward_one, checks the vertices agree
bit for bit, and writes their speed ratio to profiles/cpu_calibration.json.

    python tools/calibrate_cpu_baseline.py [--seconds 5]
"""
import os

os.environ["OMP_NUM_THREADS"] = "1"
os.environ["OPENBLAS_NUM_THREADS"] = "1"

import argparse  # noqa: E402
import json  # noqa: E402
import platform  # noqa: E402
import sys  # noqa: E402
import tempfile  # noqa: E402
import time  # noqa: E402

import numpy as np  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.dont_write_bytecode = True
sys.path[:0] = [REPO, os.path.join(REPO, "mano-hand_amd"), "/root/reference"]

from mano_amd.model_io import save_dump, synthetic_params  # noqa: E402
from mano_np import MANOModel  # noqa: E402  (the reference)
from oracle import mano_oracle  # noqa: E402


def rate(fn, n_inputs, seconds):
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        fn(n % n_inputs)
        n += 1
    return n / (time.perf_counter() - t0), n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=5.0)
    a = ap.parse_args()
    params = synthetic_params(0)
    rng = np.random.default_rng(1000)
    betas = rng.normal(0, 1, (256, 10))
    pose = rng.normal(0, 0.5, (256, 16, 3))
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "dump.pkl")
        save_dump(params, path)
        ref = MANOModel(path)
    p = {k: (np.asarray(v, dtype=np.float64) if k not in ("parents", "faces") else v)
         for k, v in params.items()}
    worst = 0.0
    for i in range(64):
        v_ref = ref.set_params(pose_abs=pose[i], shape=betas[i])
        v_port = mano_oracle.forward_one(p, betas[i], pose[i])
        worst = max(worst, float(np.abs(v_ref - v_port).max()))
    r_ref, n_ref = rate(lambda i: ref.set_params(pose_abs=pose[i], shape=betas[i]), 256, a.seconds)
    r_port, n_port = rate(lambda i: mano_oracle.forward_one(p, betas[i], pose[i]), 256, a.seconds)
    out = {"reference_hands_per_s": r_ref, "port_hands_per_s": r_port,
           "port_over_reference": r_port / r_ref, "max_abs_diff_m": worst,
           "hands_timed": {"reference": n_ref, "port": n_port}, "seconds_each": a.seconds,
           "cores": 1, "host": platform.processor() or platform.machine(),
           "numpy": np.__version__}
    dst = os.path.join(REPO, "profiles", "cpu_calibration.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
