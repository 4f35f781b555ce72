"""CPU baseline of bench.py -- MEASUREMENT INFRASTRUCTURE, not the product.

Times the float64 numpy restatement of the reference hot path
(`/root/reference/mano_np.py:81-115`, restated in `oracle/mano_oracle.py`) on
the host cores of the box bench.py runs on, in two forms (SURVEY.md §8d,
BASELINE.md's CPU plan):

  per_hand  `mano_oracle.forward_one`, one hand per call -- the reference's own
            batch-1 op sequence (what `MANOModel.set_params` runs per hand),
            in P worker processes with OMP_NUM_THREADS=1 each ("port": its
            speed equals the reference's, see DESIGN.md §6 calibration);
  batched   `forward_gemm` over 256-hand batches: the same float64 arithmetic
            cast as BLAS GEMMs (the shape + pose blend as one (B x 145) x
            (145 x 2334) product, the LBS blend as (778 x 16) x (16 x 12B)),
            the stronger CPU line, in the same P processes.

Inputs follow the GPU workload's distributions (beta ~ N(0, 1), pose ~
N(0, 0.5^2) rad).  Run as a script (bench.py starts it as a child process, so
its workers never share a process with the GPU):

    python oracle/cpu_baseline.py --procs 16 --seconds 10
"""
import os

os.environ["OMP_NUM_THREADS"] = "1"          # before numpy loads BLAS
os.environ["OPENBLAS_NUM_THREADS"] = "1"
os.environ["MKL_NUM_THREADS"] = "1"

import argparse  # noqa: E402
import json  # noqa: E402
import multiprocessing as mp  # noqa: E402
import sys  # noqa: E402
import time  # noqa: E402

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [REPO, os.path.join(REPO, "mano-hand_amd")]

from mano_amd.model_io import synthetic_params  # noqa: E402
from oracle import mano_oracle  # noqa: E402


def _params():
    p = synthetic_params(0)
    return {k: (np.asarray(v, dtype=np.float64) if k not in ("parents", "faces") else v)
            for k, v in p.items()}


def gemm_operands(p):
    """Model arrays in GEMM form (float64): basis (145, 3V) = [S ; P] rows,
    template (3V,), the J regression folded into beta space, weights (V, 16)."""
    V = p["mesh_template"].shape[0]
    basis = np.concatenate([p["mesh_shape_basis"].reshape(3 * V, -1),
                            p["mesh_pose_basis"].reshape(3 * V, -1)], axis=1).T.copy()
    jreg = p["J_regressor"]
    return {"basis": basis, "template": p["mesh_template"].reshape(-1),
            "jt": jreg @ p["mesh_template"],
            "js": np.einsum("jv,vcs->sjc", jreg, p["mesh_shape_basis"]).reshape(-1, jreg.shape[0] * 3),
            "W": p["skinning_weights"], "parents": p["parents"]}


def forward_gemm(ops, betas, pose):
    """Batched float64 forward of mano_np.py:81-115 on BLAS GEMMs -> verts (B, V, 3)."""
    B = betas.shape[0]
    R = mano_oracle.rodrigues(pose.reshape(B, -1, 3))                            # :84-86
    X = np.concatenate([betas, mano_oracle.pose_features(R)], axis=1)           # [beta | (R - I)]
    v_posed = (X @ ops["basis"] + ops["template"]).reshape(B, -1, 3)            # :81, :87-93
    J = ops["jt"] + (betas @ ops["js"]).reshape(B, -1, 3)                       # :83 (folded)
    _, G = mano_oracle.chain(R, J, ops["parents"])                              # :96-110
    nj = G.shape[1]
    T = ops["W"] @ G[:, :, :3, :].reshape(B, nj, 12)                            # :112 -> (B, V, 12)
    T = T.reshape(B, -1, 3, 4)
    return np.einsum("bvkl,bvl->bvk", T[..., :3], v_posed) + T[..., 3]          # :113-115


def _per_hand(args):
    worker, seconds = args
    p = _params()
    rng = np.random.default_rng(1000 + worker)
    betas = rng.normal(0, 1, (256, 10))
    pose = rng.normal(0, 0.5, (256, 16, 3))
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        mano_oracle.forward_one(p, betas[n % 256], pose[n % 256])
        n += 1
    return n, time.perf_counter() - t0


def _batched(args):
    worker, seconds = args
    ops = gemm_operands(_params())
    rng = np.random.default_rng(2000 + worker)
    B = 256
    betas = rng.normal(0, 1, (B, 10))
    pose = rng.normal(0, 0.5, (B, 16, 3))
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        forward_gemm(ops, betas, pose)
        n += B
    return n, time.perf_counter() - t0


def run(procs, seconds):
    ctx = mp.get_context("fork")
    out = {}
    for name, fn in (("per_hand", _per_hand), ("batched", _batched)):
        with ctx.Pool(procs) as pool:
            res = pool.map(fn, [(w, seconds) for w in range(procs)])
        hands = sum(r[0] for r in res)
        wall = max(r[1] for r in res)
        out[name] = {"value": hands / wall, "hands": hands, "seconds": wall}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=10.0)
    a = ap.parse_args()
    print(json.dumps(run(a.procs, a.seconds)), flush=True)


if __name__ == "__main__":
    main()
