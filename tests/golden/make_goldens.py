"""Generate golden vectors by running the REFERENCE MANOModel (build container only).

Run from the repo root:  python tests/golden/make_goldens.py
It needs `/root/reference/mano_np.py` (importable here, absent on the GPU box)
and writes, next to this script:

  mano_reference_steps.npz   a stateful script of set_params calls on ONE
                             reference model instance (zero pose, pose_abs in
                             (16,3) and (48,) form, pose_pca with N = 1/9/45 with
                             and without global_rot, shape-only updates, the
                             demo vectors of mano_np.py:209-218, near-zero and
                             large angles) -> verts, J, R, rest_verts, pose, rot
                             and posed joints after every call;
  mano_reference_batch.npz   24 independent hands (random beta + full pose);
  hand.obj / hand_restpose.obj   reference export_obj output for the demo call.

Posed joints are not stored by the reference; they are rebuilt from the
reference's own R, J and parents with the reference's `with_zeros` using the
recurrence of mano_np.py:96-104 (G[:, :3, 3] before the rest removal at :106).

The model is the build's deterministic synthetic model (seed 0); its SHA-256
is stored in every npz so tests can prove they regenerate the same model.
"""
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(REPO, "mano-hand_amd"))
sys.path.insert(0, "/root/reference")

from mano_amd.model_io import params_digest, save_dump, synthetic_params  # noqa: E402
from mano_np import MANOModel  # noqa: E402  (the reference)


def posed_joints(model):
    nj = model.R.shape[0]
    G = np.empty((nj, 4, 4))
    G[0] = model.with_zeros(np.hstack((model.R[0], model.J[0, :].reshape([3, 1]))))
    for i in range(1, nj):
        p = model.parents[i]
        G[i] = G[p].dot(model.with_zeros(np.hstack([model.R[i], (model.J[i, :] - model.J[p, :]).reshape([3, 1])])))
    return G[:, :3, 3].copy()


def snapshot(model):
    return {
        "verts": np.array(model.verts), "J": np.array(model.J), "R": np.array(model.R),
        "rest_verts": np.array(model.rest_verts), "pose": np.array(model.pose, dtype=np.float64).reshape(-1, 3),
        "rot": np.array(model.rot, dtype=np.float64).reshape(1, 3), "joints": posed_joints(model),
        "shape": np.array(model.shape, dtype=np.float64),
    }


def angle_pose(rng, mag):
    d = rng.normal(size=(16, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return d * mag


def main():
    params = synthetic_params(0)
    digest = params_digest(params)
    tmp = tempfile.mkdtemp()
    path = os.path.join(tmp, "dump_synth_seed0.pkl")
    save_dump(params, path)
    model = MANOModel(path)
    rng = np.random.default_rng(20250114)

    demo_pca = np.asarray([-0.32322194, 0.740878, -1.182191, 1.51246975,
                           -1.89044963, 0.68187004, -0.33078079, 0.23475931, -1.43845225])
    demo_shape = [-0.33191198, 0.88129797, -1.9995425, -0.79066971, -1.41297644,
                  -1.63064562, -1.25495915, -0.61775709, -0.4129301, 0.15526694]

    steps = []  # (description, kwargs)
    steps.append(("init", None))
    steps.append(("pose_abs normal", dict(pose_abs=rng.normal(0, 0.5, (16, 3)), shape=rng.normal(0, 1, 10))))
    steps.append(("pose_abs uniform pi", dict(pose_abs=rng.uniform(-np.pi, np.pi, (16, 3)), shape=rng.normal(0, 1, 10))))
    steps.append(("pose_abs flat48", dict(pose_abs=rng.normal(0, 0.5, 48))))
    steps.append(("shape only", dict(shape=rng.normal(0, 2, 10))))
    steps.append(("pca N=9 no rot", dict(pose_pca=rng.normal(0, 1, 9))))
    steps.append(("pca N=1 rot", dict(pose_pca=rng.normal(0, 1, 1), global_rot=rng.normal(0, 1, 3))))
    steps.append(("pca N=45 rot carried", dict(pose_pca=rng.normal(0, 1, 45))))
    steps.append(("pca N=45 new rot+shape", dict(pose_pca=rng.normal(0, 1, 45), global_rot=[0.3, -2.0, 0.5], shape=rng.normal(0, 1, 10))))
    steps.append(("pose_abs after pca", dict(pose_abs=rng.normal(0, 0.3, (16, 3)))))
    steps.append(("zero pose", dict(pose_abs=np.zeros((16, 3)), shape=np.zeros(10))))
    for mag in (1e-20, 1e-12, 1e-8, 1e-6, 1e-4, 1e-2):
        steps.append((f"angle {mag:g}", dict(pose_abs=angle_pose(rng, mag), shape=rng.normal(0, 1, 10))))
    for mag in (np.pi, 2 * np.pi, 3.0, 6.0):
        steps.append((f"angle {mag:g}", dict(pose_abs=angle_pose(rng, mag))))
    mixed = rng.normal(0, 0.5, (16, 3))
    mixed[1] = 0.0
    mixed[5] = [1e-9, 0, 0]
    mixed[9] = [np.pi, 0, 0]
    mixed[12] = [0, 0, 2 * np.pi]
    steps.append(("mixed edge joints", dict(pose_abs=mixed)))
    steps.append(("demo mano_np.py:209-218", dict(pose_pca=demo_pca, shape=demo_shape, global_rot=[1, 0, 0])))

    arrays = {"model_sha256": np.array(digest)}
    manifest = []
    for i, (desc, kw) in enumerate(steps):
        if kw is not None:
            model.set_params(**{k: (np.asarray(v) if k != "global_rot" and k != "shape" else v) for k, v in kw.items()})
        snap = snapshot(model)
        entry = {"step": i, "desc": desc, "args": []}
        if kw is not None:
            for k, v in kw.items():
                arrays[f"s{i}_in_{k}"] = np.asarray(v, dtype=np.float64)
                entry["args"].append(k)
        for k, v in snap.items():
            arrays[f"s{i}_out_{k}"] = v
        manifest.append(entry)
    arrays["manifest"] = np.array(json.dumps(manifest))
    np.savez_compressed(os.path.join(HERE, "mano_reference_steps.npz"), **arrays)

    # The demo call's OBJ export (mano_np.py:219) for the export_obj writer.
    model.export_obj(os.path.join(HERE, "hand.obj"))

    # Independent hands, fresh full pose + betas each (data_explore.py:12-15 style loop).
    B = 24
    betas = rng.normal(0, 1, (B, 10))
    poses = rng.normal(0, 0.5, (B, 16, 3))
    poses[:8] = rng.uniform(-np.pi, np.pi, (8, 16, 3))
    out = {k: [] for k in ("verts", "J", "R", "rest_verts", "joints")}
    for b in range(B):
        model.set_params(pose_abs=poses[b], shape=betas[b])
        snap = snapshot(model)
        for k in out:
            out[k].append(snap[k])
    np.savez_compressed(os.path.join(HERE, "mano_reference_batch.npz"), model_sha256=np.array(digest),
                        betas=betas, pose=poses, **{k: np.stack(v) for k, v in out.items()})
    print(f"wrote {len(steps)} steps, {B} batch hands; model sha256 {digest}")


if __name__ == "__main__":
    main()
