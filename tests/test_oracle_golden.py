"""Pin the CPU oracle to the reference's own outputs (tests/golden/, made by
tests/golden/make_goldens.py importing /root/reference/mano_np.py)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, step_kwargs
from oracle import mano_oracle

TOL = 1e-12  # float64 restatement vs float64 reference


def test_synthetic_model_matches_fixture_digest(params, golden_steps, golden_batch):
    from mano_amd import params_digest
    d = params_digest(params)
    assert d == str(golden_steps[1]["model_sha256"])
    assert d == str(golden_batch["model_sha256"])


def test_stateful_script_matches_reference(params, golden_steps):
    manifest, data = golden_steps
    assert len(manifest) >= 20
    model = None
    for entry in manifest:
        i = entry["step"]
        if model is None:
            assert entry["desc"] == "init"
            model = mano_oracle.StatefulOracle(params)
        else:
            model.set_params(**step_kwargs(entry, data))
        for key, got in (("verts", model.verts), ("J", model.J), ("R", model.R),
                         ("rest_verts", model.rest_verts), ("joints", model.joints),
                         ("rot", model.rot), ("pose", np.reshape(model.pose, (-1, 3)))):
            ref = data[f"s{i}_out_{key}"]
            err = np.abs(np.asarray(got) - ref).max()
            assert err <= TOL, (entry["desc"], key, err)


def test_init_is_template(params, golden_steps):
    _, data = golden_steps
    assert np.abs(data["s0_out_verts"] - params["mesh_template"]).max() < 1e-15


def test_batched_oracle_matches_reference(params, golden_batch):
    g = golden_batch
    out = mano_oracle.forward(params, g["betas"], g["pose"])
    for key, gk in (("verts", "verts"), ("joints", "joints"), ("rest_verts", "rest_verts"),
                    ("rest_joints", "J"), ("rot", "R")):
        err = np.abs(out[key] - g[gk]).max()
        assert err <= TOL, (key, err)


def test_per_hand_oracle_matches_reference(params, golden_batch):
    g = golden_batch
    for b in range(0, g["betas"].shape[0], 5):
        v = mano_oracle.forward_one(params, g["betas"][b], g["pose"][b])
        assert np.abs(v - g["verts"][b]).max() <= TOL


def test_translation_extension_is_additive(params, golden_batch):
    g = golden_batch
    t = np.random.default_rng(0).uniform(-1, 1, (g["betas"].shape[0], 3))
    a = mano_oracle.forward(params, g["betas"], g["pose"])
    b = mano_oracle.forward(params, g["betas"], g["pose"], t)
    assert np.abs(b["verts"] - a["verts"] - t[:, None]).max() < 1e-14
    assert np.abs(b["joints"] - a["joints"] - t[:, None]).max() < 1e-14


def test_rodrigues_edge_angles():
    r = np.array([[0, 0, 0], [1e-20, 0, 0], [0, np.pi, 0], [0, 0, 2 * np.pi], [1, 2, 3]], float)
    R = mano_oracle.rodrigues(r)
    assert np.allclose(R[0], np.eye(3))
    assert np.allclose(R[1], np.eye(3))
    assert np.allclose(np.einsum("nij,nkj->nik", R, R), np.eye(3), atol=1e-14)


def test_export_obj_matches_reference_text(golden_steps, tmp_path):
    """The OBJ writer reproduces the reference's export_obj bytes for the demo call."""
    from mano_amd.model import write_obj
    from mano_amd import synthetic_params
    manifest, data = golden_steps
    last = manifest[-1]["step"]
    faces = synthetic_params(0)["faces"]
    p = str(tmp_path / "hand.obj")
    write_obj(p, data[f"s{last}_out_verts"], faces)
    write_obj(str(tmp_path / "hand_restpose.obj"), data[f"s{last}_out_rest_verts"], faces)
    for name in ("hand.obj", "hand_restpose.obj"):
        with open(os.path.join(GOLDEN, name)) as a, open(tmp_path / name) as b:
            assert a.read() == b.read(), name


@pytest.mark.parametrize("n", [1, 9, 45])
def test_pca_branch(params, n):
    rng = np.random.default_rng(n)
    c = rng.normal(size=n)
    rot = rng.normal(size=3)
    pose = mano_oracle.pose_from_pca(params, c, rot)[0]
    ref = (c @ params["pose_pca_basis"][:n] + params["pose_pca_mean"]).reshape(15, 3)
    assert np.allclose(pose[1:], ref) and np.allclose(pose[0], rot)


def test_check_sample_leg(tmp_path):
    """bench.py's correctness leg (oracle/check_sample.py, run as a child
    process by the bench): exact oracle outputs read as ~0 error, a 2e-5 m
    perturbation of one hand is found and reported with its global index."""
    import json
    import subprocess
    import sys
    from mano_amd.model_io import synthetic_params
    from oracle import mano_oracle
    from conftest import REPO
    rng = np.random.default_rng(3)
    n = 7
    betas = rng.normal(0, 1, (n, 10)).astype(np.float32)
    pose = rng.normal(0, 0.5, (n, 16, 3)).astype(np.float32)
    trans = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    ref = mano_oracle.forward(synthetic_params(0), betas.astype(np.float64), pose.astype(np.float64),
                              trans.astype(np.float64))
    verts = ref["verts"].astype(np.float64)
    verts[4, 100, 1] += 2e-5
    path = tmp_path / "s.npz"
    np.savez(path, index=np.arange(1000, 1000 + n), betas=betas, pose=pose, trans=trans, verts=verts,
             joints=ref["joints"], model=np.array("synthetic:0"))
    r = subprocess.run([sys.executable, f"{REPO}/oracle/check_sample.py", str(path)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["n_sampled"] == n and res["finite"]
    assert 1.5e-5 < res["max_abs_err_verts"] < 2.5e-5 and res["worst_hand_verts"] == 1004
    assert res["max_abs_err_joints"] < 1e-12
