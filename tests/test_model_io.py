"""Model-asset layout (dump_model.py:4-21) and the code-free loader."""
import os
import pickle

import numpy as np
import pytest

from mano_amd import model_io


def test_dump_roundtrip(params, tmp_path):
    p = str(tmp_path / "dump.pkl")
    model_io.save_dump(params, p)
    back = model_io.load_dump(p)
    assert set(back) == set(model_io.MODEL_KEYS)
    assert back["parents"] == model_io.MANO_PARENTS
    for k in model_io.MODEL_KEYS:
        if k != "parents":
            assert np.array_equal(np.asarray(back[k]), np.asarray(params[k])), k
    assert model_io.params_digest(back) == model_io.params_digest(params)


def test_reference_loader_reads_our_dump(params, tmp_path):
    """The file we write is exactly what mano_np.py:17-18 reads (plain dict pickle)."""
    p = str(tmp_path / "dump.pkl")
    model_io.save_dump(params, p)
    with open(p, "rb") as f:
        raw = pickle.load(f, encoding="bytes")  # our own file: safe to unpickle
    assert sorted(raw) == sorted(model_io.MODEL_KEYS)
    assert raw["parents"][0] is None


def test_npz_model(params, tmp_path):
    p = str(tmp_path / "m.npz")
    arrs = {k: np.asarray(params[k]) for k in model_io.MODEL_KEYS if k != "parents"}
    np.savez(p, parents=model_io.parents_to_int(params["parents"]), **arrs)
    back = model_io.load_dump(p)
    assert back["parents"] == model_io.MANO_PARENTS
    assert model_io.params_digest(back) == model_io.params_digest(params)


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned",))


def test_loader_refuses_code(tmp_path):
    p = str(tmp_path / "evil.pkl")
    with open(p, "wb") as f:
        pickle.dump({"mesh_template": _Evil()}, f)
    with pytest.raises(pickle.UnpicklingError):
        model_io.load_dump(p)


def test_missing_key_is_keyerror(params, tmp_path):
    p = str(tmp_path / "partial.pkl")
    with open(p, "wb") as f:
        pickle.dump({k: params[k] for k in model_io.MODEL_KEYS if k != "faces"}, f)
    with pytest.raises(KeyError):
        model_io.load_dump(p)


def test_missing_file_is_oserror(tmp_path):
    with pytest.raises(OSError):
        model_io.load_dump(str(tmp_path / "nope.pkl"))


def test_layout_checks(params):
    model_io.check_layout(params)
    bad = dict(params)
    bad["mesh_pose_basis"] = np.zeros((778, 3, 134))
    with pytest.raises(ValueError):
        model_io.check_layout(bad)
    bad = dict(params)
    bad["parents"] = [None, 0, 5] + list(params["parents"][3:])
    with pytest.raises(ValueError):
        model_io.check_layout(bad)


def test_synthetic_model_properties(params):
    assert params["mesh_template"].shape == (778, 3)
    assert params["mesh_shape_basis"].shape == (778, 3, 10)
    assert params["mesh_pose_basis"].shape == (778, 3, 135)
    assert params["faces"].shape == (1538, 3)
    assert np.allclose(params["J_regressor"].sum(1), 1.0) and (params["J_regressor"] >= 0).all()
    assert np.allclose(params["skinning_weights"].sum(1), 1.0)
    assert model_io.params_digest(model_io.synthetic_params(0)) == model_io.params_digest(params)
