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


# ---- official-pickle ingestion without chumpy ----------
# chumpy is not installed and no official MANO pickle exists here, so the
# official file is imitated: a stand-in `chumpy.ch.Ch` class (same module and
# class name, value kept in `x` as chumpy leaves do) and a real scipy CSC
# matrix.  Parity with a real MANO_*.pkl is unpinned.
import sys
import types


def _official_like(params, protocol):
    scipy_sparse = pytest.importorskip("scipy.sparse")
    mods = {}
    for name in ("chumpy", "chumpy.ch"):
        mods[name] = sys.modules.get(name)
    pkg = types.ModuleType("chumpy")
    ch = types.ModuleType("chumpy.ch")

    class Ch(object):
        def __init__(self, x):
            self.x = np.asarray(x)
            self._dirty_vars = set()
            self.label = None

    Ch.__module__, Ch.__qualname__ = "chumpy.ch", "Ch"
    ch.Ch = Ch
    pkg.ch = ch
    sys.modules["chumpy"], sys.modules["chumpy.ch"] = pkg, ch
    try:
        kintree = np.array([[4294967295] + [p for p in params["parents"][1:]], list(range(16))],
                           dtype=np.int64)
        official = {
            "hands_components": np.asarray(params["pose_pca_basis"]),
            "hands_mean": np.asarray(params["pose_pca_mean"]),
            "J_regressor": scipy_sparse.csc_matrix(np.asarray(params["J_regressor"])),
            "weights": Ch(params["skinning_weights"]),
            "posedirs": Ch(params["mesh_pose_basis"]),
            "shapedirs": Ch(params["mesh_shape_basis"]),
            "v_template": Ch(params["mesh_template"]),
            "f": np.asarray(params["faces"], dtype=np.uint32),
            "kintree_table": kintree,
            "J": np.zeros((16, 3)),
            "bs_style": "lbs",
            "bs_type": "lrotmin",
        }
        return pickle.dumps(official, protocol=protocol)
    finally:
        for name, m in mods.items():
            if m is None:
                sys.modules.pop(name, None)
            else:
                sys.modules[name] = m


@pytest.mark.parametrize("protocol", [0, 2])
def test_load_official_without_chumpy(params, tmp_path, protocol):
    src = tmp_path / "MANO_LEFT.pkl"
    src.write_bytes(_official_like(params, protocol))
    assert "chumpy" not in sys.modules
    got = model_io.load_official(str(src))
    assert got["parents"] == model_io.MANO_PARENTS
    for k in model_io.MODEL_KEYS:
        if k == "parents":
            continue
        a, b = np.asarray(got[k]), np.asarray(params[k])
        assert a.shape == b.shape and np.array_equal(a, b.astype(a.dtype)), k
    # dump_model(): official -> dump layout file, readable by load_dump
    dst = tmp_path / "dump.pkl"
    model_io.dump_model(str(src), str(dst))
    back = model_io.load_dump(str(dst))
    model_io.check_layout(back)
    assert np.array_equal(np.asarray(back["J_regressor"]), np.asarray(params["J_regressor"]))


def test_load_official_refuses_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))

    p = tmp_path / "evil.pkl"
    p.write_bytes(pickle.dumps({"hands_components": Evil()}, protocol=2))
    with pytest.raises(pickle.UnpicklingError):
        model_io.load_official(str(p))


def _scan_fixture():
    from conftest import GOLDEN
    with np.load(os.path.join(GOLDEN, "mano_reference_scans.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_dump_scans_matches_reference(tmp_path):
    """dump_scans (dump_model.py:24-43) on official-layout pickles, against the
    reference's own output (tests/golden/make_scan_goldens.py ran it)."""
    g = _scan_fixture()
    paths = {}
    for side in ("left", "right"):
        official = {k: g[f"{side}_{k}"] for k in ("hands_components", "hands_mean", "hands_coeffs")}
        paths[side] = str(tmp_path / f"MANO_{side.upper()}.pkl")
        with open(paths[side], "wb") as f:
            pickle.dump(official, f, protocol=2)
    dst = str(tmp_path / "axangles.npy")
    got = model_io.dump_scans(paths["left"], paths["right"], dst)
    assert got.shape == g["axangles"].shape == (73, 15, 3)
    assert np.array_equal(got, g["axangles"])
    assert np.array_equal(np.load(dst, allow_pickle=False), g["axangles"])
    pose = model_io.scans_to_pose(got)                  # data_explore.py:13
    assert pose.shape == (73, 16, 3) and np.all(pose[:, 0] == 0) and np.array_equal(pose[:, 1:], got)
