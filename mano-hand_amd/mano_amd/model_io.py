"""MANO model-asset I/O: the `dump_model.py` layout, loaded without executing code.

The reference stores the model as a plain dict pickle written by
`dump_model()` (reference `dump_model.py:4-21`) and reads it back with
`pickle.load(f, encoding='bytes')` (reference `mano_np.py:17-18`).  The nine
keys and their shapes are the layout contract this module keeps:

    pose_pca_basis    (45, 45)        dump_model.py:8   (hands_components)
    pose_pca_mean     (45,)           dump_model.py:9   (hands_mean)
    J_regressor       (16, 778) dense dump_model.py:10  (.toarray())
    skinning_weights  (778, 16)       dump_model.py:11
    mesh_pose_basis   (778, 3, 135)   dump_model.py:13  (posedirs)
    mesh_shape_basis  (778, 3, 10)    dump_model.py:14  (shapedirs)
    mesh_template     (778, 3)        dump_model.py:15  (v_template)
    faces             (1538, 3) int   dump_model.py:16
    parents           list[16], parents[0] is None      dump_model.py:17-18

Unlike the reference we never run an unrestricted unpickler: `load_dump`
accepts only the globals numpy needs to rebuild arrays, so a hostile pickle
raises `pickle.UnpicklingError` instead of executing.  `.npz` files with the
same keys (``parents`` stored with -1 for the root) load too.

`synthetic_params()` is the deterministic stand-in for the licensed official
model (absent here): random arrays of the official shapes and magnitudes
(SURVEY.md §8d).  It is workload data for tests and benchmarks, not an oracle.
"""
from __future__ import annotations

import hashlib
import io
import pickle
from typing import Dict

import numpy as np

MODEL_KEYS = (
    "pose_pca_basis",
    "pose_pca_mean",
    "J_regressor",
    "skinning_weights",
    "mesh_pose_basis",
    "mesh_shape_basis",
    "mesh_template",
    "faces",
    "parents",
)

# MANO kinematic tree: wrist + 5 fingers x 3 joints (dump_model.py:17 kintree_table[0]).
MANO_PARENTS = [None, 0, 1, 2, 0, 4, 5, 0, 7, 8, 0, 10, 11, 0, 13, 14]
N_VERTS, N_JOINTS, N_SHAPE, N_FACES = 778, 16, 10, 1538
N_POSE_FEATS = 9 * (N_JOINTS - 1)  # 135

_SAFE_GLOBALS = {
    ("numpy.core.multiarray", "_reconstruct"),
    ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"),
    ("numpy._core.multiarray", "scalar"),
    ("numpy", "ndarray"),
    ("numpy", "dtype"),
    ("_codecs", "encode"),
}


class _ArrayOnlyUnpickler(pickle.Unpickler):
    """Unpickler that can rebuild numpy arrays and builtin containers only."""

    def find_class(self, module, name):  # noqa: D401 - pickle hook
        if (module, name) in _SAFE_GLOBALS:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(
            f"refusing to load global {module}.{name} from a model file "
            "(only numpy arrays are allowed)")


def _norm_key(k):
    return k.decode("latin1") if isinstance(k, bytes) else k


def load_dump(path: str) -> Dict[str, object]:
    """Load a `dump_model.py` dict pickle (or an .npz with the same keys).

    Mirrors reference `mano_np.py:17-33`: the returned dict carries the nine
    keys; a missing key raises KeyError and file errors raise OSError, as the
    reference's own loader does.
    """
    with open(path, "rb") as f:
        head = f.read(4)
        f.seek(0)
        if head[:2] == b"PK":  # npz archive
            with np.load(f, allow_pickle=False) as z:
                raw = {k: z[k] for k in z.files}
            if "parents" in raw:
                par = [int(p) for p in raw["parents"].tolist()]
                raw["parents"] = [None if p < 0 else p for p in par]
        else:
            raw = _ArrayOnlyUnpickler(f, encoding="bytes").load()
    if not isinstance(raw, dict):
        raise pickle.UnpicklingError("model file does not hold a dict")
    params = {_norm_key(k): v for k, v in raw.items()}
    out = {}
    for key in MODEL_KEYS:
        out[key] = params[key]  # KeyError on a missing key, like mano_np.py:20-33
    return out


def save_dump(params: Dict[str, object], path: str) -> None:
    """Write `params` in the exact `dump_model.py:20-21` form (dict pickle)."""
    out = {}
    for key in MODEL_KEYS:
        v = params[key]
        out[key] = list(v) if key == "parents" else np.asarray(v)
    with open(path, "wb") as f:
        pickle.dump(out, f)


# ---------------------------------------------------------------------------
# Official MANO_{LEFT,RIGHT}.pkl ingestion without chumpy.
#
# The official pickle (Python 2, read by the reference with
# `pickle.load(f, encoding='latin1')`, dump_model.py:6) stores chumpy `Ch`
# objects for weights / posedirs / shapedirs / v_template, a scipy CSC matrix
# for J_regressor and numpy arrays for the rest.  dump_model.py needs chumpy
# and scipy installed to rebuild them and then converts each to an array
# (dump_model.py:8-18).  `load_official` rebuilds the same arrays with a
# restricted unpickler that executes nothing: chumpy / scipy globals resolve to
# inert record classes that only keep their pickled state, and the arrays are
# read out of that state (a leaf `Ch` keeps its value in `x`; a CSC matrix in
# `data` / `indices` / `indptr` / `_shape`).  Parity unpinned: no official
# pickle exists here; tests/test_model_io.py checks the loader on pickles made
# with stand-in classes of the same module/class names and state fields.
# ---------------------------------------------------------------------------
class _Record:
    """Inert stand-in for a chumpy / scipy object: keeps the pickled state."""

    _origin = ""

    def __init__(self, *args, **kwargs):
        self.__dict__["_args"] = args

    def __setstate__(self, state):
        if isinstance(state, tuple) and len(state) == 2:  # (dict, slots) form
            state = {**(state[0] or {}), **(state[1] or {})}
        if isinstance(state, dict):
            self.__dict__.update({_norm_key(k): v for k, v in state.items()})


class _ChRecord(_Record):
    _origin = "chumpy"


class _CscRecord(_Record):
    _origin = "scipy.sparse csc_matrix"


def _safe_reconstructor(cls, base, state):
    """copyreg._reconstructor restricted to the record classes (protocol 0/1 pickles)."""
    if not (isinstance(cls, type) and issubclass(cls, _Record)) or base is not object:
        raise pickle.UnpicklingError(f"refusing to reconstruct {cls!r} from a model file")
    obj = cls.__new__(cls)
    obj.__dict__["_args"] = ()
    return obj


# builtins a chumpy object's state may hold (its caches and flags); constructing
# them from pickled data runs no user code.
_INERT_BUILTINS = {"object": object, "set": set, "frozenset": frozenset, "list": list,
                   "dict": dict, "tuple": tuple}


class _OfficialUnpickler(_ArrayOnlyUnpickler):
    """numpy arrays + inert records of chumpy / scipy.sparse objects, nothing else."""

    def find_class(self, module, name):
        if module.startswith("chumpy"):
            return _ChRecord
        if module.startswith("scipy.sparse") and name == "csc_matrix":
            return _CscRecord
        if (module, name) in (("copy_reg", "_reconstructor"), ("copyreg", "_reconstructor")):
            return _safe_reconstructor
        if module in ("__builtin__", "builtins") and name in _INERT_BUILTINS:
            return _INERT_BUILTINS[name]
        return super().find_class(module, name)


def _as_array(v, key):
    if isinstance(v, _ChRecord):
        if "x" not in v.__dict__:
            raise ValueError(f"{key}: chumpy object without a stored value 'x' "
                             "(a derived expression); cannot convert without chumpy")
        return np.asarray(v.__dict__["x"])
    if isinstance(v, _CscRecord):
        return _csc_dense(v, key)
    return np.asarray(v)


def _csc_dense(v, key):
    d = v.__dict__
    try:
        data, indices, indptr = (np.asarray(d[k]) for k in ("data", "indices", "indptr"))
        shape = tuple(int(x) for x in d.get("_shape", d.get("shape")))
    except (KeyError, TypeError) as e:
        raise ValueError(f"{key}: unrecognised CSC matrix state {sorted(d)}") from e
    out = np.zeros(shape, dtype=data.dtype)
    for c in range(shape[1]):  # column c holds rows indices[indptr[c]:indptr[c+1]]
        lo, hi = int(indptr[c]), int(indptr[c + 1])
        out[indices[lo:hi], c] += data[lo:hi]
    return out


def load_official(path: str) -> Dict[str, object]:
    """Official MANO pickle -> the nine-key dump layout (dump_model.py:4-18), no chumpy."""
    with open(path, "rb") as f:
        data = _OfficialUnpickler(f, encoding="latin1").load()
    if not isinstance(data, dict):
        raise pickle.UnpicklingError("official model file does not hold a dict")
    data = {_norm_key(k): v for k, v in data.items()}
    out = {
        "pose_pca_basis": _as_array(data["hands_components"], "hands_components"),  # :8
        "pose_pca_mean": _as_array(data["hands_mean"], "hands_mean"),               # :9
        "J_regressor": _as_array(data["J_regressor"], "J_regressor"),               # :10
        "skinning_weights": _as_array(data["weights"], "weights"),                   # :11
        "mesh_pose_basis": _as_array(data["posedirs"], "posedirs"),                  # :13
        "mesh_shape_basis": _as_array(data["shapedirs"], "shapedirs"),               # :14
        "mesh_template": _as_array(data["v_template"], "v_template"),                # :15
        "faces": _as_array(data["f"], "f"),                                          # :16
    }
    parents = _as_array(data["kintree_table"], "kintree_table")[0].tolist()         # :17
    parents[0] = None                                                                # :18
    out["parents"] = parents
    return out


def dump_model(src_path: str, dst_path: str) -> None:
    """dump_model.py:4-21 without chumpy: official pickle -> dump-layout pickle."""
    save_dump(load_official(src_path), dst_path)


def _scan_poses(path: str) -> np.ndarray:
    """One official pickle's captured hand poses: hands_coeffs . hands_components
    + hands_mean, as (M, 15, 3) finger axis-angles (dump_model.py:25-30)."""
    with open(path, "rb") as f:
        data = _OfficialUnpickler(f, encoding="latin1").load()
    if not isinstance(data, dict):
        raise pickle.UnpicklingError("official model file does not hold a dict")
    data = {_norm_key(k): v for k, v in data.items()}
    basis = _as_array(data["hands_components"], "hands_components")
    mean = _as_array(data["hands_mean"], "hands_mean")
    coeffs = _as_array(data["hands_coeffs"], "hands_coeffs")
    return np.reshape(np.matmul(coeffs, basis) + mean, [-1, N_JOINTS - 1, 3])


# The right hand's scans are mirrored into the left hand's frame (dump_model.py:38).
RIGHT_TO_LEFT = np.array([[[1, -1, -1]]])


def dump_scans(left_path: str, right_path: str, dst_path: str = None) -> np.ndarray:
    """dump_model.py:24-43 without chumpy: the captured scan poses of both
    official pickles as one (M_left + M_right, 15, 3) array of finger
    axis-angles (left, then right mirrored by [1, -1, -1]), saved with
    `np.save` when `dst_path` is given (the reference writes axangles.npy).
    This is the realistic pose source of data_explore.py:12-15."""
    left = _scan_poses(left_path)
    right = _scan_poses(right_path)
    right *= RIGHT_TO_LEFT
    axangles = np.concatenate([left, right])
    if dst_path is not None:
        np.save(dst_path, axangles)
    return axangles


def scans_to_pose(axangles) -> np.ndarray:
    """(M, 15, 3) scan axis-angles -> (M, 16, 3) full poses with a zero global
    rotation prepended, as data_explore.py:13 feeds them to set_params."""
    a = np.asarray(axangles, dtype=np.float64).reshape(-1, N_JOINTS - 1, 3)
    return np.concatenate([np.zeros((a.shape[0], 1, 3)), a], axis=1)


def parents_to_int(parents) -> np.ndarray:
    """`parents` list with None at the root -> int32 array with -1 at the root."""
    return np.array([-1 if p is None else int(p) for p in parents], dtype=np.int32)


def synthetic_params(seed: int = 0) -> Dict[str, object]:
    """Deterministic random MANO model of the official shapes.

    template ~ N(0, 0.05^2) m, shapedirs ~ N(0, 5e-3^2), posedirs ~ N(0, 2e-3^2);
    J_regressor non-negative, 32 supporting vertices per joint, rows sum to 1;
    skinning weights dense, non-negative, rows sum to 1 (worst case for LBS);
    PCA basis orthonormal rows scaled like the official `hands_components`.
    """
    rng = np.random.default_rng(seed)
    template = rng.normal(0.0, 0.05, (N_VERTS, 3))
    shapedirs = rng.normal(0.0, 5e-3, (N_VERTS, 3, N_SHAPE))
    posedirs = rng.normal(0.0, 2e-3, (N_VERTS, 3, N_POSE_FEATS))
    jreg = np.zeros((N_JOINTS, N_VERTS))
    for j in range(N_JOINTS):
        idx = rng.choice(N_VERTS, 32, replace=False)
        w = rng.random(32) + 0.05
        jreg[j, idx] = w / w.sum()
    weights = rng.random((N_VERTS, N_JOINTS)) ** 4 + 1e-3
    weights /= weights.sum(axis=1, keepdims=True)
    faces = np.stack([rng.choice(N_VERTS, 3, replace=False) for _ in range(N_FACES)]).astype(np.int64)
    q, _ = np.linalg.qr(rng.normal(size=(45, 45)))
    pca_basis = q.T * rng.uniform(0.2, 1.0, (45, 1))
    pca_mean = rng.normal(0.0, 0.15, 45)
    return {
        "pose_pca_basis": pca_basis,
        "pose_pca_mean": pca_mean,
        "J_regressor": jreg,
        "skinning_weights": weights,
        "mesh_pose_basis": posedirs,
        "mesh_shape_basis": shapedirs,
        "mesh_template": template,
        "faces": faces,
        "parents": list(MANO_PARENTS),
    }


def params_digest(params: Dict[str, object]) -> str:
    """SHA-256 over the nine arrays (fixtures pin the synthetic model with it)."""
    h = hashlib.sha256()
    for key in MODEL_KEYS:
        v = params[key]
        if key == "parents":
            v = parents_to_int(v)
        a = np.ascontiguousarray(np.asarray(v))
        h.update(key.encode())
        h.update(str(a.dtype).encode())
        h.update(str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def check_layout(params: Dict[str, object]) -> None:
    """Validate shapes against the dump layout; raise ValueError on mismatch."""
    tmpl = np.asarray(params["mesh_template"])
    if tmpl.ndim != 2 or tmpl.shape[1] != 3:
        raise ValueError(f"mesh_template must be (V, 3), got {tmpl.shape}")
    nv = tmpl.shape[0]
    par = params["parents"]
    nj = len(par)
    exp = {
        "mesh_shape_basis": (nv, 3, None),
        "mesh_pose_basis": (nv, 3, 9 * (nj - 1)),
        "J_regressor": (nj, nv),
        "skinning_weights": (nv, nj),
    }
    for key, shp in exp.items():
        a = np.asarray(params[key])
        if a.ndim != len(shp) or any(s is not None and s != d for s, d in zip(shp, a.shape)):
            raise ValueError(f"{key} has shape {a.shape}, expected {shp}")
    pi = parents_to_int(par)
    if pi[0] != -1 or any(not (0 <= pi[i] < i) for i in range(1, nj)):
        raise ValueError("parents must be None at the root and parents[i] < i elsewhere")


def to_bytes(params: Dict[str, object]) -> bytes:
    buf = io.BytesIO()
    pickle.dump({k: params[k] for k in MODEL_KEYS}, buf)
    return buf.getvalue()
