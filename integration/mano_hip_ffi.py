"""mano_hip_ffi.py -- the binding a reyuwei/MANO-Hand maintainer drops next to mano_np.py.

numpy + ctypes only: no torch, no other framework.  It binds the C-ABI of
libmano_hip.so (include/mano_hip.h) and replaces the numpy body of
`MANOModel.update()` (mano_np.py:79-115) with one `mano_forward` launch on an
MI355X, keeping every attribute the reference sets there (`J` :83, `R` :86,
`rest_verts` :93, `verts` :114) as float64 arrays:

    from mano_np import MANOModel
    import mano_hip_ffi
    mano_hip_ffi.patch(MANOModel)          # update() now runs on the GPU
    model = MANOModel('dump_mano_left.pkl')
    verts = model.set_params(pose_pca=c, shape=beta, global_rot=[1, 0, 0])

Memory comes from the library itself, so the process never needs a GPU
framework: by default the inputs and outputs live in one pinned host block
(mano_host_alloc, mapped into the device's address space) that the kernels
read and write directly -- a call is one mano_forward and one
mano_synchronize, no copy; `Engine(..., zero_copy=False)` keeps them in
device buffers (mano_alloc) moved by mano_memcpy.  `Engine.forward` is the
batched form: (B, 10) betas and (B, 16, 3) poses in one launch pair.

The library is found at $MANO_HIP_LIB, else at the build's in-tree path.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "MANO_HIP_LIB", os.path.join(_HERE, "..", "mano-hand_amd", "mano_amd", "libmano_hip.so"))

_p, _i32, _i64, _sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t
_d = ctypes.POINTER(ctypes.c_double)
H2D, D2H = 1, 2  # MANO_MEMCPY_HOST_TO_DEVICE, MANO_MEMCPY_DEVICE_TO_HOST
STATUS_CLEAR, STATUS_NO_WAIT = 1, 2  # MANO_STATUS_CLEAR, MANO_STATUS_NO_WAIT
N_JOINTS, N_SHAPE = 16, 10

_lib = ctypes.CDLL(LIB_PATH)
for _name, _res, _args in (
        ("mano_model_create", ctypes.c_int, [ctypes.c_int, _i32, _d, _d, _d, _d, _d,
                                             ctypes.POINTER(_i32), _d, _d, ctypes.POINTER(_p)]),
        ("mano_model_destroy", ctypes.c_int, [_p]),
        ("mano_forward_workspace_bytes", _sz, [_p, _i64]),
        ("mano_forward", ctypes.c_int, [_p, _i64, _p, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _sz, _p]),
        ("mano_alloc", ctypes.c_int, [ctypes.c_int, _sz, ctypes.POINTER(_p)]),
        ("mano_free", ctypes.c_int, [ctypes.c_int, _p]),
        ("mano_memcpy", ctypes.c_int, [ctypes.c_int, _p, _p, _sz, _i32, _p]),
        ("mano_host_alloc", ctypes.c_int, [_sz, ctypes.POINTER(_p)]),
        ("mano_host_free", ctypes.c_int, [_p]),
        ("mano_synchronize", ctypes.c_int, [ctypes.c_int]),
        ("mano_model_device_status", ctypes.c_int, [_p, ctypes.POINTER(_i32), _i32]),
        ("mano_last_error", ctypes.c_char_p, [])):
    _fn = getattr(_lib, _name)
    _fn.restype, _fn.argtypes = _res, _args


def _check(rc):
    if rc != 0:
        raise RuntimeError(f"libmano_hip: {rc}: {_lib.mano_last_error().decode()}")


_IO = (("betas", N_SHAPE), ("pose", N_JOINTS * 3), ("verts", None), ("joints", N_JOINTS * 3),
       ("rest_verts", None), ("rest_joints", N_JOINTS * 3), ("rot_mats", N_JOINTS * 9))
_OUTS = ("verts", "joints", "rest_verts", "rest_joints", "rot_mats")


class Engine:
    """A device-resident MANO model plus I/O buffers for up to `capacity` hands
    (a pinned host block the kernels use directly, or device buffers)."""

    def __init__(self, model, device=0, capacity=1, zero_copy=True):
        """model: anything with the reference's array attributes (mano_np.py:20-33)."""
        self.zero_copy = zero_copy
        self._host, self._views = None, {}
        f = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float64))  # noqa: E731
        arrs = [f(model.mesh_template), f(model.mesh_shape_basis), f(model.mesh_pose_basis),
                f(model.J_regressor), f(model.skinning_weights)]
        par = np.array([-1 if p is None else int(p) for p in model.parents], dtype=np.int32)
        pca, mean = f(model.pose_pca_basis), f(model.pose_pca_mean)
        self.device, self.n_verts = device, arrs[0].shape[0]
        self._h = _p()
        _check(_lib.mano_model_create(device, self.n_verts, *[a.ctypes.data_as(_d) for a in arrs],
                                      par.ctypes.data_as(ctypes.POINTER(_i32)), pca.ctypes.data_as(_d),
                                      mean.ctypes.data_as(_d), ctypes.byref(self._h)))
        self._bufs = {}
        self.capacity = 0
        self._reserve(capacity)

    def _alloc(self, name, nbytes):
        ptr = _p()
        _check(_lib.mano_alloc(self.device, nbytes, ctypes.byref(ptr)))
        self._bufs[name] = ptr

    def _free_bufs(self):
        for name, ptr in self._bufs.items():
            if name == "workspace" or not self.zero_copy:
                _check(_lib.mano_free(self.device, ptr))
        self._bufs, self._views = {}, {}
        if self._host is not None:
            _check(_lib.mano_host_free(self._host))
            self._host = None

    def _reserve(self, n):
        if n <= self.capacity:
            return
        self._free_bufs()
        sizes = [(name, n * (f if f is not None else 3 * self.n_verts)) for name, f in _IO]
        if self.zero_copy:
            # one pinned block, each array at a 256-B boundary; the outputs
            # follow the inputs, so one float64 conversion reads them all
            offs, o = {}, 0
            for name, k in sizes:
                offs[name] = o
                o += (4 * k + 255) // 256 * 256
            self._host = _p()
            _check(_lib.mano_host_alloc(o, ctypes.byref(self._host)))
            block = np.ctypeslib.as_array(ctypes.cast(self._host, ctypes.POINTER(ctypes.c_uint8)), shape=(o,))
            for name, k in sizes:
                self._views[name] = block[offs[name]:offs[name] + 4 * k].view(np.float32)
                self._bufs[name] = _p(self._host.value + offs[name])
            self._out_block = block[offs["verts"]:].view(np.float32)
            self._out_at = {name: (offs[name] - offs["verts"]) // 4 for name, _ in sizes if name in _OUTS}
        else:
            for name, k in sizes:
                self._alloc(name, 4 * k)
        self._ws_bytes = _lib.mano_forward_workspace_bytes(self._h, n)
        self._alloc("workspace", self._ws_bytes)
        self.capacity = n

    def _put(self, name, a):
        a = np.ascontiguousarray(a, dtype=np.float32)
        if self.zero_copy:
            self._views[name][:a.size] = a.reshape(-1)
        else:
            _check(_lib.mano_memcpy(self.device, self._bufs[name], a.ctypes.data_as(_p), a.nbytes, H2D, None))

    def _get(self, name, shape):
        if self.zero_copy:
            return self._views[name][:int(np.prod(shape))].reshape(shape).astype(np.float64)
        out = np.empty(shape, dtype=np.float32)
        _check(_lib.mano_memcpy(self.device, out.ctypes.data_as(_p), self._bufs[name], out.nbytes, D2H, None))
        return out.astype(np.float64)

    def forward(self, betas, pose):
        """betas (B, 10), pose (B, 16, 3) axis-angle -> float64 host arrays:
        verts (B,V,3), J (B,16,3) rest joints, R (B,16,3,3), rest_verts (B,V,3),
        joints (B,16,3) posed joints."""
        pose = np.reshape(pose, (-1, N_JOINTS, 3))
        B = pose.shape[0]
        betas = np.reshape(betas, (B, N_SHAPE))
        self._reserve(B)
        self._put("betas", betas)
        self._put("pose", pose)
        b = self._bufs
        _check(_lib.mano_forward(self._h, B, b["betas"], N_SHAPE, b["pose"], None, b["verts"],
                                 b["joints"], b["rest_verts"], b["rest_joints"], b["rot_mats"],
                                 b["workspace"], self._ws_bytes, None))
        V = self.n_verts
        shapes = {"verts": (B, V, 3), "J": ("rest_joints", (B, N_JOINTS, 3)),
                  "R": ("rot_mats", (B, N_JOINTS, 3, 3)), "rest_verts": (B, V, 3), "joints": (B, N_JOINTS, 3)}
        shapes = {k: (v if isinstance(v[0], str) else (k, v)) for k, v in shapes.items()}
        if self.zero_copy:  # the outputs are in the host block once the launches completed
            _check(_lib.mano_synchronize(self.device))
            self._check_status()
            if B == self.capacity:
                # the whole output region is this call's: one conversion, then views of it
                out = self._out_block.astype(np.float64)
                at = self._out_at
                return {k: out[at[n]:at[n] + int(np.prod(s))].reshape(s) for k, (n, s) in shapes.items()}
            # B < capacity: only each output's first B rows (cost follows B, not capacity)
            return {k: self._get(n, s) for k, (n, s) in shapes.items()}
        out = {k: self._get(n, s) for k, (n, s) in shapes.items()}
        self._check_status()
        return out

    def _check_status(self):
        """The kernels finished: raise if one raised a MANO_DEVICE_* bit (its
        outputs are not valid; include/mano_hip.h mano_model_device_status).
        The bits are taken (MANO_STATUS_CLEAR) when they are reported: the
        error is raised once, for the call whose launches set them, and the
        next forward launches again -- left set, every later launch on the
        model would be refused with MANO_EDEVICE and the Engine unusable."""
        st = _i32(0)
        _check(_lib.mano_model_device_status(self._h, ctypes.byref(st), STATUS_NO_WAIT))
        if st.value:
            taken = _i32(0)
            _check(_lib.mano_model_device_status(self._h, ctypes.byref(taken), STATUS_NO_WAIT | STATUS_CLEAR))
            raise RuntimeError(f"libmano_hip: device status 0x{st.value | taken.value:x}: outputs not valid "
                               "(status cleared)")

    def close(self):
        if self._h:
            self._free_bufs()
            _check(_lib.mano_model_destroy(self._h))
            self._h = None


def patch(cls, device=0):
    """Replace cls.update (mano_np.py:79-115) with the GPU forward."""
    def update(self):
        pose = self.pose.reshape((-1, 3))  # a list pose raises AttributeError, as at :84
        shape = np.asarray(self.shape, dtype=np.float64)
        if shape.shape != (N_SHAPE,):  # the reference's shapedirs.dot(shape) raises too (:81)
            raise ValueError(f"shape has shape {shape.shape}, ({N_SHAPE},) expected")
        eng = self.__dict__.get("_hip_engine")
        if eng is None:
            eng = self._hip_engine = Engine(self, device)
        out = eng.forward(shape[None], pose[None])
        self.J, self.R, self.rest_verts, self.verts = (out[k][0] for k in ("J", "R", "rest_verts", "verts"))
    cls.update = update
    return cls
