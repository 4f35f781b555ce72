"""Host layer over the gfx950 C-ABI: the batched engine and the drop-in MANOModel.

`ManoHip`   -- device-resident model + batched forward over torch device
               tensors (betas (B,10), pose (B,16,3), trans (B,3) -> verts,
               joints, ...).  Every computation is a launch of libmano_hip.so;
               torch only supplies device memory and the stream.
`MANOModel` -- the reference's object API (/root/reference/mano_np.py:5-201):
               same constructor argument, `set_params` / `update` semantics and
               quirks, attributes `verts J R rest_verts pose shape rot faces
               parents`, `rodrigues`, `with_zeros`, `pack`, `export_obj`.
               Outputs are float64 numpy copies as in the reference; the
               forward itself runs on the GPU (float32).
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import numpy as np
import torch

from . import _abi
from .model_io import (MODEL_KEYS, N_JOINTS, N_SHAPE, check_layout, load_dump,
                       parents_to_int)

_F64P = ctypes.POINTER(ctypes.c_double)


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(_F64P)


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream_handle(device: torch.device, stream=None):
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return ctypes.c_void_p(s.cuda_stream)


# Workspace row layout of the blend-GEMM A operand (mano_internal.h x_pos):
# element k of a hand's X row sits at X_POS[k], so that a 16x16x4 MFMA
# fragment lane reads its four consecutive K steps with one 16-byte load.
X_STRIDE = 160
X_POS = np.array([16 * (k >> 4) + 4 * (k & 3) + ((k >> 2) & 3) for k in range(X_STRIDE)])


class ManoHip:
    """Device-resident MANO model on one GPU (wraps a `mano_model*` handle)."""

    def __init__(self, params: Dict[str, object], device=None, precision: str = "fp32"):
        """`precision`: "fp32" (exact fp32 MFMA, default) or "f16x3" (split-half
        MFMA, same error order; include/mano_hip.h MANO_PRECISION_*)."""
        check_layout(params)
        if device is None:
            idx = torch.cuda.current_device()
        elif isinstance(device, int):
            idx = device
        else:
            d = torch.device(device)
            idx = d.index if d.index is not None else torch.cuda.current_device()
        self.device = torch.device("cuda", idx)
        lib = _abi.lib()
        f64 = lambda k: np.ascontiguousarray(np.asarray(params[k], dtype=np.float64))  # noqa: E731
        tmpl = f64("mesh_template")
        self.n_verts = int(tmpl.shape[0])
        sdirs, pdirs = f64("mesh_shape_basis"), f64("mesh_pose_basis")
        if sdirs.shape[2] != N_SHAPE:
            raise ValueError(f"mesh_shape_basis must have {N_SHAPE} shape directions, got {sdirs.shape}")
        if len(params["parents"]) != N_JOINTS:
            raise ValueError(f"the HIP kernels are built for {N_JOINTS} joints")
        jreg, wts = f64("J_regressor"), f64("skinning_weights")
        par = parents_to_int(params["parents"])
        pca = params.get("pose_pca_basis")
        mean = params.get("pose_pca_mean")
        pca = None if pca is None else np.ascontiguousarray(np.asarray(pca, dtype=np.float64))
        mean = None if mean is None else np.ascontiguousarray(np.asarray(mean, dtype=np.float64))
        if pca is not None and (pca.shape != (45, 45) or mean.shape != (45,)):
            raise ValueError(f"pose_pca_basis/mean must be (45,45)/(45,), got {pca.shape}/{mean.shape}")
        torch.cuda.init()
        handle = ctypes.c_void_p()
        _abi.check(lib.mano_model_create(
            self.device.index, self.n_verts, _dptr(tmpl), _dptr(sdirs), _dptr(pdirs), _dptr(jreg),
            _dptr(wts), par.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
            None if pca is None else _dptr(pca), None if mean is None else _dptr(mean),
            ctypes.byref(handle)))
        self._h = handle
        self._ws: Dict[int, torch.Tensor] = {}  # stream handle -> workspace
        self.set_precision(precision)

    def set_precision(self, precision: str) -> None:
        """Arithmetic of forward / stage_blend_skin / stage_skin ("fp32" | "f16x3")."""
        if precision not in _abi.PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(_abi.PRECISIONS)}, got {precision!r}")
        _abi.check(_abi.lib().mano_model_set_precision(self._h, _abi.PRECISIONS[precision]))
        self.precision = precision

    # ------------------------------------------------------------------ utils
    def device_status(self, clear: bool = True, wait: bool = True) -> int:
        """The model's device status (include/mano_hip.h
        mano_model_device_status): 0, or MANO_DEVICE_* bits raised by a launch
        whose outputs are not valid.  `wait`: for every launch on the device
        first; `clear`: reset the bits (until then every launching call on
        the model raises DeviceStatusError, MANO_EDEVICE)."""
        st = ctypes.c_int32()
        flags = (_abi.MANO_STATUS_CLEAR if clear else 0) | (0 if wait else _abi.MANO_STATUS_NO_WAIT)
        _abi.check(_abi.lib().mano_model_device_status(self._h, ctypes.byref(st), flags))
        return st.value

    def check_device(self) -> None:
        """Raise DeviceStatusError if any launch since the last check raised a
        MANO_DEVICE_* bit (the bits are cleared)."""
        st = self.device_status(clear=True)
        if st:
            raise _abi.DeviceStatusError(st)

    def synchronize(self, stream=None) -> None:
        """Wait for `stream` (default: the device's current stream), then raise
        DeviceStatusError if a launch raised a MANO_DEVICE_* bit -- the point
        at which the asynchronous stage calls' outputs are known valid.  The
        bits stay set (later launches keep failing) until check_device() or
        device_status(clear=True)."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        s.synchronize()
        st = self.device_status(clear=False, wait=False)
        if st:
            raise _abi.DeviceStatusError(st)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _abi.check(_abi.lib().mano_model_destroy(self._h))
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter teardown order varies
        try:
            self.close()
        except Exception:
            pass

    def workspace_bytes(self, n: int) -> int:
        return int(_abi.lib().mano_workspace_bytes(self._h, n))

    def forward_workspace_bytes(self, n: int) -> int:
        return int(_abi.lib().mano_forward_workspace_bytes(self._h, n))

    def workspace_offsets(self, n: int):
        a, b, c = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        _abi.check(_abi.lib().mano_workspace_offsets(self._h, n, ctypes.byref(a), ctypes.byref(b),
                                                     ctypes.byref(c)))
        return a.value, b.value, c.value

    def workspace(self, n: int, forward_only: bool = False, stream=None) -> torch.Tensor:
        """Device workspace large enough for `n` hands (all stage calls, or with
        `forward_only` just mano_forward's X rows + transforms), one per stream.

        Launches on different streams never share a workspace (the header's
        rule for concurrent calls), and each workspace is allocated ON its
        stream, so when it grows the caching allocator hands the old block out
        again only in that stream's order -- never while a queued launch on the
        stream may still read it.  A grown workspace starts with the old one's
        contents (same offsets, workspace_layout depends on n only), so the
        X rows and transforms of a preceding forward() stay valid for the stage
        calls that need the larger, unfused layout."""
        lib = _abi.lib()
        need = int(lib.mano_forward_workspace_bytes(self._h, n) if forward_only
                   else lib.mano_workspace_bytes(self._h, n))
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        key = s.cuda_stream
        ws = self._ws.get(key)
        if ws is None or ws.numel() < need + 256:
            old = ws
            with torch.cuda.stream(s):
                ws = torch.empty(max(need, 256) + 256, dtype=torch.uint8, device=self.device)
                if old is not None:
                    src, dst = self._aligned_view(old), self._aligned_view(ws)
                    k = min(src.numel(), dst.numel())
                    dst[:k].copy_(src[:k])
            self._ws[key] = ws
        return ws

    @staticmethod
    def _aligned_view(ws: torch.Tensor) -> torch.Tensor:
        """The 256-B-aligned part of a workspace tensor (what the ABI is given)."""
        base = ws.data_ptr()
        return ws[((base + 255) & ~255) - base:]

    def _ws_args(self, n, forward_only: bool = False, stream=None, workspace=None):
        if workspace is not None:
            # the caller's own workspace (e.g. one a captured HIP graph holds),
            # never one of the per-stream entries above
            need = int(_abi.lib().mano_forward_workspace_bytes(self._h, n) if forward_only
                       else _abi.lib().mano_workspace_bytes(self._h, n))
            if (not isinstance(workspace, torch.Tensor) or workspace.device != self.device
                    or workspace.dtype != torch.uint8 or not workspace.is_contiguous()):
                raise ValueError(f"workspace must be a contiguous uint8 tensor on {self.device}")
            if workspace.numel() < need + 256:
                raise ValueError(f"workspace has {workspace.numel()} bytes, {need + 256} needed for {n} hands")
            ws = workspace
        else:
            ws = self.workspace(n, forward_only, stream)
        base = ws.data_ptr()
        aligned = (base + 255) & ~255
        return ctypes.c_void_p(aligned), ctypes.c_size_t(ws.numel() - (aligned - base))

    def _check(self, t: Optional[torch.Tensor], name: str, shape) -> Optional[torch.Tensor]:
        if t is None:
            return None
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"{name} must be a torch tensor on {self.device}")
        if t.device != self.device or t.dtype != torch.float32:
            raise ValueError(f"{name} must be float32 on {self.device}, got {t.dtype} on {t.device}")
        if tuple(t.shape) != tuple(shape):
            raise ValueError(f"{name} has shape {tuple(t.shape)}, expected {tuple(shape)}")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
        return t

    def _inputs(self, betas, pose, trans):
        if not isinstance(pose, torch.Tensor):
            raise TypeError("pose must be a torch tensor")
        B = pose.shape[0]
        pose = self._check(pose.reshape(B, N_JOINTS, 3) if pose.dim() == 2 else pose, "pose",
                           (B, N_JOINTS, 3))
        if betas.dim() == 1:
            betas = self._check(betas, "betas", (N_SHAPE,))
            bstride = 0
        else:
            betas = self._check(betas, "betas", (B, N_SHAPE))
            bstride = N_SHAPE
        trans = self._check(trans, "trans", (B, 3))
        return B, betas, bstride, pose, trans

    # --------------------------------------------------------------- forward
    def _outputs(self, out, stream, specs):
        """Output tensors: the caller's (checked) or new ones allocated on the
        launch stream (so the caching allocator orders their reuse after it)."""
        res = dict(out) if out else {}
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        for name, shape, want in specs:
            if not want:
                continue
            t = res.get(name)
            if t is None:
                with torch.cuda.stream(s):
                    t = torch.empty(shape, dtype=torch.float32, device=self.device)
                res[name] = t
            self._check(t, name, shape)
        return res

    def forward(self, betas: torch.Tensor, pose: torch.Tensor, trans: Optional[torch.Tensor] = None,
                *, joints: bool = True, rest_verts: bool = False, rest_joints: bool = False,
                rot_mats: bool = False, out: Optional[Dict[str, torch.Tensor]] = None,
                stream=None, workspace: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
        """Batched MANOModel.update() (mano_np.py:79-115) on the GPU.

        betas (B,10) or (10,) shared, pose (B,16,3) or (B,48) axis-angle,
        trans (B,3) optional.  Returns float32 device tensors: verts (B,V,3),
        and on request joints (B,16,3) posed, rest_verts (B,V,3),
        rest_joints (B,16,3), rot_mats (B,16,3,3).  `workspace`: a uint8
        device tensor of at least forward_workspace_bytes(B) + 256 bytes that
        the caller owns (default: the engine's per-stream workspace).
        """
        B, betas, bstride, pose, trans = self._inputs(betas, pose, trans)
        V = self.n_verts
        res = self._outputs(out, stream, (
            ("verts", (B, V, 3), True), ("joints", (B, N_JOINTS, 3), joints),
            ("rest_verts", (B, V, 3), rest_verts), ("rest_joints", (B, N_JOINTS, 3), rest_joints),
            ("rot_mats", (B, N_JOINTS, 3, 3), rot_mats)))
        g = lambda k: _ptr(res.get(k))  # noqa: E731
        ws, wsb = self._ws_args(B, forward_only=True, stream=stream, workspace=workspace)
        _abi.check(_abi.lib().mano_forward(
            self._h, B, _ptr(betas), bstride, _ptr(pose), _ptr(trans), g("verts"),
            g("joints") if joints else None, g("rest_verts") if rest_verts else None,
            g("rest_joints") if rest_joints else None, g("rot_mats") if rot_mats else None,
            ws, wsb, _stream_handle(self.device, stream)))
        return res

    def forward_pca(self, betas: torch.Tensor, pca: torch.Tensor, rot: Optional[torch.Tensor] = None,
                    trans: Optional[torch.Tensor] = None, *, joints: bool = True,
                    pose: bool = False, rest_verts: bool = False, rest_joints: bool = False,
                    rot_mats: bool = False, out: Optional[Dict[str, torch.Tensor]] = None,
                    stream=None) -> Dict[str, torch.Tensor]:
        """Batched set_params(pose_pca=c, global_rot=rot, shape=beta)
        (mano_np.py:66-77): the PCA map runs as the articulation prologue.

        pca (B,N) (0 <= N <= 45) or (N,) shared, rot (B,3) / (3,) shared / None
        (zero root rotation), betas as in `forward`.  `pose=True` also returns
        the (B,16,3) pose the kernels used."""
        if not isinstance(pca, torch.Tensor):
            raise TypeError("pca must be a torch tensor")
        if pca.dim() == 1:
            N = pca.shape[0]
            pca_stride = 0
        else:
            N = pca.shape[1]
            pca_stride = N
        if not 0 <= N <= 45:
            raise ValueError(f"pca has {N} coefficients; at most 45 (mano_np.py:55-56)")
        B = pca.shape[0] if pca.dim() == 2 else (betas.shape[0] if betas.dim() == 2 else None)
        if B is None:
            raise ValueError("batch size unknown: give (B,N) pca or (B,10) betas")
        self._check(pca, "pose_pca", tuple(pca.shape))
        if pca.dim() == 2 and pca.shape[0] != B:
            raise ValueError("pca rows must match the batch")
        if betas.dim() == 1:
            betas = self._check(betas, "betas", (N_SHAPE,))
            bstride = 0
        else:
            betas = self._check(betas, "betas", (B, N_SHAPE))
            bstride = N_SHAPE
        rot_stride = 0
        if rot is not None:
            if rot.dim() == 1 or (rot.dim() == 2 and rot.shape[0] == 1):
                rot = self._check(rot.reshape(3), "global_rot", (3,))
            else:
                rot = self._check(rot, "global_rot", (B, 3))
                rot_stride = 3
        trans = self._check(trans, "trans", (B, 3))
        V = self.n_verts
        res = self._outputs(out, stream, (
            ("verts", (B, V, 3), True), ("joints", (B, N_JOINTS, 3), joints),
            ("pose", (B, N_JOINTS, 3), pose),
            ("rest_verts", (B, V, 3), rest_verts), ("rest_joints", (B, N_JOINTS, 3), rest_joints),
            ("rot_mats", (B, N_JOINTS, 3, 3), rot_mats)))
        g = lambda k, want: _ptr(res.get(k)) if want else None  # noqa: E731
        ws, wsb = self._ws_args(B, forward_only=True, stream=stream)
        _abi.check(_abi.lib().mano_forward_pca(
            self._h, B, _ptr(betas), bstride, _ptr(pca), N, pca_stride, _ptr(rot), rot_stride,
            _ptr(trans), g("verts", True), g("joints", joints), g("pose", pose),
            g("rest_verts", rest_verts), g("rest_joints", rest_joints), g("rot_mats", rot_mats),
            ws, wsb, _stream_handle(self.device, stream)))
        return res

    # ---- the forward pass as separate kernels (per-kernel timing / intermediates) ----
    def stage_articulate(self, betas, pose, trans=None, joints=None, rest_joints=None,
                         rot_mats=None, stream=None):
        B, betas, bstride, pose, trans = self._inputs(betas, pose, trans)
        ws, wsb = self._ws_args(B, stream=stream)
        _abi.check(_abi.lib().mano_stage_articulate(
            self._h, B, _ptr(betas), bstride, _ptr(pose), _ptr(trans), _ptr(joints),
            _ptr(rest_joints), _ptr(rot_mats), ws, wsb, _stream_handle(self.device, stream)))

    def stage_blend(self, n: int, rest_verts=None, stream=None):
        ws, wsb = self._ws_args(n, stream=stream)
        _abi.check(_abi.lib().mano_stage_blend(self._h, n, _ptr(rest_verts), ws, wsb,
                                               _stream_handle(self.device, stream)))

    def stage_skin(self, n: int, verts: torch.Tensor, rest_verts=None, trans=None, stream=None):
        """Standalone LBS (mano_stage_skin).  Asynchronous: a lost hand-over
        inside the kernel (MANO_DEVICE_SKIN_HANDOFF_TIMEOUT) surfaces at
        `synchronize()` and makes every later launch on this model raise
        DeviceStatusError until `check_device()` clears it."""
        ws, wsb = self._ws_args(n, stream=stream)
        _abi.check(_abi.lib().mano_stage_skin(self._h, n, _ptr(rest_verts), _ptr(trans),
                                              _ptr(verts), ws, wsb,
                                              _stream_handle(self.device, stream)))

    def stage_blend_skin(self, n: int, verts: torch.Tensor, rest_verts=None, trans=None,
                         stream=None):
        """Fused blend GEMM + LBS (the second half of `forward`)."""
        ws, wsb = self._ws_args(n, stream=stream)
        _abi.check(_abi.lib().mano_stage_blend_skin(self._h, n, _ptr(rest_verts), _ptr(trans),
                                                    _ptr(verts), ws, wsb,
                                                    _stream_handle(self.device, stream)))

    def intermediates(self, n: int, stream=None) -> Dict[str, torch.Tensor]:
        """Views of the workspace after the stage calls over `n` hands:
        `features` (n, 160) the blend-GEMM A operand rows X = [beta | R-I
        features | 1 | 0...] in the kernels' k-permuted order (`X[:, k] =
        features[:, X_POS[k]]`), `transforms` (n,16,3,4) skinning transforms,
        `vposed` (n,V,3)."""
        ws = self.workspace(n, stream=stream)
        base = ws.data_ptr()
        shift = ((base + 255) & ~255) - base
        fo, to, vo = self.workspace_offsets(n)
        f32 = ws[shift:shift + (ws.numel() - shift) // 4 * 4].view(torch.float32)
        return {
            "features": f32[fo // 4: fo // 4 + n * X_STRIDE].view(n, X_STRIDE),
            "transforms": f32[to // 4: to // 4 + n * 192].view(n, N_JOINTS, 3, 4),
            "vposed": f32[vo // 4: vo // 4 + n * self.n_verts * 3].view(n, self.n_verts, 3),
        }

    # ---- synthetic workload (benchmarks and shard-invariance tests) ----
    def synthetic_inputs(self, seed: int, first: int, n: int, *, beta_sigma: float = 1.0,
                         pose_sigma: float = 0.5, trans_range: float = 1.0, trans: bool = False,
                         stream=None) -> Dict[str, torch.Tensor]:
        """Hands first..first+n-1 of the counter-based (Philox) synthetic batch
        keyed by `seed` (include/mano_hip.h mano_synthetic_inputs): betas
        (n,10) ~ N(0, beta_sigma^2), pose (n,16,3) ~ N(0, pose_sigma^2), and
        with `trans` (n,3) ~ U(-trans_range, trans_range).  Any shard of a
        global batch reproduces the same hands bit for bit."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        with torch.cuda.stream(s):
            out = {"betas": torch.empty((n, N_SHAPE), dtype=torch.float32, device=self.device),
                   "pose": torch.empty((n, N_JOINTS, 3), dtype=torch.float32, device=self.device)}
            if trans:
                out["trans"] = torch.empty((n, 3), dtype=torch.float32, device=self.device)
        _abi.check(_abi.lib().mano_synthetic_inputs(
            self.device.index, seed, first, n, beta_sigma, pose_sigma, trans_range,
            _ptr(out["betas"]), _ptr(out["pose"]), _ptr(out.get("trans")),
            _stream_handle(self.device, stream)))
        return out

    # ---- set_params' PCA branch and the Rodrigues helper on device ----
    def pose_from_pca(self, pca: torch.Tensor, rot: Optional[torch.Tensor] = None,
                      stream=None) -> torch.Tensor:
        """pose (B,16,3) = [rot | pca @ pose_pca_basis[:N] + mean] (mano_np.py:66-72)."""
        if pca.dim() == 1:
            pca = pca[None]
        B, N = pca.shape
        self._check(pca, "pose_pca", (B, N))
        if rot is not None:
            rot = self._check(rot.reshape(-1, 3), "global_rot", (rot.numel() // 3, 3))
            rot_stride = 0 if rot.shape[0] == 1 else 3
            if rot.shape[0] not in (1, B):
                raise ValueError("global_rot must have 1 or B rows")
        else:
            rot_stride = 0
        pose = torch.empty((B, N_JOINTS, 3), dtype=torch.float32, device=self.device)
        _abi.check(_abi.lib().mano_pose_from_pca(self._h, B, _ptr(pca), N, N, _ptr(rot), rot_stride,
                                                 _ptr(pose), _stream_handle(self.device, stream)))
        return pose

    def rodrigues(self, axis_angle: torch.Tensor, stream=None) -> torch.Tensor:
        """(..., 3) axis-angle -> (..., 3, 3) rotations (mano_np.py:117-148)."""
        aa = axis_angle.reshape(-1, 3).contiguous()
        self._check(aa, "axis_angle", (aa.shape[0], 3))
        rot = torch.empty((aa.shape[0], 3, 3), dtype=torch.float32, device=self.device)
        _abi.check(_abi.lib().mano_rodrigues(self.device.index, aa.shape[0], _ptr(aa), _ptr(rot),
                                             _stream_handle(self.device, stream)))
        return rot.reshape(axis_angle.shape[:-1] + (3, 3))


class MANOModel:
    """Drop-in for the reference `MANOModel` (mano_np.py:5-201), GPU-backed.

    * Call `set_params` to set pose and shape params.
    * Call `export_obj` to export to obj file.
    """

    def __init__(self, model_path, device=None):
        """model_path: a model dumped by `dump_model.py` (mano_np.py:11-46)."""
        params = load_dump(model_path)
        self._init_from_params(params, device)

    @classmethod
    def from_params(cls, params: Dict[str, object], device=None) -> "MANOModel":
        self = cls.__new__(cls)
        self._init_from_params(params, device)
        return self

    def _init_from_params(self, params, device):
        self.pose_pca_basis = params["pose_pca_basis"]
        self.pose_pca_mean = params["pose_pca_mean"]
        self.J_regressor = params["J_regressor"]
        self.skinning_weights = params["skinning_weights"]
        self.mesh_pose_basis = params["mesh_pose_basis"]
        self.mesh_shape_basis = params["mesh_shape_basis"]
        self.mesh_template = params["mesh_template"]
        self.faces = params["faces"]
        self.parents = params["parents"]
        self.n_joints = 16
        self.n_shape_params = 10
        self.engine = ManoHip({k: params[k] for k in MODEL_KEYS}, device=device)
        self.device = self.engine.device
        self.pose = np.zeros((self.n_joints, 3))
        self.shape = np.zeros(self.n_shape_params)
        self.rot = np.zeros([1, 3])
        self.trans = np.zeros(3)
        self.verts = None
        self.rest_verts = None
        self.J = None
        self.R = None
        self.joints = None
        self._io = None
        self._graphs = {}
        self._zc = {}
        self.update()

    def _dev(self, a) -> torch.Tensor:
        return torch.as_tensor(np.asarray(a, dtype=np.float32)).to(self.device)

    def set_params(self, pose_abs=None, pose_pca=None, shape=None, global_rot=None, trans=None):
        """Same semantics as mano_np.py:48-77, plus an optional translation.

        pose_abs: per-joint axis-angle, shape [16, 3] (or [48]); taken verbatim.
        pose_pca: [N] PCA coefficients, N <= 45; pose = c.basis[:N] + mean
          with the stored global rotation `rot` prepended (host float64; the
          batched device form is `ManoHip.forward_pca`).
        global_rot: only read on the pose_pca branch, then kept in `rot`.
        shape: the 10 shape coefficients.
        trans: (extension) global translation [3], kept in `trans`.
        Returns a copy of the updated vertices.
        """
        if pose_abs is not None:
            self.pose = pose_abs
        if pose_pca is not None:
            # Host float64, the reference's own arithmetic (mano_np.py:67-72), so
            # `pose` keeps float64 values across later shape-only updates.  A
            # list raises AttributeError (.shape), N > 45 a ValueError (the
            # matmul), N = 0 gives the mean pose -- all as the reference does.
            n = pose_pca.shape[0]
            fingers = (np.expand_dims(pose_pca, 0) @ np.asarray(self.pose_pca_basis)[:n])[0]
            fingers = np.reshape(fingers + self.pose_pca_mean, [self.n_joints - 1, 3])
            if global_rot is not None:
                self.rot = np.reshape(global_rot, [1, 3])
            self.pose = np.concatenate([self.rot, fingers], 0)
        if shape is not None:
            self.shape = shape
        if trans is not None:
            self.trans = np.reshape(np.asarray(trans, dtype=np.float64), (3,))
        self.update()
        return self.verts.copy()

    # The batch-1 update's inputs and outputs, packed: one pinned host block
    # each way.  Default (zero_copy): the two forward kernels read the input
    # block and write the output block in host memory directly (pinned host
    # memory is mapped into the device's address space), so a call is one
    # mano_forward and one stream sync: 24.7 us for that part against 34.6 us
    # for the copy form's graph replay (H2D, kernels, D2H) and 34.3 us for
    # the same kernels launched from device buffers through ManoHip.forward
    # (tools/debug/dropin_parts.py, profiles/r04i_dropin_parts.json; the
    # kernels are the same, bit-identical results).  A block the runtime
    # does not report as device-mapped takes the copy form: a device block
    # each way, one H2D, the kernels, one D2H, captured once per translation
    # mode and precision into a HIP graph (use_graphs) or launched eagerly.
    _IN = (("shape", (1, N_SHAPE)), ("pose", (1, N_JOINTS, 3)), ("trans", (1, 3)))
    _OUT = ("verts", "joints", "rest_verts", "rest_joints", "rot_mats")
    zero_copy = True
    use_graphs = True

    def _io_buffers(self):
        if self._io is None:
            V = self.engine.n_verts
            outs = (("verts", (1, V, 3)), ("joints", (1, N_JOINTS, 3)), ("rest_verts", (1, V, 3)),
                    ("rest_joints", (1, N_JOINTS, 3)), ("rot_mats", (1, N_JOINTS, 3, 3)))

            def carve(spec, dev, pinned):
                n = sum(int(np.prod(shp)) for _, shp in spec)
                d = torch.empty(n, dtype=torch.float32, device=dev)
                h = torch.empty(n, dtype=torch.float32, pin_memory=pinned)
                views, o = {}, 0
                for name, shp in spec:
                    k = int(np.prod(shp))
                    views[name] = (d[o:o + k].view(shp), h[o:o + k].numpy().reshape(shp[1:]))
                    o += k
                return d, h, views

            d_in, h_in, v_in = carve(self._IN, self.device, True)
            d_out, h_out, v_out = carve(outs, self.device, True)
            # the outputs' places in the host block (one float64 conversion per call)
            o = 0
            layout = []
            for name, shp in outs:
                k = int(np.prod(shp))
                layout.append((name, o, o + k, shp[1:]))
                o += k
            self._out_layout = tuple(layout)
            # the batch-1 forward's own workspace: the eager calls and every
            # captured graph use it (a graph holds its raw pointer), and it is
            # never one of the engine's per-stream workspaces, which another
            # call on a pooled stream of the same handle could regrow and free
            ws = torch.empty(self.engine.forward_workspace_bytes(1) + 256, dtype=torch.uint8,
                             device=self.device)
            self._io = (d_in, h_in, v_in, d_out, h_out, v_out, ws)
        return self._io

    def update(self):
        """Recompute every output on the GPU from pose / shape (mano_np.py:79-115)."""
        pose = np.asarray(self.pose.reshape((-1, 1, 3)), dtype=np.float64)  # list -> AttributeError
        if pose.size != 3 * self.n_joints:
            raise ValueError(f"pose has {pose.size} values, {3 * self.n_joints} expected")
        shape = np.asarray(self.shape, dtype=np.float64)
        if shape.shape != (self.n_shape_params,):
            raise ValueError(f"shape has shape {shape.shape}, ({self.n_shape_params},) expected")
        d_in, h_in, v_in, d_out, h_out, v_out, _ = self._io_buffers()
        # float64 -> float32 exactly as np.asarray(..., dtype=np.float32) would
        v_in["shape"][1][...] = shape
        v_in["pose"][1][...] = pose.reshape(self.n_joints, 3)
        v_in["trans"][1][...] = self.trans
        t = self.trans  # (3,) float64; three scalar tests cost less than np.any here
        with_trans = bool(t[0] != 0 or t[1] != 0 or t[2] != 0)
        s = torch.cuda.current_stream(self.device)
        zc = self._zero_copy_args(with_trans) if self.zero_copy else None
        if zc is not None:
            # mano_forward on the pinned blocks (the handle's precision)
            _abi.check(_abi.lib().mano_forward(*zc, ctypes.c_void_p(s.cuda_stream)))
        else:
            # a graph replays the kernels of the precision it was captured with
            g = self._graph((with_trans, self.engine.precision)) if self.use_graphs else None
            if g is not None:
                g.replay()
            else:
                self._update_body(with_trans)
        s.synchronize()
        blk = h_out.numpy().astype(np.float64)  # float64 views of one conversion
        host = {k: blk[a:b].reshape(shp) for k, a, b, shp in self._out_layout}
        self.verts = host["verts"]
        self.rest_verts = host["rest_verts"]
        self.J = host["rest_joints"]
        self.R = host["rot_mats"]
        self.joints = host["joints"]

    def _zero_copy_args(self, with_trans):
        """mano_forward's arguments (all but the stream) with the pinned host
        blocks as its inputs and outputs, or None when either block is not
        device-mapped host memory (then update() takes the copy form)."""
        if with_trans not in self._zc:
            d_in, h_in, v_in, d_out, h_out, v_out, ws = self._io_buffers()
            args = None
            if _abi.host_block_mapped(h_in.data_ptr()) and _abi.host_block_mapped(h_out.data_ptr()):
                hp = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731  (numpy views of the blocks)
                base = ws.data_ptr()
                aligned = (base + 255) & ~255
                args = (self.engine._h, 1, hp(v_in["shape"][1]), N_SHAPE, hp(v_in["pose"][1]),
                        hp(v_in["trans"][1]) if with_trans else None,
                        *(hp(v_out[k][1]) for k in self._OUT),
                        ctypes.c_void_p(aligned), ctypes.c_size_t(ws.numel() - (aligned - base)))
            self._zc[with_trans] = args
        return self._zc[with_trans]

    def _update_body(self, with_trans):
        """H2D of the packed inputs, mano_forward, D2H of the packed outputs
        (on the current stream; no sync)."""
        d_in, h_in, v_in, d_out, h_out, v_out, ws = self._io_buffers()
        d_in.copy_(h_in, non_blocking=True)
        self.engine.forward(v_in["shape"][0], v_in["pose"][0], v_in["trans"][0] if with_trans else None,
                            joints=True, rest_verts=True, rest_joints=True, rot_mats=True,
                            out={k: dv for k, (dv, _) in v_out.items()}, workspace=ws)
        h_out.copy_(d_out, non_blocking=True)

    def _graph(self, key):
        """The update body captured into a HIP graph (one per translation
        mode and engine precision), built on first use after an eager run on
        the capture stream.  The graph reads and writes only this object's
        packed I/O blocks and its private batch-1 workspace (`_io_buffers`),
        which live as long as the object."""
        with_trans = key[0]
        if key not in self._graphs:
            g = None
            cur = torch.cuda.current_stream(self.device)
            side = torch.cuda.Stream(self.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                self._update_body(with_trans)
            side.synchronize()
            try:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=side):
                    self._update_body(with_trans)
            except RuntimeError:
                g = None  # capture refused: keep the eager launches (same kernels)
            cur.wait_stream(side)
            # the graph holds raw pointers into the private workspace and the
            # I/O blocks; keep them referenced beside it
            self._graphs[key] = (g, side, self._io)
        return self._graphs[key][0]

    def forward_batch(self, betas, pose, trans=None, **kw):
        """Batched forward on device tensors; see `ManoHip.forward`."""
        return self.engine.forward(betas, pose, trans, **kw)

    def rodrigues(self, r):
        """Batched axis-angle [N,1,3] -> rotation [N,3,3] (mano_np.py:117-148), on the GPU."""
        r = np.asarray(r, dtype=np.float64)
        return self.engine.rodrigues(self._dev(r.reshape(-1, 3))).double().cpu().numpy()

    def with_zeros(self, x):
        """Append a [0, 0, 0, 1] row to a [3, 4] matrix (mano_np.py:150-163)."""
        return np.vstack((x, np.array([[0.0, 0.0, 0.0, 1.0]])))

    def pack(self, x):
        """[B,4,1] -> [B,4,4] with zero columns in front (mano_np.py:165-179)."""
        return np.dstack((np.zeros((x.shape[0], 4, 3)), x))

    def export_obj(self, path):
        """Write `path` and `<stem>_restpose.obj` in the format of mano_np.py:181-201."""
        write_obj(path, self.verts, self.faces)
        write_obj(path[:path.index(".obj")] + "_restpose.obj", self.rest_verts, self.faces)


def write_obj(path, verts, faces):
    """OBJ text exactly as mano_np.py:190-194: 'v %f %f %f' and 1-based 'f %d %d %d'."""
    v = np.asarray(verts, dtype=np.float64).reshape(-1, 3)
    f = np.asarray(faces).reshape(-1, 3) + 1
    with open(path, "w") as fp:
        fp.write("".join("v %f %f %f\n" % (a, b, c) for a, b, c in v))
        fp.write("".join("f %d %d %d\n" % (a, b, c) for a, b, c in f))
