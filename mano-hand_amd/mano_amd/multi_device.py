"""One process, one host thread, n GPUs: the single-process multi-device forward.

The reference is a single process whose batch is a Python loop over hands
(`data_explore.py:12-15` calling `mano_np.py:48-115` per hand); hands are
independent, so this host layer splits a batch into contiguous shards
(`distributed.shard_range`), runs each shard's forward on its own GPU and
stream -- every launch is asynchronous, so one thread keeps all devices busy
-- and, when the caller wants every vertex on one device, assembles the
shards on the root GPU with ONE RCCL group from the same thread
(`mano_comm_create_all` = ncclCommInitAll over the devices, `mano_group_start`
/ `mano_group_end` around one `mano_gather` per device: every peer sends its
shard straight to the root over its own xGMI link; include/mano_hip.h ABI 6).
The root's own shard is computed in place in the assembled buffers, so only
the peers' shards move.  `gather="copy"` assembles with peer copies instead
(hipMemcpyPeerAsync through torch), which also works when a device is listed
twice (a 1-GPU rehearsal of the sharding).

torch supplies device memory, streams and events only; every computation is a
libmano_hip.so launch.
"""
from __future__ import annotations

import ctypes
import math
from typing import Dict, List, Optional, Sequence

import torch

from . import _abi
from .distributed import shard_range
from .model import ManoHip
from .model_io import N_JOINTS


class DeviceComms:
    """One RCCL communicator per device, made in one call by this thread
    (mano_comm_create_all: rank i on devices[i]), and the grouped gather."""

    def __init__(self, devices: Sequence[int]):
        self.devices = [int(d) for d in devices]
        n = len(self.devices)
        arr = (ctypes.c_int * n)(*self.devices)
        comms = (ctypes.c_void_p * n)()
        _abi.check(_abi.lib().mano_comm_create_all(n, arr, comms))
        self._c: Optional[List[ctypes.c_void_p]] = [ctypes.c_void_p(c) for c in comms]

    def gather(self, pieces: Sequence[Sequence[torch.Tensor]], outs: Sequence[torch.Tensor],
               root: int, streams: Sequence[torch.cuda.Stream]) -> None:
        """pieces[i][k]: device i's contiguous shard of output k (rows along
        dim 0, shard_range order); outs[k] on devices[root] receives all rows
        of output k.  All 2 x n mano_gather calls go in one RCCL group: they
        are issued together when the group ends, each on its device's stream."""
        if self._c is None:
            raise RuntimeError("communicators are closed")
        lib = _abi.lib()
        n = len(self.devices)
        if len(pieces) != n or len(streams) != n or not 0 <= root < n:
            raise ValueError(f"{len(pieces)} piece lists / {len(streams)} streams / root {root} "
                             f"for {n} devices")
        # Every call's arguments, checked before the group posts anything
        # (mano_gather_check runs mano_gather's own checks): a call refused
        # half way through a group would leave the calls before it posted, and
        # ncclGroupEnd would launch a root receive whose send never comes.
        calls = []
        for k, out in enumerate(outs):
            if len(pieces[root]) <= k or out.device != pieces[root][k].device or not out.is_contiguous():
                raise ValueError(f"output {k} must be contiguous on the root's device")
            row = math.prod(out.shape[1:]) * out.element_size()
            sizes = (ctypes.c_size_t * n)(*[pieces[i][k].shape[0] * row for i in range(n)])
            if sum(sizes) != out.numel() * out.element_size():
                raise ValueError(f"output {k} holds {out.shape[0]} rows, the pieces {sum(sizes) // row}")
            for i in range(n):
                p = pieces[i][k]
                if not p.is_contiguous() or p.device != torch.device("cuda", self.devices[i]):
                    raise ValueError(f"piece {k} of device {self.devices[i]} must be contiguous on it")
                args = (self._c[i], ctypes.c_void_p(p.data_ptr()), p.shape[0] * row,
                        ctypes.c_void_p(out.data_ptr()) if i == root else None, sizes, root)
                _abi.check(lib.mano_gather_check(*args))
                calls.append(args + (ctypes.c_void_p(streams[i].cuda_stream),))
        _abi.check(lib.mano_group_start())
        try:
            for args in calls:
                _abi.check(lib.mano_gather(*args))
        except BaseException:
            # a failure past the checks (HIP / RCCL): close the group without
            # masking the original error; the streams' state is then undefined
            lib.mano_group_end()
            raise
        _abi.check(lib.mano_group_end())

    def n_ranks(self) -> List[int]:
        """Each communicator's rank count as RCCL holds it (mano_comm_info)."""
        if self._c is None:
            raise RuntimeError("communicators are closed")
        out = []
        for c in self._c:
            n = ctypes.c_int32()
            _abi.check(_abi.lib().mano_comm_info(c, ctypes.byref(n), None, None))
            out.append(n.value)
        return out

    def close(self):
        if self._c is not None:
            for c in self._c:
                _abi.check(_abi.lib().mano_comm_destroy(c))
            self._c = None


class ManoMultiDevice:
    """The MANO forward over several GPUs from one host thread.

    devices: GPU indices (default: every visible GPU); root: the index INTO
    `devices` of the GPU that receives gathered outputs."""

    def __init__(self, params: Dict[str, object], devices: Optional[Sequence[int]] = None,
                 precision: str = "fp32", root: int = 0):
        if devices is None:
            devices = list(range(torch.cuda.device_count()))
        self.devices = [int(d) for d in devices]
        if not self.devices:
            raise ValueError("no devices")
        if not 0 <= root < len(self.devices):
            raise ValueError(f"root {root} is not an index into devices {self.devices}")
        self.root = root
        self.engines = [ManoHip(params, device=d, precision=precision) for d in self.devices]
        self.streams = [torch.cuda.Stream(device=d) for d in self.devices]
        self.n_verts = self.engines[0].n_verts
        self._comms: Optional[DeviceComms] = None

    @property
    def root_device(self) -> torch.device:
        return torch.device("cuda", self.devices[self.root])

    def shard_ranges(self, n_total: int):
        n = len(self.devices)
        return [shard_range(n_total, r, n) for r in range(n)]

    def comms(self) -> DeviceComms:
        """The RCCL communicators (made on first use)."""
        if self._comms is None:
            self._comms = DeviceComms(self.devices)
        return self._comms

    # ---------------------------------------------------------------- forward
    def _enter(self):
        """Order this call's work after everything the caller has queued on
        each device's current stream.  The returned tensors are allocated on
        the internal streams, so when the caller frees one, the caching
        allocator may hand its block to the next call's allocations on those
        streams at once; with the internal streams waiting here, the next
        call's writes cannot overtake the caller's reads of the old result
        (nor its writes of this call's inputs)."""
        for d, s in zip(self.devices, self.streams):
            s.wait_stream(torch.cuda.current_stream(torch.device("cuda", d)))

    def _alloc_outputs(self, n_total, joints, gather):
        """Per device: the (verts, joints) its forward writes.  With a gather,
        the root's rows of the assembled buffers (allocated on the root's
        stream) are its outputs, so its shard never moves."""
        V = self.n_verts
        ranges = self.shard_ranges(n_total)
        assembled = None
        if gather:
            rd, rs = self.root_device, self.streams[self.root]
            with torch.cuda.device(rd), torch.cuda.stream(rs):
                assembled = {"verts": torch.empty((n_total, V, 3), device=rd)}
                if joints:
                    assembled["joints"] = torch.empty((n_total, N_JOINTS, 3), device=rd)
        per = []
        for i, (d, s) in enumerate(zip(self.devices, self.streams)):
            a, b = ranges[i]
            if gather and i == self.root:
                per.append({k: t[a:b] for k, t in assembled.items()})
                continue
            with torch.cuda.device(d), torch.cuda.stream(s):
                o = {"verts": torch.empty((b - a, V, 3), device=torch.device("cuda", d))}
                if joints:
                    o["joints"] = torch.empty((b - a, N_JOINTS, 3), device=torch.device("cuda", d))
            per.append(o)
        return ranges, per, assembled

    def _finish(self, ranges, per, assembled, joints, gather):
        keys = ["verts"] + (["joints"] if joints else [])
        if gather == "rccl":
            self.comms().gather([[per[i][k] for k in keys] for i in range(len(self.devices))],
                                [assembled[k] for k in keys], self.root, self.streams)
        elif gather == "copy":
            rd, rs = self.root_device, self.streams[self.root]
            for i, s in enumerate(self.streams):
                if i == self.root:
                    continue
                a, b = ranges[i]
                if b == a:
                    continue
                rs.wait_stream(s)            # the peer's shard is written
                with torch.cuda.device(rd), torch.cuda.stream(rs):
                    for k in keys:
                        assembled[k][a:b].copy_(per[i][k], non_blocking=True)
                # the peer's buffers are read on the root's stream: their
                # memory returns to the peer's pool only after that copy
                for k in keys:
                    per[i][k].record_stream(rs)
        if gather:
            # the caller's current stream on the root orders after the gather
            # (and, for RCCL, the peers' sends ran on their own streams, which
            # the root's receive completes with)
            torch.cuda.current_stream(self.root_device).wait_stream(self.streams[self.root])
            return assembled
        for d, s in zip(self.devices, self.streams):
            torch.cuda.current_stream(torch.device("cuda", d)).wait_stream(s)
        return per

    def forward(self, betas: torch.Tensor, pose: torch.Tensor, trans: Optional[torch.Tensor] = None, *,
                joints: bool = True, gather="rccl"):
        """Batched forward of (B,10) betas and (B,16,3) poses (and (B,3)
        trans), on any one device or the host, split over the devices.

        gather "rccl" / "copy": returns {"verts": (B,V,3), "joints": (B,16,3)}
        on the root device; False: a list of per-device dicts holding rows
        shard_range(B, i, n) of the batch."""
        if gather not in ("rccl", "copy", False, None):
            raise ValueError(f"gather must be 'rccl', 'copy' or False, got {gather!r}")
        gather = gather or False
        B = pose.shape[0]
        pose = pose.reshape(B, N_JOINTS, 3)
        self._enter()
        ranges, per, assembled = self._alloc_outputs(B, joints, gather)
        src_stream = torch.cuda.current_stream(pose.device) if pose.is_cuda else None
        for i, (eng, d, s) in enumerate(zip(self.engines, self.devices, self.streams)):
            a, b = ranges[i]
            if b == a:
                continue
            dev = torch.device("cuda", d)
            if src_stream is not None:
                s.wait_stream(src_stream)    # the inputs are written
            with torch.cuda.device(dev), torch.cuda.stream(s):
                take = lambda t: None if t is None else t[a:b].to(dev, non_blocking=True).contiguous()  # noqa: E731
                bt = betas if betas.dim() == 1 else betas[a:b]
                bt = bt.to(dev, non_blocking=True).contiguous()
                eng.forward(bt, take(pose), take(trans), joints=joints, out=per[i], stream=s)
        return self._finish(ranges, per, assembled, joints, gather)

    def forward_pca(self, betas: torch.Tensor, pca: torch.Tensor, rot: Optional[torch.Tensor] = None,
                    trans: Optional[torch.Tensor] = None, *, joints: bool = True, gather="rccl"):
        """Batched set_params(pose_pca=c, global_rot=rot, shape=beta)
        (mano_np.py:66-77) split over the devices: ManoHip.forward_pca per
        shard.  pca (B,N) or (N,) shared, rot (B,3) / (3,) shared / None,
        betas (B,10) / (10,); outputs as in `forward`."""
        if gather not in ("rccl", "copy", False, None):
            raise ValueError(f"gather must be 'rccl', 'copy' or False, got {gather!r}")
        gather = gather or False
        B = pca.shape[0] if pca.dim() == 2 else (betas.shape[0] if betas.dim() == 2 else None)
        if B is None:
            raise ValueError("batch size unknown: give (B,N) pca or (B,10) betas")
        self._enter()
        ranges, per, assembled = self._alloc_outputs(B, joints, gather)
        src = next((t for t in (pca, betas, rot, trans) if t is not None and t.is_cuda), None)
        src_stream = torch.cuda.current_stream(src.device) if src is not None else None
        for i, (eng, d, s) in enumerate(zip(self.engines, self.devices, self.streams)):
            a, b = ranges[i]
            if b == a:
                continue
            dev = torch.device("cuda", d)
            if src_stream is not None:
                s.wait_stream(src_stream)
            with torch.cuda.device(dev), torch.cuda.stream(s):
                def take(t, per_hand):
                    if t is None:
                        return None
                    return (t[a:b] if per_hand else t).to(dev, non_blocking=True).contiguous()
                eng.forward_pca(take(betas, betas.dim() == 2), take(pca, pca.dim() == 2),
                                take(rot, rot is not None and rot.dim() == 2 and rot.shape[0] == B),
                                take(trans, True), joints=joints, out=per[i], stream=s)
        return self._finish(ranges, per, assembled, joints, gather)

    def forward_synthetic(self, seed: int, n_total: int, *, trans: bool = False, joints: bool = True,
                          gather="rccl"):
        """The forward of global hands 0..n_total-1 of the counter-based
        synthetic batch (mano_synthetic_inputs): each device generates its own
        shard's inputs by global index, so no input crosses a link."""
        if gather not in ("rccl", "copy", False, None):
            raise ValueError(f"gather must be 'rccl', 'copy' or False, got {gather!r}")
        gather = gather or False
        self._enter()
        ranges, per, assembled = self._alloc_outputs(n_total, joints, gather)
        for i, (eng, s) in enumerate(zip(self.engines, self.streams)):
            a, b = ranges[i]
            if b == a:
                continue
            inp = eng.synthetic_inputs(seed, a, b - a, trans=trans, stream=s)  # allocated on s
            eng.forward(inp["betas"], inp["pose"], inp.get("trans"), joints=joints, out=per[i], stream=s)
        return self._finish(ranges, per, assembled, joints, gather)

    def gather_bandwidth(self, n_total: int, reps: int = 5, seed: int = 1003) -> Dict[str, object]:
        """Measure the RCCL group gather alone: every device forwards its shard
        of `n_total` synthetic hands (the root's in place in the assembled
        buffers), then the gather of verts + joints into the root runs `reps`
        times between HIP events on the root's stream (after one untimed
        call).  Returns the mean ms and the rate of the peers' bytes into the
        root -- the xGMI figure of a multi-GPU node."""
        self._enter()
        ranges, per, assembled = self._alloc_outputs(n_total, True, True)
        for i, (eng, s) in enumerate(zip(self.engines, self.streams)):
            a, b = ranges[i]
            if b > a:
                inp = eng.synthetic_inputs(seed, a, b - a, stream=s)
                eng.forward(inp["betas"], inp["pose"], None, joints=True, out=per[i], stream=s)
        keys = ("verts", "joints")
        pieces = [[p[k] for k in keys] for p in per]
        outs = [assembled[k] for k in keys]
        comms = self.comms()
        comms.gather(pieces, outs, self.root, self.streams)
        for d in sorted(set(self.devices)):
            torch.cuda.synchronize(d)
        rs = self.streams[self.root]
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for e0, e1 in evs:
            for d in sorted(set(self.devices)):
                torch.cuda.synchronize(d)
            e0.record(rs)
            comms.gather(pieces, outs, self.root, self.streams)
            e1.record(rs)
        for d in sorted(set(self.devices)):
            torch.cuda.synchronize(d)
        ms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / max(1, reps)
        row = sum(math.prod(o.shape[1:]) * o.element_size() for o in outs)
        to_root = sum((b - a) * row for i, (a, b) in enumerate(ranges) if i != self.root)
        return {"ms": ms, "bytes_to_root": to_root, "GBs_to_root": to_root / (ms * 1e-3) / 1e9 if ms > 0 else None,
                "devices": list(self.devices), "reps": reps,
                "form": "one RCCL group of mano_gather from this thread (peers' ncclSend, the root's "
                        "ncclRecv), the root's shard in place; HIP events on the root's stream"}

    def synchronize(self) -> None:
        """Wait for every device's stream; raise DeviceStatusError if a launch
        on any device raised a MANO_DEVICE_* bit."""
        for eng, s in zip(self.engines, self.streams):
            eng.synchronize(s)

    def close(self) -> None:
        if self._comms is not None:
            self._comms.close()
            self._comms = None
        for e in self.engines:
            e.close()
        self.engines = []
