"""Debug: where the drop-in's batch-1 set_params time goes, and whether the
kernels reading / writing the pinned host blocks directly (no H2D / D2H copy
nodes) would be faster.

    python tools/debug/dropin_parts.py [--calls 400]

Parts, each the median over `calls` after 50 warm-up calls (same process,
same model, the graph of MANOModel's own update):
  set_params      the whole call (as bench.py's `dropin`)
  graph_sync      g.replay() + stream sync (H2D, two kernels, D2H)
  kernels_sync    the two forward kernels from device buffers + sync (eager)
  copies_sync     the H2D and D2H copies alone + sync (eager)
  sync_idle       a stream sync with nothing queued
  tiny_sync       one 1-element torch kernel + sync
  host_convert    update()'s float64 conversion of the five outputs
  zero_copy_sync  mano_forward with the pinned host blocks as its inputs and
                  outputs (no copies) + sync, eager; its verts compared with
                  the graph's bit for bit
  zero_copy_graph the same captured into a HIP graph, replay + sync
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "mano-hand_amd"))


def med(fn, calls, warm=50):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(calls):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts) * 1e6)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=400)
    a = ap.parse_args()
    import torch
    from mano_amd import MANOModel, synthetic_params, _abi
    params = synthetic_params(0)
    m = MANOModel.from_params(params, device=0)
    rng = np.random.default_rng(3)
    pose, shape = rng.normal(0, 0.5, (16, 3)), rng.normal(0, 1, 10)
    res = {}
    res["set_params"] = med(lambda: m.set_params(pose_abs=pose, shape=shape), a.calls)
    d_in, h_in, v_in, d_out, h_out, v_out, ws = m._io_buffers()
    s = torch.cuda.current_stream(m.device)
    g = m._graph((False, m.engine.precision))
    res["graph_sync"] = med(lambda: (g.replay(), s.synchronize()), a.calls)
    want = v_out["verts"][1].copy()

    def kernels():
        m.engine.forward(v_in["shape"][0], v_in["pose"][0], None, joints=True, rest_verts=True,
                         rest_joints=True, rot_mats=True, out={k: dv for k, (dv, _) in v_out.items()},
                         workspace=ws)
        s.synchronize()
    res["kernels_sync"] = med(kernels, a.calls)

    def copies():
        d_in.copy_(h_in, non_blocking=True)
        h_out.copy_(d_out, non_blocking=True)
        s.synchronize()
    res["copies_sync"] = med(copies, a.calls)
    res["sync_idle"] = med(s.synchronize, a.calls)
    one = torch.zeros(1, device=m.device)
    res["tiny_sync"] = med(lambda: (one.add_(1), s.synchronize()), a.calls)
    res["host_convert"] = med(lambda: {k: hv.astype(np.float64) for k, (_, hv) in v_out.items()}, a.calls)

    # zero copy: the kernels' operands are the pinned host blocks themselves
    lib = _abi.lib()
    hp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    off = {}
    o = 0
    for name, shp in m._IN:
        off[name] = o
        o += int(np.prod(shp)) * 4
    ooff = {}
    o = 0
    for name, (dv, _) in v_out.items():
        ooff[name] = o
        o += dv.numel() * 4
    hin, hout = h_in.data_ptr(), h_out.data_ptr()

    # Only launch on host blocks the runtime reports as pinned host memory
    # mapped at the same address for the device (hipHostMalloc'd).
    class Attr(ctypes.Structure):
        _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                    ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int),
                    ("allocationFlags", ctypes.c_uint)]
    hip = ctypes.CDLL("libamdhip64.so")
    for name, p in (("in", hin), ("out", hout)):
        at = Attr()
        rc = hip.hipPointerGetAttributes(ctypes.byref(at), ctypes.c_void_p(p))
        res[f"host_block_{name}"] = {"rc": rc, "type": at.type, "device_ptr_same": at.devicePointer == p,
                                     "flags": at.allocationFlags}
        if rc != 0 or at.type != 1 or at.devicePointer != p:
            print(json.dumps(res), flush=True)
            raise SystemExit(f"host block {name} is not device-mapped pinned memory: no zero-copy launch")
    wsp = (ws.data_ptr() + 255) & ~255
    wsb = ws.numel() - (wsp - ws.data_ptr())
    sh = ctypes.c_void_p(s.cuda_stream)
    h_out.zero_()

    def zc():
        _abi.check(lib.mano_forward(m.engine._h, 1, ctypes.c_void_p(hin + off["shape"]), 10,
                                    ctypes.c_void_p(hin + off["pose"]), None,
                                    ctypes.c_void_p(hout + ooff["verts"]), ctypes.c_void_p(hout + ooff["joints"]),
                                    ctypes.c_void_p(hout + ooff["rest_verts"]),
                                    ctypes.c_void_p(hout + ooff["rest_joints"]),
                                    ctypes.c_void_p(hout + ooff["rot_mats"]), ctypes.c_void_p(wsp),
                                    ctypes.c_size_t(wsb), sh))
        s.synchronize()
    zc()
    res["zero_copy_bit_exact"] = bool(np.array_equal(v_out["verts"][1], want))
    res["zero_copy_sync"] = med(zc, a.calls)
    gs = torch.cuda.Stream(m.device)
    with torch.cuda.stream(gs):
        zc()
        gz = torch.cuda.CUDAGraph()
        sh = ctypes.c_void_p(gs.cuda_stream)
        with torch.cuda.graph(gz, stream=gs):
            _abi.check(lib.mano_forward(m.engine._h, 1, ctypes.c_void_p(hin + off["shape"]), 10,
                                        ctypes.c_void_p(hin + off["pose"]), None,
                                        ctypes.c_void_p(hout + ooff["verts"]), ctypes.c_void_p(hout + ooff["joints"]),
                                        ctypes.c_void_p(hout + ooff["rest_verts"]),
                                        ctypes.c_void_p(hout + ooff["rest_joints"]),
                                        ctypes.c_void_p(hout + ooff["rot_mats"]), ctypes.c_void_p(wsp),
                                        ctypes.c_size_t(wsb), sh))
    h_out.zero_()
    gz.replay()
    s.synchronize()
    torch.cuda.synchronize()
    res["zero_copy_graph_bit_exact"] = bool(np.array_equal(v_out["verts"][1], want))
    res["zero_copy_graph"] = med(lambda: (gz.replay(), s.synchronize()), a.calls)
    res["status"] = m.engine.device_status()
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
