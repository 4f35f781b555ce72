"""Debug: the batch-1 drop-in's wait for its kernels, three ways.

    python tools/debug/sync_forms.py [--calls 400]

For the zero-copy batch-1 forward (mano_forward on MANOModel's pinned host
blocks) and for a 1-element torch kernel: medians over `calls` (after 50
warm-up calls) of launch + wait, where the wait is
  stream_sync   hipStreamSynchronize (torch Stream.synchronize, the product)
  event_sync    an event recorded after the launch, hipEventSynchronize
  event_spin    the same event polled with hipEventQuery in a Python loop
and the whole set_params call with the product's wait."""
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
    m = MANOModel.from_params(synthetic_params(0), device=0)
    rng = np.random.default_rng(3)
    pose, shape = rng.normal(0, 0.5, (16, 3)), rng.normal(0, 1, 10)
    res = {"set_params": med(lambda: m.set_params(pose_abs=pose, shape=shape), a.calls)}
    s = torch.cuda.current_stream(m.device)
    zc = m._zero_copy_args(False)
    assert zc is not None, "pinned blocks not device-mapped"
    lib = _abi.lib()
    sp = ctypes.c_void_p(s.cuda_stream)
    launch = lambda: lib.mano_forward(*zc, sp)  # noqa: E731
    ev = torch.cuda.Event()
    ev_block = torch.cuda.Event(blocking=True)

    def spin(e):
        while not e.query():
            pass

    one = torch.zeros(1, device=m.device)
    for name, work in (("forward", launch), ("tiny", lambda: one.add_(1))):
        res[f"{name}_stream_sync"] = med(lambda: (work(), s.synchronize()), a.calls)
        res[f"{name}_event_sync"] = med(lambda: (work(), ev_block.record(s), ev_block.synchronize()), a.calls)
        res[f"{name}_event_spin"] = med(lambda: (work(), ev.record(s), spin(ev)), a.calls)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
