"""The single-process multi-GPU path (mano_amd.multi_device, include/mano_hip.h
ABI 6: mano_comm_create_all + mano_group_start / mano_group_end; ABI 7:
mano_gather_check, the pre-flight of a group's calls).

One host thread drives every device: shards of one batch run on their own
GPUs and streams, and the assembled outputs on the root equal the
single-handle forward of the whole batch bit for bit (hands are independent,
mano_np.py:79-115; the batch is the reference's single-process loop,
data_explore.py:12-15).  On the 1-GPU pool the RCCL form runs at n = 1
(ncclCommInitAll over one device) and the sharding / stream / assembly logic
with one GPU listed several times (peer-copy assembly); the n = 2 RCCL case
runs wherever 2 GPUs are visible."""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _reference(params, seed, n, trans):
    from mano_amd import ManoHip
    m = ManoHip(params, device=0)
    inp = m.synthetic_inputs(seed, 0, n, trans=trans)
    out = m.forward(inp["betas"], inp["pose"], inp.get("trans"), joints=True)
    torch.cuda.synchronize()
    res = {k: v.cpu() for k, v in out.items()}, {k: v.cpu() for k, v in inp.items()}
    m.close()
    return res


def test_one_device_rccl_group_gather_bit_exact(params):
    """n = 1: mano_comm_create_all over device 0, the grouped gather (the
    root's shard in place), bit-exact against the single-handle forward --
    from synthetic inputs generated per device and from caller inputs."""
    from mano_amd import ManoMultiDevice
    n, seed = 1000, 1004
    ref, inp = _reference(params, seed, n, trans=True)
    md = ManoMultiDevice(params, devices=[0])
    try:
        out = md.forward_synthetic(seed, n, trans=True, gather="rccl")
        torch.cuda.synchronize()
        assert out["verts"].device == torch.device("cuda", 0)
        assert torch.equal(out["verts"].cpu(), ref["verts"]) and torch.equal(out["joints"].cpu(), ref["joints"])
        d = torch.device("cuda", 0)
        out2 = md.forward(inp["betas"].to(d), inp["pose"].to(d), inp["trans"].to(d), gather="rccl")
        md.synchronize()
        assert torch.equal(out2["verts"].cpu(), ref["verts"]) and torch.equal(out2["joints"].cpu(), ref["joints"])
    finally:
        md.close()


def test_abi_group_gather_not_in_place():
    """The ABI directly: one communicator from mano_comm_create_all, a
    mano_gather between mano_group_start / mano_group_end whose send is NOT
    the root's slot (the root copies its shard), bytes equal."""
    from mano_amd import _abi
    lib = _abi.lib()
    comms = (ctypes.c_void_p * 1)()
    _abi.check(lib.mano_comm_create_all(1, (ctypes.c_int * 1)(0), comms))
    try:
        src = torch.arange(3 * 1024, dtype=torch.float32, device="cuda:0")
        dst = torch.zeros(3 * 1024 + 64, dtype=torch.float32, device="cuda:0")
        s = torch.cuda.current_stream(0)
        sizes = (ctypes.c_size_t * 1)(src.numel() * 4)
        _abi.check(lib.mano_group_start())
        _abi.check(lib.mano_gather(ctypes.c_void_p(comms[0]), ctypes.c_void_p(src.data_ptr()), src.numel() * 4,
                                   ctypes.c_void_p(dst.data_ptr()), sizes, 0, ctypes.c_void_p(s.cuda_stream)))
        _abi.check(lib.mano_group_end())
        torch.cuda.synchronize()
        assert torch.equal(dst[:src.numel()], src) and not dst[src.numel():].any()
    finally:
        _abi.check(lib.mano_comm_destroy(ctypes.c_void_p(comms[0])))


def _completes(stream, seconds=60.0):
    """True when everything queued on `stream` so far finishes within
    `seconds` (an event polled from the host: a hung group fails the test
    instead of hanging it)."""
    import time
    ev = torch.cuda.Event()
    ev.record(stream)
    t_end = time.monotonic() + seconds
    while not ev.query():
        if time.monotonic() > t_end:
            return False
        time.sleep(0.005)
    return True


def test_abi_group_preflight_refuses_second_call_before_anything_posts():
    """ABI 7's rule for a group of gathers (the partial-group hang): the host
    checks EVERY call with mano_gather_check before mano_group_start.  Here
    the second call of the group is bad (rank_bytes[root] != send_bytes, then
    root out of range, then recv NULL on the root): the check returns
    MANO_EINVAL, the host never opens the group, and nothing is launched --
    the first call's out-of-place destination is untouched.  The good group
    that follows completes within a timeout and lands its bytes."""
    from mano_amd import _abi
    lib = _abi.lib()
    comms = (ctypes.c_void_p * 1)()
    _abi.check(lib.mano_comm_create_all(1, (ctypes.c_int * 1)(0), comms))
    c = ctypes.c_void_p(comms[0])
    try:
        n = ctypes.c_int32()
        _abi.check(lib.mano_comm_info(c, ctypes.byref(n), None, None))
        assert n.value == 1
        s = torch.cuda.current_stream(0)
        src_v = torch.arange(4096, dtype=torch.float32, device="cuda:0")
        src_j = torch.arange(256, dtype=torch.float32, device="cuda:0") + 0.5
        dst_v = torch.full((4096,), -7.0, device="cuda:0")
        dst_j = torch.full((256,), -7.0, device="cuda:0")
        torch.cuda.synchronize()
        vb, jb = (ctypes.c_size_t * 1)(4096 * 4), (ctypes.c_size_t * 1)(256 * 4)
        first = (c, ctypes.c_void_p(src_v.data_ptr()), 4096 * 4, ctypes.c_void_p(dst_v.data_ptr()), vb, 0)
        assert lib.mano_gather_check(*first) == _abi.MANO_OK
        bad_calls = [
            (c, ctypes.c_void_p(src_j.data_ptr()), 256 * 4, ctypes.c_void_p(dst_j.data_ptr()), vb, 0),
            (c, ctypes.c_void_p(src_j.data_ptr()), 256 * 4, ctypes.c_void_p(dst_j.data_ptr()), jb, 1),
            (c, ctypes.c_void_p(src_j.data_ptr()), 256 * 4, None, jb, 0),
        ]
        for bad in bad_calls:
            assert lib.mano_gather_check(*bad) == _abi.MANO_EINVAL
            assert _abi.last_error()
            # mano_gather runs the same checks and posts nothing either
            assert lib.mano_gather(*bad, ctypes.c_void_p(s.cuda_stream)) == _abi.MANO_EINVAL
        assert _completes(s)
        assert bool((dst_v == -7.0).all()) and bool((dst_j == -7.0).all())   # nothing launched
        good = (c, ctypes.c_void_p(src_j.data_ptr()), 256 * 4, ctypes.c_void_p(dst_j.data_ptr()), jb, 0)
        assert lib.mano_gather_check(*good) == _abi.MANO_OK
        _abi.check(lib.mano_group_start())
        _abi.check(lib.mano_gather(*first, ctypes.c_void_p(s.cuda_stream)))
        _abi.check(lib.mano_gather(*good, ctypes.c_void_p(s.cuda_stream)))
        _abi.check(lib.mano_group_end())
        assert _completes(s)
        assert torch.equal(dst_v, src_v) and torch.equal(dst_j, src_j)
    finally:
        _abi.check(lib.mano_comm_destroy(c))


def test_device_comms_bad_second_output_launches_nothing(params):
    """DeviceComms.gather validates every call of its group before the group
    opens: a bad SECOND output (its row count does not match the pieces)
    raises, the first output's out-of-place destination is untouched, and a
    following good gather completes within a timeout, bit for bit."""
    from mano_amd import DeviceComms
    d = torch.device("cuda", 0)
    v = torch.randn(100, 778, 3, device=d)
    j = torch.randn(100, 16, 3, device=d)
    out_v = torch.full((100, 778, 3), -3.0, device=d)
    bad_j = torch.full((99, 16, 3), -3.0, device=d)
    s = torch.cuda.current_stream(0)
    dc = DeviceComms([0])
    try:
        assert dc.n_ranks() == [1]
        torch.cuda.synchronize()
        with pytest.raises(ValueError):
            dc.gather([[v, j]], [out_v, bad_j], 0, [s])
        assert _completes(s)
        assert bool((out_v == -3.0).all()) and bool((bad_j == -3.0).all())
        out_j = torch.empty(100, 16, 3, device=d)
        dc.gather([[v, j]], [out_v, out_j], 0, [s])
        assert _completes(s)
        assert torch.equal(out_v, v) and torch.equal(out_j, j)
    finally:
        dc.close()


def test_results_safe_to_free_on_the_callers_stream(params):
    """The returned tensors live on ManoMultiDevice's internal streams: a
    result read on the caller's stream, freed, then the next forward_synthetic
    (whose allocations may reuse its block) must not overwrite it mid-read --
    each call orders its streams after the caller's.  A slow read of the
    first result (a long copy chain on the current stream) still sees its
    values."""
    from mano_amd import ManoMultiDevice
    n, seed = 4096, 1002
    ref, _ = _reference(params, seed, n, trans=False)
    other, _ = _reference(params, seed + 1, n, trans=False)
    md = ManoMultiDevice(params, devices=[0])
    try:
        out = md.forward_synthetic(seed, n, gather=False)[0]
        cur = torch.cuda.current_stream(0)
        acc = torch.zeros_like(out["verts"])
        for _ in range(200):            # a long read of the result on the caller's stream
            acc.copy_(out["verts"])
        del out                          # freed while the reads are still queued
        nxt = md.forward_synthetic(seed + 1, n, gather=False)[0]
        cur.wait_stream(md.streams[0])
        torch.cuda.synchronize()
        assert torch.equal(acc.cpu(), ref["verts"])
        assert torch.equal(nxt["verts"].cpu(), other["verts"])
    finally:
        md.close()


def test_duplicate_device_refused_by_rccl_form():
    from mano_amd import DeviceComms, _abi
    with pytest.raises(_abi.ManoError) as ei:
        DeviceComms([0, 0])
    assert ei.value.code == _abi.MANO_EINVAL and "twice" in str(ei.value)


@pytest.mark.parametrize("gather", ["copy", False])
def test_shards_over_one_gpu_listed_three_times(params, gather):
    """The sharding, per-device streams and assembly with 3 engines (one GPU
    listed three times): a ragged 1,003-hand batch (335 + 334 + 334) equals
    the single-handle forward bit for bit, assembled by peer copies or as
    per-device shards."""
    from mano_amd import ManoMultiDevice
    from mano_amd.distributed import shard_range
    n, seed = 1003, 1002
    ref, _ = _reference(params, seed, n, trans=False)
    md = ManoMultiDevice(params, devices=[0, 0, 0], root=1)
    try:
        out = md.forward_synthetic(seed, n, gather=gather)
        torch.cuda.synchronize()
        if gather:
            assert torch.equal(out["verts"].cpu(), ref["verts"]) and torch.equal(out["joints"].cpu(), ref["joints"])
        else:
            assert len(out) == 3
            for i, o in enumerate(out):
                a, b = shard_range(n, i, 3)
                assert torch.equal(o["verts"].cpu(), ref["verts"][a:b])
                assert torch.equal(o["joints"].cpu(), ref["joints"][a:b])
    finally:
        md.close()


def test_host_inputs_and_shared_betas(params):
    """Caller inputs on the host with one shared beta row, split over 2
    engines: equal to the single-handle forward of the same inputs."""
    from mano_amd import ManoHip, ManoMultiDevice
    rng = np.random.default_rng(5)
    n = 77
    betas = torch.tensor(rng.normal(0, 1, 10), dtype=torch.float32)
    pose = torch.tensor(rng.normal(0, 0.5, (n, 16, 3)), dtype=torch.float32)
    m = ManoHip(params, device=0)
    ref = m.forward(betas.cuda(), pose.cuda(), joints=True)
    torch.cuda.synchronize()
    md = ManoMultiDevice(params, devices=[0, 0])
    try:
        out = md.forward(betas, pose, gather="copy")
        md.synchronize()
        assert torch.equal(out["verts"], ref["verts"]) and torch.equal(out["joints"], ref["joints"])
    finally:
        md.close()
        m.close()


@pytest.mark.parametrize("devices,gather,n_pca,rot_kind", [([0], "rccl", 45, "per_hand"),
                                                           ([0, 0, 0], "copy", 6, "shared"),
                                                           ([0, 0], False, 12, None)])
def test_forward_pca_split(params, devices, gather, n_pca, rot_kind):
    """forward_pca (mano_np.py:66-77 batched) split over the devices equals
    the single-handle forward_pca bit for bit: per-hand / shared / absent
    global rotation, 45 / 6 / 12 coefficients, per-hand betas and trans."""
    from mano_amd import ManoHip, ManoMultiDevice
    from mano_amd.distributed import shard_range
    rng = np.random.default_rng(n_pca)
    n = 1001
    d = torch.device("cuda", 0)
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=d)  # noqa: E731
    betas, pca = t(rng.normal(0, 1, (n, 10))), t(rng.normal(0, 1, (n, n_pca)))
    trans = t(rng.normal(0, 0.1, (n, 3)))
    rot = {"per_hand": t(rng.normal(0, 0.7, (n, 3))), "shared": t(rng.normal(0, 0.7, 3)), None: None}[rot_kind]
    m = ManoHip(params, device=0)
    ref = m.forward_pca(betas, pca, rot, trans, joints=True)
    torch.cuda.synchronize()
    md = ManoMultiDevice(params, devices=devices)
    try:
        out = md.forward_pca(betas, pca, rot, trans, gather=gather)
        md.synchronize()
        if gather:
            assert torch.equal(out["verts"], ref["verts"]) and torch.equal(out["joints"], ref["joints"])
        else:
            for i, o in enumerate(out):
                a, b = shard_range(n, i, len(devices))
                assert torch.equal(o["verts"], ref["verts"][a:b]) and torch.equal(o["joints"], ref["joints"][a:b])
    finally:
        md.close()
        m.close()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="the RCCL group gather needs 2 GPUs")
def test_two_devices_rccl_group_gather(params):
    """n = 2 for real: one thread, two GPUs, one RCCL group; GPU 0's
    assembled outputs of a ragged batch equal the single-handle forward."""
    from mano_amd import ManoMultiDevice
    n, seed = 1003, 1004
    ref, _ = _reference(params, seed, n, trans=True)
    md = ManoMultiDevice(params, devices=[0, 1])
    try:
        out = md.forward_synthetic(seed, n, trans=True, gather="rccl")
        md.synchronize()
        assert torch.equal(out["verts"].cpu(), ref["verts"]) and torch.equal(out["joints"].cpu(), ref["joints"])
        assert md.comms().n_ranks() == [2, 2]      # RCCL's communicators hold both devices
        # the first xGMI figure: device 1's shard of a C4-sized batch into device 0
        import warnings
        gb = md.gather_bandwidth(2 * 262144)
        assert gb["GBs_to_root"] > 0 and gb["bytes_to_root"] > 0
        warnings.warn(f"xGMI gather device 1 -> 0 (one RCCL group, ManoMultiDevice): "
                      f"{gb['GBs_to_root']:.1f} GB/s, {gb['bytes_to_root'] / 1e9:.2f} GB in {gb['ms']:.3f} ms")
    finally:
        md.close()


@pytest.mark.parametrize("extra", [["--gpus", "1", "--workload", "C4", "--batch", "8192"],
                                   ["--gpus", "3", "--devices", "0,0,0", "--workload", "C4", "--batch", "4096"],
                                   ["--gpus", "2", "--devices", "0,0", "--batch", "4096"]])
def test_bench_single_process(extra):
    """bench.py --single-process: one host thread drives the devices (one RCCL
    group gather at n = 1; peer-copy assembly with one GPU listed several
    times), every device's sampled hands pass the oracle check."""
    import json
    import os
    import subprocess
    import sys
    from conftest import REPO
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--single-process", *extra,
                        "--steps", "10", "--warmup", "2", "--ramp-seconds", "0.2"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    n = int(extra[1])
    assert line["status"] == "ok" and line["n_gpus"] == n and line["value"] > 0
    assert line["process_model"]["single_process"] and line["process_model"]["host_threads"] == 1
    assert line["correctness"]["pass"] and line["correctness"]["ranks_checked"] == n, line["correctness"]
    if "C4" in extra:
        assert line["config"]["gather_to_gpu0"]
        assert ("RCCL" in line["config"]["gather_impl"]) == (n == 1)
