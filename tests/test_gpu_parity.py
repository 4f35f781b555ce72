"""HIP path vs the float64 oracle and the reference goldens (MI355X only).

Tolerance: max |err| <= 1e-5 m on vertices and joints (north_star: float32
HIP path vs float64 numpy), 1e-6 on rotation matrices and pose features.
Every call goes through libmano_hip.so (the C-ABI); nothing here has a CPU
fallback.
"""
import numpy as np
import pytest

from conftest import step_kwargs
from oracle import mano_oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL_M = 1e-5
TOL_R = 1e-6


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def engine(params, dev):
    from mano_amd import ManoHip
    m = ManoHip(params, device=0)
    yield m
    m.close()


def f32(a, dev):
    return torch.tensor(np.asarray(a), dtype=torch.float32, device=dev)


def host(t):
    return t.double().cpu().numpy()


def run(engine, dev, betas, pose, trans=None):
    out = engine.forward(f32(betas, dev), f32(pose, dev), None if trans is None else f32(trans, dev),
                         joints=True, rest_verts=True, rest_joints=True, rot_mats=True)
    torch.cuda.synchronize()
    return {k: host(v) for k, v in out.items()}


def assert_close(got, ref, where=""):
    for k_got, k_ref, tol in (("verts", "verts", TOL_M), ("joints", "joints", TOL_M),
                              ("rest_verts", "rest_verts", TOL_M), ("rest_joints", "rest_joints", TOL_M),
                              ("rot_mats", "rot", TOL_R)):
        err = np.abs(got[k_got] - ref[k_ref]).max() if got[k_got].size else 0.0
        assert err <= tol, f"{where} {k_got}: max err {err:.3e} > {tol}"


def test_library_is_the_loaded_path(engine):
    import os
    import sys
    from mano_amd import _abi
    assert _abi._LIB is not None and _abi.LIB_PATH.endswith(os.environ.get("MANO_TEST_LIB", "libmano_hip.so"))
    assert "oracle" not in sys.modules.get("mano_amd.model").__dict__


def test_batch_golden(engine, dev, golden_batch):
    g = golden_batch
    got = run(engine, dev, g["betas"], g["pose"])
    ref = {"verts": g["verts"], "joints": g["joints"], "rest_verts": g["rest_verts"],
           "rest_joints": g["J"], "rot": g["R"]}
    assert_close(got, ref, "golden batch")


def test_stateful_script_golden(params, golden_steps):
    """The drop-in MANOModel replays the reference's set_params script."""
    from mano_amd import MANOModel
    manifest, data = golden_steps
    model = None
    for entry in manifest:
        i = entry["step"]
        if model is None:
            model = MANOModel.from_params(params, device=0)
        else:
            ret = model.set_params(**step_kwargs(entry, data))
            assert ret.dtype == np.float64 and ret.shape == (778, 3)
            assert ret is not model.verts and np.array_equal(ret, model.verts)
        for key, got, tol in (("verts", model.verts, TOL_M), ("J", model.J, TOL_M),
                              ("R", model.R, TOL_R), ("rest_verts", model.rest_verts, TOL_M),
                              ("joints", model.joints, TOL_M), ("rot", model.rot, 1e-12),
                              ("pose", np.reshape(model.pose, (-1, 3)), 1e-5)):
            err = np.abs(np.asarray(got, dtype=np.float64) - data[f"s{i}_out_{key}"]).max()
            assert err <= tol, (entry["desc"], key, err)


def test_export_obj_demo(params, golden_steps, tmp_path):
    import os
    from conftest import GOLDEN
    from mano_amd import MANOModel
    manifest, data = golden_steps
    model = MANOModel.from_params(params, device=0)
    last = manifest[-1]
    model.set_params(**step_kwargs(last, data))
    p = str(tmp_path / "hand.obj")
    model.export_obj(p)
    for name in ("hand.obj", "hand_restpose.obj"):
        a = open(os.path.join(GOLDEN, name)).read().split("\n")
        b = open(tmp_path / name).read().split("\n")
        assert len(a) == len(b)
        va = np.array([[float(x) for x in l.split()[1:]] for l in a if l.startswith("v ")])
        vb = np.array([[float(x) for x in l.split()[1:]] for l in b if l.startswith("v ")])
        assert np.abs(va - vb).max() <= 1e-5 + 1e-6
        assert [l for l in a if l.startswith("f ")] == [l for l in b if l.startswith("f ")]


@pytest.mark.parametrize("B", [1, 2, 31, 32, 33, 127, 128, 129, 1000])
def test_ragged_batches(engine, dev, params, B):
    rng = np.random.default_rng(B)
    betas = rng.normal(0, 1, (B, 10))
    pose = rng.normal(0, 0.5, (B, 16, 3))
    trans = rng.uniform(-1, 1, (B, 3))
    got = run(engine, dev, betas, pose, trans)
    ref = mano_oracle.forward(params, betas, pose, trans)
    ref["rest_joints"] = ref["rest_joints"]
    assert_close(got, ref, f"B={B}")


@pytest.mark.parametrize("mag", [0.0, 1e-20, 1e-12, 1e-8, 1e-6, 1e-4, 1e-3, 1e-2, 0.1,
                                 np.pi, 2 * np.pi, 3.0, 6.0, 10.0])
def test_edge_angles(engine, dev, params, mag):
    rng = np.random.default_rng(17)
    B = 64
    d = rng.normal(size=(B, 16, 3))
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    pose = d * mag
    betas = rng.normal(0, 1, (B, 10))
    got = run(engine, dev, betas, pose)
    ref = mano_oracle.forward(params, betas, pose)
    assert_close(got, ref, f"|theta|={mag}")


def test_uniform_pi_and_axis_aligned(engine, dev, params):
    rng = np.random.default_rng(3)
    B = 256
    pose = rng.uniform(-np.pi, np.pi, (B, 16, 3))
    pose[:16] = 0.0
    for i in range(16):
        pose[i, i, i % 3] = np.pi  # exact half turns about each axis
    betas = rng.normal(0, 2, (B, 10))
    got = run(engine, dev, betas, pose)
    assert_close(got, mano_oracle.forward(params, betas, pose), "uniform pi")


def test_shared_betas_stride_zero(engine, dev, params):
    rng = np.random.default_rng(4)
    beta = rng.normal(0, 1, 10)
    pose = rng.normal(0, 0.5, (50, 16, 3))
    out = engine.forward(f32(beta, dev), f32(pose, dev))
    ref = mano_oracle.forward(params, beta, pose)
    assert np.abs(host(out["verts"]) - ref["verts"]).max() <= TOL_M


@pytest.mark.parametrize("B", [1, 15, 16, 17, 300])
def test_joints_staged_and_unaligned(engine, dev, params, B):
    """Posed joints leave articulate as a staged dwordx4 stream when the
    caller's buffer is 16-B aligned, per lane otherwise: same bits both
    ways, with and without trans, and nothing written past row B."""
    rng = np.random.default_rng(40 + B)
    beta = f32(rng.normal(0, 1, (B, 10)), dev)
    pose = f32(rng.normal(0, 0.5, (B, 16, 3)), dev)
    trans = f32(rng.uniform(-1, 1, (B, 3)), dev)
    for tr in (None, trans):
        a = engine.forward(beta, pose, tr, joints=True)["joints"]
        raw = torch.full((B * 48 + 8,), 7.0, device=dev)
        ju = raw[1:1 + B * 48].view(B, 16, 3)  # 4-B offset: per-lane stores
        engine.forward(beta, pose, tr, joints=True, out={"joints": ju})
        assert torch.equal(a, ju)
        assert raw[0].item() == 7.0 and torch.all(raw[1 + B * 48:] == 7.0)
        raw.fill_(7.0)
        ja = raw[4:4 + B * 48].view(B, 16, 3)  # 16-B offset: the staged stream
        engine.forward(beta, pose, tr, joints=True, out={"joints": ja})
        assert torch.equal(a, ja)
        assert torch.all(raw[:4] == 7.0) and torch.all(raw[4 + B * 48:] == 7.0)
    ref = mano_oracle.forward(params, host(beta), host(pose), host(trans))
    assert np.abs(host(a) - ref["joints"]).max() <= TOL_M


def test_flat48_pose(engine, dev, params):
    rng = np.random.default_rng(5)
    pose = rng.normal(0, 0.5, (20, 48))
    betas = rng.normal(0, 1, (20, 10))
    out = engine.forward(f32(betas, dev), f32(pose, dev))
    ref = mano_oracle.forward(params, betas, pose)
    assert np.abs(host(out["verts"]) - ref["verts"]).max() <= TOL_M


def test_stage_intermediates(engine, dev, params):
    """Each kernel alone: features (R-I), skinning transforms, v_posed."""
    rng = np.random.default_rng(6)
    B = 70
    betas = rng.normal(0, 1, (B, 10))
    pose = rng.normal(0, 0.7, (B, 16, 3))
    engine.stage_articulate(f32(betas, dev), f32(pose, dev))
    engine.stage_blend(B)
    torch.cuda.synchronize()
    inter = engine.intermediates(B)
    ref = mano_oracle.forward(params, betas, pose)
    # features: the X rows, k-permuted in the workspace (model.X_POS)
    from mano_amd.model import X_POS
    X = host(inter["features"])[:, X_POS]
    assert np.abs(X[:, :10] - betas).max() < 1e-6
    feats = mano_oracle.pose_features(ref["rot"])
    assert np.abs(X[:, 10:145] - feats).max() <= TOL_R
    assert np.all(X[:, 145] == 1.0) and np.all(X[:, 146:] == 0.0)
    assert sorted(X_POS.tolist()) == list(range(160))
    # transforms: oracle G after rest removal, rows 0..2
    _, G = mano_oracle.chain(ref["rot"], ref["rest_joints"], params["parents"])
    assert np.abs(host(inter["transforms"]) - G[:, :, :3, :]).max() <= TOL_M
    assert np.abs(host(inter["vposed"]) - ref["rest_verts"]).max() <= TOL_M


def test_large_batch_sampled(engine, dev, params):
    """Full C2 size (65,536 hands): sampled hands vs the oracle + properties."""
    B = 65536
    g = torch.Generator(device=dev).manual_seed(1001)
    betas = torch.randn((B, 10), generator=g, device=dev)
    pose = 0.5 * torch.randn((B, 16, 3), generator=g, device=dev)
    trans = torch.rand((B, 3), generator=g, device=dev) * 2 - 1
    out = engine.forward(betas, pose, trans, joints=True)
    torch.cuda.synchronize()
    verts = out["verts"]
    assert torch.isfinite(verts).all()
    idx = np.random.default_rng(0).choice(B, 256, replace=False)
    idx = np.concatenate([idx, [0, 31, 32, B - 33, B - 1]])
    ref = mano_oracle.forward(params, host(betas[idx]), host(pose[idx]), host(trans[idx]))
    assert np.abs(host(verts[idx]) - ref["verts"]).max() <= TOL_M
    assert np.abs(host(out["joints"][idx]) - ref["joints"]).max() <= TOL_M
    # shard invariance: any contiguous split gives bit-identical results
    for a, b in ((0, 1000), (1000, 40000), (40000, B)):
        part = engine.forward(betas[a:b].contiguous(), pose[a:b].contiguous(),
                              trans[a:b].contiguous(), joints=False)
        assert torch.equal(part["verts"], verts[a:b])
    # determinism
    again = engine.forward(betas, pose, trans, joints=False)
    assert torch.equal(again["verts"], verts)


def test_root_rotation_equivariance(engine, dev, params):
    """Rotating the root rotates every vertex about the root joint (property at size)."""
    rng = np.random.default_rng(8)
    B = 4096
    betas = rng.normal(0, 1, (B, 10))
    pose = rng.normal(0, 0.5, (B, 16, 3))
    pose[:, 0] = 0.0
    base = run(engine, dev, betas, pose)
    rot = np.array([0.0, 0.0, np.pi / 2])
    pose2 = pose.copy()
    pose2[:, 0] = rot
    turned = run(engine, dev, betas, pose2)
    Rz = mano_oracle.rodrigues(rot)
    j0 = base["rest_joints"][:, :1]
    expect = (base["verts"] - j0) @ Rz.T + j0
    assert np.abs(turned["verts"] - expect).max() <= 2 * TOL_M


def test_scan_pose_source(engine, dev, params):
    """The realistic pose source of data_explore.py:12-15: the reference's own
    dump_scans() output (tests/golden/mano_reference_scans.npz, 73 captured
    poses; the right hand mirrored by [1, -1, -1]) with a zero root, shared
    betas and per-hand betas, through the batched forward vs the oracle."""
    import os
    from conftest import GOLDEN
    from mano_amd import scans_to_pose
    with np.load(os.path.join(GOLDEN, "mano_reference_scans.npz"), allow_pickle=False) as z:
        pose = scans_to_pose(z["axangles"])
    B = pose.shape[0]
    rng = np.random.default_rng(73)
    for betas in (np.zeros((B, 10)), rng.normal(0, 1, (B, 10))):
        out = run(engine, dev, betas, pose)
        ref = mano_oracle.forward(params, betas, pose)
        assert_close(out, ref, "scan poses")


def test_empty_batch(engine, dev):
    out = engine.forward(torch.empty((0, 10), device=dev), torch.empty((0, 16, 3), device=dev))
    assert out["verts"].shape == (0, 778, 3)


@pytest.mark.parametrize("n", [1, 9, 45])
def test_pose_from_pca(engine, dev, params, n):
    rng = np.random.default_rng(n)
    B = 40
    c = rng.normal(0, 1, (B, n))
    rot = rng.normal(0, 1, (B, 3))
    got = host(engine.pose_from_pca(f32(c, dev), f32(rot, dev)))
    ref = mano_oracle.pose_from_pca(params, c, rot)
    assert np.abs(got - ref).max() <= 1e-5


def test_rodrigues_kernel(engine, dev):
    rng = np.random.default_rng(9)
    r = np.concatenate([rng.normal(0, 1, (500, 3)), np.zeros((1, 3)), [[1e-20, 0, 0], [np.pi, 0, 0]]])
    got = host(engine.rodrigues(f32(r, dev)))
    assert np.abs(got - mano_oracle.rodrigues(r)).max() <= TOL_R


def test_errors(engine, dev):
    from mano_amd import _abi
    with pytest.raises(ValueError):
        engine.forward(torch.zeros((3, 10), device=dev, dtype=torch.float64), torch.zeros((3, 16, 3), device=dev))
    with pytest.raises(ValueError):
        engine.forward(torch.zeros((3, 9), device=dev), torch.zeros((3, 16, 3), device=dev))
    with pytest.raises(ValueError):
        engine.forward(torch.zeros((3, 10)), torch.zeros((3, 16, 3)))
    # stage calls: workspace too small -> MANO_ESMALL through the raw ABI
    import ctypes
    lib = _abi.lib()
    b = torch.zeros((64, 10), device=dev)
    p = torch.zeros((64, 16, 3), device=dev)
    v = torch.empty((64, 778, 3), device=dev)
    ws = torch.empty(1024, dtype=torch.uint8, device=dev)
    rc = lib.mano_stage_articulate(engine._h, 64, ctypes.c_void_p(b.data_ptr()), 10,
                                   ctypes.c_void_p(p.data_ptr()), None, None, None, None,
                                   ctypes.c_void_p(ws.data_ptr()), 1024, None)
    assert rc == _abi.MANO_ESMALL and "workspace" in _abi.last_error()
    # mano_forward: same workspace rule, bad arguments refused
    need = lib.mano_forward_workspace_bytes(engine._h, 64)
    assert 0 < need <= lib.mano_workspace_bytes(engine._h, 64)
    rc = lib.mano_forward(engine._h, 64, ctypes.c_void_p(b.data_ptr()), 10, ctypes.c_void_p(p.data_ptr()),
                          None, ctypes.c_void_p(v.data_ptr()), None, None, None, None,
                          ctypes.c_void_p(ws.data_ptr()), 1024, None)
    assert rc == _abi.MANO_ESMALL and "workspace" in _abi.last_error()
    rc = lib.mano_forward(engine._h, 64, ctypes.c_void_p(b.data_ptr()), 5, ctypes.c_void_p(p.data_ptr()),
                          None, ctypes.c_void_p(v.data_ptr()), None, None, None, None,
                          ctypes.c_void_p(ws.data_ptr()), 1024, None)
    assert rc == _abi.MANO_EINVAL and "betas_stride" in _abi.last_error()
    rc = lib.mano_forward(engine._h, 64, ctypes.c_void_p(b.data_ptr()), 10, None, None,
                          ctypes.c_void_p(v.data_ptr()), None, None, None, None,
                          ctypes.c_void_p(ws.data_ptr()), 1024, None)
    assert rc == _abi.MANO_EINVAL
    torch.cuda.synchronize()


def test_dropin_quirks(params):
    from mano_amd import MANOModel
    m = MANOModel.from_params(params, device=0)
    with pytest.raises(ValueError):
        m.set_params(shape=np.zeros(9))          # mano_np.py:81 dot -> ValueError
    m.shape = np.zeros(10)
    with pytest.raises(AttributeError):
        m.set_params(pose_abs=[[0.0, 0.0, 0.0]] * 16)  # list pose -> AttributeError at :84
    m.pose = np.zeros((16, 3))
    with pytest.raises(AttributeError):
        m.set_params(pose_pca=[0.1, 0.2])         # list pca -> AttributeError at :67
    # global_rot without pose_pca is ignored (read only on the PCA branch, :70-72)
    m.set_params(pose_abs=np.zeros((16, 3)), global_rot=[1.0, 0, 0])
    assert np.all(m.rot == 0)
    # translation extension: verts shift exactly, joints too
    v0 = m.verts.copy()
    j0 = m.joints.copy()
    m.set_params(trans=[0.1, -0.2, 0.3])
    assert np.abs(m.verts - v0 - [0.1, -0.2, 0.3]).max() < 1e-6
    assert np.abs(m.joints - j0 - [0.1, -0.2, 0.3]).max() < 1e-6


@pytest.mark.parametrize("io", ["zero_copy", "graph", "eager"])
def test_dropin_packed_io_matches_batched(engine, dev, params, io):
    """The drop-in's packed batch-1 I/O (the kernels on the pinned host
    blocks themselves; or one H2D, one D2H through them, replayed from a HIP
    graph or launched eagerly) returns the batched engine's bits, and its
    results are owned copies: a later call changes neither an earlier return
    nor its attributes."""
    from mano_amd import MANOModel
    m = MANOModel.from_params(params, device=0)
    m.zero_copy = io == "zero_copy"
    m.use_graphs = io == "graph"
    graphs = io == "graph"
    rng = np.random.default_rng(5)
    pose_a, pose_b = rng.normal(0, 0.5, (2, 16, 3))
    beta_a, beta_b = rng.normal(0, 1, (2, 10))
    va = m.set_params(pose_abs=pose_a, shape=beta_a, trans=[0.01, 0.02, -0.03])
    keep = {k: getattr(m, k) for k in ("verts", "rest_verts", "J", "R", "joints")}
    snap = {k: v.copy() for k, v in keep.items()}
    va_copy = va.copy()
    m.set_params(pose_abs=pose_b, shape=beta_b)
    assert np.array_equal(va, va_copy)
    for k in keep:
        assert np.array_equal(keep[k], snap[k]), k
    out = engine.forward(torch.tensor(beta_a, dtype=torch.float32, device=dev)[None],
                         torch.tensor(pose_a, dtype=torch.float32, device=dev)[None],
                         torch.tensor([[0.01, 0.02, -0.03]], dtype=torch.float32, device=dev),
                         joints=True, rest_verts=True, rest_joints=True, rot_mats=True)
    want = {"verts": "verts", "rest_verts": "rest_verts", "J": "rest_joints", "R": "rot_mats",
            "joints": "joints"}
    for k, o in want.items():
        assert snap[k].dtype == np.float64
        assert np.array_equal(snap[k], out[o][0].double().cpu().numpy()), k
    if graphs:  # captured and replayed (not the eager fallback); trans is kept across calls
        assert all(g[0] is not None for g in m._graphs.values())
        assert set(m._graphs) == {(True, "fp32")}
    if io == "zero_copy":  # both translation modes ran on the host blocks (not the copy form)
        assert set(m._zc) == {True, False} and all(a is not None for a in m._zc.values())
        assert not m._graphs
    # alternating modes and repeated inputs reproduce the same bits
    again = m.set_params(pose_abs=pose_a, shape=beta_a, trans=[0.01, 0.02, -0.03])
    assert np.array_equal(again, va_copy)
    # a precision switch is honoured (its own graph), and switching back reproduces the fp32 bits
    m.engine.set_precision("f16x3")
    h3 = m.set_params(pose_abs=pose_a, shape=beta_a, trans=[0.0, 0.0, 0.0])  # trans is kept across calls
    ref = engine.forward(torch.tensor(beta_a, dtype=torch.float32, device=dev)[None],
                         torch.tensor(pose_a, dtype=torch.float32, device=dev)[None])["verts"][0]
    assert np.abs(h3 - ref.double().cpu().numpy()).max() <= TOL_M
    m.engine.set_precision("fp32")
    assert np.array_equal(m.set_params(pose_abs=pose_a, shape=beta_a, trans=[0.01, 0.02, -0.03]), va_copy)
    if graphs:  # the f16x3 call ran without translation: its own graph
        assert set(m._graphs) == {(True, "fp32"), (False, "f16x3")}


@pytest.mark.parametrize("B", [1, 33, 200, 4096, 4099, 16387])
def test_fused_equals_unfused(engine, dev, params, B):
    """blend_skin (fused, v_posed on chip) == blend then skin, bit for bit."""
    rng = np.random.default_rng(100 + B)
    betas = f32(rng.normal(0, 1, (B, 10)), dev)
    pose = f32(rng.normal(0, 0.6, (B, 16, 3)), dev)
    trans = f32(rng.uniform(-1, 1, (B, 3)), dev)
    fused = engine.forward(betas, pose, trans, rest_verts=True)
    engine.stage_articulate(betas, pose, trans)
    vp = torch.empty((B, 778, 3), device=dev)
    v = torch.empty((B, 778, 3), device=dev)
    engine.stage_blend(B, rest_verts=vp)
    engine.stage_skin(B, v, rest_verts=vp, trans=trans)
    torch.cuda.synchronize()
    assert torch.equal(fused["rest_verts"], vp)
    assert torch.equal(fused["verts"], v)
    ref = mano_oracle.forward(params, host(betas), host(pose), host(trans))
    assert np.abs(host(v) - ref["verts"]).max() <= TOL_M


@pytest.mark.parametrize("B,with_trans", [(2, True), (3, False), (5, True), (1023, False),
                                         (65537, True), (65538, False)])
def test_standalone_lbs_ragged(engine, dev, params, B, with_trans):
    """The standalone LBS (skin_pair: 4-hand units, a partial last quad when
    B % 4 != 0, many units per memory wave at 65,537 hands) over a v_posed
    buffer == the fused kernel's verts bit for bit; every vertex is written
    and nothing past the batch (a NaN guard row after the output stays NaN)."""
    rng = np.random.default_rng(300 + B)
    betas = f32(rng.normal(0, 1, (B, 10)), dev)
    pose = f32(rng.normal(0, 0.6, (B, 16, 3)), dev)
    trans = f32(rng.uniform(-1, 1, (B, 3)), dev) if with_trans else None
    fused = engine.forward(betas, pose, trans, rest_verts=True)
    engine.stage_articulate(betas, pose, trans)
    out = torch.full((B + 1, 778, 3), float("nan"), device=dev)
    engine.stage_skin(B, out[:B], rest_verts=fused["rest_verts"], trans=trans)
    torch.cuda.synchronize()
    assert torch.equal(fused["verts"], out[:B])
    assert torch.isnan(out[B]).all()


@pytest.mark.parametrize("B,with_trans", [(1, True), (2, False), (3, True), (5, False), (1023, True),
                                         (40000, True), (65533, False), (65536, True),
                                         (65537, True), (65538, False)])
def test_standalone_lbs_in_place(engine, dev, params, B, with_trans):
    """The LBS in place (mano_stage_skin with rest_verts == verts, ABI 7: the
    blend GEMM writes v_posed into verts, skin_pair's in-place units
    overwrite it -- the tail unit stores only its own 10 vertices, hand
    quads last-first; at 40,000-65,536 hands the spans the launcher deems
    cold -- 0-2 and 0-6 -- stream nontemporal) == the fused kernel's verts
    bit for bit, ragged batches included; the rows past the batch stay
    untouched."""
    rng = np.random.default_rng(700 + B)
    betas = f32(rng.normal(0, 1, (B, 10)), dev)
    pose = f32(rng.normal(0, 0.6, (B, 16, 3)), dev)
    trans = f32(rng.uniform(-1, 1, (B, 3)), dev) if with_trans else None
    fused = engine.forward(betas, pose, trans)
    engine.stage_articulate(betas, pose, trans)
    buf = torch.full((B + 1, 778, 3), float("nan"), device=dev)
    engine.stage_blend(B, rest_verts=buf[:B])
    engine.stage_skin(B, buf[:B], rest_verts=buf[:B], trans=trans)
    torch.cuda.synchronize()
    assert torch.equal(fused["verts"], buf[:B])
    assert torch.isnan(buf[B]).all()
    ref = mano_oracle.forward(params, host(betas[:64]), host(pose[:64]), None if trans is None else host(trans[:64]))
    assert np.abs(host(buf[:min(B, 64)]) - ref["verts"]).max() <= TOL_M


def test_standalone_lbs_in_place_f16x3_and_overlap(engine, dev, params):
    """In place under F16X3 (no in-place f16x3 kernel: the rows are staged in
    the workspace first) equals the out-of-place f16x3 LBS bit for bit; rows
    that overlap without being the same are refused with MANO_EINVAL."""
    from mano_amd import _abi
    B = 4099
    rng = np.random.default_rng(77)
    betas = f32(rng.normal(0, 1, (B, 10)), dev)
    pose = f32(rng.normal(0, 0.6, (B, 16, 3)), dev)
    engine.stage_articulate(betas, pose)
    vp = torch.empty((B, 778, 3), device=dev)
    engine.stage_blend(B, rest_verts=vp)
    engine.set_precision("f16x3")
    try:
        out = torch.empty_like(vp)
        engine.stage_skin(B, out, rest_verts=vp)
        buf = vp.clone()
        engine.stage_skin(B, buf, rest_verts=buf)
        torch.cuda.synchronize()
        assert torch.equal(out, buf)
    finally:
        engine.set_precision("fp32")
    big = torch.empty((B + 1, 778, 3), device=dev)
    with pytest.raises(_abi.ManoError) as ei:
        engine.stage_skin(B, big[1:], rest_verts=big[:B])
    assert ei.value.code == _abi.MANO_EINVAL and "overlap" in str(ei.value)


@pytest.mark.parametrize("B,shared,with_trans", [(1, False, True), (17, True, False),
                                                 (200, False, False), (4096, False, True)])
def test_forward_equals_staged(engine, dev, params, B, shared, with_trans):
    """mano_forward == its two kernels called as stages (articulate, then
    blend_skin16), bit for bit, for every output."""
    rng = np.random.default_rng(300 + B)
    betas = f32(rng.normal(0, 1, (10,) if shared else (B, 10)), dev)
    pose = f32(rng.normal(0, 0.6, (B, 16, 3)), dev)
    trans = f32(rng.uniform(-1, 1, (B, 3)), dev) if with_trans else None
    one = engine.forward(betas, pose, trans, joints=True, rest_verts=True, rest_joints=True,
                         rot_mats=True)
    j = torch.empty((B, 16, 3), device=dev)
    rj = torch.empty((B, 16, 3), device=dev)
    rm = torch.empty((B, 16, 3, 3), device=dev)
    v = torch.empty((B, 778, 3), device=dev)
    vp = torch.empty((B, 778, 3), device=dev)
    engine.stage_articulate(betas, pose, trans, joints=j, rest_joints=rj, rot_mats=rm)
    engine.stage_blend_skin(B, v, rest_verts=vp, trans=trans)
    torch.cuda.synchronize()
    for name, staged in (("verts", v), ("rest_verts", vp), ("joints", j), ("rest_joints", rj),
                         ("rot_mats", rm)):
        assert torch.equal(one[name], staged), name
    b = host(betas)
    ref = mano_oracle.forward(params, np.broadcast_to(b, (B, 10)) if shared else b, host(pose),
                              None if trans is None else host(trans))
    assert np.abs(host(one["verts"]) - ref["verts"]).max() <= TOL_M
    assert np.abs(host(one["joints"]) - ref["joints"]).max() <= TOL_M


@pytest.mark.parametrize("precision", ["fp32", "f16x3"])
@pytest.mark.parametrize("B", [1, 5, 64, 257, 1027])
def test_output_phase_independent(engine, dev, params, B, precision):
    """blend_skin16 / blend_skin_h3 pick their sector-aligned operand
    variants (mano_layout.h) from the verts address: verts / rest_verts written
    at every 4-B phase of a 32-B sector (views offset by 0..7 floats) are
    bit-identical to the plain outputs, with and without translation, and to
    the oracle.  So are the unfused stages: the blend GEMM's v_posed (fp32)
    and the standalone LBS reading and writing offset views."""
    engine.set_precision(precision)
    try:
        _phase_check(engine, dev, params, B)
    finally:
        engine.set_precision("fp32")


def _phase_check(engine, dev, params, B):
    rng = np.random.default_rng(900 + B)
    betas = f32(rng.normal(0, 1, (B, 10)), dev)
    pose = f32(rng.normal(0, 0.5, (B, 16, 3)), dev)
    trans = f32(rng.uniform(-1, 1, (B, 3)), dev)
    n = B * 778 * 3
    for tr in (None, trans):
        # plain-buffer references: with rest_verts (the fp32 kernel in either
        # precision -- f16x3 has no rest_verts kernel), verts only (the
        # precision's own fused kernel), and the standalone LBS over that v_posed
        want = engine.forward(betas, pose, tr, joints=False, rest_verts=True)
        want_v = engine.forward(betas, pose, tr, joints=False)["verts"]
        want_lbs = torch.empty_like(want_v)
        engine.stage_skin(B, want_lbs, rest_verts=want["rest_verts"], trans=tr)
        if engine.precision == "fp32":
            torch.cuda.synchronize()
            assert torch.equal(want_v, want["verts"]) and torch.equal(want_lbs, want["verts"])
        for off in range(8):
            buf = torch.full((2 * n + 64,), float("nan"), device=dev)
            v = buf[off:off + n].view(B, 778, 3)
            vp = buf[n + 32 + off:n + 32 + off + n].view(B, 778, 3)
            engine.stage_articulate(betas, pose, tr)
            engine.stage_blend_skin(B, v, rest_verts=vp, trans=tr)
            v_only = torch.full((n + 8,), float("nan"), device=dev)[off:off + n].view(B, 778, 3)
            engine.stage_blend_skin(B, v_only, trans=tr)
            # the unfused stages too: the blend GEMM's v_posed into an offset
            # view (fp32 only -- stage_blend is the fp32 GEMM in either
            # precision, so its v_posed is the fp32 kernel's), and the
            # standalone LBS from the offset rest_verts into an offset view
            vp_blend = None
            if engine.precision == "fp32":
                vp_blend = torch.full((n + 8,), float("nan"), device=dev)[off:off + n].view(B, 778, 3)
                engine.stage_blend(B, rest_verts=vp_blend)
            v_lbs = torch.full((n + 8,), float("nan"), device=dev)[off:off + n].view(B, 778, 3)
            engine.stage_skin(B, v_lbs, rest_verts=vp, trans=tr)
            torch.cuda.synchronize()
            assert torch.equal(v, want["verts"]), (off, tr is None)
            assert torch.equal(vp, want["rest_verts"]), (off, tr is None)
            assert torch.equal(v_only, want_v), (off, tr is None)
            if vp_blend is not None:
                assert torch.equal(vp_blend, want["rest_verts"]), (off, tr is None, "blend")
            assert torch.equal(v_lbs, want_lbs), (off, tr is None, "unfused")
            assert torch.isnan(buf[:off]).all() and torch.isnan(buf[off + n:n + 32 + off]).all()
            assert torch.isnan(buf[2 * n + 32 + off:]).all()
    ref = mano_oracle.forward(params, host(betas), host(pose), host(trans))
    assert np.abs(host(want["verts"]) - ref["verts"]).max() <= TOL_M
    assert np.abs(host(want_v) - ref["verts"]).max() <= TOL_M
    assert np.abs(host(want_lbs) - ref["verts"]).max() <= TOL_M


def truncated_params(params, V):
    """The synthetic model cut to its first V vertices: a smaller mesh of the
    same layout (exercises every span / tail-group case of the kernels)."""
    p = dict(params)
    for k in ("mesh_template", "mesh_shape_basis", "mesh_pose_basis", "skinning_weights"):
        p[k] = np.ascontiguousarray(np.asarray(params[k])[:V])
    p["J_regressor"] = np.ascontiguousarray(np.asarray(params["J_regressor"])[:, :V])
    f = np.asarray(params["faces"])
    p["faces"] = f[(f < V).all(axis=1)]
    return p


@pytest.mark.parametrize("precision", ["fp32", "f16x3"])
@pytest.mark.parametrize("V", [32, 50, 64, 100, 130, 200])
def test_other_mesh_sizes(dev, params, V, precision):
    """Meshes of V vertices: full 64-vertex spans (V // 64 of them) plus
    1-4 tail groups, or tail groups only; fused == staged LBS bit for bit and
    both within the tolerance of the oracle."""
    from mano_amd import ManoHip
    p = truncated_params(params, V)
    m = ManoHip(p, device=0, precision=precision)
    try:
        B = 37
        rng = np.random.default_rng(V)
        betas = f32(rng.normal(0, 1, (B, 10)), dev)
        pose = f32(rng.normal(0, 0.6, (B, 16, 3)), dev)
        trans = f32(rng.uniform(-1, 1, (B, 3)), dev)
        fused = m.forward(betas, pose, trans, joints=True, rest_verts=True)
        fused_v = m.forward(betas, pose, trans)["verts"]   # the precision's verts-only kernel
        m.stage_articulate(betas, pose, trans)
        v = torch.empty((B, V, 3), device=dev)
        m.stage_skin(B, v, rest_verts=fused["rest_verts"], trans=trans)
        torch.cuda.synchronize()
        if precision == "fp32":   # f16x3 builds no rest_verts kernel: its fused LBS has no v_posed to share
            assert torch.equal(fused["verts"], v) and torch.equal(fused_v, v)
        ref = mano_oracle.forward(p, host(betas), host(pose), host(trans))
        for key, got in (("verts", fused["verts"]), ("joints", fused["joints"]),
                         ("rest_verts", fused["rest_verts"]), ("verts", fused_v), ("verts", v)):
            err = np.abs(host(got) - ref[key]).max()
            assert err <= TOL_M, (V, precision, key, err)
    finally:
        m.close()
