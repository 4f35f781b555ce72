"""Whole-batch properties at BASELINE's C2 size (65,536 hands, MI355X).

The oracle checks sampled hands; these check EVERY hand of a full-size batch
against properties the math of `mano_np.py:79-115` guarantees exactly, so a
fault confined to some tile, residue class or sector phase of the fused
kernel's layout (mano_layout.h) cannot hide between the samples:

* position independence -- hands are independent (no cross-hand term), so a
  permuted batch gives the permuted outputs bit for bit, although every hand
  lands in another tile row, quad, residue class and basis variant;
* translation is a final fp32 add (`trans`): the outputs with
  per-hand trans equal the outputs without it plus trans, bit for bit;
* root-rotation equivariance -- G_0 = [R_0 | J_0] (`:97`) multiplies every
  joint's transform from the left, so verts(root r) = R(r)(verts(root 0) -
  J_0) + J_0 and the same for the posed joints (float64 on the fp32 outputs,
  within the north_star 1e-5 m)."""
import pytest

from oracle import mano_oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

B = 65536          # BASELINE configs[1] (C2)
SEED = 1001
TOL_M = 1e-5       # north_star: max |err| <= 1e-5 m


@pytest.fixture(scope="module", params=["fp32", "f16x3"])
def engine(params, request):
    from mano_amd import ManoHip
    m = ManoHip(params, device=0, precision=request.param)
    yield m
    m.close()


def test_permuted_batch_is_permuted_output(engine):
    inp = engine.synthetic_inputs(SEED, 0, B, trans=True)
    out = engine.forward(inp["betas"], inp["pose"], inp["trans"], joints=True)
    g = torch.Generator().manual_seed(5)
    perm = torch.randperm(B, generator=g).to(inp["pose"].device)
    outp = engine.forward(inp["betas"][perm], inp["pose"][perm], inp["trans"][perm], joints=True)
    torch.cuda.synchronize()
    assert engine.device_status() == 0
    for k in ("verts", "joints"):
        same = (outp[k] == out[k][perm]).flatten(1).all(dim=1)
        assert bool(same.all()), (engine.precision, k, int((~same).sum()), perm[~same][:8].tolist())


def test_translation_is_a_final_add(params):
    """fp32 (the f16x3 apply fuses trans into its last fma by design)."""
    from mano_amd import ManoHip
    m = ManoHip(params, device=0)
    try:
        inp = m.synthetic_inputs(SEED, 0, B, trans=True)
        with_t = m.forward(inp["betas"], inp["pose"], inp["trans"], joints=True)
        no_t = m.forward(inp["betas"], inp["pose"], None, joints=True)
        # the unfused path: articulate -> blend GEMM -> standalone LBS with trans
        vp = torch.empty_like(no_t["verts"])
        v = torch.empty_like(no_t["verts"])
        m.stage_articulate(inp["betas"], inp["pose"], inp["trans"])
        m.stage_blend(B, rest_verts=vp)
        m.stage_skin(B, v, rest_verts=vp, trans=inp["trans"])
        torch.cuda.synchronize()
        assert m.device_status() == 0
        t = inp["trans"][:, None, :]
        assert torch.equal(with_t["verts"], no_t["verts"] + t)
        assert torch.equal(with_t["joints"], no_t["joints"] + t)
        assert torch.equal(v, with_t["verts"])
    finally:
        m.close()


def test_root_rotation_equivariance(engine):
    inp = engine.synthetic_inputs(SEED, 0, B)
    pose0 = inp["pose"].clone()
    pose0[:, 0] = 0.0
    out = engine.forward(inp["betas"], inp["pose"], joints=True)
    out0 = engine.forward(inp["betas"], pose0, joints=True, rest_joints=True)
    torch.cuda.synchronize()
    assert engine.device_status() == 0
    R = torch.as_tensor(mano_oracle.rodrigues(inp["pose"][:, 0].double().cpu().numpy()),
                        device=pose0.device)                                   # (B,3,3) float64
    J0 = out0["rest_joints"][:, :1].double()                                   # (B,1,3)
    for k in ("verts", "joints"):
        want = torch.einsum("bij,bvj->bvi", R, out0[k].double() - J0) + J0
        err = (out[k].double() - want).abs().amax(dim=(1, 2))
        worst = int(err.argmax())
        print(f"root-rotation equivariance {engine.precision} {k}: max {float(err.max()):.3e} m (hand {worst})")
        assert float(err.max()) <= TOL_M, (engine.precision, k, worst, float(err.max()))
