"""Non-finite inputs stay inside their own hand (MI355X).

The reference has no input checks: a NaN or Inf in one hand's pose, shape or
(our extension) translation runs through `mano_np.py:79-115` and comes out as
non-finite values of that hand only (numpy propagates them; which joints go
non-finite follows the kinematic tree, `:96-104`).  The batched kernels mix
hands in every MFMA tile (16 hands per tile, rows past the batch end repeat
the last hand) and the f16x3 kernels split every operand into halves, so this
checks, in both precisions and along the fused and the unfused path:

* each poisoned hand's verts / joints are non-finite exactly where the float64
  oracle's are (the per-joint mask of the kinematic chain included);
* every other hand is bit-identical to the same forward on clean inputs."""
import numpy as np
import pytest

from oracle import mano_oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

B = 1000
# hand -> (what, value): a pose joint component (non-root and root), a shape
# coefficient, a translation, and the last hand of the batch (whose row the
# partial tile repeats)
POISON = {17: ("pose", (5, 1), float("nan")), 333: ("pose", (0, 2), float("inf")),
          500: ("betas", 3, float("inf")), 777: ("trans", 0, float("nan")),
          999: ("pose", (15, 0), float("nan"))}


def _inputs():
    rng = np.random.default_rng(77)
    betas = rng.normal(0, 1, (B, 10))
    pose = rng.normal(0, 0.6, (B, 16, 3))
    trans = rng.uniform(-1, 1, (B, 3))
    bad = [betas.copy(), pose.copy(), trans.copy()]
    for h, (what, idx, val) in POISON.items():
        arr = {"betas": bad[0], "pose": bad[1], "trans": bad[2]}[what]
        arr[(h,) + (idx if isinstance(idx, tuple) else (idx,))] = val
    return (betas, pose, trans), tuple(bad)


def _forward_all(m, betas, pose, trans):
    """verts / joints of the fused forward, plus the unfused stages' verts
    (articulate -> blend GEMM -> standalone LBS) in fp32."""
    out = m.forward(betas, pose, trans, joints=True)
    res = {"verts": out["verts"], "joints": out["joints"]}
    if m.precision == "fp32":
        j = torch.empty_like(out["joints"])
        m.stage_articulate(betas, pose, trans, joints=j)
        vp = torch.empty_like(out["verts"])
        v = torch.empty_like(out["verts"])
        m.stage_blend(B, rest_verts=vp)
        m.stage_skin(B, v, rest_verts=vp, trans=trans)
        res["verts_unfused"] = v
    else:
        res["verts_lbs"] = torch.empty_like(out["verts"])
        fp = m.forward(betas, pose, trans, joints=False, rest_verts=True)  # fp32 kernel, f16x3 LBS below
        m.stage_skin(B, res["verts_lbs"], rest_verts=fp["rest_verts"], trans=trans)
    torch.cuda.synchronize()
    return {k: v.cpu() for k, v in res.items()}


@pytest.mark.parametrize("precision", ["fp32", "f16x3"])
def test_poisoned_hands_stay_isolated(params, precision):
    from mano_amd import ManoHip
    dev = torch.device("cuda", 0)
    (betas, pose, trans), (bbad, pbad, tbad) = _inputs()
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=dev)  # noqa: E731
    m = ManoHip(params, device=0, precision=precision)
    try:
        clean = _forward_all(m, t(betas), t(pose), t(trans))
        dirty = _forward_all(m, t(bbad), t(pbad), t(tbad))
        assert m.device_status() == 0
    finally:
        m.close()
    hands = sorted(POISON)
    good = torch.ones(B, dtype=torch.bool)
    good[hands] = False
    for k in clean:
        assert torch.equal(dirty[k][good], clean[k][good]), (precision, k)
    with np.errstate(all="ignore"):
        ref = mano_oracle.forward(params, bbad[hands], pbad[hands], tbad[hands])
    for i, h in enumerate(hands):
        rv = ~np.isfinite(ref["verts"][i])
        rj = ~np.isfinite(ref["joints"][i])
        assert rv.any(), (h, "the oracle keeps this hand finite: the poison missed")
        for k in clean:
            got = ~np.isfinite(dirty[k][h].numpy())
            want = rj if k == "joints" else rv
            assert np.array_equal(got, want), (precision, k, h, int(got.sum()), int(want.sum()))
