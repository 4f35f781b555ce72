"""Randomized batch sizes and output address phases (MI355X).

The fused kernel tiles hands in residue classes of the verts address phase
(mano_layout.h: quads of 64 hands of one class, shifted operand variants) and
the standalone LBS in 4-hand x 64-vertex units; the index math has many
cases (partial quads, classes with one hand more than others, tiles past the
batch end recomputing the last tile).  Twenty seeded batch sizes between 1
and 300,000, each written at a random 4-B phase of a 32-B sector: the first,
last, tile / quad / class-boundary and random hands of verts and joints
against the float64 oracle (north_star 1e-5 m), the whole batch finite, and
the standalone LBS over the fused kernel's own v_posed equal to it bit for bit
on every hand (the two kernels' tilings are unrelated, so agreement on all
rows also covers every tile the sample misses)."""
import numpy as np
import pytest

from oracle import mano_oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL_M = 1e-5


def _sizes():
    rng = np.random.default_rng(2026)
    sizes = set(int(x) for x in np.exp(rng.uniform(0, np.log(300000), 16)).astype(int) + 1)
    sizes |= {63, 64, 257, 4 * 64 * 8 + 3}     # one quad short, one quad, a quad + 1, 8 classes + 3
    return sorted(sizes)


def _check_rows(B):
    P = 8  # address-phase period of the residue classes (hands)
    edges = {0, 1, 2, B - 1, B - 2, B - 3}
    for q in (63, 64, 65, 64 * P - 1, 64 * P, 64 * P + 1, B // 2):
        edges |= {q, B - 1 - q}
    rnd = np.random.default_rng(B).integers(0, B, 24)
    return np.unique(np.clip(np.array(sorted(edges | set(int(x) for x in rnd))), 0, B - 1))


@pytest.mark.parametrize("B", _sizes())
def test_random_batch_and_phase(params, B):
    from mano_amd import ManoHip
    dev = torch.device("cuda", 0)
    m = ManoHip(params, device=0)
    try:
        rng = np.random.default_rng(B + 7)
        off = int(rng.integers(0, 8))                    # float offset: the 4-B phase in a 32-B sector
        inp = m.synthetic_inputs(4000 + B % 97, 0, B, trans=True)
        n = B * 778 * 3
        buf = torch.full((n + 16,), float("nan"), device=dev)
        verts = buf[off:off + n].view(B, 778, 3)
        joints = torch.empty((B, 16, 3), device=dev)
        rest = torch.empty((B, 778, 3), device=dev)
        m.forward(inp["betas"], inp["pose"], inp["trans"], joints=True, rest_verts=True,
                  out={"verts": verts, "joints": joints, "rest_verts": rest})
        v_only = torch.full((n + 16,), float("nan"), device=dev)[off:off + n].view(B, 778, 3)
        m.forward(inp["betas"], inp["pose"], inp["trans"], joints=False, out={"verts": v_only})
        lbs = torch.empty_like(rest)
        m.stage_skin(B, lbs, rest_verts=rest, trans=inp["trans"])
        torch.cuda.synchronize()
        assert m.device_status() == 0
        assert torch.isfinite(verts).all() and torch.isfinite(joints).all()
        assert torch.isnan(buf[:off]).all() and torch.isnan(buf[off + n:]).all()
        assert torch.equal(v_only, verts)                  # with / without rest_verts: same bits
        assert torch.equal(lbs, verts)                     # standalone LBS == fused, every hand
        idx = _check_rows(B)
        ti = torch.as_tensor(idx, device=dev)
        h = lambda t: t.index_select(0, ti).double().cpu().numpy()  # noqa: E731
        ref = mano_oracle.forward(params, h(inp["betas"]), h(inp["pose"]), h(inp["trans"]))
        ev = np.abs(h(verts) - ref["verts"]).max()
        ej = np.abs(h(joints) - ref["joints"]).max()
        assert ev <= TOL_M and ej <= TOL_M, (B, off, ev, ej)
    finally:
        m.close()
