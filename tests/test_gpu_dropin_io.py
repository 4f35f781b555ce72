"""The drop-in's own constructors on the GPU (mano_np.py:11-46, dump_model.py:4-21).

`MANOModel(model_path)` is the reference's constructor and the first line of
README / INTEGRATION: it is run here from the files a user would hold -- a
`dump_model.py` dict pickle written by `save_dump`, the same arrays as an
`.npz`, and an official-style pickle ingested by `load_official` (the stand-in
of tests/test_model_io.py: chumpy `Ch` leaves and a scipy CSC J_regressor;
parity with a real official file is unpinned, none exists here).  Each model
replays the reference's 23-step `set_params` script (tests/golden) at 1e-5 m.
"""
import numpy as np
import pytest

from conftest import step_kwargs

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL_M = 1e-5
TOL_R = 1e-6


def replay_script(model_factory, golden_steps):
    """Construct the model (the script's step 0 is the constructor's own
    update(), mano_np.py:46) and replay every set_params step."""
    manifest, data = golden_steps
    model = None
    for entry in manifest:
        i = entry["step"]
        if model is None:
            model = model_factory()
        else:
            model.set_params(**step_kwargs(entry, data))
        for key, got, tol in (("verts", model.verts, TOL_M), ("J", model.J, TOL_M),
                              ("R", model.R, TOL_R), ("rest_verts", model.rest_verts, TOL_M),
                              ("joints", model.joints, TOL_M)):
            err = np.abs(np.asarray(got, dtype=np.float64) - data[f"s{i}_out_{key}"]).max()
            assert err <= tol, (entry["desc"], key, err)
    return model


def test_constructor_from_dump_pickle(params, golden_steps, tmp_path):
    from mano_amd import MANOModel, save_dump
    path = tmp_path / "MANO_RIGHT_dump.pkl"
    save_dump(params, str(path))
    m = replay_script(lambda: MANOModel(str(path), device=0), golden_steps)
    assert m.parents == params["parents"] and m.parents[0] is None
    assert np.array_equal(np.asarray(m.faces), np.asarray(params["faces"]))


def test_constructor_from_npz(params, golden_steps, tmp_path):
    from mano_amd import MANOModel
    from mano_amd.model_io import MODEL_KEYS
    path = tmp_path / "mano.npz"
    arrays = {k: np.asarray(params[k]) for k in MODEL_KEYS if k != "parents"}
    arrays["parents"] = np.array([-1 if p is None else p for p in params["parents"]], dtype=np.int64)
    np.savez(path, **arrays)
    replay_script(lambda: MANOModel(str(path), device=0), golden_steps)


def test_constructor_from_official_pickle(params, golden_steps, golden_batch, tmp_path):
    """dump_model.py's input format: load_official -> from_params, and the
    dump_model() file it writes -> MANOModel(path)."""
    from test_model_io import _official_like
    from mano_amd import ManoHip, MANOModel
    from mano_amd.model_io import dump_model, load_official
    src = tmp_path / "MANO_RIGHT.pkl"
    src.write_bytes(_official_like(params, 2))
    official = load_official(str(src))
    replay_script(lambda: MANOModel.from_params(official, device=0), golden_steps)
    dst = tmp_path / "MANO_RIGHT_dumped.pkl"
    dump_model(str(src), str(dst))
    replay_script(lambda: MANOModel(str(dst), device=0), golden_steps)
    # the golden batch through the batched engine built from the official file
    g = golden_batch
    eng = ManoHip(official, device=0)
    dev = torch.device("cuda", 0)
    out = eng.forward(torch.tensor(g["betas"], dtype=torch.float32, device=dev),
                      torch.tensor(g["pose"], dtype=torch.float32, device=dev), joints=True)
    torch.cuda.synchronize()
    assert np.abs(out["verts"].double().cpu().numpy() - g["verts"]).max() <= TOL_M
    assert np.abs(out["joints"].double().cpu().numpy() - g["joints"]).max() <= TOL_M
    eng.close()


@pytest.mark.parametrize("zero_copy", [True, False])
def test_dropin_graph_workspace_is_private(params, golden_steps, zero_copy):
    """The drop-in's batch-1 launches (on the pinned host blocks, or the
    captured HIP graph of the copy form) read and write their own batch-1
    workspace: batched calls on the same engine over every pooled stream
    (torch.cuda.Stream() hands out a pool of handles), each growing that
    stream's workspace, must not disturb them."""
    from mano_amd import MANOModel
    manifest, data = golden_steps
    m = MANOModel.from_params(params, device=0)
    m.zero_copy = zero_copy
    assert m.use_graphs
    first = next(e for e in manifest if e["step"] > 0)
    kw = step_kwargs(first, data)
    m.set_params(**kw)                      # builds and replays the graph
    want = m.verts.copy()
    dev = m.device
    B = 4096
    betas = torch.randn(B, 10, device=dev)
    pose = 0.5 * torch.randn(B, 16, 3, device=dev)
    for _ in range(40):                     # more streams than the pool holds
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            m.forward_batch(betas, pose, joints=True, rest_verts=True)
    torch.cuda.synchronize()
    for _ in range(3):
        got = m.set_params(**kw)
        assert np.array_equal(got, want)
    err = np.abs(want - data[f"s{first['step']}_out_verts"]).max()
    assert err <= TOL_M
