"""The C ABI from a plain C program (integration/mano_c_host.c): model
create from the dump_model.py arrays, on-device synthetic inputs, mano_forward,
the single-process RCCL group gather (ABI 6) and the status read -- its
verts and posed joints equal the Python engine's forward of the same hands
bit for bit."""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

C_HOST = os.path.join(REPO, "integration", "mano_c_host")


def write_model_bin(path, params):
    f64 = lambda k: np.ascontiguousarray(np.asarray(params[k], dtype=np.float64))  # noqa: E731
    from mano_amd.model_io import parents_to_int
    V = f64("mesh_template").shape[0]
    with open(path, "wb") as f:
        f.write(np.int32(V).tobytes())
        for k in ("mesh_template", "mesh_shape_basis", "mesh_pose_basis", "J_regressor", "skinning_weights"):
            f.write(f64(k).tobytes())
        f.write(parents_to_int(params["parents"]).astype(np.int32).tobytes())
        f.write(f64("pose_pca_basis").tobytes())
        f.write(f64("pose_pca_mean").tobytes())
    return V


@pytest.mark.parametrize("n", [1, 777, 4099])
def test_c_host_matches_engine(params, tmp_path, n):
    assert os.path.exists(C_HOST), "built by __graft_entry__.build()"
    V = write_model_bin(str(tmp_path / "model.bin"), params)
    out = str(tmp_path / "out.bin")
    r = subprocess.run([C_HOST, str(tmp_path / "model.bin"), str(n), "1001", out], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    raw = np.fromfile(out, dtype=np.float32)
    verts = raw[:n * V * 3].reshape(n, V, 3)
    joints = raw[n * V * 3:].reshape(n, 16, 3)
    from mano_amd import ManoHip
    m = ManoHip(params, device=0)
    inp = m.synthetic_inputs(1001, 0, n)
    ref = m.forward(inp["betas"], inp["pose"], joints=True)
    torch.cuda.synchronize()
    assert np.array_equal(verts, ref["verts"].cpu().numpy())
    assert np.array_equal(joints, ref["joints"].cpu().numpy())
    m.close()
