"""The maintainer's binding (integration/mano_hip_ffi.py): numpy + ctypes only.

A child process that never imports torch drives libmano_hip.so through the
C-ABI alone (mano_host_alloc / mano_alloc / mano_forward / mano_synchronize,
and the copy form's mano_memcpy): the golden batch through `Engine.forward`
in both I/O forms (bit-identical), and the reference's stateful set_params
script with `update` patched onto a stand-in of the reference class (the
oracle's restatement of mano_np.py:35-77, its arrays bound under the
reference's attribute names), each within 1e-5 m of the reference goldens.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, sys
import numpy as np
sys.path[:0] = [REPO + "/integration", REPO + "/mano-hand_amd", REPO]
import mano_hip_ffi
from mano_amd.model_io import synthetic_params
from oracle.mano_oracle import StatefulOracle

params = synthetic_params(0)
g = dict(np.load(REPO + "/tests/golden/mano_reference_batch.npz", allow_pickle=False))
eng = mano_hip_ffi.Engine(type("M", (), params), device=0, capacity=4)
out = eng.forward(g["betas"], g["pose"])   # grows the buffers 4 -> 24 hands
for k_got, k_ref in (("verts", "verts"), ("J", "J"), ("R", "R"), ("rest_verts", "rest_verts"),
                     ("joints", "joints")):
    err = np.abs(out[k_got] - g[k_ref]).max()
    assert err <= 1e-5, (k_got, err)
# a smaller batch after a larger one converts only its own rows, same bits
small = eng.forward(g["betas"][:3], g["pose"][:3])
for k in out:
    assert small[k].shape[0] == 3 and np.array_equal(small[k], out[k][:3]), k
eng.close()
# the copy form (device buffers + mano_memcpy) gives the zero-copy form's bits
eng_c = mano_hip_ffi.Engine(type("M", (), params), device=0, capacity=24, zero_copy=False)
out_c = eng_c.forward(g["betas"], g["pose"])
for k in out:
    assert np.array_equal(out[k], out_c[k]), k
eng_c.close()

class Ref(StatefulOracle):
    """Stand-in for mano_np.MANOModel: the reference's attributes + set_params."""
    def __init__(self, p):
        for k, v in p.items():
            setattr(self, k, v)
        super().__init__(p)

mano_hip_ffi.patch(Ref, device=0)
z = dict(np.load(REPO + "/tests/golden/mano_reference_steps.npz", allow_pickle=False))
manifest = json.loads(str(z.pop("manifest")))
model = None
worst = 0.0
for entry in manifest:
    i = entry["step"]
    if model is None:
        model = Ref(params)
    else:
        kw = {k: z[f"s{i}_in_{k}"] for k in entry["args"]}
        ret = model.set_params(**kw)
        assert ret.dtype == np.float64 and ret.shape == (778, 3)
    for key in ("verts", "J", "R", "rest_verts"):
        err = np.abs(np.asarray(getattr(model, key)) - z[f"s{i}_out_{key}"]).max()
        assert err <= 1e-5, (entry["desc"], key, err)
        worst = max(worst, err)
model._hip_engine.close()
assert "torch" not in sys.modules, "the binding pulled in torch"
print("FFI_OK", len(manifest), "steps, worst err", worst)
'''


def test_numpy_ctypes_binding_without_torch():
    code = "REPO = %r\n" % REPO + CHILD
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "FFI_OK" in r.stdout
