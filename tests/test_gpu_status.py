"""The device status word (include/mano_hip.h mano_model_device_status).

skin_pair's memory and compute waves hand units over through bounded LDS
waits; a wait that gives up must be reported, never return MANO_OK with
un-skinned vertices silently.  The timeout path is forced with the
diagnostic library libmano_hip_polltest.so (waits give up after one poll;
built by __graft_entry__.build()), in a child process."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

POLLTEST = os.path.join(REPO, "mano-hand_amd", "mano_amd", "libmano_hip_polltest.so")

_CHILD = r"""
import sys
sys.path.insert(0, sys.argv[1] + "/mano-hand_amd")
from mano_amd import _abi
_abi.LIB_PATH = sys.argv[2]          # the diagnostic library, this child only
import torch
from mano_amd import ManoHip, synthetic_params
m = ManoHip(synthetic_params(0), device=0)
assert m.device_status() == 0
B = 4096
inp = m.synthetic_inputs(1001, 0, B)
verts = torch.full((B, 778, 3), float("nan"), device="cuda:0")
m.stage_articulate(inp["betas"], inp["pose"])
m.stage_blend(B)
m.stage_skin(B, verts)
st = m.device_status(clear=True)
again = m.device_status(clear=True)
unwritten = int(torch.isnan(verts).any(dim=2).any(dim=1).sum())
print("STATUS", st, again, unwritten)
m.close()
"""


def test_status_clean_after_every_kernel(params):
    from mano_amd import ManoHip
    m = ManoHip(params, device=0)
    try:
        assert m.device_status() == 0
        for prec in ("fp32", "f16x3"):
            m.set_precision(prec)
            inp = m.synthetic_inputs(1001, 0, 20000, trans=True)
            m.forward(inp["betas"], inp["pose"], inp["trans"], joints=True, rest_verts=True)
            m.stage_articulate(inp["betas"], inp["pose"], inp["trans"])
            m.stage_blend(20000)
            v = torch.empty((20000, 778, 3), device="cuda:0")
            m.stage_skin(20000, v, trans=inp["trans"])
            m.check_device()
        assert m.device_status() == 0
    finally:
        m.close()


def test_handoff_timeout_is_reported():
    assert os.path.exists(POLLTEST), "build with __graft_entry__.build()"
    r = subprocess.run([sys.executable, "-c", _CHILD, REPO, POLLTEST], capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("STATUS")][-1].split()
    st, again, unwritten = int(line[1]), int(line[2]), int(line[3])
    from mano_amd import _abi
    assert st & _abi.MANO_DEVICE_SKIN_HANDOFF_TIMEOUT, line
    assert again == 0                 # cleared by the first read
    assert unwritten > 0              # the unconfirmed units' verts were not stored
