"""The device status of a model (include/mano_hip.h mano_model_device_status).

skin_pair's memory and compute waves hand units over through bounded LDS
waits; a wait that gives up must be reported, never return MANO_OK with
un-skinned vertices silently: the flag it raises makes `synchronize()` raise
and every later launch on the model fail with MANO_EDEVICE until it is read
and cleared.  The timeout path is forced with the diagnostic library
libmano_hip_polltest.so (waits give up after one poll; built by
__graft_entry__.build()), in a child process."""
import os
import subprocess
import sys

import pytest

from conftest import REPO

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

POLLTEST = os.path.join(REPO, "mano-hand_amd", "mano_amd", "libmano_hip_polltest.so")

_CHILD = r"""
import sys, threading
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
try:
    m.synchronize()
    sync_raised = 0
except _abi.DeviceStatusError as e:
    sync_raised = e.status
# every launching call fails loudly while the flag is set
blocked = 0
for call in (lambda: m.stage_articulate(inp["betas"], inp["pose"]), lambda: m.stage_skin(B, verts),
             lambda: m.forward(inp["betas"], inp["pose"])):
    try:
        call()
    except _abi.DeviceStatusError as e:
        blocked += e.code == _abi.MANO_EDEVICE
st = m.device_status(clear=True)
again = m.device_status(clear=True)
unwritten = int(torch.isnan(verts).any(dim=2).any(dim=1).sum())
m.forward(inp["betas"], inp["pose"])   # launches again once cleared
m.synchronize()
# two threads read-and-clear at once: each raised bit is reported exactly once
reports = []
for it in range(8):
    m.stage_articulate(inp["betas"], inp["pose"])
    m.stage_blend(B)
    m.stage_skin(B, verts)
    torch.cuda.synchronize()
    go = threading.Barrier(2)
    got = [None, None]
    def take(i):
        go.wait()
        got[i] = m.device_status(clear=True)
    ts = [threading.Thread(target=take, args=(i,)) for i in range(2)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    reports.append(sum(1 for g in got if g & _abi.MANO_DEVICE_SKIN_HANDOFF_TIMEOUT))
print("STATUS", sync_raised, blocked, st, again, unwritten, ",".join(map(str, reports)))
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
            m.synchronize()
            m.check_device()
        assert m.device_status() == 0
        assert m.device_status(clear=False, wait=False) == 0
    finally:
        m.close()


def test_handoff_timeout_is_reported():
    assert os.path.exists(POLLTEST), "build with __graft_entry__.build()"
    r = subprocess.run([sys.executable, "-c", _CHILD, REPO, POLLTEST], capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("STATUS")][-1].split()
    sync_raised, blocked, st, again, unwritten = (int(x) for x in line[1:6])
    reports = [int(x) for x in line[6].split(",")]
    from mano_amd import _abi
    bit = _abi.MANO_DEVICE_SKIN_HANDOFF_TIMEOUT
    assert sync_raised & bit, line      # synchronize() raised
    assert blocked == 3                  # every launching call refused with MANO_EDEVICE
    assert st & bit, line
    assert again == 0                    # cleared by the first read
    assert unwritten > 0                 # the unconfirmed units' verts were not stored
    assert reports == [1] * len(reports), reports   # concurrent read-and-clear: reported once, never lost
