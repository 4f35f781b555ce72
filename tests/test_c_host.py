"""The plain-C host of the C ABI (integration/mano_c_host.c) compiles with
-Wall -Wextra -Werror against include/mano_hip.h alone and links against
libmano_hip.so (no GPU needed)."""
import os
import shutil
import subprocess

import pytest

from conftest import REPO


def test_c_host_compiles_and_links(tmp_path):
    if shutil.which("gcc") is None:
        pytest.skip("gcc not installed")
    import __graft_entry__ as g
    out = str(tmp_path / "mano_c_host")
    g.build_c_host(out)
    assert os.access(out, os.X_OK)
    env = dict(os.environ, LD_LIBRARY_PATH=os.path.dirname(g.LIB))  # the rpath is relative to integration/
    r = subprocess.run([out], capture_output=True, text=True, env=env)  # usage only: no model, no GPU call
    assert r.returncode == 1 and "usage" in r.stderr
