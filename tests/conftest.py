import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "mano-hand_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")

# Diagnostic A/B runs only: MANO_TEST_LIB=<file in mano_amd/> runs the suite
# against another build of the library (a tools/ variant).  The driver never
# sets it; test_library_is_the_loaded_path then checks the named file loaded.
if os.environ.get("MANO_TEST_LIB"):
    from mano_amd import _abi as _abi_mod
    _abi_mod.LIB_PATH = os.path.join(os.path.dirname(_abi_mod.LIB_PATH), os.environ["MANO_TEST_LIB"])


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def params():
    from mano_amd import synthetic_params
    return synthetic_params(0)


@pytest.fixture(scope="session")
def golden_steps():
    import json
    with np.load(os.path.join(GOLDEN, "mano_reference_steps.npz"), allow_pickle=False) as z:
        data = {k: z[k] for k in z.files}
    manifest = json.loads(str(data.pop("manifest")))
    return manifest, data


@pytest.fixture(scope="session")
def golden_batch():
    with np.load(os.path.join(GOLDEN, "mano_reference_batch.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def step_kwargs(entry, data):
    """Rebuild the set_params kwargs of one golden step (as the generator passed them)."""
    i = entry["step"]
    kw = {}
    for k in entry["args"]:
        v = data[f"s{i}_in_{k}"]
        kw[k] = v if k not in ("global_rot",) else list(v)
    return kw
