"""Golden vectors for dump_scans() by running the REFERENCE (build container only).

Run from the repo root:  python tests/golden/make_scan_goldens.py
It needs `/root/reference/dump_model.py` (importable here, absent on the GPU
box).  `dump_scans()` (dump_model.py:24-43) reads '../model/MANO_LEFT.pkl' and
'../model/MANO_RIGHT.pkl' relative to the working directory and writes
'./axangles.npy'; this script builds two official-layout pickles holding the
three arrays dump_scans reads (hands_components, hands_mean, hands_coeffs --
numpy arrays, as in the official files) in a temporary tree, runs the
reference there, and stores inputs + output in mano_reference_scans.npz.
"""
import os
import pickle
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(REPO, "mano-hand_amd"))
sys.path.insert(0, "/root/reference")

from mano_amd.model_io import synthetic_params  # noqa: E402
import dump_model as reference  # noqa: E402  (the reference)


def main():
    rng = np.random.default_rng(42)
    arrays = {}
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "model"))
        os.makedirs(os.path.join(tmp, "work"))
        for side, seed, m in (("LEFT", 0, 40), ("RIGHT", 1, 33)):
            p = synthetic_params(seed)
            official = {"hands_components": np.asarray(p["pose_pca_basis"]),
                        "hands_mean": np.asarray(p["pose_pca_mean"]),
                        "hands_coeffs": rng.normal(0, 1, (m, 45))}
            with open(os.path.join(tmp, "model", f"MANO_{side}.pkl"), "wb") as f:
                pickle.dump(official, f, protocol=2)
            for k, v in official.items():
                arrays[f"{side.lower()}_{k}"] = v
        cwd = os.getcwd()
        os.chdir(os.path.join(tmp, "work"))
        try:
            reference.dump_scans()
            arrays["axangles"] = np.load("axangles.npy", allow_pickle=False)
        finally:
            os.chdir(cwd)
    np.savez(os.path.join(HERE, "mano_reference_scans.npz"), **arrays)
    print("axangles", arrays["axangles"].shape)


if __name__ == "__main__":
    main()
