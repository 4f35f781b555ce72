"""Per-call latency of the drop-in MANOModel.set_params (batch 1): the kernels
on the pinned host blocks (zero copy, the default), packed I/O through them
(model.py: one pinned H2D, one D2H) replayed from a HIP graph, the same
launched eagerly, and the round-2 form (a device tensor per input, a
.double().cpu() per output); same model, same inputs, same process.

    python tools/debug/dropin_latency.py [--calls 300]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "mano-hand_amd"))


def per_array_update(self):
    """The round-2 MANOModel.update (per-array copies), for the comparison."""
    pose = np.asarray(self.pose.reshape((-1, 1, 3)), dtype=np.float64)
    shape = np.asarray(self.shape, dtype=np.float64)
    trans = None if not np.any(self.trans) else self._dev(self.trans)[None]
    out = self.engine.forward(self._dev(shape)[None], self._dev(pose.reshape(1, self.n_joints, 3)),
                              trans, joints=True, rest_verts=True, rest_joints=True, rot_mats=True)
    host = {k: v[0].double().cpu().numpy() for k, v in out.items()}
    self.verts = host["verts"]
    self.rest_verts = host["rest_verts"]
    self.J = host["rest_joints"]
    self.R = host["rot_mats"]
    self.joints = host["joints"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=300)
    a = ap.parse_args()
    from mano_amd import MANOModel, synthetic_params
    from mano_amd import model as model_mod
    params = synthetic_params(0)
    rng = np.random.default_rng(3)
    poses = rng.normal(0, 0.5, (a.calls, 16, 3))
    shapes = rng.normal(0, 1, (a.calls, 10))
    res = {}
    packed = model_mod.MANOModel.update
    for name, upd, graphs, zc in (("zero_copy", packed, True, True), ("graph", packed, True, False),
                                  ("packed", packed, False, False), ("per_array", per_array_update, False, False),
                                  ("zero_copy_again", packed, True, True)):
        model_mod.MANOModel.update = upd
        model_mod.MANOModel.use_graphs = graphs
        model_mod.MANOModel.zero_copy = zc
        m = MANOModel.from_params(params, device=0)
        outs = []
        for i in range(30):
            m.set_params(pose_abs=poses[i], shape=shapes[i])
        ts = []
        for i in range(a.calls):
            t0 = time.perf_counter()
            outs.append(m.set_params(pose_abs=poses[i], shape=shapes[i]))
            ts.append(time.perf_counter() - t0)
        ts = np.sort(np.asarray(ts)) * 1e6
        res[name] = {"median_us": float(np.median(ts)), "p90_us": float(ts[int(0.9 * len(ts))]),
                     "digest": float(np.sum(np.stack(outs)[:, ::7]))}
        m.engine.close()
    model_mod.MANOModel.update = packed
    model_mod.MANOModel.use_graphs = True
    model_mod.MANOModel.zero_copy = True
    res["same_results"] = len({res[k]["digest"] for k in ("zero_copy", "graph", "packed", "per_array")}) == 1
    print(json.dumps(res))


if __name__ == "__main__":
    main()
