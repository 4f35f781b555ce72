"""CPU oracle for the MANO forward pass -- TEST INFRASTRUCTURE ONLY.

This is a float64 numpy restatement of the reference hot path
(`/root/reference/mano_np.py`, `MANOModel.update` :79-115 and its helpers
`rodrigues` :117-148, `with_zeros` :150-163, `pack` :165-179) and of the
`set_params` argument semantics (:48-77).  It exists to CHECK the HIP path:
only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg
may import it.  The product (`mano-hand_amd/`) never imports, links or
executes anything under `oracle/`.

Parity pinning: `tests/test_oracle_golden.py` checks this restatement against
fixtures in `tests/golden/`, which `tests/golden/make_goldens.py` produced by
importing the reference `MANOModel` itself in the build container on the
deterministic synthetic model (the official MANO pickle is licensed and absent).
The restatement agrees with the reference to ~1e-16 m on every fixture.

Two forms are provided:
  * `forward`      -- batched over hands (einsum), the checker for large batches;
  * `forward_one`  -- one hand at a time, the reference's op sequence verbatim
                      (shape blend, J regression, Rodrigues, pose blend, chain
                      loop, rest removal, W.G, LBS apply); `bench.py` times it as
                      the CPU baseline (`cpu_baseline.kind == "port"`).
"""
from __future__ import annotations

import numpy as np

EPS64 = np.finfo(np.float64).eps  # mano_np.py:132


def rodrigues(r):
    """Axis-angle (..., 3) -> rotation (..., 3, 3); restates mano_np.py:117-148.

    theta = |r| clamped to float64 eps (:130-132), r_hat = r/theta (:133),
    R = cos I + (1 - cos) r_hat r_hat^T + sin [r_hat]_x (:136-147).
    """
    r = np.asarray(r, dtype=np.float64)
    theta = np.linalg.norm(r, axis=-1, keepdims=True)
    theta = np.maximum(theta, EPS64)
    rh = r / theta
    c = np.cos(theta)[..., None]
    s = np.sin(theta)[..., None]
    x, y, z = rh[..., 0], rh[..., 1], rh[..., 2]
    zero = np.zeros_like(x)
    m = np.stack([zero, -z, y, z, zero, -x, -y, x, zero], axis=-1).reshape(r.shape[:-1] + (3, 3))
    dot = rh[..., :, None] * rh[..., None, :]
    eye = np.eye(3)
    return c * eye + (1.0 - c) * dot + s * m


def pose_features(R):
    """(R[1:] - I).ravel() per hand: feature k = 9(j-1) + 3 row + col (mano_np.py:87-91)."""
    R = np.asarray(R)
    return (R[..., 1:, :, :] - np.eye(3)).reshape(R.shape[:-3] + (-1,))


def chain(R, J, parents):
    """Kinematic chain (mano_np.py:96-104) and rest-pose removal (:106-110).

    R (B,16,3,3), J (B,16,3) rest joints.  Returns
      posed_joints (B,16,3) = G[:, :, :3, 3] before removal (not stored by the
      reference; derived exactly as the recurrence defines it),
      G (B,16,4,4) after removal (the skinning transforms of :112).
    """
    B, nj = R.shape[0], R.shape[1]
    G = np.zeros((B, nj, 4, 4))
    G[:, :, 3, 3] = 1.0
    G[:, 0, :3, :3] = R[:, 0]
    G[:, 0, :3, 3] = J[:, 0]
    for i in range(1, nj):
        p = parents[i]
        local = np.zeros((B, 4, 4))
        local[:, :3, :3] = R[:, i]
        local[:, :3, 3] = J[:, i] - J[:, p]
        local[:, 3, 3] = 1.0
        G[:, i] = G[:, p] @ local
    posed = G[:, :, :3, 3].copy()
    Jh = np.concatenate([J, np.zeros((B, nj, 1))], axis=-1)
    G[:, :, :, 3] -= np.einsum("bjkl,bjl->bjk", G, Jh)
    return posed, G


def forward(params, betas, pose, trans=None):
    """Batched fp64 restatement of mano_np.py:79-115 (+ optional translation).

    betas (B,10) or (10,), pose (B,16,3) or (B,48).  Returns a dict with
    verts (B,V,3), joints (B,16,3) posed, rest_verts (B,V,3) (= .rest_verts),
    rest_joints (B,16,3) (= .J), rot (B,16,3,3) (= .R).
    `trans` (B,3) is the build's extension: added to verts
    and joints after skinning; the reference has no translation parameter.
    """
    pose = np.asarray(pose, dtype=np.float64)
    B = pose.shape[0]
    pose = pose.reshape(B, -1, 3)
    betas = np.asarray(betas, dtype=np.float64)
    if betas.ndim == 1:
        betas = np.broadcast_to(betas, (B, betas.shape[0]))
    tmpl = np.asarray(params["mesh_template"], dtype=np.float64)
    sdirs = np.asarray(params["mesh_shape_basis"], dtype=np.float64)
    pdirs = np.asarray(params["mesh_pose_basis"], dtype=np.float64)
    jreg = np.asarray(params["J_regressor"], dtype=np.float64)
    W = np.asarray(params["skinning_weights"], dtype=np.float64)
    parents = params["parents"]
    v_shaped = tmpl[None] + np.einsum("vcs,bs->bvc", sdirs, betas)          # :81
    J = np.einsum("jv,bvc->bjc", jreg, v_shaped)                            # :83
    R = rodrigues(pose)                                                     # :84-86
    v_posed = v_shaped + np.einsum("vcp,bp->bvc", pdirs, pose_features(R))  # :87-93
    posed, G = chain(R, J, parents)                                         # :96-110
    T = np.einsum("vj,bjkl->bvkl", W, G)                                    # :112
    verts = np.einsum("bvkl,bvl->bvk", T[:, :, :3, :3], v_posed) + T[:, :, :3, 3]  # :113-115
    if trans is not None:
        t = np.asarray(trans, dtype=np.float64).reshape(B, 1, 3)
        verts = verts + t
        posed = posed + t
    return {"verts": verts, "joints": posed, "rest_verts": v_posed,
            "rest_joints": J, "rot": R}


def forward_one(params, beta, pose):
    """One hand, the reference op sequence of mano_np.py:81-115 (CPU baseline)."""
    tmpl = params["mesh_template"]
    v_shaped = tmpl + params["mesh_shape_basis"].dot(beta)                          # :81
    J = params["J_regressor"].dot(v_shaped)                                          # :83
    R = rodrigues(np.asarray(pose).reshape(-1, 3))                                   # :84-86
    v_posed = v_shaped + params["mesh_pose_basis"].dot((R[1:] - np.eye(3)).ravel())  # :87-93
    parents = params["parents"]
    nj = R.shape[0]
    G = np.empty((nj, 4, 4))
    bottom = np.array([[0.0, 0.0, 0.0, 1.0]])
    G[0] = np.vstack((np.hstack((R[0], J[0].reshape(3, 1))), bottom))              # :97
    for i in range(1, nj):                                                          # :98-104
        p = parents[i]
        G[i] = G[p].dot(np.vstack((np.hstack([R[i], (J[i] - J[p]).reshape(3, 1)]), bottom)))
    Jh = np.hstack([J, np.zeros((nj, 1))]).reshape(nj, 4, 1)
    G = G - np.dstack((np.zeros((nj, 4, 3)), np.matmul(G, Jh)))                     # :106-110
    T = np.tensordot(params["skinning_weights"], G, axes=[[1], [0]])                # :112
    rest_h = np.hstack((v_posed, np.ones((v_posed.shape[0], 1))))
    return np.matmul(T, rest_h.reshape(-1, 4, 1)).reshape(-1, 4)[:, :3]             # :113-115


def pose_from_pca(params, pose_pca, rot):
    """set_params' PCA branch (mano_np.py:66-72): 16x3 pose from N coefficients.

    pose = c(1xN) @ basis[:N] + mean, reshaped (15,3), with `rot` (1,3)
    prepended as the root rotation.  Batched: pose_pca (B,N), rot (B,3).
    """
    c = np.atleast_2d(np.asarray(pose_pca, dtype=np.float64))
    n = c.shape[1]
    basis = np.asarray(params["pose_pca_basis"], dtype=np.float64)
    mean = np.asarray(params["pose_pca_mean"], dtype=np.float64)
    fingers = (c @ basis[:n] + mean).reshape(c.shape[0], -1, 3)
    rot = np.asarray(rot, dtype=np.float64).reshape(c.shape[0], 1, 3)
    return np.concatenate([rot, fingers], axis=1)


class StatefulOracle:
    """Restates MANOModel's stateful set_params/update protocol (mano_np.py:35-77).

    Holds pose (16,3), shape (10), rot (1,3) exactly as the reference does,
    including its quirks: `global_rot` is honoured only on the PCA branch and
    persists in `rot` across calls (:70-72); `pose_pca_mean` is added only on
    that branch (:67); `pose_abs` is taken verbatim (:64-65).
    """

    def __init__(self, params):
        self.params = params
        self.pose = np.zeros((16, 3))
        self.shape = np.zeros(10)
        self.rot = np.zeros((1, 3))
        self.update()

    def set_params(self, pose_abs=None, pose_pca=None, shape=None, global_rot=None):
        if pose_abs is not None:
            self.pose = np.asarray(pose_abs, dtype=np.float64)
        if pose_pca is not None:
            if global_rot is not None:
                self.rot = np.reshape(np.asarray(global_rot, dtype=np.float64), (1, 3))
            self.pose = pose_from_pca(self.params, pose_pca, self.rot)[0]
        if shape is not None:
            self.shape = np.asarray(shape, dtype=np.float64)
        self.update()
        return self.verts.copy()

    def update(self):
        out = forward(self.params, self.shape[None], np.reshape(self.pose, (1, -1, 3)))
        self.verts = out["verts"][0]
        self.J = out["rest_joints"][0]
        self.R = out["rot"][0]
        self.rest_verts = out["rest_verts"][0]
        self.joints = out["joints"][0]
