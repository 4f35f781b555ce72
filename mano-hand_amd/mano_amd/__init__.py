"""mano_amd -- MI355X-native (gfx950) MANO forward pass.

Drop-in for reyuwei/MANO-Hand's `mano_np.MANOModel`:

    from mano_amd import MANOModel          # instead of: from mano_np import MANOModel
    model = MANOModel('dump_mano_left.pkl')
    verts = model.set_params(pose_pca=c, shape=beta, global_rot=[1, 0, 0])

Batched device API: `ManoHip(params).forward(betas, pose, trans)`; one host
thread over several GPUs: `ManoMultiDevice(params, devices).forward(...)`.
"""
from .model_io import (MANO_PARENTS, MODEL_KEYS, dump_model, dump_scans, load_dump,  # noqa: F401
                       load_official, params_digest, save_dump, scans_to_pose, synthetic_params)


def __getattr__(name):
    # torch-backed classes load lazily so that model I/O works without torch/HIP.
    if name in ("MANOModel", "ManoHip", "write_obj"):
        from . import model
        return getattr(model, name)
    if name in ("ManoMultiDevice", "DeviceComms"):
        from . import multi_device
        return getattr(multi_device, name)
    raise AttributeError(name)


__all__ = ["MANOModel", "ManoHip", "ManoMultiDevice", "DeviceComms", "write_obj", "load_dump", "save_dump", "synthetic_params",
           "load_official", "dump_model", "dump_scans", "scans_to_pose",
           "params_digest", "MANO_PARENTS", "MODEL_KEYS"]
