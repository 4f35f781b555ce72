"""Debug: where does fused f16x3 LBS differ from standalone skin_h3?"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mano-hand_amd"), REPO]
import numpy as np, torch
from mano_amd import ManoHip, synthetic_params
params = synthetic_params(0)
m = ManoHip(params, device=0, precision="f16x3")
dev = torch.device("cuda", 0)
for B, with_trans in ((1, False), (1, True), (33, True), (33, False), (200, True), (4096, True)):
    rng = np.random.default_rng(100 + B)
    f = lambda a: torch.tensor(a, dtype=torch.float32, device=dev)
    betas = f(rng.normal(0, 1, (B, 10))); pose = f(rng.normal(0, 0.6, (B, 16, 3)))
    trans = f(rng.uniform(-1, 1, (B, 3))) if with_trans else None
    fused = m.forward(betas, pose, trans, rest_verts=True)
    v = torch.empty((B, 778, 3), device=dev)
    m.stage_articulate(betas, pose, trans)
    m.stage_skin(B, v, rest_verts=fused["rest_verts"], trans=trans)
    torch.cuda.synchronize()
    d = (fused["verts"] - v).abs()
    bad = (d > 0).nonzero()
    print(B, with_trans, "max diff", d.max().item(), "n diff", bad.shape[0], "of", d.numel())
    if bad.shape[0]:
        print("  first:", bad[:8].tolist(), "group hist", torch.bincount(bad[:, 1] // 16).tolist()[:50])
        print("  hand hist", torch.bincount(bad[:, 0]).tolist()[:64])
        print("  coord hist", torch.bincount(bad[:, 2]).tolist())
    from oracle import mano_oracle
    ref = mano_oracle.forward(params, betas.double().cpu().numpy(), pose.double().cpu().numpy(),
                              None if trans is None else trans.double().cpu().numpy())
    ef = np.abs(fused["verts"].double().cpu().numpy() - ref["verts"]).max()
    es = np.abs(v.double().cpu().numpy() - ref["verts"]).max()
    ep = np.abs(fused["rest_verts"].double().cpu().numpy() - ref["rest_verts"]).max()
    print("  err fused", ef, "err skin", es, "err vposed", ep)
