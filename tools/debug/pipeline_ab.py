"""Debug: the C2 step (articulate + blend_skin16) sequential on one stream vs
pipelined over two streams (articulate of batch i + 1 on a side stream, into
the other of two workspaces, while blend_skin16 of batch i runs).

    python tools/debug/pipeline_ab.py [--steps 200] [--rounds 3]

Prints one JSON line: ms per step of each form per round (wall clock over
`steps` steps between device syncs, after a 1-s ramp), and whether the
pipelined outputs equal the sequential ones bit for bit."""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "mano-hand_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--hands", type=int, default=65536)
    a = ap.parse_args()
    import torch
    from mano_amd import ManoHip, _abi, synthetic_params
    B = a.hands
    m = ManoHip(synthetic_params(0), device=0)
    dev = m.device
    lib = _abi.lib()
    inp = m.synthetic_inputs(1001, 0, B)
    need = int(lib.mano_forward_workspace_bytes(m._h, B))
    ws = [torch.empty(need + 512, dtype=torch.uint8, device=dev) for _ in range(2)]
    wsp = [ctypes.c_void_p((w.data_ptr() + 255) & ~255) for w in ws]
    wsb = ctypes.c_size_t(need + 256)
    verts = [torch.empty((B, 778, 3), device=dev) for _ in range(2)]
    joints = [torch.empty((B, 16, 3), device=dev) for _ in range(2)]
    sA = torch.cuda.Stream(device=dev)
    sB = torch.cuda.Stream(device=dev)
    hA, hB = ctypes.c_void_p(sA.cuda_stream), ctypes.c_void_p(sB.cuda_stream)
    pb, pp = ctypes.c_void_p(inp["betas"].data_ptr()), ctypes.c_void_p(inp["pose"].data_ptr())

    def art(k, h):
        _abi.check(lib.mano_stage_articulate(m._h, B, pb, 10, pp, None, ctypes.c_void_p(joints[k].data_ptr()),
                                             None, None, wsp[k], wsb, h))

    def blend(k, h):
        _abi.check(lib.mano_stage_blend_skin(m._h, B, None, None, ctypes.c_void_p(verts[k].data_ptr()),
                                             wsp[k], wsb, h))

    def run_seq(steps):
        for _ in range(steps):
            art(0, hA)
            blend(0, hA)

    ev_art = [torch.cuda.Event() for _ in range(2)]
    ev_blend = [torch.cuda.Event() for _ in range(2)]
    state = {"primed": False, "i": 0}

    def run_pipe(steps, art_first=False):
        # articulate(i) -> W[i%2] on sB; blend(i) reads W[i%2] on sA.
        if not state["primed"]:
            art(0, hB)
            ev_art[0].record(sB)
            ev_blend[1].record(sA)
            state["primed"] = True
        for _ in range(steps):
            i = state["i"]
            k, k1 = i % 2, (i + 1) % 2

            def issue_art():
                sB.wait_event(ev_blend[k1])      # blend(i - 1) has read W[k1]
                art(k1, hB)
                ev_art[k1].record(sB)

            if art_first:
                issue_art()
            sA.wait_event(ev_art[k])
            blend(k, hA)
            ev_blend[k].record(sA)
            if not art_first:
                issue_art()
            state["i"] = i + 1

    def timed(fn, steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(steps)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        run_seq(20)
        torch.cuda.synchronize()
    res = {"hands": B, "steps": a.steps, "seq": [], "pipe": [], "pipe_art_first": []}
    for _ in range(a.rounds):
        res["seq"].append(timed(run_seq, a.steps))
        res["pipe"].append(timed(run_pipe, a.steps))
        res["pipe_art_first"].append(timed(lambda s: run_pipe(s, True), a.steps))
    torch.cuda.synchronize()
    run_seq(1)
    torch.cuda.synchronize()
    ref_v, ref_j = verts[0].clone(), joints[0].clone()
    run_pipe(3)
    torch.cuda.synchronize()
    k_last = (state["i"] - 1) % 2
    res["pipe_bit_exact"] = bool(torch.equal(verts[k_last], ref_v) and torch.equal(joints[k_last], ref_j))
    for key in ("seq", "pipe", "pipe_art_first"):
        res[key + "_min"] = min(res[key])
    print(json.dumps(res), flush=True)
    m.close()


if __name__ == "__main__":
    main()
