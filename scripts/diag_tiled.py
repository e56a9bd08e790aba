"""Diagnostics of the tiled pipeline on one GPU: per rank, the CDEF tables before and after the pick's exchange.
usage: python scripts/diag_tiled.py <case> <world> [<world> ...]"""
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "svt-av1_pro-anchor-v2.1.0-_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)


def worker(rank, world, port, case):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.init()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import svtgpu
    import pipeline_cases as pc
    import pipeline_run as prun
    calls = []

    def allreduce(words):
        calls.append(words.size)
        dist.all_reduce(torch.from_numpy(words.view(np.int64)))

    comm = svtgpu.Comm.host(world, rank, allreduce)
    ctx = svtgpu.Context(0)
    c = pc.CASES[case]
    g = pc.load(case)
    src, rec, mi = pc.inputs(case)
    bd, w, h = c["bd"], c["w"], c["h"]
    us = [c["us"][0], c["us"][1], c["us"][1]]
    gx, gy = svtgpu.tile_grid(world)
    plan = svtgpu.tile_plan(w, h, us, gx, gy, rank, sb=c["sb"]).rects()
    S, R, D = (svtgpu.Frame(ctx, w, h, bd) for _ in range(3))
    S.upload(src)
    R.upload(rec)
    dl = svtgpu.DlfState(ctx, w, h)
    dl.set_mode_info(mi)
    dl.set_tile(plan["tile"], plan["dlf_out"], comm)
    lfp = prun.gpu_dlf_pick(dl, R, S, c)
    n_dlf = len(calls)
    dl.filter_to(R, D, lfp)
    st = svtgpu.CdefState(ctx, w, h)
    st.set_block_mask(pc.cdef_mask(mi))
    st.set_tile(plan["fb_rect"], plan["cdef_out"], comm)
    ctrls = svtgpu.cdef_controls(c["cdef_level"])
    ctrls.pred_y_f, ctrls.pred_uv_f = c["pred"]
    st.search(D, S, ctrls, c["q"])
    before = st.read()
    prm, fbs = st.pick(ctrls, c["q"], int(g["cdef_lambda"][0]))
    after = st.read()
    dist.barrier()
    for r in range(world):
        if r == rank:
            print("rank %d fb_rect %s lf %s dlf calls %d cdef calls %s skip before %s after %s" % (
                rank, plan["fb_rect"], lfp.levels(), n_dlf, calls[n_dlf:], before[1].tolist(), after[1].tolist()),
                flush=True)
        dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    case = sys.argv[1]
    for world in map(int, sys.argv[2:]):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        print("== %s world %d" % (case, world), flush=True)
        mp.spawn(worker, args=(world, port, case), nprocs=world, join=True)
