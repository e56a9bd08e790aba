"""The N > 1 decomposition of bench.py, on the CPU with torch.distributed gloo (world size 2).

bench.py splits one frame over ranks: CDEF filter-block rows (the [2][nFB][64] mse table and skip flags are
all-reduce-summed), MD superblock ranges (no exchange), and loop-restoration unit rows (each rank searches
its units; the per-unit records are all-gathered and every rank runs the host RD finish).  These tests run
the same helpers (svtgpu.band / lr_unit_rows / gather_lr_records / lr_finish_plane) in two gloo processes,
with the CPU oracle standing in for the device search, and check the merged result equals the one-rank
result.  The library is loaded but no device call is made (svtgpu_lr_finish_plane is host-only)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle
import svtgpu
import synth


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _lr_ctrls():
    return oracle.lr_controls(1, 1, rdmult=7000, switchable=(300, 700, 900), wiener=(250, 800), sgrproj=(250, 900))


def _lr_case():
    w, h, bd, usize = 320, 200, 10, 64
    src, rec = synth.frame_pair(w, h, bd, seed=0x5EED0900)
    unit_size = [usize, usize >> 1, usize >> 1]
    ft, units, recs = oracle.lr_search_frame(rec, src, bd, unit_size, _lr_ctrls())
    grid = [(oracle.lr_units(unit_size[p], rec[p].shape[1]), oracle.lr_units(unit_size[p], rec[p].shape[0]))
            for p in range(3)]
    return ft, units, recs, grid


def _worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ft, units, recs, grid = _lr_case()
        ctrls = _lr_ctrls()
        # LR: this rank keeps only its unit-row band of the records (what svtgpu_lr_search_units writes)
        rb, re_ = svtgpu.lr_unit_rows(grid, world, rank)
        mine = []
        for p, (hu, vu) in enumerate(grid):
            r = np.zeros(hu * vu, svtgpu.LR_UNIT_SEARCH_DTYPE)
            r[rb[p] * hu:re_[p] * hu] = recs[p][rb[p] * hu:re_[p] * hu]
            mine.append(r)
        merged = svtgpu.gather_lr_records(mine, grid, world, rank)
        lr_ok = all(np.array_equal(merged[p], recs[p]) for p in range(3))
        fin = [svtgpu.lr_finish_plane(ctrls, p, merged[p]) for p in range(3)]
        finish_ok = all(fin[p][0] == ft[p] and np.array_equal(fin[p][1], units[p]) for p in range(3))
        # CDEF: zero-padded band tables all-reduce-summed = the full table; the pick on it is unchanged
        import torch
        w, h, bd, q = 256, 192, 10, 128
        src, rec = synth.frame_pair(w, h, bd, seed=0x5EED0901)
        cc = oracle.controls(1)
        mse, skip, _, _ = oracle.cdef_search_frame(rec, src, bd, cc, q)
        nhfb, nvfb = (w // 4 + 15) // 16, (h // 4 + 15) // 16
        b, e = svtgpu.band(nvfb, world, rank)
        part = torch.zeros((2, nvfb * nhfb, 64), dtype=torch.int64)
        part[:, b * nhfb:e * nhfb] = torch.from_numpy(np.ascontiguousarray(mse).reshape(2, -1, 64)[:, b * nhfb:e * nhfb])
        sk = torch.zeros(nvfb * nhfb, dtype=torch.uint8)
        sk[b * nhfb:e * nhfb] = torch.from_numpy(np.ascontiguousarray(skip).reshape(-1)[b * nhfb:e * nhfb])
        dist.all_reduce(part)
        dist.all_reduce(sk)
        cdef_ok = np.array_equal(part.numpy().reshape(np.shape(mse)), mse) and \
            np.array_equal(sk.numpy().reshape(np.shape(skip)), skip)
        lam = 60000
        p1 = oracle.cdef_pick(w, h, part.numpy().reshape(np.shape(mse)), sk.numpy().reshape(np.shape(skip)), cc, q, lam)
        p0 = oracle.cdef_pick(w, h, mse, skip, cc, q, lam)
        pick_ok = p1[0].as_tuple() == p0[0].as_tuple() and np.array_equal(p1[1], p0[1])
        # MD: SB ranges cover the frame exactly once
        nsb = 37
        cover = torch.zeros(nsb, dtype=torch.int32)
        b, e = svtgpu.band(nsb, world, rank)
        cover[b:e] += 1
        dist.all_reduce(cover)
        md_ok = bool((cover == 1).all())
        out.put((rank, lr_ok, finish_ok, cdef_ok, pick_ok, md_ok))
    finally:
        dist.destroy_process_group()


def test_bands_partition():
    for count in (1, 2, 7, 8, 9, 135):
        for n in (1, 2, 3, 8):
            bands = [svtgpu.band(count, n, r) for r in range(n)]
            assert bands[0][0] == 0 and bands[-1][1] == count
            assert all(bands[r][1] == bands[r + 1][0] for r in range(n - 1))


def test_two_rank_decomposition():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, lr_ok, finish_ok, cdef_ok, pick_ok, md_ok in res:
        assert lr_ok, "rank %d: gathered LR records differ" % rank
        assert finish_ok, "rank %d: LR finish on gathered records differs from the one-rank finish" % rank
        assert cdef_ok and pick_ok, "rank %d: CDEF band all-reduce" % rank
        assert md_ok, "rank %d: MD SB bands" % rank
