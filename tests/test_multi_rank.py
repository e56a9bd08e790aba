"""A picture tiled over ranks (bench.py --gpus N > 1), host side, on the CPU with torch.distributed gloo.

Each rank takes a tile of svtgpu_tile_plan (2 x 4 for 8 GPUs); the frame-level calls exchange, through the C ABI's
communicator (svtgpu.Comm.host: the library's host transport, here over gloo), the DLF trial SSEs, the
zero-padded CDEF search tables and the zero-padded LR search records, and every rank then takes the same
frame-level decisions.  Here the CPU oracle stands in for the device search (no device call is made: the host
transport on host buffers and svtgpu_lr_finish_plane touch no GPU): each rank keeps only its tile's part of the
oracle's outputs, sums them over the ranks through the library, and the decisions on the sums must equal the
one-rank decisions.  The device path of the same split runs in tests/test_tiled_gpu.py."""
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


@pytest.mark.parametrize("w,h,us", [(3840, 2160, 256), (1920, 1080, 256), (640, 360, 64), (328, 200, 64)])
@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_tile_plan_partitions(w, h, us, n):
    """Tiles, filter blocks, LR units and LR outputs of the ranks cover the frame exactly once; every rank's CDEF
    output covers its LR output plus 3 samples, its DLF output covers its tile and CDEF output plus 2."""
    gx, gy = svtgpu.tile_grid(n)
    unit = [us, us >> 1, us >> 1]
    try:
        plans = [svtgpu.tile_plan(w, h, unit, gx, gy, r).rects() for r in range(n)]
    except svtgpu.SvtGpuError:
        assert (w + us // 2) // us < gx or (h + us // 2) // us < gy  # fewer units than ranks
        return
    cover = np.zeros((h, w), np.int32)
    fb = np.zeros(((h + 63) // 64, (w + 63) // 64), np.int32)
    for pl in plans:
        t, f = pl["tile"], pl["fb_rect"]
        cover[t[1]:t[3], t[0]:t[2]] += 1
        fb[f[1]:f[3], f[0]:f[2]] += 1
    assert (cover == 1).all() and (fb == 1).all()
    for p in range(3):
        pw, ph = (w, h) if p == 0 else (w // 2, h // 2)
        hu, vu = oracle.lr_units(unit[p], pw), oracle.lr_units(unit[p], ph)
        cu = np.zeros((vu, hu), np.int32)
        co = np.zeros((ph, pw), np.int32)
        for pl in plans:
            u, o = pl["lr_units"][p], pl["lr_out"][p]
            cu[u[1]:u[3], u[0]:u[2]] += 1
            co[o[1]:o[3], o[0]:o[2]] += 1
        assert (cu == 1).all() and (co == 1).all(), p
    for pl in plans:
        o, c, d, t = pl["lr_out"][0], pl["cdef_out"], pl["dlf_out"], pl["tile"]
        assert c[0] <= max(0, o[0] - 3) and c[1] <= max(0, o[1] - 3) and c[2] >= min(w, o[2] + 3) and c[3] >= min(h, o[3] + 3)
        for q in (c, t):
            assert d[0] <= max(0, q[0] - 2) and d[1] <= max(0, q[1] - 2) and d[2] >= min(w, q[2] + 2) and \
                d[3] >= min(h, q[3] + 2)


def _worker(rank, world, port, out):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def allreduce(words):
            dist.all_reduce(torch.from_numpy(words.view(np.int64)))

        comm = svtgpu.Comm.host(world, rank, allreduce)
        gx, gy = svtgpu.tile_grid(world)
        # LR: the records of this rank's units, zero elsewhere, summed over the ranks = every unit's record
        w, h, bd, usize = 320, 200, 10, 64
        src, rec = synth.frame_pair(w, h, bd, seed=0x5EED0900)
        unit = [usize, usize >> 1, usize >> 1]
        ctrls = _lr_ctrls()
        ft, units, recs = oracle.lr_search_frame(rec, src, bd, unit, ctrls)
        plan = svtgpu.tile_plan(w, h, unit, gx, gy, rank).rects()
        merged = []
        for p in range(3):
            hu = oracle.lr_units(unit[p], rec[p].shape[1])
            mine = np.zeros_like(recs[p])
            u = plan["lr_units"][p]
            for r in range(u[1], u[3]):
                mine[r * hu + u[0]:r * hu + u[2]] = recs[p][r * hu + u[0]:r * hu + u[2]]
            words = np.ascontiguousarray(mine).view(np.uint64).copy()
            merged.append(comm.allreduce(words).view(svtgpu.LR_UNIT_SEARCH_DTYPE))
        lr_ok = all(merged[p].tobytes() == np.ascontiguousarray(recs[p]).tobytes() for p in range(3))
        fin = [svtgpu.lr_finish_plane(ctrls, p, merged[p]) for p in range(3)]
        finish_ok = all(fin[p][0] == ft[p] and np.array_equal(fin[p][1], units[p]) for p in range(3))
        # CDEF: the tables of this rank's filter blocks, zero elsewhere, summed = the full tables; the pick agrees
        w, h, bd, q = 512, 256, 10, 128
        src, rec = synth.frame_pair(w, h, bd, seed=0x5EED0901)
        cc = oracle.controls(1)
        mse, skip, dd, vv = oracle.cdef_search_frame(rec, src, bd, cc, q)
        nhfb, nvfb = (w // 4 + 15) // 16, (h // 4 + 15) // 16
        f = svtgpu.tile_plan(w, h, [64, 32, 32], gx, gy, rank).rects()["fb_rect"]
        sel = np.zeros((nvfb, nhfb), bool)
        sel[f[1]:f[3], f[0]:f[2]] = True
        sel = sel.reshape(-1)
        m = np.where(sel[None, :, None], np.asarray(mse).reshape(2, -1, 64), 0).astype(np.uint64)
        s = np.zeros(((nvfb * nhfb + 7) // 8) * 8, np.uint8)
        s[:nvfb * nhfb] = np.where(sel, np.asarray(skip).reshape(-1), 0)
        d = np.where(sel[:, None], np.asarray(dd).reshape(-1, 64), 0).astype(np.uint8)
        v = np.where(sel[:, None], np.asarray(vv).reshape(-1, 64), 0).astype(np.int32)
        m = comm.allreduce(m.reshape(-1)).reshape(np.shape(mse))
        s = comm.allreduce(s.view(np.uint64)).view(np.uint8)[:nvfb * nhfb].reshape(np.shape(skip))
        d = comm.allreduce(d.reshape(-1).view(np.uint64)).view(np.uint8).reshape(np.shape(dd))
        v = comm.allreduce(v.reshape(-1).view(np.uint64)).view(np.int32).reshape(np.shape(vv))
        cdef_ok = np.array_equal(m, mse) and np.array_equal(s, skip) and np.array_equal(d, dd) and np.array_equal(v, vv)
        lam = 60000
        p1 = oracle.cdef_pick(w, h, m, s, cc, q, lam)
        p0 = oracle.cdef_pick(w, h, mse, skip, cc, q, lam)
        pick_ok = p1[0].as_tuple() == p0[0].as_tuple() and np.array_equal(p1[1], p0[1])
        # DLF: the per-tile SSEs of a trial summed over the ranks = the frame SSE (picture_sse_calculations)
        t = svtgpu.tile_plan(w, h, [64, 32, 32], gx, gy, rank).rects()["tile"]
        a, b = src[0].astype(np.int64), rec[0].astype(np.int64)
        sse = np.array([((a - b)[t[1]:t[3], t[0]:t[2]] ** 2).sum()], np.uint64)
        dlf_ok = int(comm.allreduce(sse)[0]) == int(((a - b) ** 2).sum())
        # MD: superblock ranges cover the frame exactly once
        nsb = 37
        cover = torch.zeros(nsb, dtype=torch.int32)
        b0, e0 = svtgpu.band(nsb, world, rank)
        cover[b0:e0] += 1
        dist.all_reduce(cover)
        md_ok = bool((cover == 1).all())
        comm.close()
        out.put((rank, lr_ok, finish_ok, cdef_ok, pick_ok, dlf_ok, md_ok))
    finally:
        dist.destroy_process_group()


def test_bands_partition():
    for count in (1, 2, 7, 8, 9, 135):
        for n in (1, 2, 3, 8):
            bands = [svtgpu.band(count, n, r) for r in range(n)]
            assert bands[0][0] == 0 and bands[-1][1] == count
            assert all(bands[r][1] == bands[r + 1][0] for r in range(n - 1))


@pytest.mark.parametrize("world", [2, 4])
def test_tiled_exchanges(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, lr_ok, finish_ok, cdef_ok, pick_ok, dlf_ok, md_ok in res:
        assert lr_ok, "rank %d: gathered LR records differ" % rank
        assert finish_ok, "rank %d: LR finish on the gathered records differs from the one-rank finish" % rank
        assert cdef_ok and pick_ok, "rank %d: CDEF table exchange" % rank
        assert dlf_ok, "rank %d: DLF SSE sum" % rank
        assert md_ok, "rank %d: MD SB bands" % rank


def _skip_worker(rank, world, port, out):
    """Rank 1 skips an exchange (and stays alive past the deadline); rank 0's exchange must end with the named error
    within the deadline instead of hanging."""
    import datetime
    import time
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    grp = dist.new_group(backend="gloo")  # the data exchanges' own group; the default group stays for control
    try:
        def allreduce(words, timeout_ms):  # the host transport bounds its wait by the communicator's deadline
            w = dist.all_reduce(torch.from_numpy(words.view(np.int64)), group=grp, async_op=True)
            w.wait(timeout=datetime.timedelta(milliseconds=timeout_ms))

        comm = svtgpu.Comm.host(world, rank, allreduce)
        comm.set_timeout(1500)
        comm.set_slot(3)
        assert comm.timeout_ms == 1500
        a = np.arange(8, dtype=np.uint64)
        ok = np.array_equal(comm.allreduce(a.copy()), a * world)  # one matched exchange first
        if rank == 0:
            t0 = time.monotonic()
            try:
                comm.allreduce(a.copy())
                msg = "no error"
            except svtgpu.SvtGpuError as e:
                msg = str(e)
            dt = time.monotonic() - t0
            try:  # the communicator fails every later call
                comm.allreduce(a.copy())
                later = "no error"
            except svtgpu.SvtGpuError as e:
                later = str(e)
            out.put((ok, msg, dt, comm.failed, later))
        else:
            time.sleep(4.0)  # skipped the exchange; alive past rank 0's deadline
        dist.barrier()
        comm.close()
    finally:
        dist.destroy_process_group()


def test_host_transport_skipped_exchange_times_out():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_skip_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok, msg, dt, failed, later = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert ok
    assert "exchange failed" in msg and "caller's words" in msg and "frame slot 3" in msg and "exchange #2" in msg, msg
    assert dt < 1.5 + 2.0, dt  # the deadline, not a hang
    assert failed and "exchange #2" in later
    assert all(p.exitcode == 0 for p in procs)
