"""A picture tiled over ranks (BASELINE.json config 4) on the device path, bit-exact.

World sizes 2, 4 and 8 (svtgpu.tile_grid: 1 x 2, 2 x 2 and the 2 x 4 grid of the 8-GPU run): that many processes
(torch.distributed gloo) share the one GPU of the test box; each runs the whole pipeline of a case on its tile through
the library's frame-level calls with a host-transport communicator (svtgpu.Comm.host over gloo: RCCL needs one rank
per device), so every exchange goes through the C ABI: the DLF trial SSEs before each bisection step, the CDEF search
tables before the pick, the LR search records before the finish.  The ranks' crops (DLF output over each tile, CDEF
and LR outputs over each rank's LR units) are assembled on rank 0 and compared with the reference's outputs of the
case, digests included for the 4K 10-bit bench configuration (tests/golden/pipe_c3_4k10.npz) — the same check as the
one-rank run.  The cases are chosen so that tile columns cross the frame at 64-sample edges that are not multiples of
128 (mini10b, mini10e, mini8c), at 128 in a SB128 picture (sb128_10) and at 1792 / 1024 in the 4K / 1080p bench
pictures; the rows at 64-sample steps (mini8c at 2 x 4).

The RCCL transport runs too: a one-rank RCCL communicator takes the tiled path (svtgpu_comm_tiled) with every
exchange an ncclAllReduce — host buffers (DLF trial SSEs, LR records) and device buffers (CDEF tables) — on the whole
pipeline of the 4K bench case; the 8-GPU bench runs exactly these calls."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import pipeline_cases as pc
import pipeline_run as prun

WORLD_CASES = {
    2: ["mini10", "sb128_10", "c3_4k10"],
    4: ["mini10b", "mini10e", "sb128_10", "sbdlf8_key", "c3_4k10"],
    8: ["mini8c", "c1_1080p8", "c3_4k10"],
}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, cases, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if torch.cuda.is_available():
        torch.cuda.init()  # torch's HIP runtime first (conftest.py)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import svtgpu

        def allreduce(words):  # uint64 sums as int64 (two's complement: the same bits)
            t = torch.from_numpy(words.view(np.int64))
            dist.all_reduce(t)

        comm = svtgpu.Comm.host(world, rank, allreduce)
        ctx = svtgpu.Context(0)
        for case in cases:
            part = prun.run_gpu_tiled(case, rank, world, comm, ctx)
            parts = [None] * world
            dist.all_gather_object(parts, part)
            if rank == 0:
                try:
                    prun.check(case, prun.assemble_tiled(case, parts), "tiled x%d" % world)
                    q.put((case, "ok"))
                except AssertionError as e:
                    q.put((case, "FAIL: %s" % str(e)[:2000]))
            print("rank %d/%d: %s done" % (rank, world, case), flush=True)
        comm.close()
    except BaseException as e:  # reported to the parent
        q.put(("rank %d" % rank, "ERROR: %r" % e))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_ranks_one_gpu_bit_exact(world):
    cases = WORLD_CASES[world]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    try:
        while len(res) < len(cases):
            item = q.get(timeout=300)
            res.append(item)
            assert not item[1].startswith("ERROR"), item
    finally:
        for p in procs:
            p.join(timeout=120)
            if p.exitcode is None:
                p.kill()
    for case, status in res:
        assert status == "ok", (case, status)
    assert all(p.exitcode == 0 for p in procs)


def test_world_cases_cross_tile_columns():
    """CPU check of the case choice: every listed world really cuts the case into its grid, and the grids include
    column edges off the 128-sample grid."""
    import svtgpu
    off128 = False
    for world, cases in WORLD_CASES.items():
        gx, gy = svtgpu.tile_grid(world)
        for case in cases:
            c = pc.CASES[case]
            us = [c["us"][0], c["us"][1], c["us"][1]]
            plans = [svtgpu.tile_plan(c["w"], c["h"], us, gx, gy, r, sb=c["sb"]).rects() for r in range(world)]
            xs = sorted({p["tile"][0] for p in plans})
            assert len(xs) == gx and len({p["tile"][1] for p in plans}) == gy, (world, case)
            off128 |= any(x % 128 for x in xs)
            if c["sb"] == 128:
                assert all(x % 128 == 0 for x in xs), (world, case, xs)
    assert off128


@pytest.fixture(scope="module")
def rccl1():
    import svtgpu
    ctx = svtgpu.Context(0)
    comm = svtgpu.Comm.rccl(ctx, 1, 0, svtgpu.Comm.unique_id())
    yield ctx, comm
    comm.close()


@pytest.mark.gpu
def test_rccl_one_rank_allreduce(rccl1):
    """svtgpu_comm_create (RCCL) with one rank: ncclAllReduce runs on host buffers (staged through the comm's device
    buffer) and on device buffers (on the caller's stream); one rank's sum is the identity."""
    import torch
    ctx, comm = rccl1
    assert comm.nranks == 1
    a = np.arange(17, dtype=np.uint64) * np.uint64(0x100000001)
    assert np.array_equal(comm.allreduce(a.copy()), a)
    big = np.random.default_rng(3).integers(0, 1 << 62, size=300001, dtype=np.uint64)
    assert np.array_equal(comm.allreduce(big.copy()), big)
    t = torch.from_numpy(big.view(np.int64)).cuda()
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    comm.allreduce_device(t.data_ptr(), t.numel(), stream=s.cuda_stream)
    s.synchronize()
    assert np.array_equal(t.cpu().numpy().view(np.uint64), big)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["sb128_10", "c3_4k10"])
def test_rccl_one_rank_pipeline(rccl1, case):
    """The whole tiled pipeline over a one-rank RCCL communicator (every exchange an ncclAllReduce) equals the
    reference's outputs of the case."""
    ctx, comm = rccl1
    part = prun.run_gpu_tiled(case, 0, 1, comm, ctx)
    prun.check(case, prun.assemble_tiled(case, [part]), "rccl x1")


@pytest.mark.gpu
def test_cdef_bound_tables_exact_size_tiled_pick_twice(rccl1):
    """1080p (510 filter blocks, not a multiple of 8): a bound skip table of exactly nfb bytes is never written past
    its end by the tiled search / pick (guard bytes after it), and a second pick on the same search (tiled: the tables
    are summed once) gives the same result as the first and as an untiled state."""
    import torch
    import svtgpu
    import synth
    ctx, comm = rccl1
    w, h, bd, q, lam = 1920, 1080, 8, 160, 60000
    src, rec = synth.frame_pair(w, h, bd, seed=0x5EED0099)
    R, S = svtgpu.Frame(ctx, w, h, bd), svtgpu.Frame(ctx, w, h, bd)
    R.upload(rec)
    S.upload(src)
    ctrls = svtgpu.cdef_controls(1)
    ref = svtgpu.CdefState(ctx, w, h)
    ref.search(R, S, ctrls, q)
    prm0, fbs0 = ref.pick(ctrls, q, lam)
    st = svtgpu.CdefState(ctx, w, h)
    nfb = st.nfb
    assert nfb % 8
    mse = torch.zeros((2, nfb, 64), dtype=torch.int64, device="cuda")
    guard = torch.full((nfb + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    st.bind_tables(mse.data_ptr(), guard.data_ptr())
    st.set_tile(None, None, comm)
    st.search(R, S, ctrls, q)
    prm1, fbs1 = st.pick(ctrls, q, lam)
    prm2, fbs2 = st.pick(ctrls, q, lam)
    torch.cuda.synchronize()
    g = guard.cpu().numpy()
    assert (g[nfb:] == 0xA5).all(), "skip table written past nfb bytes"
    assert prm1.as_tuple() == prm0.as_tuple() == prm2.as_tuple()
    assert np.array_equal(fbs1, fbs0) and np.array_equal(fbs2, fbs0)
    for x in (R, S, ref, st):
        x.close()


@pytest.mark.gpu
def test_rccl_exchange_deadline_aborts():
    """The RCCL branch of the exchange deadline (one rank): a collective held behind a stalled stream is still
    outstanding when the deadline expires, so the bounded wait names it, aborts the communicator (ncclCommAbort) and
    fails every later call; the stream itself drains (the stall ends on its own clock).  A deadline that expires with
    no exchange enqueued on the stream since its last completed wait is an ordinary wait (no false timeout)."""
    import time
    import torch
    import svtgpu
    ctx = svtgpu.Context(0)
    comm = svtgpu.Comm.rccl(ctx, 1, 0, svtgpu.Comm.unique_id())
    comm.set_timeout(400)
    comm.set_slot(2)
    s = torch.cuda.Stream()
    t = torch.arange(64, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    # no exchange outstanding (the last one completed at a wait): a stall longer than the deadline is waited for,
    # not reported
    comm.allreduce_device(t.data_ptr(), t.numel(), stream=s.cuda_stream)
    comm.sync(s.cuda_stream)
    ctx.debug_stall(900, s.cuda_stream)
    time.sleep(0.05)
    comm.sync(s.cuda_stream)
    assert not comm.failed
    # the collective queued behind the stall: outstanding at the deadline
    ctx.debug_stall(2500, s.cuda_stream)
    comm.allreduce_device(t.data_ptr(), t.numel(), stream=s.cuda_stream)
    t0 = time.monotonic()
    with pytest.raises(svtgpu.SvtGpuError) as ei:
        comm.sync(s.cuda_stream)
    dt = time.monotonic() - t0
    msg = str(ei.value)
    assert "exchange timed out" in msg and "caller's words" in msg and "frame slot 2" in msg and "aborted" in msg, msg
    # detected at the deadline; the abort itself may then wait for the stalled (non-RCCL) kernel on the stream -- a
    # hung collective's own kernel ends on ncclCommAbort's abort flag
    import re
    detected = int(re.search(r"detected after (\d+) ms", msg).group(1))
    assert 400 <= detected < 1000, msg
    assert dt < 2.5 + 1.0, dt
    assert comm.failed
    with pytest.raises(svtgpu.SvtGpuError):
        comm.allreduce_device(t.data_ptr(), t.numel(), stream=s.cuda_stream)
    ctx.synchronize(s.cuda_stream)  # the stall drains on its own
    assert torch.equal(t.cpu(), torch.arange(64, dtype=torch.int64))
    comm.close()
    ctx.close()


@pytest.mark.gpu
def test_rccl_comm_init_bounded_peer_never_joins():
    """communicator creation is bounded like the exchanges.  Rank 0 of a two-rank RCCL communicator whose
    rank 1 never joins (it died between the id broadcast and its init) returns SVTGPU_ERR_HIP within the deadline,
    with "communicator init", the frame slot, the rank and the rank count in the message; the partial communicator is
    aborted and the device stays usable (a one-rank communicator afterwards works)."""
    import time
    import torch
    import svtgpu
    ctx = svtgpu.Context(0)
    uid = svtgpu.Comm.unique_id()
    t0 = time.monotonic()
    with pytest.raises(svtgpu.SvtGpuError) as ei:
        svtgpu.Comm.rccl(ctx, 2, 0, uid, timeout_ms=1500, slot=3)
    dt = time.monotonic() - t0
    msg = str(ei.value)
    assert "communicator init" in msg and "frame slot 3" in msg and "rank 0 of 2" in msg, msg
    assert 1.4 <= dt < 1.5 + 8.0, dt  # detected at the deadline (the abort of the bootstrap may take a moment)
    c = svtgpu.Comm.rccl(ctx, 1, 0, svtgpu.Comm.unique_id(), timeout_ms=5000, slot=0)
    t = torch.arange(16, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    c.allreduce_device(t.data_ptr(), t.numel(), stream=torch.cuda.current_stream().cuda_stream)
    c.sync(torch.cuda.current_stream().cuda_stream)
    assert torch.equal(t.cpu(), torch.arange(16, dtype=torch.int64))
    c.close()
    ctx.close()


def _skip_pick_worker(rank, world, port, q):
    import datetime
    import time
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.init()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    grp = dist.new_group(backend="gloo")
    try:
        import svtgpu
        import synth

        def allreduce(words, timeout_ms):
            w = dist.all_reduce(torch.from_numpy(words.view(np.int64)), group=grp, async_op=True)
            w.wait(timeout=datetime.timedelta(milliseconds=timeout_ms))

        comm = svtgpu.Comm.host(world, rank, allreduce)
        comm.set_timeout(2000)
        comm.set_slot(1)
        ctx = svtgpu.Context(0)
        w, h, bd, qi, lam = 640, 384, 10, 128, 60000
        src, rec = synth.frame_pair(w, h, bd, seed=0x5EED0777)
        R, S = svtgpu.Frame(ctx, w, h, bd), svtgpu.Frame(ctx, w, h, bd)
        R.upload(rec)
        S.upload(src)
        plan = svtgpu.tile_plan(w, h, [64, 32, 32], *svtgpu.tile_grid(world), rank).rects()
        st = svtgpu.CdefState(ctx, w, h)
        st.set_tile(plan["fb_rect"], plan["cdef_out"], comm)
        ctrls = svtgpu.cdef_controls(1)
        st.search(R, S, ctrls, qi)
        if rank == 0:
            t0 = time.monotonic()
            try:
                st.pick(ctrls, qi, lam)
                msg = "no error"
            except svtgpu.SvtGpuError as e:
                msg = str(e)
            q.put((msg, time.monotonic() - t0, comm.failed))
        else:
            time.sleep(5.0)  # skips the pick's exchange, alive past rank 0's deadline
        dist.barrier()
        for x in (st, R, S, comm):
            x.close()
    except BaseException as e:
        q.put(("ERROR: %r" % e, 0.0, False))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(180)
def test_skipped_cdef_exchange_times_out_named():
    """Two ranks of a tiled picture on the one GPU (host transport over gloo): rank 1 searches its filter blocks but
    never reaches the pick; rank 0's pick returns the named error ("CDEF search tables", frame slot, exchange number)
    within the communicator's deadline instead of hanging."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_skip_pick_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        msg, dt, failed = q.get(timeout=150)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    assert "exchange failed" in msg and "CDEF search tables" in msg and "frame slot 1" in msg, msg
    assert dt < 2.0 + 3.0, dt
    assert failed


@pytest.mark.gpu
def test_cdef_rebind_tables_between_picks_sums_again():
    """binding other tables (or another tile / comm) between two picks with no search in between must make
    the next pick sum the tables over the ranks again.  A two-rank host communicator in one process whose other rank
    contributes zeros (the transport is the identity and counts its calls): after a rebind the pick exchanges again
    and picks from the new tables, equal to an untiled pick over them."""
    import torch
    import svtgpu
    ctx = svtgpu.Context(0)
    calls = []
    comm = svtgpu.Comm.host(2, 0, lambda words: calls.append(words.size))
    w, h, q, lam = 1024, 512, 128, 60000
    ctrls = svtgpu.cdef_controls(1)
    st, ref = svtgpu.CdefState(ctx, w, h), svtgpu.CdefState(ctx, w, h)
    st.set_tile(None, None, comm)
    rng = np.random.default_rng(77)
    picks = []
    for k in range(2):
        mse = rng.integers(1 << 20, 1 << 30, size=(2, st.nfb, 64), dtype=np.int64).astype(np.uint64)
        skip = (rng.random(st.nfb) < 0.1).astype(np.uint8)
        mse_t = torch.from_numpy(mse.view(np.int64)).cuda()
        skip_t = torch.from_numpy(skip).cuda()
        torch.cuda.synchronize()
        n0 = len(calls)
        st.bind_tables(mse_t.data_ptr(), skip_t.data_ptr())
        prm, fbs = st.pick(ctrls, q, lam)
        assert len(calls) > n0, "pick %d after a rebind did not exchange the tables" % k
        ref.bind_tables(mse_t.data_ptr(), skip_t.data_ptr())
        rprm, rfbs = ref.pick(ctrls, q, lam)
        assert prm.as_tuple() == rprm.as_tuple() and np.array_equal(fbs, rfbs), k
        picks.append(prm.as_tuple())
        n1 = len(calls)
        st.pick(ctrls, q, lam)  # same tables, no rebind: gathered already, no second exchange
        assert len(calls) == n1
        del mse_t, skip_t
    for x in (st, ref, comm, ctx):
        x.close()


# a picture off the 8-sample grid tiled over the ranks (svtgpu_tile_plan_crop): coded size 8-aligned, crop below it
CROP_CASES = {
    2: [(dict(w=336, h=184, bd=10, q=150, us=(64, 32), mi=("random", 31, 0.3), seed=131), (330, 182))],
    4: [(dict(w=1368, h=768, bd=10, q=170, us=(64, 32), mi=("random", 32, 0.3), seed=132), (1366, 766)),
        (dict(w=640, h=368, bd=8, q=90, us=(64, 32), cdef_level=3, mi=("random", 33, 0.4), seed=133), (634, 362))],
}


def _crop_worker(rank, world, port, cases, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if torch.cuda.is_available():
        torch.cuda.init()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pipeline_cases as pcs
        import svtgpu

        def allreduce(words):
            dist.all_reduce(torch.from_numpy(words.view(np.int64)))

        comm = svtgpu.Comm.host(world, rank, allreduce)
        ctx = svtgpu.Context(0)
        for i, (kw, crop) in enumerate(cases):
            c = pcs._case(**kw)
            part = prun.run_crop(c, crop, rank, world, comm, ctx)
            parts = [None] * world
            dist.all_gather_object(parts, part)
            if rank == 0:
                try:
                    prun.compare_crop_parts(prun.run_crop(c, crop, ctx=ctx), parts)
                    q.put((i, "ok"))
                except AssertionError as e:
                    q.put((i, "FAIL: %s" % str(e)[:2000]))
        comm.close()
    except BaseException as e:
        q.put(("rank %d" % rank, "ERROR: %r" % e))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4])
def test_ranks_one_gpu_crop_size(world):
    """A picture whose crop size is off the 8-sample grid (1366 x 766 in a 1368 x 768 coded frame, 330 x 182, 634 x 362),
    tiled over 2 / 4 ranks on one GPU with svtgpu_tile_plan_crop: every rank's decisions (DLF levels, CDEF strengths,
    LR frame types and the summed unit records) and its outputs over its rects equal the single-GPU run, whose crop
    handling the reference fixtures pin (DLF: gen_golden_dlf.c cases 8-10; LR: the crop-size search / frame goldens)."""
    cases = CROP_CASES[world]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_crop_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    try:
        while len(res) < len(cases):
            item = q.get(timeout=300)
            res.append(item)
            assert not str(item[1]).startswith("ERROR"), item
    finally:
        for p in procs:
            p.join(timeout=120)
            if p.exitcode is None:
                p.kill()
    for case, status in res:
        assert status == "ok", (case, status)
    assert all(p.exitcode == 0 for p in procs)


def test_tile_plan_crop_units_cover_the_crop():
    """CPU check of svtgpu_tile_plan_crop: the ranks' LR units partition each plane's unit grid of the crop size, their
    sample rects reach the crop edge (not the coded edge), the tiles reach the coded edge; invalid crops are refused."""
    import svtgpu
    for (w, h), (cw, ch) in (((1368, 768), (1366, 766)), ((336, 184), (330, 182))):
        us = [64, 32, 32]
        for world in (2, 4):
            gx, gy = svtgpu.tile_grid(world)
            plans = [svtgpu.tile_plan(w, h, us, gx, gy, r, crop=(cw, ch)).rects() for r in range(world)]
            assert max(p["tile"][2] for p in plans) == w and max(p["tile"][3] for p in plans) == h
            for p, (pw, ph) in enumerate(((cw, ch), ((cw + 1) // 2, (ch + 1) // 2), ((cw + 1) // 2, (ch + 1) // 2))):
                assert max(q["lr_out"][p][2] for q in plans) == pw and max(q["lr_out"][p][3] for q in plans) == ph
                covered = sum((q["lr_units"][p][2] - q["lr_units"][p][0]) * (q["lr_units"][p][3] - q["lr_units"][p][1])
                              for q in plans)
                nx = max(q["lr_units"][p][2] for q in plans)
                ny = max(q["lr_units"][p][3] for q in plans)
                assert covered == nx * ny
    with pytest.raises(svtgpu.SvtGpuError):
        svtgpu.tile_plan(1368, 768, [64, 32, 32], 2, 2, 0, crop=(1360, 766))  # the coded size is not the crop's alignment
