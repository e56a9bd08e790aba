"""A picture tiled over ranks (BASELINE.json config 4) on the device path, bit-exact.

Two processes (torch.distributed gloo, world size 2) share the one GPU of the test box; each runs the whole
pipeline of a case on its tile through the library's frame-level calls with a host-transport communicator
(svtgpu.Comm.host over gloo: RCCL needs one rank per device), so every exchange goes through the C ABI:
the DLF trial SSEs before each bisection step, the CDEF search tables before the pick, the LR search records
before the finish.  The ranks' crops (DLF output over each tile, CDEF and LR outputs over each rank's LR
units) are assembled on rank 0 and compared with the reference's outputs of the case, digests included for
the 4K 10-bit bench configuration (tests/golden/pipe_c3_4k10.npz) — the same check as the one-rank run.
A one-rank RCCL communicator is exercised on its own (the 8-GPU path of bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import pipeline_run as prun

CASES = ["mini10", "sb128_10", "c3_4k10"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
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
        for case in CASES:
            part = prun.run_gpu_tiled(case, rank, world, comm, ctx)
            parts = [None] * world
            dist.all_gather_object(parts, part)
            if rank == 0:
                try:
                    prun.check(case, prun.assemble_tiled(case, parts), "tiled x%d" % world)
                    q.put((case, "ok"))
                except AssertionError as e:
                    q.put((case, "FAIL: %s" % str(e)[:2000]))
        comm.close()
    except BaseException as e:  # reported to the parent
        q.put(("rank %d" % rank, "ERROR: %r" % e))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_two_ranks_one_gpu_bit_exact():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = []
    try:
        while len(res) < len(CASES):
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


@pytest.mark.gpu
def test_rccl_one_rank_comm():
    """svtgpu_comm_create (RCCL) with one rank: the sums are the identity, and the tiled calls accept it."""
    import svtgpu
    ctx = svtgpu.Context(0)
    comm = svtgpu.Comm.rccl(ctx, 1, 0, svtgpu.Comm.unique_id())
    assert comm.nranks == 1
    a = np.arange(17, dtype=np.uint64) * np.uint64(0x100000001)
    assert np.array_equal(comm.allreduce(a.copy()), a)
    comm.close()
