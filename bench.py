#!/usr/bin/env python
"""bench.py — MI355X in-loop-filter hot path throughput (BASELINE.json metric).

A "step" = one 4K 10-bit 4:2:0 frame per frame slot through the device-resident in-loop filter pipeline:
  mode info: the frame's mode-info grid uploaded and its deblocking edge records rebuilt (an encoder hands over a new
      grid every frame);
  DLF stage (EbDlfProcess.c, dlf level 1): full-image level search (svt_av1_pick_filter_level) and the frame filter
      (svt_av1_loop_filter_frame);
  CDEF stage (EbCdefProcess.c / EbEncCdef.c): strength search over all 64x64 filter blocks (64 strengths, cdef_level
      1) -> frame-level strength pick (finish_cdef_search) -> apply (svt_av1_cdef_frame);
  LR stage (EbRestProcess.c): loop-restoration search (restoration_seg_search + rest_finish_search, wn/sg filter level
      1: 7-tap Wiener with refinement, 16 SGR eps with refinement) on the CDEF output and the apply
      (svt_av1_loop_restoration_filter_frame; RU 256 luma / 128 chroma; stripe boundary lines from the DLF output);
  MD distortion stage: SAD / SSE / variance of every AV1 block shape of every SB against 7 reference frames at one
      full-pel motion vector per (SB, reference) (SURVEY.md §8d config 5 workload at 4K).
Inputs: the 4K 10-bit (and 1080p 8-bit) frames, mode info and frame-level controls (base_q_idx, starting
loop-filter levels, the CDEF lambda, the LR rate inputs) are those of the reference-pinned pipeline cases
(tests/pipeline_cases.py c3_4k10 / c1_1080p8; tests/golden/pipe_*.npz hold the reference's own outputs on them and
tests/test_pipeline_golden.py checks the GPU against them bit-exact): the timed frames are the checked frames.
Other sizes use the same integer generator, unpinned.  Inputs are resident in HBM before timing.

N = 1: the whole frame on one GPU.  N > 1 (one rank per GPU; `--gpus N` spawns its ranks, or torchrun):
  tiles (default): every frame is tiled over the ranks (svtgpu_tile_plan: 1x2, 2x2, 2x4 grids on the restoration-unit
      grid); each rank runs the DLF trials, the CDEF search, the LR search and all three applies on its tile, and the
      frame-level calls exchange over RCCL (libsvtgpu's own communicator, one per frame slot): the DLF trial SSEs
      before every bisection step, the CDEF search tables before the pick, the LR search records before the RD
      finish; the MD batch takes an SB range per rank.  Strong scaling: a step is the same F frames at every N.
  frames (opt-in, secondary): every rank filters whole pictures of its own, no exchange (weak scaling).

Prints ONE JSON line on rank 0 (contract in the task description): value = luma Mpixels/s of the whole job, plus
`roofline` for the largest device-time kernel of the step (timed live on the stream it runs on; traffic and VALU
issue from the committed PMC profile) and `cpu_baseline` (the reference's own CPU path on this host, rank 0, N = 1,
bounded sample).
"""
import argparse
import datetime
import json
import os
import sys
import threading
import time

import numpy as np

FRAMES_IN_FLIGHT = 4  # default frames pipelined per GPU (round 3 final kernels: 2 -> 2672, 3 -> 2846, 4 -> 2914, 5 -> 2772 Mpx/s)
# default when a rank filters a tile of the picture (N > 1, or an emulated rank): its stages are shorter but their
# latency chains are not, so more frames overlap (round 4, emulated 8-GPU rank, 16 hardware queues: F = 4 5.9-6.0,
# F = 5 7.1, F = 6 7.6-7.7 Gpx/s; profiles/r04/queues).  Round 6, library streams, the MD batch on the main stream
# (2 streams per frame): F = 7 fills the 16 queues exactly (14 + the context's + the null stream) and beats F = 6 at
# every rank count (emulated 8 / 4 / 2-GPU ranks 10.38-10.40 / 8.21-8.22 / 5.28-5.35 vs 9.48-9.52 / 7.59-7.69 /
# 5.03-5.06 Gpx/s, two runs each, profiles/r06/fsweep_tiled.txt); F = 8 oversubscribes the queues (8.7)
TILED_FRAMES_IN_FLIGHT = 7
# hardware queues per process: HIP's default 4 would serialize the frames' streams, but past 16 the queues are
# time-sliced and every frame's latency chain stretches (emulated 8-GPU rank: F = 6 with 16 queues 7.6 Gpx/s, with 18
# 4.8; F = 8 with 32 queues 1.7); whole frames run the same with 8, 12 or 16 (3.03-3.06 Gpx/s at F = 4)
MAX_HW_QUEUES = 16


def _arg(argv, name):
    for i, w in enumerate(argv):
        if w == name and i + 1 < len(argv):
            return argv[i + 1]
        if w.startswith(name + "="):
            return w.split("=", 1)[1]
    return None


def _tiled(argv):
    """A rank of a tiled picture: N > 1 (the default split) or an emulated rank."""
    n = int(_arg(argv, "--gpus") or os.environ.get("WORLD_SIZE", 1))
    return (n > 1 and (_arg(argv, "--split") or "tiles") == "tiles") or int(_arg(argv, "--emulate-rank") or 0) > 1


def _frames_in_flight(argv):
    f = _arg(argv, "--frames-in-flight")
    return int(f) if f else (TILED_FRAMES_IN_FLIGHT if _tiled(argv) else FRAMES_IN_FLIGHT)


# set before the HIP runtime starts: 4 queues per frame in flight (3 streams each), at most MAX_HW_QUEUES
_want_queues = int(os.environ.get("SVTGPU_BENCH_QUEUES", 0)) or min(MAX_HW_QUEUES, max(8, 4 * _frames_in_flight(sys.argv[1:])))
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < _want_queues:
    os.environ["GPU_MAX_HW_QUEUES"] = str(min(_want_queues, 32))

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "svt-av1_pro-anchor-v2.1.0-_amd"))

import svtgpu  # noqa: E402
import synth  # noqa: E402

def pmc_summary(path, kernel, bd):
    """Per-launch PMC figures of `kernel` from the committed summary (scripts/pmc_traffic.py / pmc_sq.py over
    rocprofv3 --pmc passes of this bench, which cannot run inside it): traffic bytes (2 x FETCH_SIZE + WRITE_SIZE)
    and SQ_INSTS_VALU.  ({}, None) when no summary covers the kernel."""
    try:
        summary = json.load(open(path))
    except (OSError, ValueError):
        return {}, None
    ty = "unsigned short" if bd > 8 else "unsigned char"
    ks = summary.get("kernels", {})
    k = ks.get("%s<%s>" % (kernel, ty))
    if not k:  # a kernel with more template arguments (sgr_res_kernel<T, TREE>): the instance that ran most
        cand = [v for n, v in ks.items() if n.startswith("%s<%s," % (kernel, ty))]
        k = max(cand, key=lambda v: v.get("launches", 0)) if cand else None
    if not k:
        return {}, None
    return k, "%s (%s; %d launches)" % (os.path.relpath(path, ROOT), summary["method"], k["launches"])


HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# VALU issue peak: 256 CUs x 4 SIMDs, a wave64 instruction every 2 cycles per SIMD (SIMD32), 2.4 GHz
VALU_PEAK_INSTS = 256 * 4 * 0.5 * 2.4e9

# BASELINE configurations whose frames and frame-level controls are the reference-pinned pipeline cases
# (tests/pipeline_cases.py; the reference's outputs on them in tests/golden/pipe_<case>.npz, checked bit-exact by
# tests/test_pipeline_golden.py; tests/test_bench_inputs.py checks these constants against the cases and fixtures)
PINNED = {
    (3840, 2160, 10): dict(case="c3_4k10", seed=0x5EED0003, q=160, lf=(16, 16, 8, 8), lam=206765, rdmult=7000,
                           sw=(300, 700, 900), wc=(250, 800), sc=(250, 900), us=(256, 128)),
    (1920, 1080, 8): dict(case="c1_1080p8", seed=0x5EED0002, q=160, lf=(16, 16, 8, 8), lam=207229, rdmult=7000,
                          sw=(300, 700, 900), wc=(250, 800), sc=(250, 900), us=(256, 128)),
}
UNPINNED = dict(case=None, q=160, lf=(16, 16, 8, 8), lam=206765, rdmult=7000, sw=(300, 700, 900), wc=(250, 800),
                sc=(250, 900), us=(256, 128))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--bit-depth", type=int, default=10)
    ap.add_argument("--cdef-level", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true", help="no device-clock timing inside the LR search")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "r06", "pmc", "kernels.json"),
                    help="per-launch traffic / VALU counters from scripts/pmc_traffic.sh (PMC passes cannot run inside "
                         "the bench)")
    ap.add_argument("--cpu-grid", default="4x4", help="crops of the frame timed on the host CPU (one per thread)")
    ap.add_argument("--cpu-passes", type=int, default=6,
                    help="reference CPU baseline: passes over the crops (sizes the sample to ~10-30 s of CPU work)")
    ap.add_argument("--cpu-kind", choices=("reference", "port"), default="reference",
                    help="CPU baseline: the reference's own C + AVX2 kernels (oracle/_ref/ref_bench, built from the "
                         "reference sources by oracle/ref.mk) or the repo's C restatement (oracle/)")
    ap.add_argument("--frames-in-flight", type=int, default=None,
                    help="frames pipelined per GPU, each on its own streams and host thread (the encoder's "
                         "picture-level parallelism); a step processes one frame per slot.  Default %d, %d for a rank "
                         "of a tiled picture (and the tile projection's emulated ranks)" % (FRAMES_IN_FLIGHT,
                                                                                            TILED_FRAMES_IN_FLIGHT))
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="the tiles' exchanges: nccl = libsvtgpu's RCCL communicator over xGMI (one rank per GPU); "
                         "gloo = the library's host transport over gloo (rehearses N > 1 ranks sharing one GPU)")
    ap.add_argument("--comm-timeout-ms", type=int, default=60000,
                    help="deadline of every tile exchange (DLF trial SSEs, CDEF tables, LR records): a rank whose peer "
                         "never arrives fails with the exchange named instead of hanging the node")
    ap.add_argument("--split", default="tiles", choices=("tiles", "frames"),
                    help="N > 1: 'tiles' = every frame tiled over the ranks with RCCL exchanges (SURVEY §8e, BASELINE "
                         "config 4; strong scaling); 'frames' = every rank filters pictures of its own (weak scaling)")
    ap.add_argument("--inputs", default="pinned", choices=("pinned", "synth"),
                    help="pinned: the reference-pinned pipeline case of this size when there is one (else synth); "
                         "synth: the float generator (synth.frame_pair)")
    ap.add_argument("--master-port", type=int, default=29517, help="rendezvous port when bench.py spawns its ranks")
    ap.add_argument("--md-main", action="store_true", default=None,
                    help="run the MD batch on the frame's main stream (after the CDEF stage) instead of its own: one "
                         "hardware queue less per frame in flight")
    ap.add_argument("--dlf-sync", action="store_true",
                    help="A/B: the synchronous DLF level search (svtgpu_dlf_pick: host-driven bisection, levels back "
                         "before the filter) instead of the asynchronous one (device bisection + filter in stream order)")
    ap.add_argument("--run-ahead", type=int, default=2, metavar="K",
                    help="steps a slot's thread may enqueue ahead of its stream's completed ones (the asynchronous "
                         "searches leave no host wait inside a step)")
    ap.add_argument("--cdef-async", dest="cdef_sync", action="store_false",
                    help="A/B: the asynchronous CDEF pick (svtgpu_cdef_pick_async + the apply from device memory, no "
                         "host wait) instead of the synchronous one (svtgpu_cdef_pick: the host waits for the settle check "
                         "and the strengths; the default: measured faster at four frames in flight, DESIGN §5)")
    ap.add_argument("--lr-sync", action="store_true",
                    help="A/B: the synchronous LR search (svtgpu_lr_search_frame: one host wait, frame types back before "
                         "the apply) instead of the asynchronous one (search + device RD finish + apply in stream order)")
    ap.add_argument("--torch-streams", action="store_true",
                    help="A/B: the frame slots' streams from torch.cuda.Stream() (torch's stream pool) instead of "
                         "svtgpu_stream_create")
    ap.add_argument("--lr-serial", action="store_true",
                    help="measurement: every LR search runs its Wiener chain after its self-guided chain on one stream, "
                         "so each search kernel has the device to itself (the condition of the roofline's isolated "
                         "phase; rocprofv3 of a --frames-in-flight 1 --lr-serial run reproduces its durations)")
    ap.add_argument("--lr-levels", default="1,1", metavar="WN,SG",
                    help="diagnostic only (sensitivity runs; the headline is 1,1): the Wiener / self-guided search levels")
    ap.add_argument("--stages", default="all", choices=("all", "cdef", "md"),
                    help="'all' = the whole step; 'cdef' = CDEF search + pick + apply on the recon alone (SURVEY §8d "
                         "configs 1/2)")
    ap.add_argument("--host-timing", action="store_true",
                    help="report the host thread's wall / CPU ms per frame-level call (config.host_ms, slot 0)")
    ap.add_argument("--emulate-rank", type=int, default=0, metavar="N",
                    help="N = 1 only: run the largest rank of an N-GPU tiled picture alone (one-rank RCCL "
                         "communicators); value is then the projected N-GPU job throughput F x W x H / step time")
    ap.add_argument("--no-tile-projection", dest="tile_projection", action="store_false",
                    help="N = 1: skip the emulated ranks of 2/4/8-GPU tiled pictures (config.tile_projection)")
    ap.add_argument("--no-matrix", action="store_true",
                    help="skip the extra configurations (north_star matrix + config 1) run as child processes")
    a = ap.parse_args()
    a.explicit_frames = a.frames_in_flight is not None
    if a.frames_in_flight is None:
        a.frames_in_flight = _frames_in_flight(sys.argv[1:])
    # one hardware queue per stream: per frame in flight the main stream, the MD stream and the LR search's Wiener
    # stream, plus the library context's and torch's null stream.  Streams beyond GPU_MAX_HW_QUEUES share queues, and
    # a shared in-order queue serializes two frames' chains (round 5's six-frames collapse, 2903 -> 1360 Mpx/s with the
    # same frame latency: the lazily created Wiener streams landed on queues in thread order).  The MD batch moves onto
    # the main stream when its own stream would not get a queue of its own.
    if a.md_main is None:
        a.md_main = 3 * a.frames_in_flight + 2 > _want_queues
    return a


# the north_star reporting matrix beside the headline 4K 10-bit line: (label, argv) of child bench runs, started
# before this process touches the GPU; their JSON lines are summarised under config.matrix
MATRIX = [
    ("config1_1080p8_cdef", ["--width", "1920", "--height", "1080", "--bit-depth", "8", "--stages", "cdef",
                             "--cpu-grid", "4x4", "--cpu-passes", "120", "--steps", "100", "--warmup", "5",
                             "--frames-in-flight", "1"]),
    ("pipeline_1080p8", ["--width", "1920", "--height", "1080", "--bit-depth", "8", "--no-cpu-baseline",
                         "--steps", "60", "--warmup", "5"]),
    ("pipeline_1080p10", ["--width", "1920", "--height", "1080", "--bit-depth", "10", "--no-cpu-baseline",
                          "--steps", "60", "--warmup", "5"]),
    ("pipeline_4k8", ["--width", "3840", "--height", "2160", "--bit-depth", "8", "--no-cpu-baseline",
                      "--steps", "40", "--warmup", "5"]),
    ("config5_8k10_md", ["--width", "7680", "--height", "4320", "--bit-depth", "10", "--stages", "md",
                         "--no-cpu-baseline", "--steps", "50", "--warmup", "5"]),
]


def run_matrix():
    """Each extra configuration as a child bench process (sequential, before this process initialises the GPU)."""
    import subprocess
    res = {}
    for label, argv in MATRIX:
        try:
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--no-matrix"] + argv, capture_output=True,
                               text=True, timeout=300)
            line = [l for l in r.stdout.splitlines() if l.startswith("{")]
            if r.returncode != 0 or not line:
                res[label] = {"error": "exit %d: %s" % (r.returncode, r.stderr.strip()[-300:])}
                continue
            d = json.loads(line[-1])
            c = d["config"]
            res[label] = {"value": d["value"], "unit": d["unit"], "ms_per_step": d["ms_per_step"],
                          "frames_in_flight": c["frames_in_flight"], "workload": c["workload"],
                          "pipeline_frac_hbm": c.get("pipeline_roofline", {}).get("frac")}
            if "md_roofline" in c:
                res[label]["md_roofline"] = c["md_roofline"]
            if "cpu_baseline" in d:
                res[label]["cpu_baseline"] = d["cpu_baseline"]
        except (OSError, ValueError, subprocess.TimeoutExpired) as e:
            res[label] = {"error": repr(e)[:300]}
    return res


def run_projection(a):
    """Strong-scaling projection of BASELINE config 4 on this one GPU: for N = 2, 4, 8 a child bench process runs the
    rank with the largest tile of an N-rank picture alone (--emulate-rank N: its own process and hardware queues like a
    real rank, the tiled rank's default frames in flight, one-rank RCCL communicators -- every ncclAllReduce issued,
    none crossing xGMI).  Its value is F x W x H / its step time: the N-GPU job's throughput up to the collectives'
    xGMI latency.  Sequential, before this process initialises the GPU."""
    import subprocess
    res = {}
    for nn in (2, 4, 8):
        argv = ["--no-matrix", "--no-tile-projection", "--no-cpu-baseline", "--emulate-rank", str(nn),
                "--width", str(a.width), "--height", str(a.height), "--bit-depth", str(a.bit_depth),
                "--cdef-level", str(a.cdef_level), "--steps", str(max(10, min(a.steps, 40))), "--warmup", "5"]
        if a.explicit_frames:
            argv += ["--frames-in-flight", str(a.frames_in_flight)]
        try:
            r = subprocess.run([sys.executable, os.path.abspath(__file__)] + argv, capture_output=True, text=True,
                               timeout=300)
            line = [l for l in r.stdout.splitlines() if l.startswith("{")]
            if r.returncode != 0 or not line:
                res["n%d" % nn] = {"error": "exit %d: %s" % (r.returncode, r.stderr.strip()[-300:])}
                continue
            d = json.loads(line[-1])
            c = d["config"]
            e = c.get("emulated", {})
            res["n%d" % nn] = {"grid": e.get("grid"), "rank": e.get("rank"), "tile": e.get("tile"),
                               "tile_share": e.get("tile_share"), "frames_in_flight": c["frames_in_flight"],
                               "ms_per_step": d["ms_per_step"], "projected_Mpx_s": d["value"],
                               "frame_latency_ms": c["frame_latency_ms"],
                               "stage_ms": {k: v for k, v in c["stage_ms"].items() if k != "note"},
                               "cdef_pick_ms": e.get("cdef_pick_ms")}
        except (OSError, ValueError, subprocess.TimeoutExpired) as ex:
            res["n%d" % nn] = {"error": repr(ex)[:300]}
    res["note"] = ("one rank of an N-GPU tiled picture emulated on this GPU as its own process (bench --emulate-rank N: "
                   "the rank with the largest tile, frames_in_flight frames in flight, one-rank RCCL communicators): "
                   "ms_per_step ~ the N-GPU job's step time without the xGMI latency of its collectives (DLF trial SSEs "
                   "per bisection step, CDEF tables 2.1 MB, LR records); projected_Mpx_s = F x W x H / ms_per_step.  "
                   "Replicated per rank whatever N: the CDEF pick (cdef_pick_ms), the DLF bisection's host decisions "
                   "and the LR RD finish")
    return res


def spawn_ranks(a):
    """`--gpus N` outside a torch.distributed launcher: start the N ranks as children (one process per GPU) before
    this process touches the device, and return their exit code.  Inside a launcher WORLD_SIZE must equal N."""
    world = int(os.environ.get("WORLD_SIZE", "0"))
    if world:
        if world != a.gpus:
            raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d: refusing to report one as the other"
                             % (a.gpus, world))
        return None
    if a.gpus <= 1:
        return None
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(a.master_port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def cpu_threads():
    """Host threads for the CPU baseline: the cores this process may use, at most 16 (a GPU box's CPU share is 16 cores
    per GPU while os.cpu_count() reports the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


REF_BENCH = os.path.join(ROOT, "oracle", "_ref", "ref_bench")


def write_ref_bench_input(f, src, rec, mi, ctrls, bd, q, lam, grid, lr_ctrls, md_refs, md_mvs, lf_start):
    """The input file of oracle/_ref/ref_bench (layout in oracle/ref_harness/ref_bench.c's main)."""
    gx, gy = (int(x) for x in grid.split("x"))
    H, W = rec[0].shape
    hdr = np.array([W, H, bd, len(md_refs), q, lam, gx, gy, lr_ctrls.rdmult, *lr_ctrls.switchable_restore_cost,
                    *lr_ctrls.wiener_restore_cost, *lr_ctrls.sgrproj_restore_cost, *lf_start], np.int32)
    f.write(hdr.tobytes())
    f.write(bytes(ctrls))
    for planes in (src, rec):
        for p in planes:
            f.write(np.ascontiguousarray(p, np.uint16).tobytes())
    f.write(np.ascontiguousarray(mi).tobytes())
    for r in md_refs:
        f.write(np.ascontiguousarray(r, np.uint16).tobytes())
    f.write(np.ascontiguousarray(md_mvs, np.int32).tobytes())


def cpu_baseline_reference(src, rec, mi, ctrls, bd, level, q, lam, grid, lr_ctrls, md_refs, md_mvs, passes,
                           lf_start, stages="all"):
    """The reference's own CPU path (oracle/_ref/ref_bench: its C with the AVX2/SSE2 kernels an AVX2 host binds) on the
    host's cores, over the same crops as cpu_baseline. The frame, mode info, CDEF controls, LR rate inputs, MD
    references and MVs are handed over in a file; the binary times itself (input loading excluded)."""
    import subprocess
    import tempfile
    gx, gy = (int(x) for x in grid.split("x"))
    H, W = rec[0].shape
    nthr = min(cpu_threads(), gx * gy)
    def run(f, threads, npass):
        env = dict(os.environ, REF_BENCH_STAGES="2" if stages == "cdef" else "15")
        res = subprocess.run([REF_BENCH, f.name, str(threads), str(npass)], capture_output=True, text=True, timeout=600,
                             env=env)
        if res.returncode != 0:
            raise RuntimeError("ref_bench failed (%d): %s" % (res.returncode, res.stderr.strip()[-400:]))
        kv = dict(t.split("=") for t in res.stdout.split()[1:])
        return int(kv["px"]), float(kv["seconds"])

    with tempfile.NamedTemporaryFile(prefix="ref_bench_", suffix=".bin", dir="/tmp", delete=True) as f:
        write_ref_bench_input(f, src, rec, mi, ctrls, bd, q, lam, grid, lr_ctrls, md_refs, md_mvs, lf_start)
        f.flush()
        px, dt = run(f, nthr, passes)
        px1, dt1 = run(f, 1, 1)  # one thread, one pass: the per-core rate
    model = "unknown CPU"
    try:
        with open("/proc/cpuinfo") as ci:
            model = next(l.split(":", 1)[1].strip() for l in ci if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    cw, ch = (W // gx) & ~63, (H // gy) & ~63
    return {"value": round(px / dt / 1e6, 4), "unit": "Mpixels/s", "cores": nthr, "kind": "reference",
            "single_thread_value": round(px1 / dt1 / 1e6, 4), "cpu": model,
            "sample": ("the %d-bit frame cut into %dx%d crops of %dx%d, each through " % (bd, gx, gy, cw, ch)) +
                      ("CDEF search + strength selection + apply at cdef_level %d on the recon (the reference's "
                       "%s path)" % (level, "8-bit (is_16bit_pipeline = 0)" if bd == 8 else "16-bit")
                       if stages == "cdef" else
                       "the same stages (DLF level search + filter, CDEF search + strength selection + apply at "
                       "cdef_level %d, LR search + apply at wn/sg level 1, MD SAD/SSE/variance over 7 refs)" % level) +
                      (" by the reference's own C with its AVX2/SSE2 kernels (oracle/_ref/ref_bench), %d passes, %d "
                       "host threads, %.1f s" % (passes, nthr, dt))}


def cpu_baseline(src, rec, mi, lf_start, bd, level, q, lam, grid, lr_ctrls, lr_us, md_refs, md_mvs):
    """The repo's C restatement (oracle/, gcc -O2) on the host's cores: the frame is cut into gx x gy crops and each
    host thread runs the same stages as the GPU step (DLF pick + filter, CDEF search + pick + apply, LR search + apply,
    MD batch) on one crop at a time (ctypes releases the GIL, so the threads run in parallel)."""
    import threading as th
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: used here only as the reported CPU baseline
    gx, gy = (int(x) for x in grid.split("x"))
    H, W = rec[0].shape
    cw, ch = (W // gx) & ~63, (H // gy) & ~63  # crops on the 64-px grid (whole FBs, units, SBs)
    ctrls = oracle.controls(level)
    octrls = oracle.lr_controls(1, 1, rdmult=lr_ctrls.rdmult, switchable=tuple(lr_ctrls.switchable_restore_cost),
                                wiener=tuple(lr_ctrls.wiener_restore_cost), sgrproj=tuple(lr_ctrls.sgrproj_restore_cost))
    nsbx = (W + 63) // 64

    def one(cx, cy):
        y0, x0 = cy * ch, cx * cw
        mi_c = np.ascontiguousarray(mi[y0 // 4:(y0 + ch) // 4, x0 // 4:(x0 + cw) // 4])
        crop = [np.ascontiguousarray(rec[0][y0:y0 + ch, x0:x0 + cw])] + \
               [np.ascontiguousarray(p[y0 // 2:(y0 + ch) // 2, x0 // 2:(x0 + cw) // 2]) for p in rec[1:]]
        cs = [np.ascontiguousarray(src[0][y0:y0 + ch, x0:x0 + cw])] + \
             [np.ascontiguousarray(p[y0 // 2:(y0 + ch) // 2, x0 // 2:(x0 + cw) // 2]) for p in src[1:]]
        lfp = oracle.dlf_pick(crop, cs, bd, mi_c, lf_start, 0, 0, 0, 0, 0)
        crop = oracle.dlf_frame(crop, bd, mi_c, lfp)
        mse, skip, d, v = oracle.cdef_search_frame(crop, cs, bd, ctrls, q)
        prm, fbs = oracle.cdef_pick(cw, ch, mse, skip, ctrls, q, lam)
        cdef_out = oracle.cdef_apply_frame(crop, bd, None, d, v, prm, fbs)
        ft, units, _ = oracle.lr_search_frame(cdef_out, cs, bd, lr_us, octrls)
        oracle.lr_apply_frame(crop, cdef_out, bd, ft, lr_us, units)
        sbs = [(y0 // 64 + r) * nsbx + x0 // 64 + c for r in range(ch // 64) for c in range(cw // 64)]
        oracle.md_dist_batch(cs[0], [np.ascontiguousarray(r[y0:y0 + ch, x0:x0 + cw]) for r in md_refs], bd,
                             np.ascontiguousarray(md_mvs[sbs], np.int32))

    jobs = [(cx, cy) for cy in range(gy) for cx in range(gx)]
    nthr = min(cpu_threads(), len(jobs))
    lock, errors = th.Lock(), []

    def worker():
        while True:
            with lock:
                if not jobs:
                    return
                job = jobs.pop()
            try:
                one(*job)
            except BaseException as e:
                errors.append(e)
                return

    t0 = time.perf_counter()
    threads = [th.Thread(target=worker) for _ in range(nthr)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    dt = time.perf_counter() - t0
    if errors:
        raise errors[0]
    px = gx * gy * cw * ch
    return {"value": round(px / dt / 1e6, 4), "unit": "Mpixels/s", "cores": nthr, "kind": "port",
            "sample": "the %d-bit frame cut into %dx%d crops of %dx%d, each through the same stages (DLF pick+filter, "
                      "CDEF search+pick+apply at cdef_level %d, LR search+apply at wn/sg level 1, MD batch 7 refs) by the "
                      "C restatement (oracle/, gcc -O2), %d host threads, %.1f s"
                      % (bd, gx, gy, cw, ch, level, nthr, dt)}


def measure_next_rows(ctx, torch, W, H, reps=20):
    """The §8(f) rows beside the pipeline, timed with HIP events on the stream they run on (rank 0, N = 1): the
    frame-buffer kernels against the HBM roofline (their bytes are the algorithmic bytes: every touched sample read or
    written once), and the open-loop ME full-pel search (VALU-bound: v_sad_u8 over every position)."""
    import ctypes
    L = svtgpu.lib()
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    out = {}

    def timed(fn):
        fn()  # warm
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    def hbm(name, ms, nbytes, what):
        out[name] = {"ms": round(ms, 5), "alg_MB": round(nbytes / 1e6, 3),
                     "achieved_GBs": round(nbytes / (ms * 1e-3) / 1e9, 1),
                     "frac": round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "what": what}

    src8, _ = synth.frame_pair(W, H, 8, seed=0x5EED0031)
    f8, f16, g8 = svtgpu.Frame(ctx, W, H, 8), svtgpu.Frame(ctx, W, H, 10), svtgpu.Frame(ctx, W, H, 8)
    f8.upload(src8)
    torch.cuda.synchronize()
    S = 1.5 * W * H
    hbm("convert_8to16", timed(lambda: L.svtgpu_frame_convert(f8.h, f16.h, sp)), 3 * S,
        "svt_convert_pic_8bit_to_16bit, 3 planes (1 B read + 2 B written per sample)")
    hbm("convert_16to8", timed(lambda: L.svtgpu_frame_convert(f16.h, g8.h, sp)), 3 * S,
        "16 -> 8 copy-back of a non-reference picture, 3 planes (2 B read + 1 B written per sample)")
    pw = ph = 80
    stride = W + 2 * pw
    buf = torch.zeros((H + 2 * ph) * stride, dtype=torch.int16, device="cuda")
    border = (H + 2 * ph) * stride - W * H
    hbm("pad_ref_luma_16bit", timed(lambda: L.svtgpu_pad_plane(ctypes.c_void_p(buf.data_ptr()), 16, stride, W, H, pw, ph,
                                                                sp)),
        2 * (border + 2 * H + 2 * stride), "svt_aom_generate_padding16_bit of a 4K luma plane, 80-sample border "
                                           "(border samples written, edge samples read)")
    # open-loop ME: every 64x64 block x 2 references, 32 x 32 full-pel positions
    nref, saw, sah = 2, 32, 32
    refs = []
    for k in range(nref):
        rf = svtgpu.Frame(ctx, W, H, 8)
        rf.upload(synth.frame_pair(W, H, 8, seed=0x5EED0032 + k)[0])
        refs.append(rf)
    me = svtgpu.MeBatch(ctx, W, H, nref)
    me.set_origins(np.random.default_rng(3).integers(-24, -8, size=(me.nsb, nref, 2)).astype(np.int16))
    torch.cuda.synchronize()
    ms = timed(lambda: me.search(f8, refs, saw, sah, 0, stream=st.cuda_stream))
    tasks = me.nsb * nref
    out["me_fullpel_search"] = {"ms": round(ms, 4), "blocks_x_refs": tasks, "positions": saw * sah,
                                "block_positions_per_s": round(tasks * saw * sah / (ms * 1e-3), 1),
                                "sad_Gops": round(tasks * saw * sah * 4096 / (ms * 1e-3) / 1e9, 1),
                                "what": "svtgpu_me_search: %dx%d 8-bit, %d refs, %dx%d positions, 85 bests per block "
                                        "(VALU-bound: v_sad_u8)" % (W, H, nref, saw, sah)}
    return out


class HostClock:
    """--host-timing: the host thread's wall and CPU time in each frame-level call of a step (CPU time includes the
    library's spin-waits on mapped memory; wall time includes every wait)."""

    def __init__(self, on):
        self.on, self.t = on, {}
        if on:
            self.w, self.c = time.perf_counter(), time.thread_time()

    def __call__(self, name):
        if self.on:
            w, c = time.perf_counter(), time.thread_time()
            self.t[name] = ((w - self.w) * 1e3, (c - self.c) * 1e3)
            self.w, self.c = w, c


def roofline_of(kernels, bd, pmc_json):
    """The `roofline` object for the largest device-time kernel of the step.  kernels: name -> {ms (device time per
    frame), launches (per frame), alg_bytes (SURVEY §8(d) bytes per frame: the samples the kernel's job reads once and
    the outputs it must write), what}.  traffic / SQ_INSTS_VALU per launch come from the committed PMC summary."""
    name = max(kernels, key=lambda k: kernels[k]["ms"])
    k = kernels[name]
    per_launch_ms = k["ms"] / max(k["launches"], 1)
    alg = k["alg_bytes"] / max(k["launches"], 1)
    ach = alg / (per_launch_ms * 1e-3) / 1e9
    pmc, src = pmc_summary(pmc_json, name, bd)
    traffic = pmc.get("traffic_bytes")
    valu = pmc.get("SQ_INSTS_VALU")
    out = {"kernel": name, "bound": "hbm", "achieved": round(ach, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(ach / HBM_PEAK_GBS, 6), "traffic": traffic, "alg_bytes_per_launch": round(alg),
           "avg_launch_ms": round(per_launch_ms, 5), "launches_per_frame": k["launches"],
           "avg_launch_ms_device_clock": (round(k["ms_clock"] / max(k["launches"], 1), 5) if "ms_clock" in k else None),
           "ms_per_frame": round(k["ms"], 4),
           "valu": round(valu / (per_launch_ms * 1e-3 * VALU_PEAK_INSTS), 4) if valu else None,
           "valu_insts_per_launch": valu, "pmc_source": src,
           "all_kernels_ms_per_frame": {n: round(v["ms"], 4) for n, v in sorted(kernels.items(), key=lambda x: -x[1]["ms"])},
           "note": "the largest device-time kernel of the step (device time per frame, timed live with HIP events "
                   "on the stream each kernel runs on: the CDEF search and MD batch by the bench, the LR search "
                   "kernels inside the library around each launch (svtgpu_lr_profile ms_events, the span rocprofv3's "
                   "kernel trace reports); avg_launch_ms_device_clock = the device's s_memrealtime clock, first "
                   "workgroup start to last workgroup end); achieved = SURVEY §8(d) algorithmic "
                   "bytes (%s) / its launch duration; traffic = 2 x FETCH_SIZE + WRITE_SIZE per launch and valu = "
                   "SQ_INSTS_VALU / (launch duration x %.3g wave-instructions/s VALU issue peak), both from %s" %
                   (k["what"], VALU_PEAK_INSTS, os.path.relpath(pmc_json, ROOT))}
    return out


def bench_md(a, torch, dist, n, rank, local):
    """BASELINE configs[4]: the mode-decision distortion batch of one frame -- SAD, SSE and variance of every AV1 block
    shape <= 64x64 of every SB against NREF references (md_dist_kernel) -- split over the ranks by SB ranges (strong
    scaling, no exchange), with each GPU's HBM rate against the roofline ((1 + refs) x 64 x 64 x B per
    SB read once; the per-shape outputs written once)."""
    W, H, bd = a.width, a.height, a.bit_depth
    B = 2 if bd > 8 else 1
    NREF = 7
    ctx = svtgpu.Context(local)
    src, _ = synth.frame_pair_int(W, H, bd, 0x5EED0008)
    S = svtgpu.Frame(ctx, W, H, bd)
    S.upload(src)
    refs = []
    for r in range(NREF):
        rs, _ = synth.frame_pair_int(W, H, bd, 0x5EED0009 + 17 * r)
        f = svtgpu.Frame(ctx, W, H, bd)
        f.upload(rs)
        refs.append(f)
    md = svtgpu.MdBatch(ctx, W, H, NREF)
    md.set_mvs(np.random.default_rng(8).integers(-16, 17, size=(md.nsb, NREF, 2)))
    sb0, sb1 = svtgpu.band(md.nsb, n, rank)
    stream = torch.cuda.Stream()
    sp = stream.cuda_stream
    for _ in range(a.warmup):
        md.run(S, refs, sb0, sb1, sp)
    torch.cuda.synchronize()
    if n > 1:
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(a.steps):
        md.run(S, refs, sb0, sb1, sp)
    e1.record(stream)
    torch.cuda.synchronize()
    if n > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    gpu_ms = e0.elapsed_time(e1) / a.steps  # this rank's device time per step
    # the on-demand expansion of the moments into every shape's values (svtgpu_md_expand), timed apart: a consumer
    # that wants the per-shape table pays it once per frame
    e2, e3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e2.record(stream)
    for _ in range(5):
        md.expand(sb0, sb1, sp)
    e3.record(stream)
    torch.cuda.synchronize()
    expand_ms = e2.elapsed_time(e3) / 5
    if n > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = dt * 1e3 / a.steps
    nsb_mine = sb1 - sb0
    alg_in = nsb_mine * (1 + NREF) * 64 * 64 * B
    alg_out = nsb_mine * NREF * 256 * 8  # the cell moments
    gbs = (alg_in + alg_out) / (gpu_ms * 1e-3) / 1e9
    out = {"metric": "MD SAD/SSE/variance Mpixels/s on 8K10b; per-GPU HBM GB/s vs roofline", "value": round(W * H / (ms_per_step * 1e-3) / 1e6, 3),
           "unit": "Mpixels/s", "n_gpus": n, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms_per_step, 4),
           "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u16" if bd > 8 else "u8",
           "data": "synthetic",
           "config": {"workload": "md_dist_kernel: every SB x %d refs x all %d block shapes <= 64x64 (SAD, SSE, variance); "
                                  "%dx%d %d-bit, %d SBs split over %d rank(s) by SB ranges" % (NREF, svtgpu.MD_BLOCKS, W, H, bd,
                                                                                            md.nsb, n),
                      "width": W, "height": H, "bit_depth": bd, "frames_in_flight": 1, "nsb": md.nsb,
                      "sb_range": [sb0, sb1], "parallelism": "sb%d (SB ranges, no exchange)" % n if n > 1 else "single",
                      "md_roofline": {"alg_in_MB_per_gpu": round(alg_in / 1e6, 2), "out_MB_per_gpu": round(alg_out / 1e6, 2),
                                      "gpu_ms_per_frame": round(gpu_ms, 4), "achieved_GBs_per_gpu": round(gbs, 1),
                                      "peak": HBM_PEAK_GBS, "frac": round(gbs / HBM_PEAK_GBS, 4),
                                      "expand_ms_per_frame": round(expand_ms, 4),
                                      "note": "rank 0's HIP-event time per step; bytes = the SB samples of the source and "
                                              "every reference read once (SURVEY §8(d)) + the 8-byte moments of every "
                                              "4x4 cell x ref written once (every shape's SAD / SSE / variance are exact "
                                              "sums of them; svtgpu_md_expand derives the u32 [SB][ref][3][%d] table "
                                              "on demand: expand_ms_per_frame)" % svtgpu.MD_BLOCKS}}}
    if rank == 0:
        print(json.dumps(out), flush=True)
    md.close()


def main():
    a = parse()
    rc = spawn_ranks(a)
    if rc is not None:
        sys.exit(rc)
    matrix = None
    if not a.no_matrix and int(os.environ.get("WORLD_SIZE", "1")) == 1 and a.stages == "all":
        matrix = run_matrix()  # before this process touches the GPU
    projection = None
    if (a.tile_projection and a.emulate_rank <= 1 and a.stages == "all" and a.gpus == 1
            and int(os.environ.get("WORLD_SIZE", "1")) == 1):
        projection = run_projection(a)  # likewise
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    local = local % max(1, torch.cuda.device_count())  # ranks > GPUs only in a gloo rehearsal on one GPU
    torch.cuda.set_device(local)
    n = world
    if n > 1:  # control only (barriers, the max-over-ranks time, the RCCL ids): the data path is libsvtgpu's RCCL
        dist.init_process_group("gloo", timeout=datetime.timedelta(milliseconds=4 * a.comm_timeout_ms))
    if a.stages == "md":
        bench_md(a, torch, dist, n, rank, local)
        if n > 1:
            dist.destroy_process_group()
        return
    tiled = n > 1 and a.split == "tiles"
    W, H, bd = a.width, a.height, a.bit_depth
    pin = PINNED.get((W, H, bd)) if a.inputs == "pinned" else None
    cfg = pin or UNPINNED
    q, lam = cfg["q"], cfg["lam"]
    lr_us = [cfg["us"][0], cfg["us"][1], cfg["us"][1]]

    ctx = svtgpu.Context(local)
    ctrls = svtgpu.cdef_controls(a.cdef_level)
    mi = synth.mode_info(W, H, 3)
    mi_bytes = mi.nbytes
    # the mode-info grid is a frame input like the pictures: resident in HBM before the timed region (an encoder
    # whose mode decision runs on the device hands it over there); each step copies it into the DLF state
    mi_dev = torch.from_numpy(np.ascontiguousarray(mi).view(np.uint8).reshape(-1).copy()).cuda(local)
    lf_start = svtgpu.LfParams.make(*cfg["lf"])  # the previous frame's levels (search start)
    wn_lv, sg_lv = (int(x) for x in a.lr_levels.split(","))
    lr_ctrls = svtgpu.lr_controls(wn_lv, sg_lv, rdmult=cfg["rdmult"], switchable=cfg["sw"], wiener=cfg["wc"],
                                  sgrproj=cfg["sc"])
    gx, gy = svtgpu.tile_grid(n) if tiled else (1, 1)
    md_nsb = ((W + 63) // 64) * ((H + 63) // 64)
    plan = svtgpu.tile_plan(W, H, lr_us, gx, gy, rank).rects() if tiled else None
    emu_rank = None
    if a.emulate_rank > 1 and n == 1 and a.stages == "all":  # one rank of an N-GPU tiled picture, alone on this GPU
        egx, egy = svtgpu.tile_grid(a.emulate_rank)
        eplans = [svtgpu.tile_plan(W, H, lr_us, egx, egy, r).rects() for r in range(a.emulate_rank)]
        emu_rank = int(np.argmax([(p_["tile"][2] - p_["tile"][0]) * (p_["tile"][3] - p_["tile"][1]) for p_ in eplans]))
        plan = eplans[emu_rank]
    NREF = 7
    md_refs, md_ref_y = [], []  # reference frames of the MD batch, shared by the frames in flight
    for r in range(NREF):
        rs, _ = synth.frame_pair(W, H, bd, seed=0x5EED0005 + 17 * (r + 1))
        f = svtgpu.Frame(ctx, W, H, bd)
        f.upload(rs)
        md_refs.append(f)
        md_ref_y.append(rs[0])
    torch.cuda.synchronize()

    def frame_inputs(k):
        if pin:  # the pinned case's frames (every slot the same pictures; nothing is cached between frames)
            return synth.frame_pair_int(W, H, bd, pin["seed"])
        return synth.frame_pair_int(W, H, bd, 0x5EED0010 + 0x100 * k + 0x10000 * (0 if tiled else rank)) \
            if a.inputs == "pinned" else synth.frame_pair(W, H, bd, seed=0x5EED0003 + 0x100 * k + 0x10000 * rank)

    def make_comm(k):
        """One communicator per frame slot (created in slot order on every rank: RCCL's init is collective)."""
        if not tiled:
            return None
        if a.dist_backend == "nccl":
            uid = [svtgpu.Comm.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            # bounded init: a rank that died after the broadcast makes the others fail with the slot named
            c = svtgpu.Comm.rccl(ctx, n, rank, uid[0], timeout_ms=a.comm_timeout_ms, slot=k)
        else:
            grp = dist.new_group(backend="gloo")

            def allreduce(words, timeout_ms):  # bounded by the communicator's deadline
                w = dist.all_reduce(torch.from_numpy(words.view(np.int64)), group=grp, async_op=True)
                w.wait(timeout=datetime.timedelta(milliseconds=timeout_ms))
            c = svtgpu.Comm.host(n, rank, allreduce)
        # every exchange bounded: a rank whose peer never arrives exits non-zero with the exchange named
        c.set_timeout(a.comm_timeout_ms)
        c.set_slot(k)
        return c

    lib_streams = []

    def frame_stream():
        """A frame slot's stream: made by the library (svtgpu_stream_create), one hardware queue each, wrapped for
        torch's events; --torch-streams: torch.cuda.Stream() (its pool of 32 streams per priority puts the process
        past GPU_MAX_HW_QUEUES, and the queues later streams share then depend on creation order: 1080p 10-bit F = 4
        1870 vs 2440 Mpx/s)."""
        if a.torch_streams:
            return torch.cuda.Stream()
        p = ctx.stream_create(0)
        lib_streams.append(p)
        return torch.cuda.ExternalStream(p)

    class Slot:
        """One frame in flight: its own input frames, stage states, streams and (tiles) communicator."""

        def __init__(self, k, tplan=None, comm=None, md_range=None):
            """tplan: this rank's SvtGpuTilePlan rects (a tiled picture; comm its communicator), None: the whole frame.
            md_range: the MD batch's superblock range (default: all)."""
            self.k = k
            self.stream = frame_stream()     # the library launches on it, torch events time it
            # the MD batch (memory-bound) runs beside the VALU-bound LR search on its own stream, or (--md-main) on the
            # main stream: one hardware queue less per frame in flight
            self.md_stream = self.stream if a.md_main else frame_stream()
            sp = self.stream.cuda_stream
            self.src, self.rec = frame_inputs(k)
            self.R, self.S, self.D, self.O, self.L = (svtgpu.Frame(ctx, W, H, bd) for _ in range(5))
            # a rank of a tiled picture receives only the part of the inputs its calls read (the plan's in_rect)
            inr = tplan["in_rect"] if tplan else None
            self.R.upload(self.rec, sp, rect=inr)
            self.S.upload(self.src, sp, rect=inr)
            self.in_rect = inr
            self.dl = svtgpu.DlfState(ctx, W, H)
            self.lr = svtgpu.LrState(ctx, W, H, lr_us)
            self.md = svtgpu.MdBatch(ctx, W, H, NREF)
            self.md_mvs = np.random.default_rng(5 + k).integers(-16, 17, size=(self.md.nsb, NREF, 2))
            self.md.set_mvs(self.md_mvs, sp)
            self.st = svtgpu.CdefState(ctx, W, H)
            self.comm = comm
            if tplan:
                self.dl.set_tile(tplan["tile"], tplan["dlf_out"], comm)
                self.st.set_tile(tplan["fb_rect"], tplan["cdef_out"], comm)
                self.lr.set_tile(tplan["lr_units"], tplan["lr_out"], comm)
            self.md_range = md_range or (0, self.md.nsb)
            self.ev = []  # per timed step: events on the streams the kernels run on
            self.ht = []  # --host-timing: per timed step, {call: (wall ms, thread CPU ms)}
            self.lf_levels = []
            self.inflight = []  # completion events of the steps this slot's thread has enqueued
            self.at_lr = threading.Event()  # this slot's step has reached its LR stage (staggers the next slot)

        def close(self):
            for x in (self.R, self.S, self.D, self.O, self.L, self.dl, self.lr, self.md, self.st, self.comm):
                if x is not None and hasattr(x, "close"):
                    x.close()

        def step(self, timed):
            torch.cuda.set_stream(self.stream)  # per thread
            stream, md_stream, sp = self.stream, self.md_stream, self.stream.cuda_stream
            R, S, D, O, L, st, lr, dl = self.R, self.S, self.D, self.O, self.L, self.st, self.lr, self.dl
            es = [torch.cuda.Event(enable_timing=True) for _ in range(9)] if timed else None
            if timed:
                es[0].record(stream)
            if a.stages == "cdef":  # CDEF search + pick + apply on the recon (configs 1/2); events keep the layout
                if timed:
                    es[1].record(stream)
                st.search(R, S, ctrls, q, sp)
                if timed:
                    es[2].record(stream)
                if a.cdef_sync:
                    prm, _ = st.pick(ctrls, q, lam, sp)
                else:
                    st.pick_async(ctrls, q, lam, sp)
                    prm = None
                st.apply(R, O, prm, sp)
                self.at_lr.set()
                if timed:
                    for i in (8, 3, 4, 5):
                        es[i].record(stream)
                    es[6].record(stream), es[7].record(stream)
                    self.ev.append(es)
                return
            # the frame's mode info: upload + edge records; DLF level search + frame filter
            hc = HostClock(timed and a.host_timing)
            dl.set_mode_info_device(mi_dev, sp)
            hc("mode_info")
            if a.dlf_sync:
                lfp = dl.pick(R, S, lf_start, dlf_avg=0, dlf_avg_uv=0, temporal_layer_index=0, early_exit=0, stream=sp)
                hc("dlf_pick")
                dl.filter_to(R, D, lfp, 0, 3, sp)
            else:  # the bisection on the device, the filter with its levels: no host wait in the DLF stage
                dl.pick_async(R, S, lf_start, dlf_avg=0, dlf_avg_uv=0, temporal_layer_index=0, early_exit=0, stream=sp)
                hc("dlf_pick")
                dl.filter_to(R, D, None, 0, 3, sp)
            hc("dlf_filter")
            if timed:
                es[1].record(stream)
                if a.dlf_sync:
                    self.lf_levels.append(lfp.levels())
            # CDEF stage on the deblocked frame (tiles: this rank's filter blocks; the pick sums the tables)
            st.search(D, S, ctrls, q, sp)
            hc("cdef_search")
            if timed:
                es[2].record(stream)
            if a.cdef_sync:
                prm, _ = st.pick(ctrls, q, lam, sp)
            else:  # the strength search and RD choice in stream order, the apply reading their result on the device
                st.pick_async(ctrls, q, lam, sp)
                prm = None
            hc("cdef_pick")
            if timed:
                es[8].record(stream)
            st.apply(D, O, prm, sp)
            hc("cdef_apply")
            if timed:
                es[3].record(stream)
            # MD distortion batch (source vs 7 references, every block shape): independent of the filter chain, on
            # its own stream from here to the end of the step
            md_stream.wait_stream(stream)
            if timed:
                es[6].record(md_stream)
            self.md.run(S, md_refs, self.md_range[0], self.md_range[1], md_stream.cuda_stream)
            hc("md")
            if timed:
                es[7].record(md_stream)
            # LR search + apply on the CDEF output (tiles: this rank's units; the records are summed before the
            # finish) with the boundary lines from the DLF output
            self.at_lr.set()
            if a.lr_sync:
                lr_ft = lr.search(O, S, lr_ctrls, sp)
                hc("lr_search")
                lr.apply(D, O, L, lr_ft, sp)
            else:  # search, device RD finish and apply in stream order: no host wait in the LR stage
                lr.search_async(O, S, lr_ctrls, sp)
                hc("lr_search")
                lr.apply(D, O, L, None, sp)
            hc("lr_apply")
            if hc.on:
                self.ht.append(hc.t)
            if timed:
                es[4].record(stream)
            stream.wait_stream(md_stream)  # the step ends when both streams are done
            if timed:
                es[5].record(stream)
                self.ev.append(es)
            # with no host wait inside a step the thread runs ahead of its stream: at most two steps enqueued
            done = torch.cuda.Event()
            done.record(stream)
            self.inflight.append(done)
            if len(self.inflight) > a.run_ahead:
                self.inflight.pop(0).synchronize()

    F = a.frames_in_flight
    if emu_rank is not None:
        slots = [Slot(k, plan, svtgpu.Comm.rccl(ctx, 1, 0, svtgpu.Comm.unique_id()),
                      svtgpu.band(md_nsb, a.emulate_rank, emu_rank)) for k in range(F)]
    else:
        slots = [Slot(k, plan, make_comm(k), svtgpu.band(md_nsb, n, rank)) if tiled else Slot(k) for k in range(F)]
    torch.cuda.synchronize()
    lr = slots[0].lr
    # host -> device bytes of a frame's inputs (recon + source + mode-info grid; resident before timing) and their
    # PCIe-inclusive upload rate from pageable host memory, measured once here
    s0 = slots[0]
    t_up = time.perf_counter()
    for _ in range(3):
        s0.R.upload(s0.rec, s0.stream.cuda_stream)
        s0.S.upload(s0.src, s0.stream.cuda_stream)
        if a.stages == "all":
            s0.dl.set_mode_info(mi, s0.stream.cuda_stream)
    torch.cuda.synchronize()
    up_s = (time.perf_counter() - t_up) / 3
    in_bytes = sum(p.nbytes for p in s0.rec) + sum(p.nbytes for p in s0.src) + (mi_bytes if a.stages == "all" else 0)

    errors = []

    def run(slot, steps, timed, slots=slots):
        t_start = time.perf_counter()
        try:
            # frame k starts when frame k - 1 reaches its LR stage: the frames stay offset by part of a frame, so one's
            # VALU-bound search overlaps the other's latency-bound stages (started together they run in lockstep and
            # contend for the same units)
            if slot.k > 0:
                slots[slot.k - 1].at_lr.wait(60)  # bounded: a failed slot must not hang the next
            for _ in range(steps):
                slot.step(timed)
            slot.wall_ms = (time.perf_counter() - t_start) * 1e3  # the thread's enqueue span (its last waits included)
        except BaseException as e:  # re-raised on the main thread
            errors.append(e)

    def run_all(steps, timed, slots=slots):
        for sl in slots:
            sl.at_lr.clear()
        if len(slots) == 1:
            run(slots[0], steps, timed, slots)
        else:
            th = [threading.Thread(target=run, args=(sl, steps, timed, slots)) for sl in slots]
            for t in th:
                t.start()
            for t in th:
                t.join()
        if errors:
            raise errors[0]

    if a.lr_serial:
        for s_ in slots:
            s_.lr.profile([], serial=True)
    run_all(a.warmup, False)
    svtgpu.transfer_bytes(reset=True)
    # LR search kernel classes timed on the device clock over the timed steps (first WG start -> last WG end
    # of every launch, accumulated on the device and read once after the timed region) -- slot 0's searches
    lr.profile(not a.no_kernel_timing, serial=a.lr_serial)
    torch.cuda.synchronize()
    if n > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_all(a.steps, True)
    torch.cuda.synchronize()
    if n > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if a.stages == "all" and not a.lr_sync:  # the asynchronous searches' results: a device-side failure raises here
        for sl in slots:
            sl.lr.read_result(sl.stream.cuda_stream)
    dlf_rounds = None
    if a.stages in ("all", "cdef") and not a.cdef_sync:  # every slot's last asynchronous pick (errors raise)
        for sl in slots:
            sl.cdef_last = sl.st.read_params(sl.stream.cuda_stream)[0]
    if a.stages == "all" and not a.dlf_sync:  # the last asynchronous level search of every slot
        for sl in slots:
            sl.lf_levels.append(sl.dl.read_levels(sl.stream.cuda_stream).levels())
        dlf_rounds = slots[0].dl.async_rounds()
    lr_tot = lr.profile(False) if not a.no_kernel_timing else None
    h2d, d2h = svtgpu.transfer_bytes(reset=True)
    if n > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    stage_ms = np.mean([[es[i].elapsed_time(es[i + 1]) for i in range(4)] + [es[6].elapsed_time(es[7])]
                        for es in slots[0].ev], axis=0)
    frame_ms = float(np.mean([es[0].elapsed_time(es[5]) for es in slots[0].ev]))
    # frames really in flight: the sum over the slots of their mean frame latency over the step time (F when every
    # frame overlaps the others for the whole step); round 5's collapse read 2.3 of 6 with unchanged latencies
    slot_lat = [float(np.mean([es[0].elapsed_time(es[5]) for es in sl.ev])) for sl in slots if sl.ev]
    ht_main = list(slots[0].ht)  # --host-timing: the main run's (the iso phase below appends its own)
    dlf_ms, search_ms, cdef_rest_ms, lr_ms, md_ms = (float(x) for x in stage_ms)

    ms_per_step = dt * 1e3 / a.steps
    concurrency = sum(slot_lat) / ms_per_step if slot_lat else None
    if concurrency is not None and F > 1 and concurrency < F / 2:
        print("bench: WARNING: frames in flight overlap poorly: concurrency %.2f of %d (slot latencies %s ms, step %.2f "
              "ms) -- frames are serializing (shared hardware queues?)" % (concurrency, F,
              [round(x, 2) for x in slot_lat], ms_per_step), file=sys.stderr)
    frames_per_step = F * (1 if tiled else n)  # frames split: every rank filters F frames per step
    value = frames_per_step * W * H / (ms_per_step * 1e-3) / 1e6  # the whole job's luma pixels per second
    def lr_classes(tot):
        return {c: {k: tot[c][k] / max(tot["searches"], 1) if tot else 0.0
                    for k in ("launches", "ms", "ms_events", "bytes")}
                for c in svtgpu.LrState.PROFILE_CLASSES}
    lr_cls = lr_classes(lr_tot)
    # SURVEY §8(d) algorithmic bytes; per rank: its share of the frame (tiles)
    S_samples = 1.5 * W * H
    B = 2 if bd > 8 else 1
    share = 1.0
    if tiled:
        t_ = plan["tile"]
        share = (t_[2] - t_[0]) * (t_[3] - t_[1]) / float(W * H)
    SB = S_samples * B * share
    st0 = slots[0].st
    nfb_mine = st0.nfb * share
    nsb = ((W + 63) // 64) * ((H + 63) // 64)
    nsb_mine = slots[0].md_range[1] - slots[0].md_range[0]
    cdef_alg = 2 * SB + nfb_mine * (2 * 64 * 8 + 64 + 64 * 4 + 1)

    def kernel_table(search_ms_, md_ms_, lr_cls_, have_lr):
        kernels = {"cdef_search_kernel": dict(ms=search_ms_, launches=1, alg_bytes=cdef_alg,
                                              what="recon + source read once, 2*S*B, + the per-FB mse/dir/var/skip "
                                                   "outputs")}
        if a.stages == "all":
            kernels["md_dist_kernel"] = dict(ms=md_ms_, launches=1, alg_bytes=nsb_mine * (1 + NREF) * 64 * 64 * B,
                                             what="(1 + refs) x 64 x 64 x B per superblock")
            if have_lr:
                lr_kern = {"wiener_trials": ("wiener_res_kernel", 2 * SB, "the CDEF output and source of the searched "
                                                                          "planes read once, 2*S*B"),
                           "sgr_filters": ("sgr_flt_kernel", SB, "the CDEF output read once, S*B"),
                           "projection": ("sgr_res_kernel", 2 * SB, "the CDEF output and source read once, 2*S*B")}
                for cls, (kn, alg, what) in lr_kern.items():
                    c = lr_cls_[cls]
                    if c["launches"] > 0:  # HIP events around each launch (rocprofv3's span); the device clock beside
                        kernels[kn] = dict(ms=c["ms_events"] or c["ms"], ms_clock=c["ms"], launches=c["launches"],
                                           alg_bytes=alg, what=what)
        return kernels
    kernels_f = kernel_table(search_ms, md_ms, lr_cls, bool(lr_tot))
    # The roofline's durations come from the condition its PMC counters were collected in: one frame in flight
    # (scripts/r5/pmc_r05.sh runs the bench at F = 1 with the LR chains serial).  With F > 1 slot 0 runs alone for a short timed phase after the
    # main one; the contended figures of the F-frame run are reported beside it.
    iso = None
    if F > 1:
        s0 = slots[0]
        s0.ev = []
        # the roofline's launch spans: HIP events around each launch (rocprofv3's span), the two LR chains one after
        # the other so that each kernel's duration is its own (beside the other chain, a resident descent's duration
        # is mostly its wait for the CUs the other chain's descent holds)
        lr.profile(not a.no_kernel_timing, events=True, serial=True)
        iso_steps = max(10, min(a.steps, 40))
        torch.cuda.synchronize()
        for _ in range(iso_steps):
            s0.step(True)
        torch.cuda.synchronize()
        iso_tot = lr.profile(False) if not a.no_kernel_timing else None
        iso_ms = np.mean([[es[i].elapsed_time(es[i + 1]) for i in range(4)] + [es[6].elapsed_time(es[7])]
                          for es in s0.ev], axis=0)
        iso = dict(steps=iso_steps, frame_ms=float(np.mean([es[0].elapsed_time(es[5]) for es in s0.ev])),
                   kernels=kernel_table(float(iso_ms[1]), float(iso_ms[4]), lr_classes(iso_tot), bool(iso_tot)))
    roof = roofline_of(iso["kernels"] if iso else kernels_f, bd, a.pmc_json)
    roof["condition"] = ("one frame in flight (slot 0 alone, %d timed steps after the main run, the LR search's two "
                         "chains one after the other; the PMC counters' condition)" % iso["steps"]) if iso else \
        "one frame in flight (the main run%s)" % (", LR chains serial" if a.lr_serial else "")
    if iso:
        cont = roofline_of(kernels_f, bd, a.pmc_json)
        roof["contended"] = {"frames_in_flight": F, "kernel": cont["kernel"], "avg_launch_ms": cont["avg_launch_ms"],
                             "ms_per_frame": cont["ms_per_frame"], "achieved": cont["achieved"], "frac": cont["frac"],
                             "all_kernels_ms_per_frame": cont["all_kernels_ms_per_frame"],
                             "note": "the same accounting over the main run's %d frames in flight: kernels share the "
                                     "CUs with the other frames' kernels, so launch durations include queueing" % F}
    # SURVEY §8(d) algorithmic bytes per frame by stage, over slot 0's stage times (HIP events; with several frames in
    # flight the stages share the device with the other frames), and the pipeline total over the wall time per frame
    stage_bytes = {"dlf_pick_filter": 2 * SB, "cdef_search": cdef_alg, "cdef_pick_apply": 2 * SB,
                   "lr_search_apply": 4 * SB, "md_sad_sse_var": nsb_mine * (1 + NREF) * 64 * 64 * B}
    stage_t = {"dlf_pick_filter": dlf_ms, "cdef_search": search_ms, "cdef_pick_apply": cdef_rest_ms,
               "lr_search_apply": lr_ms, "md_sad_sse_var": md_ms}
    stage_roof = {k: {"alg_MB": round(stage_bytes[k] / 1e6, 2), "ms": round(stage_t[k], 4),
                      "frac": round(stage_bytes[k] / max(stage_t[k], 1e-9) * 1e-6 / HBM_PEAK_GBS, 5)}
                  for k in stage_bytes if a.stages == "all" or k in ("cdef_search", "cdef_pick_apply")}
    pipe_bytes = (10 if a.stages == "all" else 4) * S_samples * B
    frame_wall_ms = ms_per_step / frames_per_step
    pipe_roof = {"alg_MB_per_frame": round(pipe_bytes / 1e6, 2), "ms_per_frame": round(frame_wall_ms, 4),
                 "achieved_GBs": round(pipe_bytes / (frame_wall_ms * 1e-3) / 1e9, 2),
                 "frac": round(pipe_bytes / (frame_wall_ms * 1e-3) / 1e9 / HBM_PEAK_GBS / max(n if tiled else 1, 1), 5),
                 "definition": "SURVEY §8(d): %s per frame, each input read once and each output written once; over the "
                               "whole job's wall time per frame%s" % ("10*S*B" if a.stages == "all" else "4*S*B",
                                                                      ", against N x 8 TB/s" if tiled else "")}
    nfr_timed = a.steps * F
    xfer = {"h2d_bytes_per_frame": round(h2d / nfr_timed), "d2h_bytes_per_frame": round(d2h / nfr_timed),
            "input_bytes_per_frame": in_bytes,
            "input_upload_ms": round(up_s * 1e3, 3),
            "input_upload_GBs": round(in_bytes / up_s / 1e9, 2),
            "pcie_inclusive_Mpx_s": round(W * H / (frame_wall_ms * 1e-3 + up_s) / 1e6, 2) if n == 1 else None,
            "note": "h2d/d2h: host<->device bytes of the frame-level entry points during the timed steps on this rank "
                    "(DLF trial SSEs, CDEF pick, LR records and units); the frame inputs (recon + source + the "
                    "mode-info grid, input_bytes_per_frame) are resident before timing -- an encoder uploads them "
                    "per frame at input_upload_GBs (pageable host memory, measured here), giving "
                    "pcie_inclusive_Mpx_s if the upload were serialized with the step (never `value`)"}
    if tiled:
        xfer["rccl_exchange_bytes_per_frame"] = {
            "cdef_tables": st0.nfb * (2 * 64 * 8 + 64 + 64 * 4) + ((st0.nfb + 7) // 8) * 8,
            "lr_records": sum(hu * vu for hu, vu in lr.units) * svtgpu.LR_UNIT_SEARCH_DTYPE.itemsize,
            "dlf_trial_sses": "6 x 8 B per bisection step"}
    out = {
        "metric": "CDEF+restoration+SAD Mpixels/s on 4K10b",
        "value": round(value, 3),
        "unit": "Mpixels/s",
        "n_gpus": n,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak" if (n > 1 and not tiled) else "strong",
        "vs_baseline": None,
        "dtype": "u16" if bd > 8 else "u8",
        "data": "synthetic",
        "config": {"workload": "mode info -> dlf_pick+filter -> cdef_search+pick+apply -> lr_search+apply, + md batch; "
                               "%dx%d %d-bit 4:2:0, dlf level 1 (full-image search), cdef_level %d (%d strengths); MD "
                               "SAD/SSE/var 7 refs x 849 blocks/SB; LR search+apply (RU %d/%d, wn/sg level 1)"
                               % (W, H, bd, a.cdef_level, len(ctrls.strengths()), lr_us[0], lr_us[1]),
                   "inputs": ("the reference-pinned pipeline case %s (integer generator seed %#x, base_q_idx %d, start "
                              "levels %s, CDEF lambda %d; tests/golden/pipe_%s.npz)" %
                              (pin["case"], pin["seed"], q, cfg["lf"], lam, pin["case"])) if pin else
                             "synthetic, unpinned (%s generator)" % ("integer" if a.inputs == "pinned" else "float"),
                   "width": W, "height": H, "bit_depth": bd, "frames_per_step": frames_per_step,
                   "frames_in_flight": F, "frame_latency_ms": round(frame_ms, 4), "ranks_requested": a.gpus,
                   "concurrency": {"value": round(concurrency, 3) if concurrency is not None else None,
                                   "slot_latency_ms": [round(x, 3) for x in slot_lat],
                                   "slot_wall_ms": [round(getattr(sl, "wall_ms", 0.0), 2) for sl in slots],
                                   "streams_per_frame": 2 if a.md_main else 3,
                                   "stream_source": "torch.cuda.Stream (pool)" if a.torch_streams
                                   else "svtgpu_stream_create",
                                   "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                                   "low": bool(concurrency is not None and F > 1 and concurrency < F / 2),
                                   "note": "sum over the frame slots of their mean frame latency / step time"},
                   "lr_search_mode": "sync (host wait)" if a.lr_sync else "async (device RD finish, no host wait)",
                   "cdef_pick_mode": "sync (host waits: settle check, strengths)" if a.cdef_sync
                   else "async (device settle flag and parameters, no host wait)",
                   "dlf_search_mode": "sync (host-driven bisection)" if a.dlf_sync
                   else "async (device bisection, no host wait; trial rounds taken / enqueued %s)" % (dlf_rounds,),
                   "ranks": n,
                   "parallelism": ("tiles%dx%d (each frame tiled over the ranks: DLF trials/filter, CDEF search/apply, "
                                   "LR search/apply per tile; RCCL sums of the DLF trial SSEs, CDEF tables, LR records "
                                   "through libsvtgpu's communicator; MD by SB ranges)" % (gx, gy) if tiled
                                   else "frames%d (each rank filters its own pictures; no data-path collective)" % n
                                   if n > 1 else "single"),
                   "tile": plan["tile"] if tiled else None,
                   "stage_ms": {"dlf_pick_filter": round(dlf_ms, 4), "cdef_search": round(search_ms, 4),
                                "cdef_pick_apply": round(cdef_rest_ms, 4), "lr_search_apply": round(lr_ms, 4),
                                "md_sad_sse_var": round(md_ms, 4),
                                "note": "slot 0, rank 0, HIP events; dlf_pick_filter includes the mode-info upload and "
                                        "edge records; the MD batch runs on a second stream concurrently with the LR "
                                        "stage; the LR search runs its Wiener and self-guided chains on two streams"},
                   "lr_search_kernel_ms": {c: round(v["ms"], 4) for c, v in lr_cls.items()},
                   "dlf_levels": list(slots[0].lf_levels[-1]) if slots[0].lf_levels else None,
                   "tile_projection": projection,
                   "stage_roofline": stage_roof, "pipeline_roofline": pipe_roof, "transfers": xfer},
        "roofline": roof,
    }
    if a.stages == "cdef":
        out["config"]["workload"] = ("cdef_search+pick+apply on the recon (SURVEY §8d configs 1/2); %dx%d %d-bit 4:2:0, "
                                     "cdef_level %d (%d strengths)" % (W, H, bd, a.cdef_level, len(ctrls.strengths())))
        out["metric"] = "CDEF search+apply Mpixels/s"
        out["config"].pop("lr_search_kernel_ms")
    if matrix is not None:
        out["config"]["matrix"] = matrix
    if a.host_timing and ht_main:
        def host_table(ht):
            return {k: [round(float(np.mean([t[k][0] for t in ht])), 4), round(float(np.mean([t[k][1] for t in ht])), 4)]
                    for k in ht[0]}
        out["config"]["host_ms"] = host_table(ht_main)
        out["config"]["host_ms"]["note"] = ("slot 0 per timed step: [wall ms, thread CPU ms] in each call, %d frames in "
                                            "flight" % F)
        if iso and len(slots[0].ht) > len(ht_main):
            out["config"]["host_ms_f1"] = host_table(slots[0].ht[len(ht_main):])
    if emu_rank is not None:
        tl = plan["tile"]
        out["config"]["emulated"] = {"ranks": a.emulate_rank, "rank": emu_rank, "tile": tl,
                                     "grid": "%dx%d" % svtgpu.tile_grid(a.emulate_rank),
                                     "tile_share": round((tl[2] - tl[0]) * (tl[3] - tl[1]) / float(W * H), 4),
                                     "cdef_pick_ms": round(float(np.mean([es[2].elapsed_time(es[8])
                                                                          for es in slots[0].ev])), 4),
                                     "note": "this GPU ran one rank of an N-GPU tiled picture alone (one-rank RCCL "
                                             "communicators: every exchange issued, none over xGMI); value = F x W x H "
                                             "/ this rank's step time, the N-GPU job's rate up to the collectives' "
                                             "latency"}
    if rank == 0 and n == 1 and a.stages == "all" and not a.no_matrix:
        out["config"]["next_rows"] = measure_next_rows(ctx, torch, W, H)
    if rank == 0 and n == 1 and not a.no_cpu_baseline:
        s0 = slots[0]
        if a.cpu_kind == "reference" and os.path.exists(REF_BENCH):
            out["cpu_baseline"] = cpu_baseline_reference(s0.src, s0.rec, mi, ctrls, bd, a.cdef_level, q, lam,
                                                         a.cpu_grid, lr_ctrls, md_ref_y, s0.md_mvs, a.cpu_passes,
                                                         cfg["lf"], a.stages)
        else:
            out["cpu_baseline"] = cpu_baseline(s0.src, s0.rec, mi, lf_start, bd, a.cdef_level, q, lam, a.cpu_grid,
                                               lr_ctrls, lr_us, md_ref_y, s0.md_mvs)
    if rank == 0:
        print(json.dumps(out), flush=True)
    for sl in slots:
        if sl.comm is not None:
            sl.comm.close()
    torch.cuda.synchronize()
    for p in lib_streams:
        svtgpu.Context.stream_destroy(p)
    if n > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
