// comm.hip — the frame-level exchanges of a picture tiled over several GPUs (BASELINE.json config 4).
//
// One communicator per frame in flight and rank; every exchange of the path is an element-wise sum of uint64 words
// over the ranks:
//   * DLF level search: the trial SSEs of the rank's tile (search_filter_level, EbDeblockingFilter.c:886-991, sums
//     picture_sse_calculations over the whole frame; the tiles partition it);
//   * CDEF pick: the zero-padded mse / skip / dir / var tables of the rank's filter blocks (cdef_seg_search's
//     per-segment outputs gathered for finish_cdef_search, EbCdefProcess.c:114 / EbEncCdef.c:728): one contributor
//     per entry, so the word sums are the gather;
//   * LR finish: the zero-padded per-unit search records (restoration_seg_search's outputs gathered for
//     rest_finish_search, EbRestorationPick.c:1471 / :1555).
// Two transports behind one object:
//   * RCCL over xGMI (ncclAllReduce on the caller's stream, buffers in device memory) — the GPU path;
//   * a host transport supplied by the caller (a function that sums uint64 words over the ranks, e.g. an MPI or gloo
//     binding): device buffers are staged through pinned host memory.  Used by the CPU-side rehearsals and by tests
//     that run several ranks on one GPU (RCCL refuses two ranks on one device).
//
// Every exchange is bounded (round 5): a rank whose peer never arrives (a skipped exchange, a peer that failed before
// its all-reduce) must not hang the node.  The device-side collectives are enqueued without a host wait (the CDEF
// tables before the pick, the DLF trial SSEs between a trial and its step kernel), so each one is noted in a small ring
// (what, sequence number, stream -- no event: a marker packet per exchange lengthened the tiled rank's latency chains),
// and every host wait of a frame-level call that may sit behind a collective goes through svtgpu_comm_wait: one event
// on the waited stream, polled against the communicator's deadline; when it expires with exchanges of that stream
// outstanding it names the oldest (what, frame slot, sequence number), aborts the RCCL communicator (ncclCommAbort ends
// the pending collectives on this rank) and returns SVTGPU_ERR_HIP; the communicator then fails every later call.
// A host transport gets the deadline from svtgpu_comm_timeout_ms and reports an expired wait by returning non-zero.
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <thread>

#include "svtgpu_internal.h"

namespace {
constexpr int XCH_RING = 32;
struct XchRecord {
    hipStream_t st   = nullptr; // the stream the collective was enqueued on
    const char *what = nullptr;
    uint64_t    seq  = 0;
    size_t      words = 0;
    bool        live = false;
};
int default_timeout_ms() {
    static const int v = [] {
        const char *e = std::getenv("SVTGPU_COMM_TIMEOUT_MS");
        const int   t = e ? std::atoi(e) : 0;
        return t > 0 ? t : 60000;
    }();
    return v;
}
} // namespace

struct SvtGpuComm {
    int32_t             nranks = 1, rank = 0;
    ncclComm_t          nccl   = nullptr;
    SvtGpuHostTransport host{};
    bool                is_host = false;
    uint64_t           *pin = nullptr; // host staging (host transport: device buffers; RCCL: host buffers go via dev)
    size_t              pin_words = 0;
    uint64_t           *dev = nullptr; // device staging of host buffers (RCCL)
    size_t              dev_words = 0;
    int                 device = 0;
    int32_t             timeout_ms = 0;  // deadline of every exchange
    int32_t             slot       = -1; // the frame slot it serves (error messages only)
    uint64_t            seq        = 0;  // exchanges issued
    bool                failed     = false;
    bool                nonblocking = false; // created with ncclConfig_t::blocking = 0: calls may return ncclInProgress
    char                fail_msg[320] = {0};
    XchRecord           ring[XCH_RING]; // the device-side collectives not yet seen complete
    hipEvent_t          wait_ev = nullptr;
};

namespace {
int nccl_fail(ncclResult_t r, const char *what) {
    char msg[256];
    std::snprintf(msg, sizeof msg, "%s: %s", what, ncclGetErrorString(r));
    svtgpu_set_last_hip_error(hipErrorUnknown, msg, __FILE__, __LINE__);
    return SVTGPU_ERR_HIP;
}
int grow_pin(SvtGpuComm *c, size_t n) {
    if (n <= c->pin_words) return SVTGPU_OK;
    if (c->pin) (void)hipHostFree(c->pin);
    c->pin = nullptr, c->pin_words = 0;
    HIP_TRY(hipHostMalloc((void **)&c->pin, n * 8, hipHostMallocDefault));
    c->pin_words = n;
    return SVTGPU_OK;
}
// a communicator that timed out (or whose RCCL call failed) fails every later call with the first message
int comm_failed(SvtGpuComm *c) {
    svtgpu_set_last_hip_error(hipErrorUnknown, c->fail_msg, __FILE__, __LINE__);
    return SVTGPU_ERR_HIP;
}
void slot_str(const SvtGpuComm *c, char *b, size_t n) {
    if (c->slot >= 0) std::snprintf(b, n, "frame slot %d", c->slot);
    else std::snprintf(b, n, "frame slot unset");
}
// the deadline expired with `r` outstanding: name it, abort RCCL, fail from now on
int comm_timeout(SvtGpuComm *c, const XchRecord &r, long long waited_ms) {
    char sl[32];
    slot_str(c, sl, sizeof sl);
    std::snprintf(c->fail_msg, sizeof c->fail_msg,
                  "exchange timed out: the all-reduce of the %s (%s, rank %d of %d, exchange #%llu, %zu words) did not "
                  "complete within %d ms (detected after %lld ms) -- a peer rank skipped or never reached it; RCCL "
                  "communicator aborted",
                  r.what, sl, c->rank, c->nranks, (unsigned long long)r.seq, r.words, c->timeout_ms, waited_ms);
    c->failed = true;
    if (c->nccl) (void)ncclCommAbort(c->nccl); // ends this rank's pending collectives
    c->nccl = nullptr;
    return comm_failed(c);
}
// the oldest exchange enqueued on `st` not yet seen complete; else the oldest one enqueued on any other stream (a wait
// on another stream can reach it through events: the CDEF pick's priority lane waits behind the caller's stream,
// ADVICE r5), or null
const XchRecord *outstanding(SvtGpuComm *c, hipStream_t st) {
    const XchRecord *oldest = nullptr, *other = nullptr;
    for (auto &r : c->ring) {
        if (!r.live) continue;
        if (r.st == st) {
            if (!oldest || r.seq < oldest->seq) oldest = &r;
        } else if (!other || r.seq < other->seq) {
            other = &r;
        }
    }
    return oldest ? oldest : other;
}
// RCCL calls of a non-blocking communicator may return ncclInProgress: poll its state against the deadline
ncclResult_t nccl_settle(ncclComm_t comm, ncclResult_t r, int timeout_ms, long long *waited_ms) {
    const auto t0 = std::chrono::steady_clock::now();
    *waited_ms    = 0;
    while (r == ncclInProgress) {
        const auto w = std::chrono::steady_clock::now() - t0;
        *waited_ms   = std::chrono::duration_cast<std::chrono::milliseconds>(w).count();
        if (*waited_ms > timeout_ms) return ncclInProgress;
        std::this_thread::yield();
        if (ncclResult_t q = ncclCommGetAsyncError(comm, &r)) return q;
    }
    return r;
}
int grow_dev(SvtGpuComm *c, size_t n) {
    if (n <= c->dev_words) return SVTGPU_OK;
    if (c->dev) (void)hipFree(c->dev);
    c->dev = nullptr, c->dev_words = 0;
    HIP_TRY(hipMalloc((void **)&c->dev, n * 8));
    c->dev_words = n;
    return SVTGPU_OK;
}
} // namespace

extern "C" int svtgpu_comm_unique_id(uint8_t id[SVTGPU_COMM_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == SVTGPU_COMM_ID_BYTES, "ncclUniqueId is 128 bytes");
    if (!id) return SVTGPU_ERR_INVALID_ARG;
    ncclUniqueId u;
    if (ncclResult_t r = ncclGetUniqueId(&u)) return nccl_fail(r, "ncclGetUniqueId");
    std::memcpy(id, &u, sizeof u);
    return SVTGPU_OK;
}

// Communicator creation is bounded like the exchanges: a non-blocking ncclCommInitRankConfig polled with
// ncclCommGetAsyncError against the deadline, so a rank whose peer died between the id broadcast and its init returns
// a named error instead of blocking in the bootstrap until the job is killed.  SVTGPU_COMM_INIT=blocking: the plain
// blocking ncclCommInitRank (A/B).
extern "C" int svtgpu_comm_create_bounded(SvtGpuContext *ctx, int32_t nranks, int32_t rank,
                                          const uint8_t id[SVTGPU_COMM_ID_BYTES], int32_t timeout_ms, int32_t slot,
                                          SvtGpuComm **out) {
    if (!ctx || !id || !out || nranks < 1 || rank < 0 || rank >= nranks || timeout_ms < 0) return SVTGPU_ERR_INVALID_ARG;
    static const bool blocking = [] {
        const char *e = std::getenv("SVTGPU_COMM_INIT");
        return e && !std::strcmp(e, "blocking");
    }();
    const int tmo = timeout_ms > 0 ? timeout_ms : default_timeout_ms();
    HIP_TRY(hipSetDevice(ctx->device));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    ncclComm_t comm = nullptr;
    if (blocking) {
        if (ncclResult_t r = ncclCommInitRank(&comm, nranks, u, rank)) return nccl_fail(r, "ncclCommInitRank");
    } else {
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking     = 0;
        ncclResult_t r   = ncclCommInitRankConfig(&comm, nranks, u, rank, &cfg);
        long long    waited = 0;
        if (r == ncclInProgress && comm) r = nccl_settle(comm, r, tmo, &waited);
        if (r != ncclSuccess) {
            char msg[320];
            if (r == ncclInProgress)
                std::snprintf(msg, sizeof msg,
                              "communicator init timed out: frame slot %d, rank %d of %d did not complete "
                              "ncclCommInitRankConfig within %d ms (waited %lld ms) -- a peer rank never joined; "
                              "RCCL communicator aborted", slot, rank, nranks, tmo, waited);
            else
                std::snprintf(msg, sizeof msg, "communicator init failed: frame slot %d, rank %d of %d: %s", slot, rank,
                              nranks, ncclGetErrorString(r));
            if (comm) (void)ncclCommAbort(comm);
            svtgpu_set_last_hip_error(hipErrorUnknown, msg, __FILE__, __LINE__);
            return SVTGPU_ERR_HIP;
        }
    }
    auto *c   = new SvtGpuComm();
    c->nranks = nranks, c->rank = rank, c->nccl = comm, c->device = ctx->device;
    c->timeout_ms = tmo, c->slot = slot;
    c->nonblocking = !blocking;
    if (hipEventCreateWithFlags(&c->wait_ev, hipEventDisableTiming) != hipSuccess) {
        svtgpu_comm_destroy(c);
        svtgpu_set_last_hip_error(hipErrorOutOfMemory, "comm event", __FILE__, __LINE__);
        return SVTGPU_ERR_HIP;
    }
    *out      = c;
    return SVTGPU_OK;
}

extern "C" int svtgpu_comm_create(SvtGpuContext *ctx, int32_t nranks, int32_t rank,
                                  const uint8_t id[SVTGPU_COMM_ID_BYTES], SvtGpuComm **out) {
    return svtgpu_comm_create_bounded(ctx, nranks, rank, id, 0, -1, out);
}

extern "C" int svtgpu_comm_create_host(int32_t nranks, int32_t rank, const SvtGpuHostTransport *t, SvtGpuComm **out) {
    if (!t || !t->allreduce_u64 || !out || nranks < 1 || rank < 0 || rank >= nranks) return SVTGPU_ERR_INVALID_ARG;
    auto *c    = new SvtGpuComm();
    c->nranks  = nranks, c->rank = rank, c->host = *t, c->is_host = true;
    c->timeout_ms = default_timeout_ms();
    *out       = c;
    return SVTGPU_OK;
}

extern "C" void svtgpu_comm_destroy(SvtGpuComm *c) {
    if (!c) return;
    if (c->nccl) (void)ncclCommDestroy(c->nccl);
    if (c->wait_ev) (void)hipEventDestroy(c->wait_ev);
    if (c->pin) (void)hipHostFree(c->pin);
    if (c->dev) (void)hipFree(c->dev);
    delete c;
}

extern "C" int32_t svtgpu_comm_nranks(const SvtGpuComm *c) { return c ? c->nranks : 0; }
bool svtgpu_comm_tiled(const SvtGpuComm *c) { return c && (c->nranks > 1 || !c->is_host); }
extern "C" int32_t svtgpu_comm_rank(const SvtGpuComm *c) { return c ? c->rank : -1; }

extern "C" int svtgpu_comm_set_timeout(SvtGpuComm *c, int32_t timeout_ms) {
    if (!c || timeout_ms <= 0) return SVTGPU_ERR_INVALID_ARG;
    c->timeout_ms = timeout_ms;
    return SVTGPU_OK;
}
extern "C" int32_t svtgpu_comm_timeout_ms(const SvtGpuComm *c) { return c ? c->timeout_ms : 0; }
extern "C" int svtgpu_comm_set_slot(SvtGpuComm *c, int32_t slot) {
    if (!c) return SVTGPU_ERR_INVALID_ARG;
    c->slot = slot;
    return SVTGPU_OK;
}
extern "C" int32_t svtgpu_comm_failed(const SvtGpuComm *c) { return c && c->failed ? 1 : 0; }

// Host wait for `st` bounded by the communicator's deadline while one of its device-side collectives is outstanding
// (any stream: the caller's waits reach the collective through stream order or events).  No communicator, a host
// transport (its sums are synchronous) or nothing outstanding: the runtime's own wait.
int svtgpu_comm_wait(SvtGpuComm *c, hipStream_t st) {
    static const bool plain = [] { // SVTGPU_COMM_WAIT=sync (diagnostic A/B): an unbounded stream synchronize
        const char *e = std::getenv("SVTGPU_COMM_WAIT");
        return e && !std::strcmp(e, "sync");
    }();
    const XchRecord *r = c && !c->is_host && !plain ? outstanding(c, st) : nullptr;
    if (!r) {
        HIP_TRY(hipStreamSynchronize(st));
        return SVTGPU_OK;
    }
    HIP_TRY(hipEventRecord(c->wait_ev, st));
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 0;; it++) {
        const hipError_t q = hipEventQuery(c->wait_ev);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) HIP_TRY(q);
        if ((it & 63) != 63) continue;
        const auto waited = std::chrono::steady_clock::now() - t0;
        if (waited > std::chrono::milliseconds(c->timeout_ms))
            return comm_timeout(c, *r, std::chrono::duration_cast<std::chrono::milliseconds>(waited).count());
        std::this_thread::yield();
    }
    for (auto &x : c->ring) // everything enqueued on `st` before the event has completed
        if (x.live && x.st == st) x.live = false;
    return SVTGPU_OK;
}


extern "C" int svtgpu_comm_sync(SvtGpuComm *c, void *stream) {
    if (!c) return SVTGPU_ERR_INVALID_ARG;
    if (c->failed) return comm_failed(c);
    return svtgpu_comm_wait(c, stream ? (hipStream_t)stream : svtgpu_default_stream());
}

// The element-wise sum of n uint64 over the ranks, in place.  Device buffers: enqueued on `st` (RCCL) or staged through
// host memory with a synchronization (host transport).  Host buffers: synchronous either way.
// A one-rank host transport is the identity and returns at once; a one-rank RCCL communicator still runs the
// collective (the same code path, transfers and stream ordering as the N-GPU run).
int svtgpu_comm_sum(SvtGpuComm *c, void *buf, size_t n, bool on_device, hipStream_t st, const char *what) {
    if (!c || n == 0 || (c->nranks == 1 && c->is_host)) return SVTGPU_OK;
    if (!buf) return SVTGPU_ERR_INVALID_ARG;
    if (c->failed) return comm_failed(c);
    const uint64_t seq = ++c->seq;
    if (c->is_host) {
        uint64_t *h = (uint64_t *)buf;
        if (on_device) {
            if (int rc = grow_pin(c, n)) return rc;
            HIP_TRY(hipMemcpyAsync(c->pin, buf, n * 8, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            h = c->pin;
        }
        if (c->host.allreduce_u64(c->host.user, h, n) != 0) {
            char sl[32];
            slot_str(c, sl, sizeof sl);
            std::snprintf(c->fail_msg, sizeof c->fail_msg,
                          "exchange failed: the host-transport all-reduce of the %s (%s, rank %d of %d, exchange #%llu, "
                          "%zu words) returned an error or timed out (deadline %d ms)",
                          what, sl, c->rank, c->nranks, (unsigned long long)seq, n, c->timeout_ms);
            c->failed = true;
            return comm_failed(c);
        }
        if (on_device) { // the pinned staging is reused by the next sum, maybe from another stream: wait for the copy
            HIP_TRY(hipMemcpyAsync(buf, c->pin, n * 8, hipMemcpyHostToDevice, st));
            HIP_TRY(hipStreamSynchronize(st));
        }
        return SVTGPU_OK;
    }
    // the ring slot of this exchange: an exchange 32 back not yet seen complete is waited for (bounded) first, before
    // this one is enqueued (so the wait, and a timeout's message, concern the older exchange only)
    XchRecord *slot = &c->ring[seq % XCH_RING];
    if (slot->live)
        if (int rc = svtgpu_comm_wait(c, slot->st)) return rc;
    slot->live = false;
    void *d = buf;
    if (!on_device) {
        if (int rc = grow_dev(c, n)) return rc;
        HIP_TRY(hipMemcpyAsync(c->dev, buf, n * 8, hipMemcpyHostToDevice, st));
        d = c->dev;
    }
    ncclResult_t r = ncclAllReduce(d, d, n, ncclUint64, ncclSum, c->nccl, st);
    long long    waited = 0;
    if (r == ncclInProgress && c->nonblocking) r = nccl_settle(c->nccl, r, c->timeout_ms, &waited);
    if (r != ncclSuccess) {
        XchRecord me;
        me.what = what, me.seq = seq, me.words = n, me.st = st;
        if (r == ncclInProgress) return comm_timeout(c, me, waited); // never enqueued within the deadline
        std::snprintf(c->fail_msg, sizeof c->fail_msg, "ncclAllReduce of the %s (exchange #%llu): %s", what,
                      (unsigned long long)seq, ncclGetErrorString(r));
        c->failed = true;
        return comm_failed(c);
    }
    slot->st = st, slot->what = what, slot->seq = seq, slot->words = n, slot->live = true;
    if (!on_device) {
        HIP_TRY(hipMemcpyAsync(buf, c->dev, n * 8, hipMemcpyDeviceToHost, st));
        return svtgpu_comm_wait(c, st);
    }
    return SVTGPU_OK;
}

extern "C" int svtgpu_comm_allreduce_u64(SvtGpuComm *c, void *buf, size_t n, int32_t on_device, void *stream) {
    if (!c) return SVTGPU_ERR_INVALID_ARG;
    // a host transport on host memory touches no device (usable without a GPU)
    hipStream_t st = stream ? (hipStream_t)stream : (c->is_host && !on_device) ? nullptr : svtgpu_default_stream();
    return svtgpu_comm_sum(c, buf, n, on_device != 0, st, "caller's words (svtgpu_comm_allreduce_u64)");
}

// ---------------------------------------------------------------------------------------------
// tile plan (host only)
// ---------------------------------------------------------------------------------------------
namespace {
int units_of(int size, int extent) { return std::max((extent + (size >> 1)) / size, 1); } // count_units_in_tile
int split_at(int n, int k, int i) { return (int)((long long)n * i / k); }
void grow(int32_t *r, int a, int w, int h) {
    r[0] = std::max(0, r[0] - a), r[1] = std::max(0, r[1] - a);
    r[2] = std::min(w, r[2] + a), r[3] = std::min(h, r[3] + a);
}
} // namespace

// A picture whose crop size (the restored area, frm_size.frame_width x frame_height) is smaller than its 8-aligned coded
// size: the deblocking and CDEF frames are the coded size, the restoration units tile the crop (chroma rounded up, the
// reference's crop_widths).  The tiles' edges stay on the luma unit grid; the last tile column / row runs to the coded
// edge, the last unit to the crop edge.
extern "C" int svtgpu_tile_plan_crop(int32_t width, int32_t height, int32_t crop_w, int32_t crop_h,
                                     const int32_t unit_size[3], int32_t sb_size, int32_t gx, int32_t gy, int32_t rank,
                                     SvtGpuTilePlan *out) {
    if (!unit_size || !out || width <= 0 || height <= 0 || (width & 7) || (height & 7) || gx < 1 || gy < 1 ||
        rank < 0 || rank >= gx * gy || (sb_size != 64 && sb_size != 128) || crop_w <= 0 || crop_h <= 0 ||
        crop_w > width || crop_h > height || width - crop_w >= 8 || height - crop_h >= 8)
        return SVTGPU_ERR_INVALID_ARG;
    for (int p = 0; p < 3; p++)
        if (unit_size[p] < (p ? 32 : 64) || unit_size[p] > 256 || (unit_size[p] & (unit_size[p] - 1)))
            return SVTGPU_ERR_INVALID_ARG;
    SvtGpuTilePlan o;
    std::memset(&o, 0, sizeof o);
    const int tx = rank % gx, ty = rank / gx, U = unit_size[0];
    const int nux = units_of(U, crop_w), nuy = units_of(U, crop_h);
    // tile edges on the unit grid and on the superblock grid: with 64-sample units in a SB128 picture the units go in
    // pairs, so no 128x128 CDEF area (searched as one, EbCdefProcess.c:193-196) is cut
    const int k = std::max(1, sb_size / U), gux = (nux + k - 1) / k, guy = (nuy + k - 1) / k;
    if (gux < gx || guy < gy) return SVTGPU_ERR_INVALID_ARG; // a rank without a unit
    const int c0 = std::min(nux, k * split_at(gux, gx, tx)), c1 = std::min(nux, k * split_at(gux, gx, tx + 1));
    const int r0 = std::min(nuy, k * split_at(guy, gy, ty)), r1 = std::min(nuy, k * split_at(guy, gy, ty + 1));
    // the tile: unit-grid edges (multiples of 64: filter-block edges too); the frame edge closes the last tile
    o.tile[0] = c0 * U, o.tile[1] = r0 * U;
    o.tile[2] = c1 == nux ? width : c1 * U, o.tile[3] = r1 == nuy ? height : r1 * U;
    o.fb_rect[0] = o.tile[0] / 64, o.fb_rect[1] = o.tile[1] / 64;
    o.fb_rect[2] = (o.tile[2] + 63) / 64, o.fb_rect[3] = (o.tile[3] + 63) / 64;
    for (int p = 0; p < 3; p++) {
        const int pw = p ? (crop_w + 1) / 2 : crop_w, ph = p ? (crop_h + 1) / 2 : crop_h, up = unit_size[p], off = p ? 4 : 8;
        const int hx = units_of(up, pw), hy = units_of(up, ph);
        // the luma unit columns / rows when the plane's unit grid matches luma's (chroma units of half the luma size),
        // else an even split of the plane's own grid
        const bool same = hx == nux && hy == nuy;
        const int  a0 = same ? c0 : split_at(hx, gx, tx), a1 = same ? c1 : split_at(hx, gx, tx + 1);
        const int  b0 = same ? r0 : split_at(hy, gy, ty), b1 = same ? r1 : split_at(hy, gy, ty + 1);
        if (a0 >= a1 || b0 >= b1) return SVTGPU_ERR_INVALID_ARG;
        o.lr_units[p][0] = a0, o.lr_units[p][1] = b0, o.lr_units[p][2] = a1, o.lr_units[p][3] = b1;
        // the units' samples: columns [a0 U, a1 U) (the last unit to the plane edge), rows start RESTORATION_UNIT_OFFSET
        // above the unit grid (foreach_rest_unit_in_tile, EbRestoration.c:1257-1294)
        o.lr_out[p][0] = a0 * up, o.lr_out[p][2] = a1 == hx ? pw : a1 * up;
        o.lr_out[p][1] = b0 == 0 ? 0 : b0 * up - off, o.lr_out[p][3] = b1 == hy ? ph : b1 * up - off;
    }
    // CDEF output read by the LR search / apply of these units: 3 samples around them (8: whole 8x8 blocks); chroma
    // units map onto the same luma area when the grids match, else take their bounding box
    int32_t c[4];
    std::memcpy(c, o.lr_out[0], sizeof c);
    for (int p = 1; p < 3; p++) {
        c[0] = std::min(c[0], 2 * o.lr_out[p][0]), c[1] = std::min(c[1], 2 * o.lr_out[p][1]);
        c[2] = std::max(c[2], std::min(width, 2 * o.lr_out[p][2])), c[3] = std::max(c[3], std::min(height, 2 * o.lr_out[p][3]));
    }
    grow(c, 8, width, height);
    std::memcpy(o.cdef_out, c, sizeof c);
    // DLF output read by the CDEF search of the tile's filter blocks and by the CDEF apply / LR boundary lines above
    int32_t d[4] = {std::min(c[0], o.tile[0]), std::min(c[1], o.tile[1]), std::max(c[2], o.tile[2]),
                    std::max(c[3], o.tile[3])};
    grow(d, 8, width, height);
    std::memcpy(o.dlf_out, d, sizeof d);
    grow(d, 16, width, height); // the deblocking filter reads up to 8 samples across an edge of the written area
    std::memcpy(o.in_rect, d, sizeof d);
    *out = o;
    return SVTGPU_OK;
}

extern "C" int svtgpu_tile_plan_sb(int32_t width, int32_t height, const int32_t unit_size[3], int32_t sb_size,
                                   int32_t gx, int32_t gy, int32_t rank, SvtGpuTilePlan *out) {
    return svtgpu_tile_plan_crop(width, height, width, height, unit_size, sb_size, gx, gy, rank, out);
}

extern "C" int svtgpu_tile_plan(int32_t width, int32_t height, const int32_t unit_size[3], int32_t gx, int32_t gy,
                                int32_t rank, SvtGpuTilePlan *out) {
    return svtgpu_tile_plan_sb(width, height, unit_size, 64, gx, gy, rank, out);
}
