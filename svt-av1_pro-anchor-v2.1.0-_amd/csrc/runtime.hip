// runtime.hip — device/context/frame management of the C ABI (include/svtgpu.h).
#include <atomic>
#include <cstdio>
#include <vector>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <mutex>

#include "svtgpu_internal.h"

static thread_local char g_last_err[512];

void svtgpu_set_last_hip_error(hipError_t e, const char *what, const char *file, int line) {
    snprintf(g_last_err, sizeof g_last_err, "%s failed: %s (%s:%d)", what, hipGetErrorString(e), file, line);
}

void svtgpu_fatal(const char *what) {
    fprintf(stderr, "svtgpu: fatal: %s: %s\n", what, g_last_err[0] ? g_last_err : "(no detail)");
    abort();
}

extern "C" const char *svtgpu_version(void) { return SVTGPU_VERSION_STR; }
extern "C" int32_t svtgpu_abi_version(void) { return SVTGPU_ABI_VERSION; }

extern "C" const char *svtgpu_error_string(int code) {
    switch (code) {
    case SVTGPU_OK: return "ok";
    case SVTGPU_ERR_INVALID_ARG: return "invalid argument";
    case SVTGPU_ERR_HIP: return g_last_err[0] ? g_last_err : "HIP error";
    case SVTGPU_ERR_UNSUPPORTED: return "unsupported configuration";
    case SVTGPU_ERR_NO_DEVICE: return "no gfx950 device";
    case SVTGPU_ERR_OOM: return "out of device memory";
    default: return "unknown error";
    }
}

extern "C" int svtgpu_device_available(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return 0;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess)
        return 0;
    return strncmp(p.gcnArchName, "gfx950", 6) == 0;
}

extern "C" int svtgpu_context_create(int device, SvtGpuContext **out) {
    if (!out)
        return SVTGPU_ERR_INVALID_ARG;
    *out  = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
        return SVTGPU_ERR_NO_DEVICE;
    HIP_TRY(hipSetDevice(device));
    auto *c   = new SvtGpuContext;
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return SVTGPU_ERR_HIP;
    }
    *out = c;
    return SVTGPU_OK;
}

extern "C" void svtgpu_context_destroy(SvtGpuContext *ctx) {
    if (!ctx)
        return;
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

extern "C" void *svtgpu_context_stream(SvtGpuContext *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

// A caller's stream for the frame-level calls, created here in the caller's order (priority > 0: the device's
// highest, < 0: its lowest, 0: normal).  Every stream is one hardware queue while there are no more streams than
// GPU_MAX_HW_QUEUES, and beyond that streams share queues in order -- a frame's chain then waits behind another frame's
// on the shared queue.  A framework's stream pool (torch.cuda.Stream() draws from 32 streams per priority created at
// once) puts the process past that count before the first frame runs, which made the queue that each later stream
// got depend on when it was created (round 6: 1080p 10-bit at four frames in flight 1870 vs 2440 Mpx/s for the same
// streams created at state creation or at the first search).  A caller that creates exactly the streams it runs
// frames on gets one queue each.
extern "C" int svtgpu_stream_create(SvtGpuContext *ctx, int32_t priority, void **out) {
    if (!ctx || !out) return SVTGPU_ERR_INVALID_ARG;
    *out = nullptr;
    HIP_TRY(hipSetDevice(ctx->device));
    int least = 0, greatest = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
    hipStream_t s = nullptr;
    if (priority == 0)
        HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    else
        HIP_TRY(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority > 0 ? greatest : least));
    *out = (void *)s;
    return SVTGPU_OK;
}

extern "C" void svtgpu_stream_destroy(void *stream) {
    if (!stream) return;
    (void)hipStreamSynchronize((hipStream_t)stream);
    (void)hipStreamDestroy((hipStream_t)stream);
}

// Plain device buffers for the pointer-level entry points (CCSO, plane conversion) when the caller has no allocator of
// its own: hipMalloc / hipFree and stream-ordered copies that are complete when they return.
extern "C" int svtgpu_buffer_alloc(SvtGpuContext *ctx, size_t bytes, void **out) {
    if (!ctx || !out || !bytes) return SVTGPU_ERR_INVALID_ARG;
    *out = nullptr;
    HIP_TRY(hipSetDevice(ctx->device));
    if (hipMalloc(out, bytes) != hipSuccess) return *out = nullptr, SVTGPU_ERR_OOM;
    return SVTGPU_OK;
}
extern "C" void svtgpu_buffer_free(void *dev) { (void)hipFree(dev); }
extern "C" int  svtgpu_buffer_upload(void *dev, const void *host, size_t bytes, void *stream) {
    if (!dev || !host) return SVTGPU_ERR_INVALID_ARG;
    hipStream_t st = stream ? (hipStream_t)stream : svtgpu_default_stream();
    HIP_TRY(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    svtgpu_count_xfer(0, bytes);
    return SVTGPU_OK;
}
extern "C" int svtgpu_buffer_download(void *host, const void *dev, size_t bytes, void *stream) {
    if (!dev || !host) return SVTGPU_ERR_INVALID_ARG;
    hipStream_t st = stream ? (hipStream_t)stream : svtgpu_default_stream();
    HIP_TRY(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    svtgpu_count_xfer(1, bytes);
    return SVTGPU_OK;
}

// Test support (the exchange deadline's abort path): one wave that spins on the 100 MHz s_memrealtime clock for `ms`
// milliseconds (at most 10 s; every lane leaves at the same bound), holding `stream` busy.
__global__ void stall_kernel(unsigned long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}
extern "C" int svtgpu_debug_stall(SvtGpuContext *ctx, void *stream, int32_t ms) {
    if (!ctx || ms < 0 || ms > 10000) return SVTGPU_ERR_INVALID_ARG;
    hipLaunchKernelGGL(stall_kernel, dim3(1), dim3(64), 0, pick_stream(ctx, stream), 100000ull * (unsigned)ms);
    HIP_TRY(hipGetLastError());
    return SVTGPU_OK;
}

extern "C" int svtgpu_synchronize(SvtGpuContext *ctx, void *stream) {
    if (!ctx)
        return SVTGPU_ERR_INVALID_ARG;
    HIP_TRY(hipStreamSynchronize(pick_stream(ctx, stream)));
    return SVTGPU_OK;
}

// process-wide context used by the per-block RTCD shims (they have no context argument)
static std::once_flag g_default_once;
static SvtGpuContext *g_default_ctx = nullptr;
SvtGpuContext        *svtgpu_default_context() {
    std::call_once(g_default_once, [] {
        if (!svtgpu_device_available()) {
            snprintf(g_last_err, sizeof g_last_err, "no gfx950 device visible");
            return;
        }
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (svtgpu_context_create(dev, &g_default_ctx) != SVTGPU_OK)
            g_default_ctx = nullptr;
    });
    if (!g_default_ctx)
        svtgpu_fatal("svtgpu per-block shim called without a usable gfx950 device");
    return g_default_ctx;
}
// every per-block shim launches on the default context's stream; each shim entry point takes it once through
// svtgpu_shim_stream, which counts the shim calls (svtgpu_shim_calls) -- frame-level calls with a null stream and the
// communicator's waits use svtgpu_default_stream and are not counted
static std::atomic<unsigned long long> g_shim_calls{0};
hipStream_t svtgpu_default_stream() { return svtgpu_default_context()->stream; }
hipStream_t svtgpu_shim_stream() {
    g_shim_calls.fetch_add(1, std::memory_order_relaxed);
    return svtgpu_default_context()->stream;
}
extern "C" uint64_t svtgpu_shim_calls(void) { return g_shim_calls.load(); }

static std::atomic<unsigned long long> g_xfer[2];
void svtgpu_count_xfer(int d2h, size_t bytes) { g_xfer[d2h ? 1 : 0] += bytes; }
extern "C" int svtgpu_transfer_bytes(uint64_t *h2d, uint64_t *d2h, int32_t reset) {
    if (h2d) *h2d = g_xfer[0].load();
    if (d2h) *d2h = g_xfer[1].load();
    if (reset) g_xfer[0] = 0, g_xfer[1] = 0;
    return SVTGPU_OK;
}

// Off by default: measured (profiles/r04/hiprio) the lanes made every configuration slower -- 4K 10-bit at one frame
// in flight 2210 vs 2307 Mpx/s, at four 2526 vs 2870, the emulated 8-GPU rank 2248 vs 4478 -- the dispatcher's
// high-priority queue does not win CU slots from resident kernels that hold every VGPR of a CU.  SVTGPU_HIPRIO=1.
static bool prio_lanes_on() {
    static const bool on = [] {
        const char *e = std::getenv("SVTGPU_HIPRIO");
        return e && e[0] == '1';
    }();
    return on;
}

int svtgpu_prio_enter(SvtGpuPrioLane *l, hipStream_t st, hipStream_t *out) {
    *out = st;
    if (!prio_lanes_on()) return SVTGPU_OK;
    if (!l->hs) {
        int least = 0, greatest = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
        HIP_TRY(hipStreamCreateWithPriority(&l->hs, hipStreamNonBlocking, greatest));
        HIP_TRY(hipEventCreateWithFlags(&l->fork, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&l->join, hipEventDisableTiming));
    }
    HIP_TRY(hipEventRecord(l->fork, st));
    HIP_TRY(hipStreamWaitEvent(l->hs, l->fork, 0));
    *out = l->hs;
    return SVTGPU_OK;
}

int svtgpu_prio_leave(SvtGpuPrioLane *l, hipStream_t hs, hipStream_t st) {
    if (hs == st) return SVTGPU_OK;
    HIP_TRY(hipEventRecord(l->join, hs));
    HIP_TRY(hipStreamWaitEvent(st, l->join, 0));
    return SVTGPU_OK;
}

void svtgpu_prio_destroy(SvtGpuPrioLane *l) {
    if (l->hs) (void)hipStreamDestroy(l->hs);
    if (l->fork) (void)hipEventDestroy(l->fork);
    if (l->join) (void)hipEventDestroy(l->join);
    l->hs = nullptr, l->fork = l->join = nullptr;
}

int svtgpu_wait_seq(const volatile unsigned long long *flag, unsigned long long seq, hipStream_t st) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 0;; it++) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return SVTGPU_OK;
        // after ~2 ms of spinning (a long kernel, or a failed launch) hand over to the runtime's wait
        if ((it & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
    }
    HIP_TRY(hipStreamSynchronize(st));
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
        svtgpu_set_last_hip_error(hipErrorUnknown, "device result word missing after stream synchronize", __FILE__,
                                  __LINE__);
        return SVTGPU_ERR_HIP;
    }
    return SVTGPU_OK;
}

// ---------------------------------------------------------------------------------------------
// frames
// ---------------------------------------------------------------------------------------------
extern "C" int svtgpu_frame_create(SvtGpuContext *ctx, int32_t width, int32_t height, int32_t bit_depth,
                                   SvtGpuFrame **out) {
    if (!ctx || !out || width <= 0 || height <= 0 || (width & 7) || (height & 7))
        return SVTGPU_ERR_INVALID_ARG;
    if (bit_depth != 8 && bit_depth != 10)
        return SVTGPU_ERR_UNSUPPORTED;
    auto *f             = new SvtGpuFrame;
    f->ctx              = ctx;
    f->width            = width;
    f->height           = height;
    f->bit_depth        = bit_depth;
    f->bytes_per_sample = bit_depth > 8 ? 2 : 1;
    size_t off[3], total = 0;
    for (int p = 0; p < 3; p++) {
        f->pw[p] = p ? width / 2 : width;
        f->ph[p] = p ? height / 2 : height;
        // rows padded to 256 B so every row starts 256-B aligned (coalesced 16-B lane loads)
        const size_t row_bytes = ((size_t)f->pw[p] * f->bytes_per_sample + 255) & ~(size_t)255;
        f->stride[p]           = (int32_t)(row_bytes / f->bytes_per_sample);
        off[p]                 = total;
        total += row_bytes * f->ph[p];
    }
    if (hipMalloc(&f->base, total) != hipSuccess) {
        delete f;
        return SVTGPU_ERR_OOM;
    }
    for (int p = 0; p < 3; p++) f->plane[p] = (char *)f->base + off[p];
    *out = f;
    return SVTGPU_OK;
}

extern "C" void svtgpu_frame_destroy(SvtGpuFrame *f) {
    if (!f)
        return;
    (void)hipFree(f->base);
    delete f;
}

extern "C" int32_t svtgpu_frame_stride(const SvtGpuFrame *f, int plane) {
    return (f && plane >= 0 && plane < 3) ? f->stride[plane] : -1;
}
extern "C" void *svtgpu_frame_plane_ptr(SvtGpuFrame *f, int plane) {
    return (f && plane >= 0 && plane < 3) ? f->plane[plane] : nullptr;
}

extern "C" int svtgpu_frame_upload(SvtGpuFrame *f, int plane, const void *host, int32_t host_stride, void *stream) {
    if (!f || !host || plane < 0 || plane > 2 || host_stride < f->pw[plane])
        return SVTGPU_ERR_INVALID_ARG;
    const size_t b = f->bytes_per_sample;
    HIP_TRY(hipMemcpy2DAsync(f->plane[plane], f->stride[plane] * b, host, host_stride * b, f->pw[plane] * b,
                             f->ph[plane], hipMemcpyHostToDevice, pick_stream(f->ctx, stream)));
    return SVTGPU_OK;
}

extern "C" int svtgpu_frame_upload_rect(SvtGpuFrame *f, int plane, const void *host, int32_t host_stride,
                                        const int32_t rect[4], void *stream) {
    if (!f || !host || !rect || plane < 0 || plane > 2 || host_stride < f->pw[plane] || rect[0] < 0 || rect[1] < 0 ||
        rect[2] > f->pw[plane] || rect[3] > f->ph[plane] || rect[0] > rect[2] || rect[1] > rect[3])
        return SVTGPU_ERR_INVALID_ARG;
    if (rect[0] == rect[2] || rect[1] == rect[3]) return SVTGPU_OK;
    const size_t b = f->bytes_per_sample;
    svtgpu_count_xfer(0, (size_t)(rect[2] - rect[0]) * (rect[3] - rect[1]) * b);
    HIP_TRY(hipMemcpy2DAsync((uint8_t *)f->plane[plane] + ((size_t)rect[1] * f->stride[plane] + rect[0]) * b,
                             f->stride[plane] * b,
                             (const uint8_t *)host + ((size_t)rect[1] * host_stride + rect[0]) * b, host_stride * b,
                             (size_t)(rect[2] - rect[0]) * b, rect[3] - rect[1], hipMemcpyHostToDevice,
                             pick_stream(f->ctx, stream)));
    return SVTGPU_OK;
}

extern "C" int svtgpu_frame_download(const SvtGpuFrame *f, int plane, void *host, int32_t host_stride, void *stream) {
    if (!f || !host || plane < 0 || plane > 2 || host_stride < f->pw[plane])
        return SVTGPU_ERR_INVALID_ARG;
    const size_t b  = f->bytes_per_sample;
    hipStream_t  st = pick_stream(f->ctx, stream);
    HIP_TRY(hipMemcpy2DAsync(host, host_stride * b, f->plane[plane], f->stride[plane] * b, f->pw[plane] * b,
                             f->ph[plane], hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return SVTGPU_OK;
}

extern "C" int svtgpu_frame_copy(SvtGpuFrame *dst, const SvtGpuFrame *src, void *stream) {
    if (!dst || !src || dst->width != src->width || dst->height != src->height || dst->bit_depth != src->bit_depth)
        return SVTGPU_ERR_INVALID_ARG;
    const size_t b = src->bytes_per_sample;
    for (int p = 0; p < 3; p++)
        HIP_TRY(hipMemcpy2DAsync(dst->plane[p], dst->stride[p] * b, src->plane[p], src->stride[p] * b, src->pw[p] * b,
                                 src->ph[p], hipMemcpyDeviceToDevice, pick_stream(dst->ctx, stream)));
    return SVTGPU_OK;
}

// ---- diagnostics: per-workgroup clocks (svtgpu_internal.h wgclk_mark) ----
namespace {
unsigned long long *g_wgclk     = nullptr;
size_t              g_wgclk_cap = 0;
} // namespace
unsigned long long *svtgpu_wgclk_begin(int nblocks) {
    static const char *path = std::getenv("SVTGPU_WGCLK");
    if (!path || nblocks <= 0) return nullptr;
    const size_t bytes = 64 * (size_t)nblocks;
    if (bytes > g_wgclk_cap) {
        if (g_wgclk) (void)hipFree(g_wgclk);
        g_wgclk = nullptr, g_wgclk_cap = 0;
        if (hipMalloc(&g_wgclk, bytes) != hipSuccess) return nullptr;
        g_wgclk_cap = bytes;
    }
    (void)hipMemset(g_wgclk, 0, bytes);
    return g_wgclk;
}
void svtgpu_wgclk_end(const char *kernel, int nblocks, hipStream_t st) {
    static const char *path = std::getenv("SVTGPU_WGCLK");
    if (!path || !g_wgclk || nblocks <= 0) return;
    std::vector<unsigned long long> h(8 * (size_t)nblocks);
    if (hipStreamSynchronize(st) != hipSuccess ||
        hipMemcpy(h.data(), g_wgclk, 64 * (size_t)nblocks, hipMemcpyDeviceToHost) != hipSuccess)
        return;
    if (FILE *f = std::fopen(path, "ab")) {
        char name[64] = {0};
        std::strncpy(name, kernel, sizeof name - 1);
        const long long n = nblocks;
        std::fwrite(name, 1, sizeof name, f);
        std::fwrite(&n, 8, 1, f);
        std::fwrite(h.data(), 8, h.size(), f);
        std::fclose(f);
    }
}
