// Calibration of the TCC FETCH_SIZE / WRITE_SIZE counters for the access widths the LR and CDEF kernels use
// (2, 4, 8 and 16 bytes per lane, coalesced rows).  Each read launch streams BYTES from a buffer 4x the size of the
// Infinity Cache, so every byte comes from HBM once; the write launch stores BYTES with 16-B lanes.  Run under
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./fetch_cal      (and a second pass with WRITE_SIZE)
// and divide the counter (KB) by the known byte count.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr size_t BYTES = size_t(1) << 30;

template <typename V>
__global__ __launch_bounds__(256) void read_w(const V *__restrict__ p, size_t n, uint32_t *out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const V x = p[i];
        const uint32_t *w = (const uint32_t *)&x;
        if constexpr (sizeof(V) >= 4) {
#pragma unroll
            for (unsigned k = 0; k < sizeof(V) / 4; k++) acc ^= w[k];
        } else {
            acc ^= (uint32_t)x;
        }
    }
    if (acc == (uint32_t)n + 1u) out[blockIdx.x] = acc; // a run-time comparison keeps every load; never true here
}

__global__ __launch_bounds__(256) void write_16(uint4 *p, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

int main() {
    void     *buf;
    uint32_t *out;
    if (hipMalloc(&buf, BYTES) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
    hipMemset(buf, 1, BYTES);
    const int grid = 256 * 16;
    for (int rep = 0; rep < 2; rep++) {
        read_w<uint16_t><<<grid, 256>>>((const uint16_t *)buf, BYTES / 2, out);
        read_w<uint32_t><<<grid, 256>>>((const uint32_t *)buf, BYTES / 4, out);
        read_w<uint2><<<grid, 256>>>((const uint2 *)buf, BYTES / 8, out);
        read_w<uint4><<<grid, 256>>>((const uint4 *)buf, BYTES / 16, out);
        write_16<<<grid, 256>>>((uint4 *)buf, BYTES / 16);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("bytes per launch %zu (%.1f KB)\n", BYTES, BYTES / 1024.0);
    hipFree(buf);
    hipFree(out);
    return 0;
}
