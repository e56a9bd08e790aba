// Microbenchmark: issue rate of v_dot2_i32_i16 vs v_mad_i32_i24 (dev tool)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef short v2i16 __attribute__((ext_vector_type(2)));
__device__ inline int dot2(uint32_t a, uint32_t b, int c) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, a), __builtin_bit_cast(v2i16, b), c, false);
}
template <int MODE>
__global__ __launch_bounds__(256) void k(int *out, uint32_t a0, uint32_t b0, int n) {
    int acc[8];
    uint32_t a = a0 + threadIdx.x, b = b0 ^ threadIdx.x;
    for (int j = 0; j < 8; j++) acc[j] = j;
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (MODE == 0) acc[j] = dot2(a + j, b, acc[j]);
            else if (MODE == 1) acc[j] = __mul24((int)(a + j), (int)b) + acc[j];
            else acc[j] = (int)((a + j) * b) + acc[j];
        }
        a = a * 3 + 1;
    }
    int s = 0;
    for (int j = 0; j < 8; j++) s += acc[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
    int *o;
    (void)hipMalloc(&o, 4 << 20);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0), (void)hipEventCreate(&e1);
    const int n = 4096, grid = 256 * 8;
    auto run = [&](auto kern, const char *name) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, o, 1u, 2u, n);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, o, 1u, 2u, n);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double ops = (double)grid * 256 * n * 8; // lane-ops
        printf("%-12s %.3f ms  %.1f Gop/s (lane ops)  %.2f lane-ops/clk/CU @2.4GHz\n", name, ms, ops / ms / 1e6,
               ops / (ms * 1e-3) / 256 / 2.4e9);
    };
    run(k<0>, "dot2");
    run(k<1>, "mad_i24");
    run(k<2>, "mul_lo+add");
    return 0;
}
