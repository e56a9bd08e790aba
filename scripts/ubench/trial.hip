// Microbenchmark: where does a Wiener trial round spend its time?  (dev tool, not part of the library)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef short v2i16 __attribute__((ext_vector_type(2)));
__device__ inline int dot2(uint32_t a, uint32_t b, int c) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, a), __builtin_bit_cast(v2i16, b), c, false);
}
__device__ inline uint32_t pack2(int lo, int hi) { return (uint32_t)(lo & 0xFFFF) | ((uint32_t)hi << 16); }
struct Tile { int x0, y0, w, h; };

template <int MODE>
__global__ __launch_bounds__(256) void trial(const uint16_t *d, const uint16_t *s, int stride, int W, int H,
                                             const Tile *tiles, int n, const int16_t *taps, unsigned long long *err) {
    constexpr int VS = 72;
    __shared__ __align__(16) uint16_t v[71 * VS];
    __shared__ __align__(16) uint32_t tq[36 * 64];
    for (int it = blockIdx.x; it < n; it += gridDim.x) {
        const Tile t = tiles[it];
        int h[8], w[8];
        for (int k = 0; k < 8; k++) h[k] = taps[k], w[k] = taps[8 + k];
        const uint32_t He[4] = {pack2(0, h[0]), pack2(h[1], h[2]), pack2(h[3], h[4]), pack2(h[5], h[6])};
        const uint32_t Ho[4] = {pack2(h[0], h[1]), pack2(h[2], h[3]), pack2(h[4], h[5]), pack2(h[6], h[7])};
        const uint32_t Ve[4] = {pack2(w[0], w[1]), pack2(w[2], w[3]), pack2(w[4], w[5]), pack2(w[6], w[7])};
        const uint32_t Vo[4] = {pack2(0, w[0]), pack2(w[1], w[2]), pack2(w[3], w[4]), pack2(w[5], w[6])};
        __syncthreads();
        const int rows = t.h + 7, ng = (t.w + 8) >> 2, nyp = (t.h + 1) >> 1;
        if (MODE != 2) {
            for (int k = 0; k < 5; k++) {
                const int i = threadIdx.x + k * 256, r = i / 18, g = i - r * 18;
                if (r >= rows || g >= ng) continue;
                int yy = t.y0 + r - 3, xx = t.x0 - 4 + 4 * g;
                yy = min(max(yy, 0), H - 1);
                xx = min(max(xx, 0), W - 4);
                const uint2 q = *(const uint2 *)(d + (size_t)yy * stride + xx);
                *(uint2 *)(v + r * VS + 4 * g) = q;
            }
        }
        __syncthreads();
        unsigned long long e = 0;
        if (MODE != 1) {
            uint16_t *tq16 = (uint16_t *)tq;
            const int xh = 2 * (threadIdx.x & 31);
            for (int r = threadIdx.x >> 5; r < rows; r += 8) {
                const uint32_t *pr = (const uint32_t *)(v + r * VS + xh);
                const uint32_t p0 = pr[0], p1 = pr[1], p2 = pr[2], p3 = pr[3], p4 = pr[4];
                const int s0 = dot2(p0, He[0], dot2(p1, He[1], dot2(p2, He[2], dot2(p3, He[3], 4096 + (int)((p2 & 0xFFFF) << 7)))));
                const int s1 = dot2(p1, Ho[0], dot2(p2, Ho[1], dot2(p3, Ho[2], dot2(p4, Ho[3], 4096 + (int)((p2 >> 16) << 7)))));
                const int o = ((r >> 1) * 64 + xh) * 2 + (r & 1);
                tq16[o] = (uint16_t)min(max(s0 >> 3, 0), 32767);
                tq16[o + 2] = (uint16_t)min(max(s1 >> 3, 0), 32767);
            }
            __syncthreads();
            const int x = threadIdx.x & 63;
            for (int yp = threadIdx.x >> 6; yp < nyp; yp += 4) {
                const int y = 2 * yp;
                const uint32_t *c = tq + yp * 64 + x;
                const uint32_t q0 = c[0], q1 = c[64], q2 = c[128], q3 = c[192];
                const int s0 = dot2(q0, Ve[0], dot2(q1, Ve[1], dot2(q2, Ve[2], dot2(q3, Ve[3], (int)((q1 >> 16) << 7)))));
                const int s1 = dot2(q0, Vo[0], dot2(q1, Vo[1], dot2(q2, Vo[2], dot2(q3, Vo[3], (int)((q2 & 0xFFFF) << 7)))));
                int sv0 = 0, sv1 = 0;
                if (MODE != 3) {
                    const uint16_t *sp = s + (size_t)(t.y0 + y) * stride + t.x0 + x;
                    sv0 = sp[0], sv1 = sp[stride];
                }
                const int d0 = min(max(s0 >> 11, 0), 1023) - sv0, d1 = min(max(s1 >> 11, 0), 1023) - sv1;
                e += (unsigned long long)(d0 * d0 + d1 * d1);
            }
        }
        for (int o = 32; o > 0; o >>= 1) e += __shfl_down(e, o, 64);
        if ((threadIdx.x & 63) == 0) atomicAdd(&err[it >> 4], e);
    }
}

int main() {
    const int W = 3840, H = 2160, stride = 3840;
    uint16_t *d, *s;
    hipMalloc(&d, (size_t)stride * H * 2);
    hipMalloc(&s, (size_t)stride * H * 2);
    hipMemset(d, 1, (size_t)stride * H * 2);
    hipMemset(s, 2, (size_t)stride * H * 2);
    std::vector<Tile> tl;
    for (int y = 0; y < H; y += 64)
        for (int x = 0; x < W; x += 64) tl.push_back({x, y, 64, std::min(64, H - y)});
    const int n = (int)tl.size();
    Tile *dt;
    hipMalloc(&dt, n * sizeof(Tile));
    hipMemcpy(dt, tl.data(), n * sizeof(Tile), hipMemcpyHostToDevice);
    int16_t ht[16] = {3, -7, 15, -22, 15, -7, 3, 0, 3, -7, 15, -22, 15, -7, 3, 0}, *tp;
    hipMalloc(&tp, 32);
    hipMemcpy(tp, ht, 32, hipMemcpyHostToDevice);
    unsigned long long *err;
    hipMalloc(&err, 8 * 4096);
    hipEvent_t a, b;
    hipEventCreate(&a), hipEventCreate(&b);
    auto run = [&](auto kern, const char *name, int grid) {
        for (int i = 0; i < 5; i++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, d, s, stride, W, H, dt, n, tp, err);
        hipEventRecord(a);
        for (int i = 0; i < 50; i++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, d, s, stride, W, H, dt, n, tp, err);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        printf("%-28s grid %5d  %8.2f us/launch (%d tiles)\n", name, grid, ms * 1000 / 50, n);
    };
    for (int grid : {n, 2048, 1024}) {
        run(trial<0>, "full", grid);
        run(trial<1>, "staging only", grid);
        run(trial<2>, "compute+src (no staging)", grid);
        run(trial<3>, "compute only", grid);
    }
    return 0;
}
