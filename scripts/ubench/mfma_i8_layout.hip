// Probe of the gfx950 v_mfma_i32_16x16x64_i8 operand layout with exact, asymmetric integer data.
// Assumed: lane l holds A[m = l & 15][k = 16 (l >> 4) + j] and B[k = 16 (l >> 4) + j][n = l & 15] in byte j of its
// 16-byte fragment; D[row = 4 (l >> 4) + r][col = l & 15] in register r.  Prints "layout ok" or the first mismatch.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void probe(const signed char *A, const signed char *B, int *D) {
    const int l = threadIdx.x;
    v4i a, b;
    signed char *pa = (signed char *)&a, *pb = (signed char *)&b;
    for (int j = 0; j < 16; j++) {
        pa[j] = A[(l & 15) * 64 + 16 * (l >> 4) + j];
        pb[j] = B[(16 * (l >> 4) + j) * 16 + (l & 15)];
    }
    v4i c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; r++) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

int main() {
    signed char hA[16 * 64], hB[64 * 16];
    for (int m = 0; m < 16; m++)
        for (int k = 0; k < 64; k++) hA[m * 64 + k] = (signed char)((m * 7 + k * 3) % 23 - 11 + (k == 5 ? 100 : 0));
    for (int k = 0; k < 64; k++)
        for (int n = 0; n < 16; n++) hB[k * 16 + n] = (signed char)((k * 5 + n * 11) % 19 - 9 - (n == 2 ? 90 : 0));
    signed char *dA, *dB;
    int         *dD, hD[256];
    hipMalloc(&dA, sizeof hA), hipMalloc(&dB, sizeof hB), hipMalloc(&dD, sizeof hD);
    hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice), hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
    for (int m = 0; m < 16; m++)
        for (int n = 0; n < 16; n++) {
            int s = 0;
            for (int k = 0; k < 64; k++) s += hA[m * 64 + k] * hB[k * 16 + n];
            if (s != hD[m * 16 + n]) {
                printf("mismatch at %d %d: %d vs %d\n", m, n, hD[m * 16 + n], s);
                return 1;
            }
        }
    printf("layout ok\n");
    return 0;
}
