// Probe: operand/result lane layout of v_mfma_i32_32x32x32_i8 on gfx950 (exact integer check).
// Hypothesis: lane l (r = l & 31, h = l >> 5) holds A[r][16h + t], B[16h + t][r] (t = 0..15);
// C reg q holds C[(q & 3) + 8 (q >> 2) + 4 h][r].
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
__global__ void k(const signed char *A, const signed char *B, int *C) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    signed char a[16], b[16];
    for (int t = 0; t < 16; t++) { a[t] = A[r * 32 + 16 * h + t]; b[t] = B[(16 * h + t) * 32 + r]; }
    v4i av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    v16i acc = {0};
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, acc, 0, 0, 0);
    for (int q = 0; q < 16; q++) C[((q & 3) + 8 * (q >> 2) + 4 * h) * 32 + r] = acc[q];
}
int main() {
    signed char hA[1024], hB[1024];
    int ref[1024], hC[1024];
    srand(1);
    for (int i = 0; i < 1024; i++) { hA[i] = (signed char)(rand() & 255); hB[i] = (signed char)(rand() & 255); }
    for (int i = 0; i < 32; i++) for (int j = 0; j < 32; j++) { int s = 0; for (int t = 0; t < 32; t++) s += hA[i * 32 + t] * hB[t * 32 + j]; ref[i * 32 + j] = s; }
    signed char *dA, *dB; int *dC;
    hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dC, 4096);
    hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    k<<<1, 64>>>(dA, dB, dC);
    hipMemcpy(hC, dC, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 1024; i++) bad += hC[i] != ref[i];
    printf("mfma_i32_32x32x32_i8 layout: %s (%d mismatches)\n", bad ? "MISMATCH" : "OK", bad);
    return bad != 0;
}
