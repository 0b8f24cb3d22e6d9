// Probe: sustained v_mfma_i32_32x32x32_i8 rate with every CU busy (the PFKS / KS GEMMs' instruction),
// operands in registers, 4 independent accumulators per wave, random operands; 1 or 4 waves per SIMD.
// Output: POP/s (2 ops per MAC) and the implied clock if one MFMA takes 32 cycles per SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int T>
__global__ void __launch_bounds__(T, 1) k(int *out, int iters, int seed) {
    v4i a = {(int)(threadIdx.x * 2654435761u ^ seed), (int)(threadIdx.x * 40503u + seed), seed * 7, (int)threadIdx.x};
    v4i b = {a[1] ^ 0x5a5a5a5a, a[0] + 12345, a[3] * 3, a[2] ^ 0x33333333};
    v16i c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
    for (int i = 0; i < iters; i++) {
        c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, b, c3, 0, 0, 0);
    }
    int s = 0;
    for (int q = 0; q < 16; q++) s += c0[q] ^ c1[q] ^ c2[q] ^ c3[q];
    out[blockIdx.x * T + threadIdx.x] = s;
}

template <int T>
void run(int cus, int *d) {
    const int iters = 20000;
    k<T><<<cus, T>>>(d, 100, 1);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    k<T><<<cus, T>>>(d, iters, 2);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double mfma = (double)cus * (T / 64) * iters * 4;  // wave-level MFMAs
    const double pops = mfma * 32 * 32 * 32 * 2 / (ms * 1e-3) / 1e15;
    const double per_simd = mfma / (cus * 4.0);
    printf("%4d threads/CU: %.3f ms, %.2f POP/s, implied clock %.2f GHz at 32 cycles per MFMA\n", T, ms, pops,
           per_simd * 32 / (ms * 1e-3) / 1e9);
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int *d;
    (void)hipMalloc(&d, sizeof(int) * cus * 1024);
    run<256>(cus, d);
    run<1024>(cus, d);
    return 0;
}
