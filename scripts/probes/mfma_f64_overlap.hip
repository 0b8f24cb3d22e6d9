// Probe: do f64 MFMA (matrix pipe) and f64 VALU FMAs of two waves on the same SIMD overlap?
// 512-thread workgroups (2 waves per SIMD), one per CU (big LDS request). Waves 0-3 ("A") and
// 4-7 ("B") share SIMDs 0-3. Each mode times one stream combination; if "A valu + B mfma" takes
// about max(A valu alone, B mfma alone) the pipes overlap and the MAC can move to MFMA.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void __launch_bounds__(512, 1) k(double *out, int iters) {
    extern __shared__ double lds[];
    const int w = threadIdx.x >> 6;
    const bool A = w < 4;
    // MODE bits: 1 = A runs VALU, 2 = B runs VALU, 4 = A runs MFMA16, 8 = B runs MFMA16,
    //            16 = B runs MFMA 4x4x4, 32 = A runs u32 VALU, 64 = A runs permlane32 swaps
    const bool valu = (A && (MODE & 1)) || (!A && (MODE & 2));
    const bool mf16 = (A && (MODE & 4)) || (!A && (MODE & 8));
    const bool mf4 = !A && (MODE & 16);
    const bool ival = A && (MODE & 32);
    const bool perm = A && (MODE & 64);
    double s = 0;
    if (valu) {
        double a[16];
        for (int i = 0; i < 16; i++) a[i] = threadIdx.x * 1e-3 + i;
        const double b = 0.999999, c = 1e-7;
        for (int it = 0; it < iters; it++)
#pragma unroll
            for (int i = 0; i < 16; i++) a[i] = fma(a[i], b, c);
        for (int i = 0; i < 16; i++) s += a[i];
    }
    if (ival) {  // integer VALU stream (16 independent u32 chains), the decomposition / torus work
        unsigned a[16];
        for (int i = 0; i < 16; i++) a[i] = threadIdx.x * 7u + i;
        const unsigned b = 0x9E3779B9u;
        for (int it = 0; it < iters; it++)
#pragma unroll
            for (int i = 0; i < 16; i++) a[i] = (a[i] ^ b) + (unsigned)it;
        for (int i = 0; i < 16; i++) s += a[i];
    }
    if (perm) {  // the DFT16 transposes (v_permlane32_swap)
        unsigned a[16];
        for (int i = 0; i < 16; i++) a[i] = threadIdx.x * 7u + i;
        for (int it = 0; it < iters; it++)
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                auto r = __builtin_amdgcn_permlane32_swap(a[i], a[i + 1], false, false);
                a[i] = r[0];
                a[i + 1] = r[1];
            }
        for (int i = 0; i < 16; i++) s += a[i];
    }
    if (mf16) {
        d4 acc[4];
        for (int i = 0; i < 4; i++) acc[i] = d4{0, 0, 0, 0};
        const double x = threadIdx.x * 1e-3, y = 0.5;
        // 16 MFMA16 (64 cycles each at the spec rate) ~ 1024 cycles = 16 x 16 VALU f64 (4 cycles)
        for (int it = 0; it < iters / 4; it++)
#pragma unroll
            for (int i = 0; i < 4; i++) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[i], 0, 0, 0);
        for (int i = 0; i < 4; i++) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    }
    if (mf4) {
        double acc[4] = {0, 0, 0, 0};
        const double x = threadIdx.x * 1e-3, y = 0.5;
        for (int it = 0; it < iters; it++)
#pragma unroll
            for (int i = 0; i < 4; i++) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, acc[i], 0, 0, 0);
        for (int i = 0; i < 4; i++) s += acc[i];
    }
    if (threadIdx.x == 0) lds[0] = s;
    out[blockIdx.x * 512 + threadIdx.x] = s;
}

template <int MODE>
float run(double *d, int iters, const char *name) {
    const int blocks = 256;
    const size_t sh = 100 * 1024;
    hipFuncSetAttribute((const void *)k<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, sh);
    k<MODE><<<blocks, 512, sh>>>(d, 16);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    k<MODE><<<blocks, 512, sh>>>(d, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%-34s %8.3f ms\n", name, ms);
    return ms;
}

int main() {
    double *d;
    (void)hipMalloc(&d, sizeof(double) * 256 * 512);
    const int it = 40000;
    run<1>(d, it, "A valu");
    run<3>(d, it, "A valu + B valu");
    run<8>(d, it, "B mfma16x16x4");
    run<1 | 8>(d, it, "A valu + B mfma16x16x4");
    run<4 | 8>(d, it, "A mfma16 + B mfma16");
    run<32>(d, it, "A u32 valu");
    run<32 | 8>(d, it, "A u32 valu + B mfma16x16x4");
    run<64>(d, it / 2, "A permlane32 (half iters)");
    run<64 | 8>(d, it / 2, "A permlane32 + B mfma16 (half)");
    run<8>(d, it / 2, "B mfma16x16x4 (half iters)");
    run<16>(d, it, "B mfma4x4x4");
    run<1 | 16>(d, it, "A valu + B mfma4x4x4");
    return 0;
}
