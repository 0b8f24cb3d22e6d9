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
    //            16 = B runs MFMA 4x4x4
    const bool valu = (A && (MODE & 1)) || (!A && (MODE & 2));
    const bool mf16 = (A && (MODE & 4)) || (!A && (MODE & 8));
    const bool mf4 = !A && (MODE & 16);
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
    run<16>(d, it, "B mfma4x4x4");
    run<1 | 16>(d, it, "A valu + B mfma4x4x4");
    return 0;
}
