// Probe: sustained FP64 FMA rate (v_fma_f64) -- calibrates the FP64 roof used by bench.py.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void __launch_bounds__(256) k(double *out, int iters) {
    double a[16];
    for (int i = 0; i < 16; i++) a[i] = threadIdx.x * 1e-3 + i;
    const double b = 0.999999, c = 1e-7;
    for (int it = 0; it < iters; it++)
#pragma unroll
        for (int i = 0; i < 16; i++) a[i] = fma(a[i], b, c);
    double s = 0;
    for (int i = 0; i < 16; i++) s += a[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
    double *d; const int blocks = 256 * 8, iters = 20000;
    (void)hipMalloc(&d, sizeof(double) * blocks * 256);
    k<<<blocks, 256>>>(d, 10); (void)hipDeviceSynchronize();
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0); k<<<blocks, 256>>>(d, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    double flop = 2.0 * 16 * iters * (double)blocks * 256;
    printf("fp64 fma: %.2f TFLOP/s (%.3f ms)\n", flop / ms / 1e9, ms);
    return 0;
}
