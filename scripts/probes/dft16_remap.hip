// Probe (verdict r04 item 1): price a DFT16 point-to-lane remap of br512x4's forward FFT before building it.
// One 1024-thread workgroup per CU (16 waves, 4 per SIMD, <= 128 VGPRs), 15 FFT-256 jobs per CU and
// iteration as in br512x4 (3 ciphertexts x 5 polynomials), a workgroup barrier per iteration (one level).
// Each job: pass A = a DFT16 per column (16 columns), W256 twiddles, LDS 16 x 16 transpose, pass B = a DFT16
// per row, spectrum back to LDS (the next iteration's input).  Plain radix arithmetic with the same f64
// count per point in every variant (~11 per point and DFT16); only the point-to-lane map differs:
//   P = 4  (today): 64 lanes per job, one job per wave (15 waves busy); DFT16 = DFT4 in registers, 4 x 4
//          transpose over the lanes u, u+16, u+32, u+48 (16 permlane swaps per wave), DFT4
//   P = 8  : 32 lanes per job, two jobs per wave (8 waves busy); DFT16 = DFT8 in registers, radix-2 across
//          lanes u, u+16 (16 permlane16 swaps per wave = 8 per job)
//   P = 16 : 16 lanes per job, four jobs per wave (4 waves busy); DFT16 entirely in registers, no swaps
// Output: ms per launch and cycles per iteration per CU at the clock attribute.
#include <hip/hip_runtime.h>

#include <cstdio>

struct cplx {
    double re, im;
};
__device__ __forceinline__ cplx cadd(cplx a, cplx b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cplx csub(cplx a, cplx b) { return {a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cplx cmul(cplx a, cplx b) {
    return {fma(a.re, b.re, -(a.im * b.im)), fma(a.re, b.im, a.im * b.re)};
}
__device__ __forceinline__ void dft4(cplx &a, cplx &b, cplx &c, cplx &d) {
    const cplx t0 = cadd(a, c), t1 = csub(a, c), t2 = cadd(b, d), t3 = csub(b, d);
    a = cadd(t0, t2);
    c = csub(t0, t2);
    b = {t1.re + t3.im, t1.im - t3.re};
    d = {t1.re - t3.im, t1.im + t3.re};
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <bool S32>
__device__ __forceinline__ void swapc(cplx &x, cplx &y) {
    u32x4 a, b;
    __builtin_memcpy(&a, &x, 16);
    __builtin_memcpy(&b, &y, 16);
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const auto r = S32 ? __builtin_amdgcn_permlane32_swap(a[w], b[w], false, false)
                           : __builtin_amdgcn_permlane16_swap(a[w], b[w], false, false);
        a[w] = r[0];
        b[w] = r[1];
    }
    __builtin_memcpy(&x, &a, 16);
    __builtin_memcpy(&y, &b, 16);
}

constexpr int JOBS = 15, STRIDE = 272;  // cplx per job region (one pad slot per 16)
__device__ __forceinline__ int pidx(int q) { return q + (q >> 4); }

// twiddle of unit modulus (|w| = 1 up to rounding), scaled by 1/4 so that values stay bounded over iterations
__device__ __forceinline__ cplx tw(const cplx *t, int e) { return t[e & 255]; }

template <int P, int NJ = JOBS>
__global__ void __launch_bounds__(1024, 1) k(double *out, int iters, const cplx *__restrict__ gtw) {
    extern __shared__ __align__(16) unsigned char smem[];
    cplx *buf = reinterpret_cast<cplx *>(smem);
    cplx *s_tw = buf + JOBS * STRIDE;  // [256] W256^e / 4
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int t = tid; t < 256; t += 1024) s_tw[t] = gtw[t];
    for (int t = tid; t < JOBS * STRIDE; t += 1024) buf[t] = {1e-3 * (t % 97), 1e-3 * (t % 89)};
    __syncthreads();
    constexpr int LPJ = 64 / (P / 4) / 1;  // lanes per job: 64, 32, 16
    constexpr int JPW = 64 / LPJ;          // jobs per wave
    // P = 4 with NJ = 30: every job wave runs two jobs back to back between the barriers (SEQ = 2)
    constexpr int SEQ = (P == 4 && NJ > JOBS) ? NJ / JOBS : 1;
    const int job = wave * JPW + lane / LPJ;
    const bool busy = wave * JPW < (SEQ > 1 ? JOBS : NJ);  // wave-uniform (a partial last wave: a dummy job)
    // NJ > 15 (what-if, timing only): jobs share the 15 LDS regions
    cplx *X = buf + (job % JOBS) * STRIDE;
    const int u = lane & 15;
    for (int it = 0; it < iters; it++) {
      for (int sq = 0; sq < SEQ; sq++)
        if (busy) {
            if constexpr (P == 4) {
                const int r = (lane >> 4) & 3;
                // pass A: column u, points m = r + 4 i
                cplx v[4];
#pragma unroll
                for (int i = 0; i < 4; i++) v[i] = X[pidx(u + 16 * (r + 4 * i))];
                dft4(v[0], v[1], v[2], v[3]);
#pragma unroll
                for (int k1 = 1; k1 < 4; k1++) v[k1] = cmul(v[k1], tw(s_tw, 16 * r * k1));
                swapc<true>(v[0], v[2]);
                swapc<true>(v[1], v[3]);
                swapc<false>(v[0], v[1]);
                swapc<false>(v[2], v[3]);
                dft4(v[0], v[1], v[2], v[3]);
#pragma unroll
                for (int k2 = 0; k2 < 4; k2++) X[pidx(u + 16 * (r + 4 * k2))] = cmul(v[k2], tw(s_tw, u * (r + 4 * k2)));
                asm volatile("" ::: "memory");
                // pass B: row u, points 16 u + r + 4 i
#pragma unroll
                for (int i = 0; i < 4; i++) v[i] = X[pidx(16 * u + r + 4 * i)];
                dft4(v[0], v[1], v[2], v[3]);
#pragma unroll
                for (int k1 = 1; k1 < 4; k1++) v[k1] = cmul(v[k1], tw(s_tw, 16 * r * k1));
                swapc<true>(v[0], v[2]);
                swapc<true>(v[1], v[3]);
                swapc<false>(v[0], v[1]);
                swapc<false>(v[2], v[3]);
                dft4(v[0], v[1], v[2], v[3]);
#pragma unroll
                for (int k2 = 0; k2 < 4; k2++) X[pidx(16 * u + r + 4 * k2)] = v[k2];
            } else if constexpr (P == 8) {
                const int h = (lane >> 4) & 1;
                cplx v[8];
                auto dft16 = [&](int base, int stride) {
#pragma unroll
                    for (int i = 0; i < 8; i++) v[i] = X[pidx(base + stride * (h + 2 * i))];
                    // DFT8 over i: two DFT4 (even / odd i), W8 twiddles, radix-2
                    dft4(v[0], v[2], v[4], v[6]);
                    dft4(v[1], v[3], v[5], v[7]);
#pragma unroll
                    for (int k = 1; k < 4; k++) v[2 * k + 1] = cmul(v[2 * k + 1], tw(s_tw, 32 * k));
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const cplx a = v[2 * k], b = v[2 * k + 1];
                        v[2 * k] = cadd(a, b);
                        v[2 * k + 1] = csub(a, b);
                    }
                    // W16^{h k'} and the radix-2 over h across lanes u, u+16: lane h keeps k' = 4h .. 4h + 3
#pragma unroll
                    for (int k = 1; k < 8; k++) v[k] = cmul(v[k], tw(s_tw, 16 * h * k));
                    swapc<false>(v[0], v[4]);
                    swapc<false>(v[1], v[5]);
                    swapc<false>(v[2], v[6]);
                    swapc<false>(v[3], v[7]);
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const cplx a = v[k], b = v[k + 4];
                        v[k] = cadd(a, b);
                        v[k + 4] = csub(a, b);
                    }
                };
                dft16(u, 16);
#pragma unroll
                for (int k = 0; k < 8; k++) X[pidx(u + 16 * (h + 2 * k))] = cmul(v[k], tw(s_tw, u * (h + 2 * k)));
                asm volatile("" ::: "memory");
                dft16(16 * u, 1);
#pragma unroll
                for (int k = 0; k < 8; k++) X[pidx(16 * u + h + 2 * k)] = v[k];
            } else {
                cplx v[16];
                auto dft16 = [&](int base, int stride) {
#pragma unroll
                    for (int m = 0; m < 16; m++) v[m] = X[pidx(base + stride * m)];
#pragma unroll
                    for (int n1 = 0; n1 < 4; n1++) dft4(v[n1], v[n1 + 4], v[n1 + 8], v[n1 + 12]);
#pragma unroll
                    for (int n1 = 1; n1 < 4; n1++)
#pragma unroll
                        for (int k1 = 1; k1 < 4; k1++) v[n1 + 4 * k1] = cmul(v[n1 + 4 * k1], tw(s_tw, 16 * n1 * k1));
#pragma unroll
                    for (int k1 = 0; k1 < 4; k1++) dft4(v[4 * k1], v[4 * k1 + 1], v[4 * k1 + 2], v[4 * k1 + 3]);
                };
                dft16(u, 16);
#pragma unroll
                for (int k = 0; k < 16; k++) X[pidx(u + 16 * k)] = cmul(v[k], tw(s_tw, u * k));
                asm volatile("" ::: "memory");
                dft16(16 * u, 1);
#pragma unroll
                for (int k = 0; k < 16; k++) X[pidx(16 * u + k)] = v[k];
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    if (lane == 0) out[blockIdx.x * 16 + wave] = X[pidx(lane)].re;
}

template <int P, int NJ = JOBS>
void run(double *d, const cplx *tw, int cus, int iters, double ghz) {
    const size_t sh = (JOBS * STRIDE + 256) * sizeof(cplx);
    (void)hipFuncSetAttribute((const void *)k<P, NJ>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
    k<P, NJ><<<cus, 1024, sh>>>(d, 8, tw);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        (void)hipEventRecord(e0);
        k<P, NJ><<<cus, 1024, sh>>>(d, iters, tw);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    printf("P=%2d points per lane, %2d jobs: %8.3f ms, %7.0f cycles per iteration, %6.0f per job (at %.2f GHz)\n", P, NJ,
           best, best * 1e-3 * ghz * 1e9 / iters, best * 1e-3 * ghz * 1e9 / iters / NJ, ghz);
}

int main() {
    int cus = 0, clk = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    const double ghz = clk / 1e6;
    cplx htw[256];
    for (int e = 0; e < 256; e++) {
        const double a = -2.0 * 3.141592653589793 * e / 256;
        htw[e] = {0.25 * __builtin_cos(a), 0.25 * __builtin_sin(a)};
    }
    double *d;
    cplx *tw;
    (void)hipMalloc(&d, sizeof(double) * cus * 16);
    (void)hipMalloc(&tw, sizeof htw);
    (void)hipMemcpy(tw, htw, sizeof htw, hipMemcpyHostToDevice);
    const int iters = 4000;
    printf("CUs %d\n", cus);
    run<4>(d, tw, cus, iters, ghz);
    run<8>(d, tw, cus, iters, ghz);
    run<16>(d, tw, cus, iters, ghz);
    run<4>(d, tw, cus, iters, ghz);
    // what-if: as many jobs as the 16 waves hold (LDS regions shared, timing only)
    run<4, 30>(d, tw, cus, iters, ghz);
    run<8, 30>(d, tw, cus, iters, ghz);
    run<16, 30>(d, tw, cus, iters, ghz);
    run<16, 45>(d, tw, cus, iters, ghz);
    run<16, 60>(d, tw, cus, iters, ghz);
    return 0;
}
