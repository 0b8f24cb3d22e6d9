// The 8-bit model's batched PBS blind rotation (N = 1024, k = 2, 6 levels of 2^7,
// shortint_woppbs_8bit.rs:39-86) with its 36 forward FFT jobs per CMux step dealt out in ROUNDS of eight:
// two ciphertexts per 512-thread workgroup, as br1024's C = 2 kernel, but instead of one level (6 jobs
// on 8 waves: two jobs on SIMDs 0-1, one on SIMDs 2-3) per barrier interval, every wave takes one job
// of the step's sequence (level 6 first; in a level p ascending, both ciphertexts of a p together), so
// that each SIMD runs two job waves in every round: 4 full rounds and one of 4 jobs instead of 6 rounds
// whose critical SIMDs run two jobs each.
//   D  rotated difference + digits of both ciphertexts' 3 polynomials for all 6 levels, thread = coefficient
//      pair j (6 pairs per thread, the same on every SIMD), int8 digit pairs -> LDS [level][poly][t][m]
//   per round r: F  job 8 r + w on wave w (fused transform, lf1k.hpp, br1024's LF lane programs) -> LDS
//                   slot w;  M  MAC at Fourier position pos over the round's jobs in sequence order, i.e.
//                   per (q, ct) chain p ascending within a level, levels descending: the oracle's order
//   S  MAC results -> slots (ct, q);  I  inverse FFT + untwist + torus + ACC += on waves 0-5 (br1024's)
// Bit-identical to br1024 (same lane programs, same fma chains).  LDS 156 KiB: ACC [6][1024] u64,
// spectra 8 x [576] cplx, digits [6][6][64][8] u16; the transform's per-lane constants sit in registers
// (loaded from global once), its untwist table is read from global memory.
#pragma once
#include "br1024.hpp"

namespace tae {
namespace br1024r {

using br1024::BUF_STRIDE;
using br1024::dft8;
using br1024::K1;
using br1024::M;
using br1024::N;
using br1024::pidx;
using br1024::u32x4;
using br1024::wave_sync;

constexpr int LEV = 6, BLOG = 7, C = 2, CJ = C * K1, THREADS = 512, WAVES = THREADS / 64;
constexpr int JOBS = LEV * CJ;                         // 36 forward FFT jobs per CMux step
constexpr int ROUNDS = (JOBS + WAVES - 1) / WAVES;    // 5: four of 8 jobs, one of 4
constexpr int ACC_STRIDE = N;

constexpr size_t lds_bytes() {
    return (size_t)CJ * ACC_STRIDE * 8 + (size_t)WAVES * BUF_STRIDE * 16 + (size_t)LEV * CJ * M * 2;
}
static_assert(lds_bytes() <= 160 * 1024, "LDS");

// TAE_B1KR_PROF (debug builds only): per-phase cycle sums of every wave of workgroup 0: decomposition,
// its barrier, FFT rounds, their barrier, MAC, its barrier, the inverse's store barrier, inverse, I2 / its
// barrier, the step-end barrier
#ifdef TAE_B1KR_PROF
#define RPROF_DECL uint64_t rprof_[10] = {0}, rprof_t_ = clock64();
#define RPROF(i)                           \
    do {                                   \
        asm volatile("" ::: "memory");     \
        const uint64_t now_ = clock64();   \
        rprof_[i] += now_ - rprof_t_;      \
        rprof_t_ = now_;                   \
    } while (0)
#else
#define RPROF_DECL
#define RPROF(i) \
    do {         \
    } while (0)
#endif

// job j of a step: level 6 - j / 6, then (p, ct) = ((j % 6) / 2, j % 2); poly index ct * K1 + p
__device__ __forceinline__ int job_level(int j) { return LEV - j / CJ; }
__device__ __forceinline__ int job_p(int j) { return (j % CJ) >> 1; }
__device__ __forceinline__ int job_ct(int j) { return j & 1; }
// wave of job j in its round: 8 r + w for the full rounds; the last round's 4 jobs on waves 0, 1, 4, 5
// (two per SIMD on SIMDs 0-1: two waves issue ~2x as often as one)
__device__ __forceinline__ int round_job(int r, int w) {
    if (r < ROUNDS - 1) return WAVES * r + w;
    return (w & 2) ? -1 : WAVES * r + (w & 1) + ((w >> 2) << 1);
}
__device__ __forceinline__ int round_slot(int r, int i) {  // slot of the round's i-th job
    return r < ROUNDS - 1 ? i : (i & 1) + ((i >> 1) << 2);
}

__global__ void __launch_bounds__(THREADS, 1)
    br_kernel(const uint64_t *__restrict__ lwe_in, int n, const uint64_t *__restrict__ lut,
              const cplx *__restrict__ bsk, uint64_t *__restrict__ out, long B, uint64_t body_add,
              uint64_t out_add, const cplx *__restrict__ wtab, const double *__restrict__ lf,
              uint64_t *__restrict__ clk) {
    ClockStamp stamp;
    stamp.start(clk);
    constexpr int LOGN = 10;
    extern __shared__ __align__(16) unsigned char smem[];
    uint64_t *acc = reinterpret_cast<uint64_t *>(smem);                  // [CJ][ACC_STRIDE]
    cplx *buf = reinterpret_cast<cplx *>(acc + CJ * ACC_STRIDE);         // [WAVES][BUF_STRIDE]
    uint16_t *s_dig = reinterpret_cast<uint16_t *>(buf + WAVES * BUF_STRIDE);  // [LEV][CJ][64][8]
    const cplx *untw = reinterpret_cast<const cplx *>(lf + lf1k::UNTW);
    const int tid = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int t = tid & 63;
    const size_t ggsw_sz = (size_t)LEV * K1 * K1 * M;
    const long ct0 = (long)blockIdx.x * C;
    const int nct = (int)min((long)C, B - ct0);

    for (int i = tid; i < CJ * N; i += THREADS) {
        const int job = i / N, j = i - job * N;
        const int ct = job / K1, c = job - ct * K1;
        uint64_t v = 0;
        if (ct < nct) {
            const uint64_t *in = lwe_in + (size_t)(ct0 + ct) * (n + 1);
            const int bt = mod_switch(in[n] + body_add, LOGN);
            const int e0 = (2 * N - (bt % (2 * N))) % (2 * N);
            v = rotated_coeff(lut + c * N, j, e0, N);
        }
        acc[job * ACC_STRIDE + j] = v;
    }
    const uint32_t gbytes = (uint32_t)((size_t)n * ggsw_sz * sizeof(cplx));
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc((void *)bsk, (short)0, gbytes, 0x00020000);
    const int pos = br1024::mac_pos(tid);
    const int gvoff = pos * (int)sizeof(cplx);
    const cplx w81 = wtab[64], w83 = wtab[192];
    // the lane's fused-DFT8 constants (as br1024's register-held ones) and pass 0's lane-uniform ones
    const lf1k::K8 kf1 = lf1k::k8(lf, lf1k::F1, 8, t >> 3), kf2 = lf1k::k8(lf, lf1k::F2, 64, t);
    const lf1k::K8 ki1 = lf1k::k8(lf, lf1k::I1, 8, t & 7), ki0 = lf1k::k8(lf, lf1k::I0, 64, t);
    const lf1k::P0c k0 = lf1k::p0(lf);
    br512::lds_sync();

    cplx accr[K1 * C];
    RPROF_DECL
    for (int step = 0; step < n; step++) {
        br1024::s_setprio_c<2>();
        const int gstep = step * (int)(ggsw_sz * sizeof(cplx));
        // ---- D: coefficient pair (j, j + M), j = tid, of all 6 polynomials ----
        {
            int ec[C];
#pragma unroll
            for (int ct = 0; ct < C; ct++)
                ec[ct] = ct < nct ? mod_switch(lwe_in[(size_t)(ct0 + ct) * (n + 1) + step], LOGN) % (2 * N) : 0;
            int jj = tid;
            asm volatile("" : "+v"(jj));
            const int dt = jj & 63, dm = jj >> 6;
#pragma unroll
            for (int poly = 0; poly < CJ; poly++) {
                const uint64_t *pl = acc + poly * ACC_STRIDE;
                const int ti = (jj - ec[poly / K1]) & (2 * N - 1);  // entry of [ACC, -ACC]
                const int ph = ti & (N - 1);
                const uint64_t m0 = (uint64_t)(int64_t)((ti << 21) >> 31);
                const uint64_t m1 = (uint64_t)(int64_t)(((ti + M) << 21) >> 31);
                const uint64_t v0 = pl[ph], v1 = pl[ph ^ M];
                const uint64_t p0 = pl[jj], p1 = pl[jj + M];
                const uint64_t x0 = (v0 ^ m0) - (p0 + m0), x1 = (v1 ^ m1) - (p1 + m1);
                uint32_t dp[LEV];  // level l + 1: digit of x0 | digit of x1 << 16
                decompose16p<LEV, BLOG>(x0, x1, dp);
#pragma unroll
                for (int l = 0; l < LEV; l++)
                    s_dig[(((l * CJ + poly) * 64) + dt) * 8 + dm] = (uint16_t)((dp[l] & 0xFF) | ((dp[l] >> 8) & 0xFF00));
            }
        }
#pragma unroll
        for (int a = 0; a < K1 * C; a++) accr[a] = cplx{0.0, 0.0};
        RPROF(0);
        br512::lds_sync();
        RPROF(1);
        br1024::s_setprio_c<3>();

        for (int r = 0; r < ROUNDS; r++) {
            constexpr int PAIRS = WAVES / 2;  // (level, p) pairs of a full round, each for both ciphertexts
            const int npair = r < ROUNDS - 1 ? PAIRS : (JOBS - WAVES * (ROUNDS - 1)) / 2;
            // the round's GGSW rows (q = 0..2 of each (level, p)), landing during the FFTs
            cplx gv[PAIRS * K1];
#pragma unroll
            for (int i = 0; i < PAIRS; i++) {
                if (i < npair) {
                    const int jp = WAVES * r + 2 * i;
                    const int lev = job_level(jp), p = job_p(jp);
#pragma unroll
                    for (int q = 0; q < K1; q++) {
                        const int soff = gstep + (((lev - 1) * K1 + p) * K1 + q) * M * (int)sizeof(cplx);
                        const u32x4 rv = __builtin_amdgcn_raw_buffer_load_b128(grs, gvoff, soff, 0);
                        __builtin_memcpy(&gv[i * K1 + q], &rv, sizeof(cplx));
                    }
                }
            }
            const int jw = round_job(r, wv);
            if (jw >= 0) {
                int tt = t;
                asm volatile("" : "+v"(tt));
                const int lev = job_level(jw), poly = job_ct(jw) * K1 + job_p(jw);
                cplx *X = buf + wv * BUF_STRIDE;
                cplx v[8];
                {  // fused pass 0 of the job's digits -> position t + 64 kk
                    const u32x4 dq = *reinterpret_cast<const u32x4 *>(s_dig + (((lev - 1) * CJ + poly) * 64 + tt) * 8);
                    int dr[8], di[8];
#pragma unroll
                    for (int m = 0; m < 8; m++) {
                        const uint32_t w = (dq[m >> 1] >> (16 * (m & 1))) & 0xFFFFu;
                        dr[m] = (int8_t)(w & 0xFF);
                        di[m] = (int8_t)(w >> 8);
                    }
                    lf1k::pass0(dr, di, v, k0);
                }
#pragma unroll
                for (int kk = 0; kk < 8; kk++) X[pidx(tt + 64 * kk)] = v[kk];
                wave_sync();
                br1024::s_setprio_c<2>();
                {  // fused pass 1: points 64 gg + uu + 8 m
                    const int gg = tt >> 3, uu = tt & 7;
#pragma unroll
                    for (int m = 0; m < 8; m++) v[m] = X[pidx(64 * gg + uu + 8 * m)];
                    lf1k::dft8<false>(v, kf1);
#pragma unroll
                    for (int kk = 0; kk < 8; kk++) X[pidx(64 * gg + uu + 8 * kk)] = v[kk];
                }
                wave_sync();
                br1024::s_setprio_c<1>();
#pragma unroll
                for (int m = 0; m < 8; m++) v[m] = X[pidx(8 * tt + m)];
                lf1k::dft8<false>(v, kf2);
#pragma unroll
                for (int kk = 0; kk < 8; kk++) X[pidx(8 * tt + kk)] = v[kk];
            }
            RPROF(2);
            br512::lds_sync();
            RPROF(3);
            br1024::s_setprio_c<3>();
            // ---- M: the round's jobs in sequence order; accumulator (q, ct) = accr[q * C + ct] ----
#pragma unroll
            for (int i = 0; i < 2 * PAIRS; i++) {
                if (i < 2 * npair) {
                    const int ct = i & 1;
                    const cplx x = buf[round_slot(r, i) * BUF_STRIDE + pidx(pos)];
#pragma unroll
                    for (int q = 0; q < K1; q++) {
                        const cplx g = gv[(i >> 1) * K1 + q];
                        double re = accr[q * C + ct].re, im = accr[q * C + ct].im;
                        re = fma(x.re, g.re, re);
                        re = fma(-x.im, g.im, re);
                        im = fma(x.re, g.im, im);
                        im = fma(x.im, g.re, im);
                        accr[q * C + ct] = {re, im};
                    }
                }
            }
            RPROF(4);
            br512::lds_sync();
            RPROF(5);
            br1024::s_setprio_c<3>();
        }
        // ---- S + I: inverse FFT of output (ct, q) = wave, untwist, from_torus, ACC += ----
#pragma unroll
        for (int q = 0; q < K1; q++)
#pragma unroll
            for (int ct = 0; ct < C; ct++) buf[(ct * K1 + q) * BUF_STRIDE + pidx(pos)] = accr[q * C + ct];
        RPROF(6);
        br512::lds_sync();
        RPROF(1);
        if (wv < CJ) {
            int tt = t;
            asm volatile("" : "+v"(tt));
            cplx *Y = buf + wv * BUF_STRIDE;
            cplx v[8];
#pragma unroll
            for (int kk = 0; kk < 8; kk++) v[kk] = Y[pidx(8 * tt + kk)];
            dft8<true>(v, w81, w83);
#pragma unroll
            for (int m = 0; m < 8; m++) Y[pidx(8 * tt + m)] = v[m];
            wave_sync();
            {
                const int gg = tt >> 3, uu = tt & 7;
#pragma unroll
                for (int kk = 0; kk < 8; kk++) v[kk] = Y[pidx(64 * gg + uu + 8 * kk)];
                lf1k::dft8<true>(v, ki1);
#pragma unroll
                for (int m = 0; m < 8; m++) Y[pidx(64 * gg + uu + 8 * m)] = v[m];
            }
            wave_sync();
            br1024::s_setprio_c<2>();
#pragma unroll
            for (int kk = 0; kk < 8; kk++) v[kk] = Y[pidx(tt + 64 * kk)];
            lf1k::dft8<true>(v, ki0);
#ifdef TAE_B1KR_I2
            wave_sync();  // this wave's reads of Y precede its writes below (LDS executes in order)
#pragma unroll
            for (int m = 0; m < 8; m++) Y[tt + 64 * m] = v[m];  // coefficient pair j = t + 64 m
        }
        RPROF(7);
        br512::lds_sync();
        {  // I2: untwist, from_torus, ACC += for coefficient pair j = tid of all 6 outputs, on all 8 waves
            int jj = tid;
            asm volatile("" : "+v"(jj));
            const cplx u = untw[jj];
#pragma unroll
            for (int k = 0; k < CJ; k++) {
                uint64_t *poly = acc + k * ACC_STRIDE;
                const cplx y = cmul(buf[k * BUF_STRIDE + jj], u);
                bool o0, o1;
                uint64_t a0 = torus_add_fast_sh<9>(y.re, poly[jj], o0), a1 = torus_add_fast_sh<9>(y.im, poly[jj + M], o1);
                if (__builtin_amdgcn_ballot_w64(!(o0 && o1))) {
                    a0 = poly[jj] + from_torus_bits(y.re * 0x1p-9);
                    a1 = poly[jj + M] + from_torus_bits(y.im * 0x1p-9);
                }
                poly[jj] = a0;
                poly[jj + M] = a1;
            }
#else
            uint64_t *poly = acc + wv * ACC_STRIDE;
#pragma unroll
            for (int m = 0; m < 8; m++) {
                const int j = tt + 64 * m;
                const cplx u = untw[j];
                const cplx y = cmul(v[m], u);  // conj(twist); the 2^-9 goes into the exponent (exact)
                bool o0, o1;
                uint64_t a0 = torus_add_fast_sh<9>(y.re, poly[j], o0), a1 = torus_add_fast_sh<9>(y.im, poly[j + M], o1);
                if (__builtin_amdgcn_ballot_w64(!(o0 && o1))) {  // zeros, out-of-range magnitudes (rare)
                    a0 = poly[j] + from_torus_bits(y.re * 0x1p-9);
                    a1 = poly[j + M] + from_torus_bits(y.im * 0x1p-9);
                }
                poly[j] = a0;
                poly[j + M] = a1;
            }
#endif
        }
        RPROF(8);
        br512::lds_sync();  // the next decomposition reads every polynomial
        RPROF(9);
    }
#ifdef TAE_B1KR_PROF
    if (blockIdx.x == 0 && (tid & 63) == 0)
        printf("b1krprof wave %d: dec %llu barDS %llu fft %llu barF %llu mac %llu barM %llu store %llu invI2 %llu inv %llu barE %llu\n",
               wv, (unsigned long long)rprof_[0], (unsigned long long)rprof_[1], (unsigned long long)rprof_[2],
               (unsigned long long)rprof_[3], (unsigned long long)rprof_[4], (unsigned long long)rprof_[5],
               (unsigned long long)rprof_[6], (unsigned long long)rprof_[7], (unsigned long long)rprof_[8],
               (unsigned long long)rprof_[9]);
#endif
    for (int ct = 0; ct < nct; ct++) {
        const uint64_t *a = acc + ct * K1 * ACC_STRIDE;
        uint64_t *o = out + (size_t)(ct0 + ct) * (K1 - 1) * N + (size_t)(ct0 + ct);
        for (int i = tid; i < (K1 - 1) * N; i += THREADS) {
            const int p = i / N, j = i - p * N;
            o[i] = j == 0 ? a[p * ACC_STRIDE] : (0 - a[p * ACC_STRIDE + N - j]);
        }
        if (tid == 0) o[(K1 - 1) * N] = a[(K1 - 1) * ACC_STRIDE] + out_add;
    }
    stamp.stop(clk);
}

}  // namespace br1024r
}  // namespace tae
