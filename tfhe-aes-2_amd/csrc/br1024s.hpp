// Batched blind rotation for the 8-bit model's PBS (N = 1024, k = 2, 6 levels of 2^7;
// shortint_woppbs_8bit.rs:39-86), C = 2 ciphertexts per 512-thread workgroup, with the FFT jobs of a
// CMux step STREAMED across the decomposition levels.
//
// br1024.hpp runs one level at a time: 6 FFT jobs (ciphertext, polynomial) on 8 waves, i.e. two SIMDs
// with two job waves and two with one.  A wave alone on a SIMD issues f64 work at about half the rate of
// a SIMD shared by two (scripts/probes/valu_rates.hip: one wave 15.3, two waves 7.1 cycles per f64 op per
// SIMD), so every level pass lasts as long as a lone wave's FFT while half of two SIMDs idles.  Here the
// 36 jobs of a step (level descending, then p, then ciphertext) run eight at a time, one per wave, in
// 5 passes (8, 8, 8, 8, 4) instead of 6 level passes of 6: every SIMD holds two FFT waves in the first
// four.  For that every wave must reach every polynomial's digits, so the decomposition writes them to
// LDS ([poly][level pair][m][lane] u32, 36 KiB), and it is spread over all 8 waves (wave w decomposes the
// coefficient pairs j = lane + 64 w of all six polynomials) instead of 6.
// The MAC of a pass consumes its jobs in job order, so every accumulator (q, ct) still sums its terms in
// the oracle's order (level descending, p ascending) with the same fma chain: results are bit-exact with
// br1024 and the oracle.  A pass never splits the two ciphertexts of a (level, p), so each GGSW row value
// is loaded once per pass for both.
// LDS (156 KiB): ACC [ct][k+1][N] u64, 8 spectrum slots [576] cplx, digits.  No twiddle table: the lane's
// pass-0/1 twiddles and twist factors are registers (as in br1024's 8-bit instantiations), loaded from
// global memory once, and the untwist is conj(twist) with its exact 2^-9 folded into the torus conversion
// (torus_add_fast_sh).
#pragma once
#include "br1024.hpp"

namespace tae {
namespace br1024s {

using br1024::ACC_STRIDE;
using br1024::BUF_STRIDE;
using br1024::dft8;
using br1024::K1;
using br1024::M;
using br1024::mac_pos;
using br1024::N;
using br1024::pidx;
using br1024::s_setprio_c;
using br1024::u32x4;

constexpr int C = 2, CJ = C * K1, THREADS = 512, WAVES = THREADS / 64;
constexpr int LEV = 6, BLOG = 7, LPAIRS = LEV / 2, LOG2M = 9;
constexpr int NJOB = LEV * CJ, NPASS = (NJOB + WAVES - 1) / WAVES;
static_assert(WAVES % C == 0 && WAVES == 8, "a pass holds whole (level, p) pairs, one job per wave");

constexpr size_t ACC_BYTES = (size_t)CJ * ACC_STRIDE * 8;
constexpr size_t BUF_BYTES = (size_t)WAVES * BUF_STRIDE * 16;
constexpr size_t DIG_BYTES = (size_t)CJ * LPAIRS * 8 * 64 * 4;
constexpr size_t lds_bytes() { return ACC_BYTES + BUF_BYTES + DIG_BYTES; }
static_assert(lds_bytes() <= 160 * 1024, "LDS");

// TAE_B1KS_PROF (debug builds only): per-phase cycle sums of every wave of workgroup 0
#ifdef TAE_B1KS_PROF
#define SPROF_DECL uint64_t sprof_[6] = {0}, sprof_t_ = clock64();
#define SPROF(i)                           \
    do {                                   \
        asm volatile("" ::: "memory");     \
        const uint64_t now_ = clock64();   \
        sprof_[i] += now_ - sprof_t_;      \
        sprof_t_ = now_;                   \
    } while (0)
#else
#define SPROF_DECL
#define SPROF(i) \
    do {         \
    } while (0)
#endif

__global__ void __launch_bounds__(THREADS, 1)
    br_kernel(const uint64_t *__restrict__ lwe_in, int n, const uint64_t *__restrict__ lut,
              const cplx *__restrict__ bsk, uint64_t *__restrict__ out, long B, uint64_t body_add, uint64_t out_add,
              const cplx *__restrict__ twist, const cplx *__restrict__ wtab, uint64_t *__restrict__ clk) {
    ClockStamp stamp;
    stamp.start(clk);
    constexpr int LOGN = 10;
    extern __shared__ __align__(16) unsigned char smem[];
    uint64_t *acc = reinterpret_cast<uint64_t *>(smem);                                  // [CJ][ACC_STRIDE]
    cplx *buf = reinterpret_cast<cplx *>(smem + ACC_BYTES);                              // [WAVES][BUF_STRIDE]
    uint32_t *dig = reinterpret_cast<uint32_t *>(smem + ACC_BYTES + BUF_BYTES);           // [CJ][LPAIRS][8][64]
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    int tt = tid & 63;
    const long ct0 = (long)blockIdx.x * C;
    const int nct = (int)min((long)C, B - ct0);
    const size_t ggsw_sz = (size_t)LEV * K1 * K1 * M;
    const uint32_t gbytes = (uint32_t)((size_t)n * ggsw_sz * sizeof(cplx));
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc((void *)bsk, (short)0, gbytes, 0x00020000);
    const int pos = mac_pos(tid);
    const int gvoff = pos * (int)sizeof(cplx);

    // the lane's twist factors (pass 0 and the untwist), pass-0 / pass-1 twiddles and the W8 factors
    cplx twr[8], w0r[7], w1r[7];
#pragma unroll
    for (int m = 0; m < 8; m++) twr[m] = twist[tt + 64 * m];
#pragma unroll
    for (int kk = 1; kk < 8; kk++) {
        w0r[kk - 1] = wtab[tt * kk];
        w1r[kk - 1] = wtab[8 * (tt & 7) * kk];
    }
    const cplx w81 = wtab[64], w83 = wtab[192];

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
    br512::lds_sync();

    const uint64_t *a_row0 = lwe_in + (size_t)ct0 * (n + 1), *a_row1 = a_row0 + (nct > 1 ? n + 1 : 0);
    cplx accr[K1 * C];
    cplx gv[WAVES / C * K1];  // GGSW values (q) of the pass's (level, p) pairs at this thread's position
    SPROF_DECL
    for (int step = 0; step < n; step++) {
        const int e0 = mod_switch(a_row0[step], LOGN) % (2 * N), e1 = mod_switch(a_row1[step], LOGN) % (2 * N);
        const int gstep = step * (int)(ggsw_sz * sizeof(cplx));
        s_setprio_c<3>();
        asm volatile("" : "+v"(tt));
        // ---- rotated difference + decomposition: coefficient pair j = tt + 64 w (+ M) of every polynomial ----
        {
            const int j = tt + 64 * w;
#pragma unroll
            for (int s = 0; s < CJ; s++) {
                const int ct = s / K1;
                if (ct < nct) {
                    const uint64_t *poly = acc + s * ACC_STRIDE;
                    const int ti = (j - (ct ? e1 : e0)) & (2 * N - 1);  // entry of [ACC, -ACC]
                    const int ph = ti & (N - 1);
                    const uint64_t m0 = (uint64_t)(int64_t)((ti << 21) >> 31);
                    const uint64_t m1 = (uint64_t)(int64_t)(((ti + M) << 21) >> 31);
                    const uint64_t v0 = poly[ph], v1 = poly[ph ^ M];
                    const uint64_t p0 = poly[j], p1 = poly[j + M];
                    const uint64_t x0 = (v0 ^ m0) - (p0 + m0), x1 = (v1 ^ m1) - (p1 + m1);
                    uint32_t dp[LEV];
                    decompose16p<LEV, BLOG>(x0, x1, dp);
#pragma unroll
                    for (int lp = 0; lp < LPAIRS; lp++)  // bytes (x0, x1) of level 2 lp + 1, then of level 2 lp + 2
                        dig[((s * LPAIRS + lp) * 8 + w) * 64 + tt] = perm_b32(dp[2 * lp + 1], dp[2 * lp], 0x06040200u);
                }
            }
        }
#pragma unroll
        for (int a = 0; a < K1 * C; a++) accr[a] = cplx{0.0, 0.0};
        SPROF(0);
        br512::lds_sync();
        SPROF(1);
        s_setprio_c<3>();
        for (int k = 0; k < NPASS; k++) {
            // GGSW rows (level, p, q) of the pass's (level, p) pairs at this thread's Fourier position
#pragma unroll
            for (int pr = 0; pr < WAVES / C; pr++) {
                const int jp = WAVES * k + C * pr;
                if (jp < NJOB) {
                    const int li = jp / CJ, p = (jp - li * CJ) / C;  // level LEV - li
#pragma unroll
                    for (int q = 0; q < K1; q++) {
                        const int soff = gstep + (((LEV - 1 - li) * K1 + p) * K1 + q) * M * (int)sizeof(cplx);
                        const u32x4 rv = __builtin_amdgcn_raw_buffer_load_b128(grs, gvoff, soff, 0);
                        __builtin_memcpy(&gv[pr * K1 + q], &rv, sizeof(cplx));
                    }
                }
            }
            const int jw = WAVES * k + w;  // this wave's job
            if (jw < NJOB) {
                const int li = jw / CJ, r = jw - li * CJ, p = r / C, ct = r - p * C;
                const int lev = LEV - li, s = ct * K1 + p;
                if (ct < nct) {
                    cplx *X = buf + w * BUF_STRIDE;
                    const uint32_t *dg = dig + (s * LPAIRS + ((lev - 1) >> 1)) * 8 * 64 + tt;
                    const int sh = ((lev - 1) & 1) * 16;
                    cplx v[8];
                    // pass 0: twist, DFT8 over m, w[t kk] -> position t + 64 kk
#pragma unroll
                    for (int m = 0; m < 8; m++) {
                        const uint32_t dw = dg[m * 64];
                        const double a0 = (double)(int32_t)__builtin_amdgcn_sbfe(dw, sh, 8);
                        const double a1 = (double)(int32_t)__builtin_amdgcn_sbfe(dw, sh + 8, 8);
                        v[m] = {fma(a0, twr[m].re, -(a1 * twr[m].im)), fma(a0, twr[m].im, a1 * twr[m].re)};
                    }
                    dft8<false>(v, w81, w83);
                    X[pidx(tt)] = v[0];
#pragma unroll
                    for (int kk = 1; kk < 8; kk++) X[pidx(tt + 64 * kk)] = cmul(v[kk], w0r[kk - 1]);
                    br1024::wave_sync();
                    s_setprio_c<2>();
                    // pass 1: points 64 gg + uu + 8 m, w[8 uu kk]
                    {
                        const int gg = tt >> 3, uu = tt & 7;
#pragma unroll
                        for (int m = 0; m < 8; m++) v[m] = X[pidx(64 * gg + uu + 8 * m)];
                        dft8<false>(v, w81, w83);
                        X[pidx(64 * gg + uu)] = v[0];
#pragma unroll
                        for (int kk = 1; kk < 8; kk++) X[pidx(64 * gg + uu + 8 * kk)] = cmul(v[kk], w1r[kk - 1]);
                    }
                    br1024::wave_sync();
                    s_setprio_c<1>();
                    // pass 2: points 8 t + m, no twiddles
#pragma unroll
                    for (int m = 0; m < 8; m++) v[m] = X[pidx(8 * tt + m)];
                    dft8<false>(v, w81, w83);
#pragma unroll
                    for (int kk = 0; kk < 8; kk++) X[pidx(8 * tt + kk)] = v[kk];
                }
            }
            SPROF(2);
            br512::lds_sync();
            SPROF(1);
            s_setprio_c<3>();
            // MAC at Fourier position pos over the pass's jobs in job order: accumulator (q, ct) = accr[q C + ct]
#pragma unroll
            for (int jj = 0; jj < WAVES; jj++) {
                if (WAVES * k + jj < NJOB) {
                    const int ct = jj % C;
                    const cplx x = buf[jj * BUF_STRIDE + pidx(pos)];
#pragma unroll
                    for (int q = 0; q < K1; q++) {
                        const cplx gg = gv[(jj / C) * K1 + q];
                        double re = accr[q * C + ct].re, im = accr[q * C + ct].im;
                        re = fma(x.re, gg.re, re);
                        re = fma(-x.im, gg.im, re);
                        im = fma(x.re, gg.im, im);
                        im = fma(x.im, gg.re, im);
                        accr[q * C + ct] = {re, im};
                    }
                }
            }
            SPROF(3);
            br512::lds_sync();
            SPROF(1);
            s_setprio_c<3>();
        }
        // ---- inverse FFT of the MAC results, accumulated into ACC ----
#pragma unroll
        for (int q = 0; q < K1; q++)
#pragma unroll
            for (int c = 0; c < C; c++) buf[(c * K1 + q) * BUF_STRIDE + pidx(pos)] = accr[q * C + c];
        br512::lds_sync();
        s_setprio_c<3>();
        if (w < CJ) {
            cplx *Y = buf + w * BUF_STRIDE;
            cplx v[8];
            // inverse pass 2: points 8 t + kk, no twiddles
#pragma unroll
            for (int kk = 0; kk < 8; kk++) v[kk] = Y[pidx(8 * tt + kk)];
            dft8<true>(v, w81, w83);
#pragma unroll
            for (int m = 0; m < 8; m++) Y[pidx(8 * tt + m)] = v[m];
            br1024::wave_sync();
            // inverse pass 1: conj(w[8 uu kk]) on points 64 gg + uu + 8 kk
            {
                const int gg = tt >> 3, uu = tt & 7;
                v[0] = Y[pidx(64 * gg + uu)];
#pragma unroll
                for (int kk = 1; kk < 8; kk++) v[kk] = cmul(Y[pidx(64 * gg + uu + 8 * kk)], cconj(w1r[kk - 1]));
                dft8<true>(v, w81, w83);
#pragma unroll
                for (int m = 0; m < 8; m++) Y[pidx(64 * gg + uu + 8 * m)] = v[m];
            }
            br1024::wave_sync();
            s_setprio_c<2>();
            // inverse pass 0: conj(w[t kk]) on points t + 64 kk, untwist, from_torus, ACC +=
            v[0] = Y[pidx(tt)];
#pragma unroll
            for (int kk = 1; kk < 8; kk++) v[kk] = cmul(Y[pidx(tt + 64 * kk)], cconj(w0r[kk - 1]));
            dft8<true>(v, w81, w83);
            uint64_t *poly = acc + w * ACC_STRIDE;
#pragma unroll
            for (int m = 0; m < 8; m++) {
                const int j = tt + 64 * m;
                const cplx t = cmul(v[m], cconj(twr[m]));  // = untwist[j] * 2^9 exactly
                bool o0, o1;
                uint64_t a0 = torus_add_fast_sh<LOG2M>(t.re, poly[j], o0), a1 = torus_add_fast_sh<LOG2M>(t.im, poly[j + M], o1);
                if (__builtin_amdgcn_ballot_w64(!(o0 && o1))) {  // zeros, out-of-range magnitudes (rare)
                    a0 = poly[j] + from_torus_bits(t.re * 0x1p-9);
                    a1 = poly[j + M] + from_torus_bits(t.im * 0x1p-9);
                }
                poly[j] = a0;
                poly[j + M] = a1;
            }
        }
        SPROF(4);
        br512::lds_sync();  // the next decomposition reads every polynomial
        SPROF(1);
    }
#ifdef TAE_B1KS_PROF
    if (blockIdx.x == 0 && tt == 0)
        printf("b1ksprof wave %d: dec %llu bar %llu fft %llu mac %llu inv %llu\n", w, (unsigned long long)sprof_[0],
               (unsigned long long)sprof_[1], (unsigned long long)sprof_[2], (unsigned long long)sprof_[3],
               (unsigned long long)sprof_[4]);
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

}  // namespace br1024s
}  // namespace tae
