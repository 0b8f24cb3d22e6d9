// Latency-oriented blind rotation for N = 1024, k = 2 with digits of at most 7 bits (the 8-bit model's
// PBS, shortint_woppbs_8bit.rs:39-86: 6 levels of 2^7) for batches of at most one ciphertext per CU --
// the model's extract_bits rounds, one byte per block, where br1024 runs one or two waves per SIMD in
// every phase.  ONE ciphertext per 1024-thread workgroup; per CMux step:
//   D  decomposition of the rotated difference ACC * X^e - ACC of the 3 polynomials, all levels at
//      once, 1536 coefficient pairs over all 16 waves -> int8 digit pairs in LDS
//   per pass of LP levels (levels descending):
//     F  forward FFT of the LP x 3 digit polynomials, one wave each (br1024's three radix-8 passes);
//        the MAC threads' GGSW rows of the pass's first level are loaded meanwhile
//     M  MAC chains (q, Fourier position): 1536 on 1024 threads (threads < 512 run q = 2 as well),
//        each chain p ascending with the oracle's fma order, the pass's levels descending
//   S  MAC results -> LDS;  I  inverse FFT of the 3 outputs (waves 0-2);  I2 untwist, torus, ACC +=
//      over all 16 waves
// The FFTs are br1024's fused-twiddle transform (lf1k.hpp) and every output keeps br1024's (and the
// oracle's) operation order: results are bit-identical to it.
// LDS (146 KiB): ACC [3][1024] u64, spectra [3 LP][576] cplx, the transform's table, digits [LEV][3][512]
// (int8 pairs).
#pragma once
#include "br1024.hpp"

namespace tae {
namespace br1024lat {

using br1024::BUF_STRIDE;
using br1024::csel;
using br1024::dft8;
using br1024::K1;
using br1024::M;
using br1024::N;
using br1024::pidx;
using br1024::u32x4;
using br1024::wave_sync;

constexpr int THREADS = 1024;

// TAE_B1KL_PROF (debug builds only): per-phase cycle sums of every wave of workgroup 0
#ifdef TAE_B1KL_PROF
#define QPROF_DECL uint64_t qprof_[8] = {0}, qprof_t_ = clock64();
#define QPROF(i)                           \
    do {                                   \
        asm volatile("" ::: "memory");     \
        const uint64_t now_ = clock64();   \
        qprof_[i] += now_ - qprof_t_;      \
        qprof_t_ = now_;                   \
    } while (0)
#else
#define QPROF_DECL
#define QPROF(i) \
    do {         \
    } while (0)
#endif

template <int LEV, int BLOG, int LP>
constexpr size_t lds_bytes() {
    return (size_t)K1 * N * 8 + (size_t)LP * K1 * BUF_STRIDE * 16 + (size_t)lf1k::KERNEL_DOUBLES * 8 +
           (size_t)LEV * K1 * M * 2;
}

template <int LEV, int BLOG, int LP>
__global__ void __launch_bounds__(THREADS, 1)
    br_kernel(const uint64_t *__restrict__ lwe_in, int n, const uint64_t *__restrict__ lut,
              const cplx *__restrict__ bsk, uint64_t *__restrict__ out, long B, uint64_t body_add,
              uint64_t out_add, const cplx *__restrict__ wtab, const double *__restrict__ lf) {
    static_assert(BLOG <= 7, "digits are stored as int8");
    static_assert(LEV == 6 && BLOG == 7, "the fused-twiddle transform's BSK rescale is the 8-bit model's");
    static_assert(LEV % LP == 0 && LP * K1 <= THREADS / 64, "one wave per FFT job of a pass");
    constexpr int LOGN = 10, JOBS = LP * K1, NPAIR = K1 * M;
    extern __shared__ __align__(16) unsigned char smem[];
    uint64_t *acc = reinterpret_cast<uint64_t *>(smem);           // [K1][N]
    cplx *buf = reinterpret_cast<cplx *>(acc + K1 * N);           // [JOBS][BUF_STRIDE], job = (lh, p)
    double *s_lf = reinterpret_cast<double *>(buf + JOBS * BUF_STRIDE);  // lf1k.hpp's table
    const cplx *s_untw = reinterpret_cast<const cplx *>(s_lf + lf1k::UNTW);
    uint16_t *s_dig = reinterpret_cast<uint16_t *>(s_lf + lf1k::KERNEL_DOUBLES);  // [LEV][K1][M]: digit(j) | digit(j + M) << 8
    const long ct = blockIdx.x;
    if (ct >= B) return;  // whole workgroup
    const int tid = threadIdx.x;
    const int jb = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool fjob = jb < JOBS;
    const int jlh = fjob ? jb / K1 : 0, jp = fjob ? jb - (jb / K1) * K1 : 0;
    const uint64_t *in = lwe_in + (size_t)ct * (n + 1);

    for (int i = tid; i < lf1k::KERNEL_DOUBLES; i += THREADS) s_lf[i] = lf[i];
    {
        const int bt = mod_switch(in[n] + body_add, LOGN);
        const int e0 = (2 * N - (bt % (2 * N))) % (2 * N);
        for (int i = tid; i < K1 * N; i += THREADS) {
            const int c = i / N, j = i - c * N;
            acc[i] = rotated_coeff(lut + c * N, j, e0, N);
        }
    }
    br512::lds_sync();

    const size_t ggsw_sz = (size_t)LEV * K1 * K1 * M;
    const uint32_t gbytes = (uint32_t)((size_t)n * ggsw_sz * sizeof(cplx));
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc((void *)bsk, (short)0, gbytes, 0x00020000);
    // MAC chains: (qa = tid >> 9, pos) for every thread, (q = 2, pos) for threads < 512
    const int qa = __builtin_amdgcn_readfirstlane(tid >> 9);  // wave-uniform: the loads' scalar offset
    const bool two = tid < M;
    int pos = 0, goff = 0;  // set per step (see t below)
    auto gload = [&](int gstep, int lev, int p, int q) {
        const int soff = gstep + (((lev - 1) * K1 + p) * K1 + q) * M * (int)sizeof(cplx);
        const u32x4 rv = __builtin_amdgcn_raw_buffer_load_b128(grs, goff, soff, 0);
        cplx g;
        __builtin_memcpy(&g, &rv, sizeof(cplx));
        return g;
    };

    QPROF_DECL
    for (int step = 0; step < n; step++) {
        const int gstep = step * (int)(ggsw_sz * sizeof(cplx));
        // lane index re-materialised per step: hoisted out of the loop, the per-lane LDS addresses of
        // the passes (dozens of them) do not fit beside the FFT state and spill
        int tq = tid;
        asm volatile("" : "+v"(tq));
        pos = br1024::mac_pos(tq & (M - 1));  // bank-conflict-free MAC reads (br1024.hpp)
        goff = pos * (int)sizeof(cplx);
        // ---- D: rotated difference and its digits, pairs (p, j), (p, j + M) ----
        {
            const int e = mod_switch(in[step], LOGN) % (2 * N);
#pragma unroll 1
            for (int i = tq; i < NPAIR; i += THREADS) {
                const int p = i / M, j = i - p * M;
                const uint64_t *poly = acc + p * N;
                const int ti = (j - e) & (2 * N - 1);  // coefficient j of ACC * X^e: entry ti of [ACC, -ACC]
                const int ph = ti & (N - 1);
                const uint64_t m0 = (uint64_t)(int64_t)((ti << 21) >> 31);
                const uint64_t m1 = (uint64_t)(int64_t)(((ti + M) << 21) >> 31);
                const uint64_t v0 = poly[ph], v1 = poly[ph ^ M];
                const uint64_t p0 = poly[j], p1 = poly[j + M];
                const uint64_t x0 = (v0 ^ m0) - (p0 + m0), x1 = (v1 ^ m1) - (p1 + m1);
                uint32_t dp[LEV];  // level l + 1: digit of x0 | digit of x1 << 16 (16-bit patterns)
                decompose16p<LEV, BLOG>(x0, x1, dp);
#pragma unroll
                for (int l = 0; l < LEV; l++) s_dig[(l * K1 + p) * M + j] = (uint16_t)((dp[l] & 0xFF) | ((dp[l] >> 8) & 0xFF00));
            }
        }
        QPROF(0);
        br512::lds_sync();
        QPROF(1);
        br1024::s_setprio_c<3>();  // progress-based priorities as in br1024 (3 after each barrier, 2 / 1 after the
        // FFT passes 0 / 1): 11.06 -> 9.76 ms per 256-ciphertext launch, same box
        double ar = 0.0, ai = 0.0, br = 0.0, bi = 0.0;
#pragma unroll 1
        for (int lev0 = LEV; lev0 >= 1; lev0 -= LP) {
            // ---- F: forward FFT of job (lev0 - jlh, jp); the pass's first-level GGSW rows load meanwhile ----
            cplx ga[LP][K1], gb[LP][K1];
#pragma unroll
            for (int p = 0; p < K1; p++) ga[0][p] = gload(gstep, lev0, p, qa);
            if (two) {
#pragma unroll
                for (int p = 0; p < K1; p++) gb[0][p] = gload(gstep, lev0, p, K1 - 1);
            }
            if (fjob) {
                int t = tq & 63;  // per pass: addresses derived from it are not kept across phases
                asm volatile("" : "+v"(t));
                const int lev = lev0 - jlh;
                const uint16_t *dg = s_dig + ((lev - 1) * K1 + jp) * M;
                cplx *X = buf + jb * BUF_STRIDE;
                cplx v[8];
                // fused pass 0 (lf1k::pass0) -> position t + 64 kk
                {
                    int dr[8], di[8];
#pragma unroll
                    for (int m = 0; m < 8; m++) {
                        const uint32_t w = dg[t + 64 * m];
                        dr[m] = (int8_t)(w & 0xFF);
                        di[m] = (int8_t)(w >> 8);
                    }
                    lf1k::pass0(dr, di, v, lf1k::p0(lf));
                }
                br1024::s_setprio_c<2>();
#pragma unroll
                for (int kk = 0; kk < 8; kk++) X[pidx(t + 64 * kk)] = v[kk];
                wave_sync();
                // fused pass 1: points 64 gg + uu + 8 m
                {
                    const int gg = t >> 3, uu = t & 7;
#pragma unroll
                    for (int m = 0; m < 8; m++) v[m] = X[pidx(64 * gg + uu + 8 * m)];
                    lf1k::dft8<false>(v, lf1k::k8(s_lf, lf1k::F1, 8, gg));
                    br1024::s_setprio_c<1>();
#pragma unroll
                    for (int kk = 0; kk < 8; kk++) X[pidx(64 * gg + uu + 8 * kk)] = v[kk];
                }
                wave_sync();
                // fused pass 2: points 8 t + m
#pragma unroll
                for (int m = 0; m < 8; m++) v[m] = X[pidx(8 * t + m)];
                lf1k::dft8<false>(v, lf1k::k8(s_lf, lf1k::F2, 64, t));
#pragma unroll
                for (int kk = 0; kk < 8; kk++) X[pidx(8 * t + kk)] = v[kk];
            }
            // the pass's other levels' GGSW rows: issued once the FFT state is dead, landing during the
            // barrier wait (before the FFT they would not fit beside it in 128 VGPRs)
            QPROF(2);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int lh = 1; lh < LP; lh++) {
#pragma unroll
                for (int p = 0; p < K1; p++) ga[lh][p] = gload(gstep, lev0 - lh, p, qa);
                if (two) {
#pragma unroll
                    for (int p = 0; p < K1; p++) gb[lh][p] = gload(gstep, lev0 - lh, p, K1 - 1);
                }
            }
            br512::lds_sync();
            QPROF(1);
            br1024::s_setprio_c<3>();
            // ---- M: levels of the pass descending, p ascending, the oracle's fma chain ----
#pragma unroll
            for (int lh = 0; lh < LP; lh++) {
#pragma unroll
                for (int p = 0; p < K1; p++) {
                    const cplx x = buf[(lh * K1 + p) * BUF_STRIDE + pidx(pos)];
                    ar = fma(x.re, ga[lh][p].re, ar);
                    ar = fma(-x.im, ga[lh][p].im, ar);
                    ai = fma(x.re, ga[lh][p].im, ai);
                    ai = fma(x.im, ga[lh][p].re, ai);
                    if (two) {
                        br = fma(x.re, gb[lh][p].re, br);
                        br = fma(-x.im, gb[lh][p].im, br);
                        bi = fma(x.re, gb[lh][p].im, bi);
                        bi = fma(x.im, gb[lh][p].re, bi);
                    }
                }
            }
            QPROF(3);
            br512::lds_sync();  // the next pass's FFTs (or the stores below) overwrite the spectra
            QPROF(1);
            br1024::s_setprio_c<3>();
        }
        // ---- S: MAC results of output q in job region q ----
        buf[qa * BUF_STRIDE + pidx(pos)] = cplx{ar, ai};
        if (two) buf[(K1 - 1) * BUF_STRIDE + pidx(pos)] = cplx{br, bi};
        br512::lds_sync();
        QPROF(4);
        // ---- I: inverse FFT of output q = jb (waves 0..2), untwist, from_torus, ACC += ----
        if (jb < K1) {
            int t = tq & 63;
            asm volatile("" : "+v"(t));
            const cplx w81 = wtab[64], w83 = wtab[192];
            cplx *Y = buf + jb * BUF_STRIDE;
            cplx v[8];
#pragma unroll
            for (int kk = 0; kk < 8; kk++) v[kk] = Y[pidx(8 * t + kk)];
            dft8<true>(v, w81, w83);
#pragma unroll
            for (int m = 0; m < 8; m++) Y[pidx(8 * t + m)] = v[m];
            wave_sync();
            {
                const int gg = t >> 3, uu = t & 7;
#pragma unroll
                for (int kk = 0; kk < 8; kk++) v[kk] = Y[pidx(64 * gg + uu + 8 * kk)];
                lf1k::dft8<true>(v, lf1k::k8(s_lf, lf1k::I1, 8, uu));
#pragma unroll
                for (int m = 0; m < 8; m++) Y[pidx(64 * gg + uu + 8 * m)] = v[m];
            }
            wave_sync();
#pragma unroll
            for (int kk = 0; kk < 8; kk++) v[kk] = Y[pidx(t + 64 * kk)];
            lf1k::dft8<true>(v, lf1k::k8(s_lf, lf1k::I0, 64, t));
            wave_sync();  // this wave's reads of Y precede its writes below (LDS executes in order)
#pragma unroll
            for (int m = 0; m < 8; m++) Y[t + 64 * m] = v[m];  // coefficient pair j = t + 64 m
        }
        br512::lds_sync();
        // ---- I2: untwist, from_torus, ACC += over all 16 waves (in I they were a fifth of the three
        // inverse waves' VALU work): item i = (q, j), wave-uniform q ----
        for (int i = tid; i < K1 * M; i += THREADS) {
            const int q = i >> 9, j = i & (M - 1);
            const cplx tt = cmul(buf[q * BUF_STRIDE + j], s_untw[j]);  // conj(twist); 2^-9 in the exponent
            uint64_t *poly = acc + q * N;
            bool o0, o1;
            uint64_t a0 = torus_add_fast_sh<9>(tt.re, poly[j], o0), a1 = torus_add_fast_sh<9>(tt.im, poly[j + M], o1);
            if (__builtin_amdgcn_ballot_w64(!(o0 && o1))) {  // zeros, out-of-range magnitudes (rare)
                a0 = poly[j] + from_torus_bits(tt.re * 0x1p-9);
                a1 = poly[j + M] + from_torus_bits(tt.im * 0x1p-9);
            }
            poly[j] = a0;
            poly[j + M] = a1;
        }
        QPROF(5);
        br512::lds_sync();  // the next decomposition reads every polynomial
        QPROF(1);
        br1024::s_setprio_c<3>();
    }
#ifdef TAE_B1KL_PROF
    if (blockIdx.x == 0 && (tid & 63) == 0)
        printf("b1klprof wave %2d: dec %llu bar %llu fft %llu mac %llu store %llu inv %llu\n", jb,
               (unsigned long long)qprof_[0], (unsigned long long)qprof_[1], (unsigned long long)qprof_[2],
               (unsigned long long)qprof_[3], (unsigned long long)qprof_[4], (unsigned long long)qprof_[5]);
#endif
    uint64_t *o = out + (size_t)ct * ((K1 - 1) * N + 1);
    for (int i = tid; i < (K1 - 1) * N; i += THREADS) {
        const int p = i / N, j = i - p * N;
        o[i] = j == 0 ? acc[p * N] : (0 - acc[p * N + N - j]);
    }
    if (tid == 0) o[(K1 - 1) * N] = acc[(K1 - 1) * N] + out_add;
}

}  // namespace br1024lat
}  // namespace tae
