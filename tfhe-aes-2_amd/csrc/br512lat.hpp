// Latency-oriented blind rotation for N = 512, k = 4 (small batches: one AES block is 128 bits):
// ONE ciphertext per 1024-thread workgroup, and the decomposition LEVELS run in parallel instead
// of one after another.  Wave jb < LEV * (k+1) owns FFT job (level jb / (k+1) + 1, polynomial
// jb % (k+1)).  A CMux step is five barrier-separated phases:
//   D  decomposition of the rotated difference ACC * X^e - ACC of all k+1 polynomials, all levels
//      at once, spread over all 16 waves (coefficient pairs (p, j), j < N/2), digits -> LDS
//   F  forward FFT of all LEV * (k+1) digit polynomials (one wave each); the MAC's GGSW loads are
//      issued before the FFT work so that they land during it
//   M  MAC: thread chain (q, position) = 15 complex terms -> out[q]; 1280 chains on 1024 threads,
//      waves 0-3 run two chains (q = 0 and 4) of one position, sharing its spectrum reads (holding
//      the next level's rows in registers as well spills: 80 VGPRs of GGSW values alone; the level
//      loop stays rolled, else the scheduler hoists all three levels' loads and spills)
//   I1 inverse FFT of the k+1 outputs (waves 0..k); the other waves issue the L2 prefetch of the
//      GGSW rows two steps ahead, so that no phase waits on it
//   I2 untwist, torus conversion and ACC += of the k+1 outputs spread over all 16 waves (in I1 they
//      were a third of the inverse waves' VALU work, on a SIMD that runs two of the five jobs)
// The per-phase profile of the previous layout (TAE_LAT_PROF) had the decomposition inside the
// inverse phase (five waves, single-wave issue rate) and three dependent GGSW load rounds per MAC
// chain behind the vmcnt of the prefetch loads.  The FFT jobs use br512x4's 4-lane DFT16
// (dft16x4), and every output keeps the oracle's operation order (levels descending, rows
// ascending, the same fma chain): results are bit-identical to br512x4 and the oracle.  Only the
// PBS flavour (homomorphic_shift_boolean) is instantiated.  Each workgroup loads the GGSW rows for
// its single ciphertext, so at large batches br512x4 (three ciphertexts per GGSW load) wins;
// Engine::bootstrap picks by batch size.
#pragma once
#include "br512.hpp"
#include "br512x4.hpp"

namespace tae {
namespace br512lat {

using br512x4::BUF_STRIDE;  // br512x4's bank-conflict-free spectrum layout (sidx), with the raw inverse
using br512x4::SF;          // outputs of I1 at natural index j < 256 in the same 290-slot regions
using br512x4::SG1;
using br512x4::SG3;
using br512x4::sidx;
using br512::K1;
using br512::lds_sync;
using br512::M;
using br512::N;
using br512::u32x4;
using br512::wave_sync;
using br512x4::dft16x4;

constexpr int THREADS = 1024;

// TAE_LAT_PROF (debug builds only): per-phase cycle sums of every wave of workgroup 0
#ifdef TAE_LAT_PROF
#define LPROF_DECL uint64_t lprof_[9] = {0}, lprof_t_ = clock64();
#define LPROF(i)                           \
    do {                                   \
        asm volatile("" ::: "memory");     \
        const uint64_t now_ = clock64();   \
        lprof_[i] += now_ - lprof_t_;      \
        lprof_t_ = now_;                   \
    } while (0)
#else
#define LPROF_DECL
#define LPROF(i) \
    do {         \
    } while (0)
#endif

template <int LEV, int BLOG>
__global__ void __launch_bounds__(THREADS, 1)
    br_kernel(const uint64_t *__restrict__ lwe_in, int n, const uint64_t *__restrict__ lut,
              const cplx *__restrict__ bsk, uint64_t *__restrict__ out, long B, uint64_t body_add,
              uint64_t out_add, const double *__restrict__ lf) {
    static_assert(LEV * K1 <= THREADS / 64, "one wave per (level, polynomial) job");
    constexpr int LOGN = 9, JOBS = LEV * K1;
    extern __shared__ __align__(16) unsigned char smem[];
    uint64_t *acc = reinterpret_cast<uint64_t *>(smem);             // [K1][N]
    cplx *buf = reinterpret_cast<cplx *>(acc + K1 * N);             // [JOBS][BUF_STRIDE] spectra
    cplx *obuf = buf + JOBS * BUF_STRIDE;                           // [K1][BUF_STRIDE] MAC results
    double *s_lf = reinterpret_cast<double *>(obuf + K1 * BUF_STRIDE);  // the fused transform's table (lf512.hpp)
    const cplx *s_untw = reinterpret_cast<const cplx *>(s_lf + lf512::UNTW);
    uint32_t *s_dig = reinterpret_cast<uint32_t *>(s_lf + lf512::KERNEL_DOUBLES);  // [LEV][K1][N/2] packed digit pairs
    const long ct = blockIdx.x;
    if (ct >= B) return;  // whole workgroup
    const int tid = threadIdx.x;
    const int jb = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63, u = lane & 15, r = lane >> 4;
    const bool fjob = jb < JOBS;
    const int jlev = fjob ? jb / K1 + 1 : 1, jp = fjob ? jb - (jb / K1) * K1 : 0;
    const uint64_t *in = lwe_in + (size_t)ct * (n + 1);

    for (int t = tid; t < lf512::KERNEL_DOUBLES; t += THREADS) s_lf[t] = lf[t];
    const double lf_s2 = lf[lf512::CONSTS], lf_c8 = lf[lf512::CONSTS + 1], lf_t8 = lf[lf512::CONSTS + 2];
    {
        const int bt = mod_switch(in[n] + body_add, LOGN);
        const int e0 = (2 * N - (bt % (2 * N))) % (2 * N);
        for (int t = tid; t < K1 * N; t += THREADS) {
            const int c = t / N, j = t - c * N;
            acc[t] = rotated_coeff(lut + c * N, j, e0, N);
        }
    }
    lds_sync();

    const size_t ggsw_sz = (size_t)LEV * K1 * K1 * M;
    const uint32_t gbytes = (uint32_t)((size_t)n * ggsw_sz * sizeof(cplx));
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc((void *)bsk, (short)0, gbytes, 0x00020000);
    // MAC chains: thread tid runs chain (q = tid >> 8, pos); threads tid < 256 also run (q = 4, pos)
    const int pos = tid & (M - 1), qa = tid >> 8, spos = sidx(pos);
    const int baseA = SF[4 * (u & 3) + r] + SG1[u >> 2], baseB = SF[4 * r + (u & 3)] + SG3[u >> 2];
    const bool two = tid < M;
    const int goff = pos * (int)sizeof(cplx);
    int ll = lane;
    asm volatile("" : "+v"(ll));

    // GGSW value (lev, p, q) of this thread's position at step offset gstep: the wave-uniform part of
    // the offset goes to the scalar operand, q (per thread for chain a) to the vector one
    auto gload = [&](int gstep, int lev, int p, int q, bool qvec) {
        const int soff = gstep + (((lev - 1) * K1 + p) * K1 + (qvec ? 0 : q)) * M * (int)sizeof(cplx);
        const int voff = goff + (qvec ? q * M * (int)sizeof(cplx) : 0);
        const u32x4 rv = __builtin_amdgcn_raw_buffer_load_b128(grs, voff, soff, 0);
        cplx g;
        __builtin_memcpy(&g, &rv, sizeof(cplx));
        return g;
    };

    // L2 prefetch of the GGSW rows two steps ahead, one dword per 128-byte line, issued by the waves
    // that are idle during the inverse phase; a prefetch's value is consumed (asm register use) a step
    // later, when it has long returned, so it never holds back a vmcnt wait of the MAC.  Every
    // workgroup reads the same rows, and workgroups b and b + 8 share an XCD (and its L2: blocks are
    // dealt round-robin over the 8 XCDs), so the workgroups of one XCD split the lines between them.
    constexpr int PFW = THREADS - K1 * 64;  // prefetching threads (waves K1..15)
    constexpr int GLINES = (int)((ggsw_sz * sizeof(cplx) + 127) / 128);
    constexpr int PF = (GLINES + PFW - 1) / PFW;
    const int xg = (int)(ct & 7), xrank = (int)(ct >> 3), xcnt = (int)((B - xg + 7) >> 3);
    const int pf_n = (GLINES + xcnt - 1) / xcnt;  // lines of this workgroup: xrank + xcnt * i
    uint32_t pf_prev[PF];
#pragma unroll
    for (int i = 0; i < PF; i++) pf_prev[i] = 0;

    LPROF_DECL
    for (int step = 0; step < n; step++) {
        const int gstep = step * (int)(ggsw_sz * sizeof(cplx));
        // ---- D: decomposition of the rotated difference, pairs (p, j) and (p, j + N/2) ----
        {
            const int e = mod_switch(in[step], LOGN) % (2 * N);
            for (int t = tid; t < K1 * M; t += THREADS) {
                const int p = t >> 8, j = t & (M - 1);
                const uint64_t *poly = acc + p * N;
                const int tt = (j - e) & (2 * N - 1);  // coefficient j of ACC * X^e: entry tt of [ACC, -ACC]
                const int ph = tt & (N - 1);
                const uint64_t m0 = (uint64_t)(int64_t)((tt << 22) >> 31);
                const uint64_t m1 = (uint64_t)(int64_t)(((tt + M) << 22) >> 31);
                const uint64_t v0 = poly[ph], v1 = poly[ph ^ M];
                const uint64_t p0 = poly[j], p1 = poly[j + M];
                const uint64_t x0 = (v0 ^ m0) - (p0 + m0), x1 = (v1 ^ m1) - (p1 + m1);
                uint32_t dp[LEV];
                decompose16p<LEV, BLOG>(x0, x1, dp);
#pragma unroll
                for (int l = 0; l < LEV; l++) s_dig[(l * K1 + p) * M + j] = dp[l];
            }
        }
        LPROF(0);
        lds_sync();
        LPROF(1);
        // ---- F: forward FFTs; this thread's first-level GGSW values are loaded meanwhile ----
        cplx ga[K1], gb[K1];
#pragma unroll
        for (int p = 0; p < K1; p++) ga[p] = gload(gstep, LEV, p, qa, true);
        if (two) {
#pragma unroll
            for (int p = 0; p < K1; p++) gb[p] = gload(gstep, LEV, p, K1 - 1, false);
        }
        if (fjob) {  // the fused-twiddle transform (lf512.hpp), as br512x4's PBS mode
            cplx *dst = buf + jb * BUF_STRIDE;
            uint32_t dw[4];
#pragma unroll
            for (int i = 0; i < 4; i++) dw[i] = s_dig[((jlev - 1) * K1 + jp) * M + ll + 64 * i];
            cplx v[4];
            lf512::a1(dw, v, lf_s2, lf_c8, lf_t8);
            br512::transpose4(v);
            lf512::dft4<false>(v, lf512::k4(s_lf, lf512::FA2, 4, r));
#pragma unroll
            for (int k2 = 0; k2 < 4; k2++) dst[baseA + SG3[k2]] = v[k2];
            wave_sync();
            // pass B (row kappa = u): positions 16 u + r + 4 i, in place
#pragma unroll
            for (int i = 0; i < 4; i++) v[i] = dst[baseB + SG1[i]];
            lf512::dft4<false>(v, lf512::k4(s_lf, lf512::FB1, 16, u));
            br512::transpose4(v);
            lf512::dft4<false>(v, lf512::k4(s_lf, lf512::FB2, 64, lane));
#pragma unroll
            for (int k2 = 0; k2 < 4; k2++) dst[baseB + SG1[k2]] = v[k2];
        }
        LPROF(2);
        lds_sync();
        LPROF(3);
        // ---- M: MAC chains, levels descending, rows ascending, the oracle's fma chain; a level's
        // GGSW values below the first are loaded at its start (L2 hits: every workgroup reads the
        // same rows this step, and the prefetch waves pulled them in two steps earlier) ----
        {
            double ar = 0.0, ai = 0.0, br = 0.0, bi = 0.0;
#pragma unroll 1
            for (int lev = LEV; lev >= 1; lev--) {
                if (lev < LEV) {
#pragma unroll
                    for (int p = 0; p < K1; p++) ga[p] = gload(gstep, lev, p, qa, true);
                    if (two) {
#pragma unroll
                        for (int p = 0; p < K1; p++) gb[p] = gload(gstep, lev, p, K1 - 1, false);
                    }
                }
#pragma unroll
                for (int p = 0; p < K1; p++) {
                    const cplx x = buf[((lev - 1) * K1 + p) * BUF_STRIDE + spos];
                    ar = fma(x.re, ga[p].re, ar);
                    ar = fma(-x.im, ga[p].im, ar);
                    ai = fma(x.re, ga[p].im, ai);
                    ai = fma(x.im, ga[p].re, ai);
                    if (two) {
                        br = fma(x.re, gb[p].re, br);
                        br = fma(-x.im, gb[p].im, br);
                        bi = fma(x.re, gb[p].im, bi);
                        bi = fma(x.im, gb[p].re, bi);
                    }
                }
            }
            obuf[qa * BUF_STRIDE + spos] = cplx{ar, ai};
            if (two) obuf[(K1 - 1) * BUF_STRIDE + spos] = cplx{br, bi};
        }
        LPROF(4);
        lds_sync();
        LPROF(5);
        // ---- I1: inverse FFT of output q = jb (waves 0..k), raw result -> obuf[q][j]; prefetch (the
        // other waves) ----
        if (jb < K1) {
            cplx *base = obuf + jb * BUF_STRIDE;
            cplx v[4];
#pragma unroll
            for (int i = 0; i < 4; i++) v[i] = base[baseB + SG1[i]];
            dft4<true>(v[0], v[1], v[2], v[3]);
            br512::transpose4(v);
            lf512::dft4<true>(v, lf512::k4(s_lf, lf512::IB2, 4, r));
#pragma unroll
            for (int k2 = 0; k2 < 4; k2++) base[baseB + SG1[k2]] = v[k2];
            wave_sync();
#pragma unroll
            for (int i = 0; i < 4; i++) v[i] = base[baseA + SG3[i]];
            lf512::dft4<true>(v, lf512::k4(s_lf, lf512::IA1, 16, u));
            br512::transpose4(v);
            lf512::dft4<true>(v, lf512::k4(s_lf, lf512::IA2, 64, lane));
            wave_sync();  // this wave's reads of base precede its writes below (LDS executes in order)
#pragma unroll
            for (int k2 = 0; k2 < 4; k2++) base[ll + 64 * k2] = v[k2];  // coefficient pair j = ll + 64 k2
        } else if (step + 2 < n) {
#pragma unroll
            for (int i = 0; i < PF; i++) {
                asm volatile("" ::"v"(pf_prev[i]));
                const int k = (tid - K1 * 64) + PFW * i, line = xrank + xcnt * k;
                if (PFW * i < pf_n)  // wave-uniform: no empty instructions for the later slots
                    pf_prev[i] = k < pf_n && line < GLINES
                                     ? __builtin_amdgcn_raw_buffer_load_b32(
                                           grs, line * 128, gstep + 2 * (int)(ggsw_sz * sizeof(cplx)), 0)
                                     : 0u;
            }
        }
        LPROF(6);
        lds_sync();
        // ---- I2: untwist, torus conversion, ACC += over all waves: item t = (q, j) ----
        for (int t = tid; t < K1 * M; t += THREADS) {
            const int q = t >> 8, j = t & (M - 1);  // wave-uniform q (64 consecutive j)
            const cplx x = cmul(obuf[q * BUF_STRIDE + j], s_untw[j]);  // x 2^-8 (exact) in the conversion
            uint64_t *poly = acc + q * N;
            bool o0, o1;
            uint64_t a0 = torus_add_fast_sh<8>(x.re, poly[j], o0), a1 = torus_add_fast_sh<8>(x.im, poly[j + M], o1);
            if (__builtin_amdgcn_ballot_w64(!(o0 && o1))) {  // zeros, out-of-range magnitudes (rare)
                a0 = poly[j] + from_torus_bits(x.re * 0x1p-8);
                a1 = poly[j + M] + from_torus_bits(x.im * 0x1p-8);
            }
            poly[j] = a0;
            poly[j + M] = a1;
        }
        LPROF(7);
        lds_sync();
        LPROF(8);
    }
#pragma unroll
    for (int i = 0; i < PF; i++) asm volatile("" ::"v"(pf_prev[i]));
#ifdef TAE_LAT_PROF
    if (blockIdx.x == 0 && lane == 0)
        printf("latprof wave %2d: dec %llu bar0 %llu fft %llu bar1 %llu mac %llu bar2 %llu inv %llu torus %llu bar3 %llu\n",
               jb, (unsigned long long)lprof_[0], (unsigned long long)lprof_[1], (unsigned long long)lprof_[2],
               (unsigned long long)lprof_[3], (unsigned long long)lprof_[4], (unsigned long long)lprof_[5],
               (unsigned long long)lprof_[6], (unsigned long long)lprof_[7], (unsigned long long)lprof_[8]);
#endif
    uint64_t *o = out + (size_t)ct * ((K1 - 1) * N + 1);
    for (int t = tid; t < (K1 - 1) * N; t += THREADS) {
        const int p = t / N, j = t - p * N;
        o[t] = j == 0 ? acc[p * N] : (0 - acc[p * N + N - j]);
    }
    if (tid == 0) o[(K1 - 1) * N] = acc[(K1 - 1) * N] + out_add;
}

// The instantiation is compiled in its own translation unit (br512lat_inst.hip) with top-down pre-RA machine
// scheduling (Makefile LATFLAGS: -6% per launch, same box; br1024 and the PFKS GEMM lose with it).
#define TAE_LAT_PARAMS                                                                                      \
    const uint64_t *__restrict__, int, const uint64_t *__restrict__, const cplx *__restrict__,            \
        uint64_t *__restrict__, long, uint64_t, uint64_t, const double *__restrict__
#ifndef TAE_LAT_INSTANTIATE
extern template __global__ void br_kernel<3, 12>(TAE_LAT_PARAMS);
#endif

inline size_t lds_bytes(int lev) {
    return (size_t)K1 * N * 8 + (size_t)(lev * K1 + K1) * BUF_STRIDE * 16 + (size_t)lf512::KERNEL_DOUBLES * 8 +
           (size_t)lev * K1 * M * 4;
}

}  // namespace br512lat
}  // namespace tae
