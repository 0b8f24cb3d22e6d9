// Latency-oriented blind rotation for N = 512, k = 4 (small batches: one AES block is 128 bits):
// ONE ciphertext per 1024-thread workgroup, and the decomposition LEVELS run in parallel instead
// of one after another.  Wave jb < LEV * (k+1) owns FFT job (level jb / (k+1) + 1, polynomial
// jb % (k+1)), so a CMux step is
//   forward FFT of all LEV * (k+1) digit polynomials                    (one wave each) | barrier
//   MAC of all levels: thread task (q, position) = 15 complex terms     -> out[q]       | barrier
//   inverse FFT of the k+1 outputs (waves 0..k), ACC +=, and the next step's decomposition of
//   that polynomial (all levels once; the finer levels to LDS for their FFT waves)       | barrier
// three barriers per step instead of the 2 LEV + 1 of br512x4 (which spends them on three
// ciphertexts per workgroup for throughput).  The FFT jobs reuse br512x4's 4-lane DFT16
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

using br512::BUF_STRIDE;
using br512::K1;
using br512::lds_sync;
using br512::M;
using br512::N;
using br512::pidx;
using br512::u32x4;
using br512::mac_pos;
using br512::wave_sync;
using br512x4::dft16x4;

constexpr int THREADS = 1024;

// TAE_LAT_PROF (debug builds only): per-phase cycle sums of every wave of workgroup 0
#ifdef TAE_LAT_PROF
#define LPROF_DECL uint64_t lprof_[8] = {0}, lprof_t_ = clock64();
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
              uint64_t out_add, const cplx *__restrict__ twist, const cplx *__restrict__ wtab) {
    static_assert(LEV * K1 <= THREADS / 64, "one wave per (level, polynomial) job");
    constexpr int LOGN = 9, JOBS = LEV * K1;
    extern __shared__ __align__(16) unsigned char smem[];
    uint64_t *acc = reinterpret_cast<uint64_t *>(smem);             // [K1][N]
    cplx *buf = reinterpret_cast<cplx *>(acc + K1 * N);             // [JOBS][BUF_STRIDE] spectra
    cplx *obuf = buf + JOBS * BUF_STRIDE;                           // [K1][BUF_STRIDE] MAC results
    cplx *s_tw = obuf + K1 * BUF_STRIDE;                            // twist e^{i pi j / N}
    cplx *s_twa = s_tw + M;                                         // [16 a + b] = W_M^{a b}
    cplx *s_utw = s_twa + M;                                        // conj(twist) 2^-8 (exact)
    cplx *s_w16 = s_utw + M;                                        // [r][3]: W16^{r k1}
    uint32_t *s_dig = reinterpret_cast<uint32_t *>(s_w16 + 12);     // [LEV-1][K1][4][64] digits
    const long ct = blockIdx.x;
    if (ct >= B) return;  // whole workgroup
    const int tid = threadIdx.x;
    const int jb = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63, u = lane & 15, r = lane >> 4;
    const bool fjob = jb < JOBS;
    const int jlev = fjob ? jb / K1 + 1 : 1, jp = fjob ? jb - (jb / K1) * K1 : 0;
    const uint64_t *in = lwe_in + (size_t)ct * (n + 1);

    for (int t = tid; t < M; t += THREADS) {
        s_tw[t] = twist[t];
        s_twa[t] = wtab[(t >> 4) * (t & 15)];
        s_utw[t] = cplx{twist[t].re * 0x1p-8, -twist[t].im * 0x1p-8};
    }
    if (tid < 12) {
        const int rr = tid / 3, k1 = tid - 3 * rr + 1;
        const int e = (rr * k1) & 15;
        const cplx w = wtab[16 * e];
        s_w16[tid] = e == 0 ? cplx{1.0, 0.0} : (e == 4 ? cplx{0.0, -1.0} : w);
    }
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
    // MAC tasks (q, position): q = tid / 256 for every thread, and q = 4 also for waves 12-15 (one
    // wave per SIMD, so each SIMD runs five task-waves)
    const int pos0 = mac_pos(tid & (M - 1)), q0 = tid >> 8;
    const cplx *my_w16 = s_w16 + 3 * r;
    int ll = lane;
    asm volatile("" : "+v"(ll));

    // MAC task (q, pos): 15 complex terms, levels descending, rows ascending, the oracle's fma chain
    // (the GGSW rows are L2 hits thanks to the prefetch below)
    auto mac_task = [&](int q, int pos, int gstep) {
        double re = 0.0, im = 0.0;
#pragma unroll
        for (int lev = LEV; lev >= 1; lev--) {
            cplx g[K1];
#pragma unroll
            for (int p = 0; p < K1; p++) {
                const int soff = gstep + (((lev - 1) * K1 + p) * K1 + q) * M * (int)sizeof(cplx);
                const u32x4 rv = __builtin_amdgcn_raw_buffer_load_b128(grs, pos * (int)sizeof(cplx), soff, 0);
                __builtin_memcpy(&g[p], &rv, sizeof(cplx));
            }
#pragma unroll
            for (int p = 0; p < K1; p++) {
                const cplx x = buf[((lev - 1) * K1 + p) * BUF_STRIDE + pidx(pos)];
                re = fma(x.re, g[p].re, re);
                re = fma(-x.im, g[p].im, re);
                im = fma(x.re, g[p].im, im);
                im = fma(x.im, g[p].re, im);
            }
        }
        obuf[q * BUF_STRIDE + pidx(pos)] = cplx{re, im};
    };

    // L2 prefetch of the GGSW rows two steps ahead: one dword per 128-byte line (the batch is small,
    // so a step's 307 KB are otherwise first touched -- from HBM -- by the MAC that needs them).  A
    // prefetch's value is consumed (asm register use) one step later, when it has long returned.
    constexpr int GLINES = (int)((ggsw_sz * sizeof(cplx) + 127) / 128);
    constexpr int PF = (GLINES + THREADS - 1) / THREADS;
    uint32_t pf_prev[PF], pf_cur[PF];
#pragma unroll
    for (int i = 0; i < PF; i++) pf_prev[i] = 0;
    // Decomposition of polynomial jb (waves 0..k, the level-1 jobs, which also own output q = jb of
    // the inverse FFT and so update ACC polynomial jb): all levels at once, once per polynomial;
    // level 1 stays in registers, the finer levels go to LDS for the waves of those jobs.
    uint32_t mydig[4];
    auto decompose_poly = [&](int e) {
        const uint64_t *poly = acc + jb * N;
        const int bt = ll - e;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int j = ll + 64 * i;
            const int t = (bt + 64 * i) & (2 * N - 1);
            const int ph = t & (N - 1);
            const uint64_t m0 = (uint64_t)(int64_t)((t << 22) >> 31);
            const uint64_t m1 = (uint64_t)(int64_t)(((t + M) << 22) >> 31);
            const uint64_t v0 = poly[ph], v1 = poly[ph ^ M];
            const uint64_t p0 = poly[j], p1 = poly[j + M];
            const uint64_t x0 = (v0 ^ m0) - (p0 + m0), x1 = (v1 ^ m1) - (p1 + m1);
            uint32_t dp[LEV];
            decompose16p<LEV, BLOG>(x0, x1, dp);
            mydig[i] = dp[0];
#pragma unroll
            for (int l = 1; l < LEV; l++) s_dig[(((l - 1) * K1 + jb) * 4 + i) * 64 + ll] = dp[l];
        }
    };
    if (jb < K1 && n > 0) decompose_poly(mod_switch(in[0], LOGN) % (2 * N));
    lds_sync();
    LPROF_DECL
    for (int step = 0; step < n; step++) {
        const int gstep = step * (int)(ggsw_sz * sizeof(cplx));
#ifndef TAE_LAT_NOPF
        if (step + 2 < n) {
#pragma unroll
            for (int i = 0; i < PF; i++) {
                const int line = tid + THREADS * i;
                pf_cur[i] = line < GLINES ? __builtin_amdgcn_raw_buffer_load_b32(
                                                grs, line * 128, gstep + 2 * (int)(ggsw_sz * sizeof(cplx)), 0)
                                          : 0u;
            }
        }
#pragma unroll
        for (int i = 0; i < PF; i++) {
            asm volatile("" ::"v"(pf_prev[i]));
            pf_prev[i] = pf_cur[i];
        }
#endif
        if (fjob) {
            uint32_t dig[4];
            if (jb < K1) {  // level 1: computed by this wave at the end of the previous step
#pragma unroll
                for (int i = 0; i < 4; i++) dig[i] = mydig[i];
            } else {
#pragma unroll
                for (int i = 0; i < 4; i++) dig[i] = s_dig[(((jlev - 2) * K1 + jp) * 4 + i) * 64 + ll];
            }
            LPROF(0);
            // pass A (column u): twist, DFT16 over m = r + 4 i, W_M^{u k} -> position u + 16 k
            cplx *dst = buf + jb * BUF_STRIDE;
            cplx v[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const double a0 = br512::lo16(dig[i]), a1 = br512::hi16(dig[i]);
                const cplx tw = s_tw[ll + 64 * i];
                v[i] = {fma(a0, tw.re, -(a1 * tw.im)), fma(a0, tw.im, a1 * tw.re)};
            }
            dft16x4<false>(v, my_w16);
#pragma unroll
            for (int k2 = 0; k2 < 4; k2++) {
                const int kq = r + 4 * k2;
                dst[pidx(u + 16 * kq)] = cmul(v[k2], s_twa[16 * kq + u]);
            }
            wave_sync();
            LPROF(1);
            // pass B (row u): DFT16 over positions 16 u + r + 4 i, in place
#pragma unroll
            for (int i = 0; i < 4; i++) v[i] = dst[pidx(16 * u + r + 4 * i)];
            dft16x4<false>(v, my_w16);
#pragma unroll
            for (int k2 = 0; k2 < 4; k2++) dst[pidx(16 * u + r + 4 * k2)] = v[k2];
        }
        LPROF(2);
        lds_sync();
        LPROF(3);
        mac_task(q0, pos0, gstep);
        if (tid >= 3 * M) mac_task(K1 - 1, pos0, gstep);
        LPROF(4);
        lds_sync();
        LPROF(5);
        if (jb < K1) {  // inverse FFT of output q = jb, ACC +=
            cplx *base = obuf + jb * BUF_STRIDE;
            cplx v[4];
#pragma unroll
            for (int i = 0; i < 4; i++) v[i] = base[pidx(16 * u + r + 4 * i)];
            dft16x4<true>(v, my_w16);
#pragma unroll
            for (int k2 = 0; k2 < 4; k2++) base[pidx(16 * u + r + 4 * k2)] = v[k2];
            wave_sync();
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int kk = r + 4 * i;
                v[i] = cmul(base[pidx(u + 16 * kk)], cconj(s_twa[16 * kk + u]));
            }
            dft16x4<true>(v, my_w16);
            uint64_t *poly = acc + jb * N;
#pragma unroll
            for (int k2 = 0; k2 < 4; k2++) {
                const int j = ll + 64 * k2;
                const cplx t = cmul(v[k2], s_utw[j]);
                poly[j] += from_torus_bits(t.re);
                poly[j + M] += from_torus_bits(t.im);
            }
            wave_sync();
            if (step + 1 < n) decompose_poly(mod_switch(in[step + 1], LOGN) % (2 * N));
        }
        LPROF(6);
        lds_sync();
        LPROF(7);
    }
#ifdef TAE_LAT_PROF
    if (blockIdx.x == 0 && lane == 0)
        printf("latprof wave %2d: dec %llu passA %llu passB %llu bar1 %llu mac %llu bar2 %llu inv %llu bar3 %llu\n", jb,
               (unsigned long long)lprof_[0], (unsigned long long)lprof_[1], (unsigned long long)lprof_[2],
               (unsigned long long)lprof_[3], (unsigned long long)lprof_[4], (unsigned long long)lprof_[5],
               (unsigned long long)lprof_[6], (unsigned long long)lprof_[7]);
#endif
    uint64_t *o = out + (size_t)ct * ((K1 - 1) * N + 1);
    for (int t = tid; t < (K1 - 1) * N; t += THREADS) {
        const int p = t / N, j = t - p * N;
        o[t] = j == 0 ? acc[p * N] : (0 - acc[p * N + N - j]);
    }
    if (tid == 0) o[(K1 - 1) * N] = acc[(K1 - 1) * N] + out_add;
}

inline size_t lds_bytes(int lev) {
    return (size_t)K1 * N * 8 + (size_t)(lev * K1 + K1) * BUF_STRIDE * 16 + 3 * (size_t)M * 16 + 12 * 16 +
           (size_t)(lev - 1) * K1 * 4 * 64 * 4;
}

}  // namespace br512lat
}  // namespace tae
