// Batched blind rotation of the 8-bit model (shortint_woppbs_8bit.rs:39-86: N = 1024, k = 2, 6 levels of 2^7)
// with FOUR ciphertexts per workgroup: 12 FFT jobs per level on 12 waves, three per SIMD.
//
// Why: br1024 runs C = 2 ciphertexts on 8 waves (256 VGPRs, two waves per SIMD), so every level
// deals its 6 FFT jobs 2:2:1:1 over the SIMDs, and a SIMD with one busy wave issues a VALU op only every
// ~11-15 cycles (scripts/probes/valu_rates.hip): the SIMDs are about half busy.  Twelve jobs on 768 threads
// keep three job waves on every SIMD through the forward transforms, the inverse and the decomposition, and
// each GGSW value loaded by the MAC feeds four ciphertexts.  The spectra of 12 jobs (108 KB) and the transform
// table (22 KB) fill the LDS, so the accumulator moves out of it:
//   - the ACC of (ciphertext, polynomial) lives in global memory (a stash [B][k+1][N] u64, L2-resident), read
//     and written only by the lane that owns the coefficient (j = t + 64 m and j + 512 of the job's wave), so
//     each lane only reads back its own stores; the first ciphertext's ACC fits the LDS that is left and stays there;
//   - after the inverse, the wave also leaves its new ACC in its own LDS job region (u64 [1024]), where the
//     next step's decomposition reads the rotated coefficients (wave-local, no barrier) before the forward
//     transform overwrites the region.
// Everything else -- the decomposition, the fused-twiddle transform (lf1k.hpp), the MAC's fma chain (levels
// descending, rows ascending), the inverse and the torus conversion -- is br1024's LFT code path operation for
// operation, so the outputs are bit-identical to br1024 and the oracle (or_lf1k_*).
#pragma once
#include "br1024.hpp"

namespace tae {
namespace br1024w {

using br1024::BUF_STRIDE;
using br1024::K1;
using br1024::M;
using br1024::mac_pos;
using br1024::N;
using br1024::pidx;
using br1024::s_setprio_c;
using br1024::wave_sync;

// TAE_B1KW_PROF (debug builds only, never the product): per-phase cycle sums of every wave of one workgroup,
// printed at exit: 0 decomposition, 1 forward transforms, 2 barrier after them, 3 MAC, 4 barrier after it,
// 5 MAC stores + barrier, 6 inverse + ACC update
#ifdef TAE_B1KW_PROF
#define WPROF_DECL uint64_t wprof_[7] = {0}, wprof_t_ = clock64();
#define WPROF(i)                         \
    do {                                 \
        asm volatile("" ::: "memory");   \
        const uint64_t now_ = clock64(); \
        wprof_[i] += now_ - wprof_t_;    \
        wprof_t_ = now_;                 \
    } while (0)
#else
#define WPROF_DECL
#define WPROF(i) \
    do {         \
    } while (0)
#endif

// TAE_B1KW_PRIO2 (A/B knob): a priority step-down after every FFT pass instead of br1024's schedule
#ifdef TAE_B1KW_PRIO2
#define B1KW_PRIO(a, b) s_setprio_c<(b)>()
#else
#define B1KW_PRIO(a, b) s_setprio_c<(a)>()
#endif

constexpr int C = 4, CJ = C * K1, THREADS = 64 * CJ;
static_assert(THREADS == 3 * 256, "one wave per FFT job; the MAC: 256 threads per GGSW column");

// LDS: the 12 job regions, lf1k's table, and the ACC of the workgroup's first ciphertext (its three polynomials
// stay in LDS; the other three ciphertexts use the global stash)
inline size_t lds_bytes() { return (size_t)CJ * BUF_STRIDE * 16 + (size_t)lf1k::KERNEL_DOUBLES * 8 + (size_t)K1 * N * 8; }

// lwe_in [B][n+1], lut the test vector GLWE [(k+1) N], bsk the conj(E2)-rescaled Fourier BSK, out [B][k N + 1],
// acc_g the ACC stash [B][k+1][N]; body_add / out_add as br1024 (homomorphic_shift_boolean); wtab the W_512
// table (its W8 entries), lf lf1k's table.
template <int LEV, int BLOG>
__global__ void __launch_bounds__(THREADS, 3)
    br_kernel(const uint64_t *__restrict__ lwe_in, int n, const uint64_t *__restrict__ lut, const cplx *__restrict__ bsk,
              uint64_t *__restrict__ out, long B, uint64_t body_add, uint64_t out_add, const cplx *__restrict__ wtab,
              const double *__restrict__ lf, uint64_t *__restrict__ acc_g, uint64_t *__restrict__ clk) {
    static_assert(LEV == 6 && BLOG == 7, "the 8-bit model's PBS shape (fused transform, byte digits)");
    constexpr int LOGN = 10, DW = (LEV + 1) / 2;
    ClockStamp stamp;
    stamp.start(clk);
    extern __shared__ __align__(16) unsigned char smem[];
    cplx *buf = reinterpret_cast<cplx *>(smem);                       // [CJ][BUF_STRIDE], job = (ct, p)
    double *s_lf = reinterpret_cast<double *>(buf + CJ * BUF_STRIDE);  // lf1k's table
    const cplx *s_untw = reinterpret_cast<const cplx *>(s_lf + lf1k::UNTW);
    const int tid = threadIdx.x;
    const int jb = __builtin_amdgcn_readfirstlane(tid >> 6);  // job = wave = (ct, p)
    const int t = tid & 63;
    const int jct = jb / K1, jp = jb - jct * K1;
    const long ct0 = (long)blockIdx.x * C;
    const int nct = (int)min((long)C, B - ct0);
    const bool jvalid = jct < nct;
    const size_t ggsw_sz = (size_t)LEV * K1 * K1 * M;
    // this job's region: spectra (cplx) during a step, the job's ACC (u64 [N]) between the inverse and the
    // next decomposition
    cplx *X = buf + jb * BUF_STRIDE;
    uint64_t *Xu = reinterpret_cast<uint64_t *>(X);
    uint64_t *ag = acc_g + ((size_t)(ct0 + jct) * K1 + jp) * N;  // this job's stash (valid jobs only)
    // ciphertext 0's ACC lives in LDS after the table (the LDS has room for one of the four): 25% less stash traffic
    const bool lacc = jct == 0;
    uint64_t *al = reinterpret_cast<uint64_t *>(s_lf + lf1k::KERNEL_DOUBLES) + jp * N;

    for (int i = tid; i < lf1k::KERNEL_DOUBLES; i += THREADS) s_lf[i] = lf[i];
    {  // ACC = X^{-b~} * test vector of this job's polynomial, by the lanes that own the coefficients
        int e0 = 0;
        if (jvalid) {
            const int bt = mod_switch(lwe_in[(size_t)(ct0 + jct) * (n + 1) + n] + body_add, LOGN);
            e0 = (2 * N - (bt % (2 * N))) % (2 * N);
        }
#pragma unroll
        for (int m = 0; m < 16; m++) {
            const int j = t + 64 * m;
            const uint64_t v = jvalid ? rotated_coeff(lut + jp * N, j, e0, N) : 0;
            Xu[j] = v;
            if (lacc) al[j] = v;
            else if (jvalid) ag[j] = v;
        }
    }
    br512::lds_sync();
    const cplx w81 = wtab[64], w83 = wtab[192];
    const lf1k::P0c k0 = lf1k::p0(lf);
    const __amdgpu_buffer_rsrc_t grs =
        __builtin_amdgcn_make_buffer_rsrc((void *)bsk, (short)0, (uint32_t)((size_t)n * ggsw_sz * sizeof(cplx)), 0x00020000);
    // MAC: thread (column q, u) owns the accumulators (q, ct) of the Fourier positions mac_pos(u) and
    // mac_pos(u + 256) for all four ciphertexts (8 accumulators, 6 GGSW values per level; the 256-thread
    // halves of br1024's mac_pos map keep every ds_read_b128 lane group on distinct banks)
    const int mq = __builtin_amdgcn_readfirstlane(tid >> 8), mu = tid & 255;
    const int mpos[2] = {mac_pos(mu), mac_pos(mu + 256)};

    uint64_t a_next = jvalid ? lwe_in[(size_t)(ct0 + jct) * (n + 1)] : 0;
    cplx accr[2 * C];  // [half h][ct]
    cplx gv[K1 * 2];   // [row p][half h]
    WPROF_DECL
    for (int step = 0; step < n; step++) {
        s_setprio_c<2>();
        const uint64_t a = a_next;
        if (step + 1 < n && jvalid) a_next = lwe_in[(size_t)(ct0 + jct) * (n + 1) + step + 1];
        const int e = mod_switch(a, LOGN) % (2 * N);
        const int gstep = step * (int)(ggsw_sz * sizeof(cplx));
        // ---- rotated difference + decomposition of coefficients j = t + 64 m (+ M), from the LDS ACC ----
        int tt = t;
        asm volatile("" : "+v"(tt));
        uint32_t dig[DW][8];
        {
            const int bt = tt - e;
#pragma unroll
            for (int m = 0; m < 8; m++) {
                const int j = tt + 64 * m;
                const int ti = (bt + 64 * m) & (2 * N - 1);  // entry of [ACC, -ACC]
                const int ph = ti & (N - 1);
                const uint64_t m0 = (uint64_t)(int64_t)((ti << 21) >> 31);
                const uint64_t m1 = (uint64_t)(int64_t)(((ti + M) << 21) >> 31);
                const uint64_t v0 = Xu[ph], v1 = Xu[ph ^ M];
                const uint64_t p0 = Xu[j], p1 = Xu[j + M];
                const uint64_t x0 = (v0 ^ m0) - (p0 + m0), x1 = (v1 ^ m1) - (p1 + m1);
                uint32_t dp[LEV];
                decompose16p<LEV, BLOG>(x0, x1, dp);
#pragma unroll
                for (int w = 0; w < DW; w++)  // bytes (x0, x1) of level 2w, then of level 2w + 1
                    dig[w][m] = 2 * w + 1 < LEV ? perm_b32(dp[2 * w + 1], dp[2 * w], 0x06040200u)
                                                : perm_b32(dp[2 * w], dp[2 * w], 0x00000200u) & 0xFFFFu;
            }
        }
        wave_sync();  // the forward transform below overwrites the region the reads above came from
        WPROF(0);
#pragma unroll
        for (int a2 = 0; a2 < 2 * C; a2++) accr[a2] = cplx{0.0, 0.0};

        for (int lev = LEV; lev >= 1; lev--) {
            asm volatile("" : "+v"(tt));  // per level: the lane's LDS / table addresses are re-derived, not held
            // the level's GGSW values (p, mq) at this thread's two positions (latency hidden by the FFTs)
#pragma unroll
            for (int p = 0; p < K1; p++)
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int soff = gstep + (((lev - 1) * K1 + p) * K1 + mq) * M * (int)sizeof(cplx);
                    const br1024::u32x4 rv =
                        __builtin_amdgcn_raw_buffer_load_b128(grs, mpos[h] * (int)sizeof(cplx), soff, 0);
                    __builtin_memcpy(&gv[p * 2 + h], &rv, sizeof(cplx));
                }
#ifdef TAE_B1KW_PRIO2
            s_setprio_c<3>();
#endif
            {
                cplx v[8];
                // fused pass 0 (lf1k::pass0) of the level's digits -> position t + 64 kk
                int dr[8], di[8];
                const int wsel = (lev - 1) >> 1, sh = ((lev - 1) & 1) * 16;
#pragma unroll
                for (int m = 0; m < 8; m++) {
                    uint32_t dw = dig[0][m];
#pragma unroll
                    for (int w = 1; w < DW; w++) {
                        const uint32_t msk = 0u - (uint32_t)(wsel == w);
                        dw = (dw & ~msk) | (dig[w][m] & msk);
                    }
                    dr[m] = __builtin_amdgcn_sbfe(dw, sh, 8);
                    di[m] = __builtin_amdgcn_sbfe(dw, sh + 8, 8);
                }
                lf1k::pass0(dr, di, v, k0);
#pragma unroll
                for (int kk = 0; kk < 8; kk++) X[pidx(tt + 64 * kk)] = v[kk];
                wave_sync();
#ifdef TAE_B1KW_PRIO2
                s_setprio_c<2>();
#else
                if (lev == LEV) s_setprio_c<1>(); else s_setprio_c<2>();
#endif
                {  // pass 1: points 64 gg + uu + 8 m
                    const int gg = tt >> 3, uu = tt & 7;
#pragma unroll
                    for (int m = 0; m < 8; m++) v[m] = X[pidx(64 * gg + uu + 8 * m)];
                    lf1k::dft8<false>(v, lf1k::k8(s_lf, lf1k::F1, 8, gg));
#pragma unroll
                    for (int kk = 0; kk < 8; kk++) X[pidx(64 * gg + uu + 8 * kk)] = v[kk];
                }
                wave_sync();
#ifdef TAE_B1KW_PRIO2
                s_setprio_c<1>();
#else
                if (lev == LEV) s_setprio_c<0>(); else s_setprio_c<1>();
#endif
                // pass 2: points 8 t + m
#pragma unroll
                for (int m = 0; m < 8; m++) v[m] = X[pidx(8 * tt + m)];
                lf1k::dft8<false>(v, lf1k::k8(s_lf, lf1k::F2, 64, tt));
#pragma unroll
                for (int kk = 0; kk < 8; kk++) X[pidx(8 * tt + kk)] = v[kk];
            }
            WPROF(1);
#ifdef TAE_B1KW_PRIO2
            s_setprio_c<0>();
#endif
            br512::lds_sync();
            WPROF(2);
            s_setprio_c<3>();
            // MAC: accumulator (mq, c) at position mpos[h] = accr[h * C + c]; rows p ascending.  The two slot
            // offsets are re-derived here (not 24 hoisted addresses held through the FFTs)
            int mslot[2] = {pidx(mpos[0]), pidx(mpos[1])};
            asm volatile("" : "+v"(mslot[0]), "+v"(mslot[1]));
#pragma unroll
            for (int p = 0; p < K1; p++)
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    cplx x[C];
#pragma unroll
                    for (int c = 0; c < C; c++) x[c] = buf[(c * K1 + p) * BUF_STRIDE + mslot[h]];
                    const cplx gg = gv[p * 2 + h];
#pragma unroll
                    for (int c = 0; c < C; c++) {
                        double re = accr[h * C + c].re, im = accr[h * C + c].im;
                        re = fma(x[c].re, gg.re, re);
                        re = fma(-x[c].im, gg.im, re);
                        im = fma(x[c].re, gg.im, im);
                        im = fma(x[c].im, gg.re, im);
                        accr[h * C + c] = {re, im};
                    }
                }
            WPROF(3);
            br512::lds_sync();
            WPROF(4);
            s_setprio_c<3>();
        }
        // ---- inverse FFT of the MAC results, accumulated into the ACC ----
        {
            int mslot[2] = {pidx(mpos[0]), pidx(mpos[1])};
            asm volatile("" : "+v"(mslot[0]), "+v"(mslot[1]));
#pragma unroll
            for (int h = 0; h < 2; h++)
#pragma unroll
                for (int c = 0; c < C; c++) buf[(c * K1 + mq) * BUF_STRIDE + mslot[h]] = accr[h * C + c];
        }
        br512::lds_sync();
        WPROF(5);
        s_setprio_c<3>();
        {
            asm volatile("" : "+v"(tt));
            // this lane's old ACC coefficients from the stash, issued first (their latency hides behind the passes)
            uint64_t old[16];
#ifdef TAE_B1KW_NOSTASH  // timing-only bound (garbage results): no ACC-stash loads or stores
            if (false) {
#else
            if (lacc) {
#pragma unroll
                for (int m = 0; m < 8; m++) {
                    old[2 * m] = al[tt + 64 * m];
                    old[2 * m + 1] = al[tt + 64 * m + M];
                }
            } else if (jvalid) {
#endif
#pragma unroll
                for (int m = 0; m < 8; m++) {
                    old[2 * m] = ag[tt + 64 * m];
                    old[2 * m + 1] = ag[tt + 64 * m + M];
                }
            } else {
#pragma unroll
                for (int m = 0; m < 16; m++) old[m] = 0;
            }
            cplx v[8];
            // inverse pass 2: points 8 t + kk, plain inverse DFT8
#pragma unroll
            for (int kk = 0; kk < 8; kk++) v[kk] = X[pidx(8 * tt + kk)];
            br1024::dft8<true>(v, w81, w83);
#pragma unroll
            for (int m = 0; m < 8; m++) X[pidx(8 * tt + m)] = v[m];
            wave_sync();
#ifdef TAE_B1KW_PRIO2
            s_setprio_c<2>();
#endif
            {  // inverse pass 1 (fused): points 64 gg + uu + 8 kk
                const int gg = tt >> 3, uu = tt & 7;
#pragma unroll
                for (int kk = 0; kk < 8; kk++) v[kk] = X[pidx(64 * gg + uu + 8 * kk)];
                lf1k::dft8<true>(v, lf1k::k8(s_lf, lf1k::I1, 8, uu));
#pragma unroll
                for (int m = 0; m < 8; m++) X[pidx(64 * gg + uu + 8 * m)] = v[m];
            }
            wave_sync();
            B1KW_PRIO(2, 1);
            // inverse pass 0 (fused): points t + 64 kk, then untwist by conj(twist) (the 2^-9 goes into the
            // torus conversion's exponent), from_torus, ACC +=
#pragma unroll
            for (int kk = 0; kk < 8; kk++) v[kk] = X[pidx(tt + 64 * kk)];
            lf1k::dft8<true>(v, lf1k::k8(s_lf, lf1k::I0, 64, tt));
            wave_sync();  // every lane's spectrum reads above come before the ACC stores into the region
#pragma unroll
            for (int m = 0; m < 8; m++) {
                const int j = tt + 64 * m;
                const cplx tv = cmul(v[m], s_untw[j]);
                bool o0, o1;
                uint64_t a0 = torus_add_fast_sh<9>(tv.re, old[2 * m], o0), a1 = torus_add_fast_sh<9>(tv.im, old[2 * m + 1], o1);
                if (__builtin_amdgcn_ballot_w64(!(o0 && o1))) {  // zeros, out-of-range magnitudes (rare)
                    a0 = old[2 * m] + from_torus_bits(tv.re * 0x1p-9);
                    a1 = old[2 * m + 1] + from_torus_bits(tv.im * 0x1p-9);
                }
                Xu[j] = a0;
                Xu[j + M] = a1;
#ifndef TAE_B1KW_NOSTASH
                if (lacc) {
                    al[j] = a0;
                    al[j + M] = a1;
                } else if (jvalid) {
                    ag[j] = a0;
                    ag[j + M] = a1;
                }
#endif
            }
        }
        wave_sync();  // the next decomposition (this wave) reads these LDS ACC writes (in-order LDS)
#ifdef TAE_B1KW_PROF
        asm volatile("s_waitcnt lgkmcnt(0) vmcnt(0)" ::: "memory");
#endif
        WPROF(6);
    }
#ifdef TAE_B1KW_PROF
    if (blockIdx.x == 100 && t == 0)
        printf("b1kwprof wave %2d: dec %llu fwd %llu barF %llu mac %llu barM %llu store %llu inv %llu\n", jb,
               (unsigned long long)wprof_[0], (unsigned long long)wprof_[1], (unsigned long long)wprof_[2],
               (unsigned long long)wprof_[3], (unsigned long long)wprof_[4], (unsigned long long)wprof_[5],
               (unsigned long long)wprof_[6]);
#endif
    br512::lds_sync();  // sample extraction reads every job's LDS ACC
    for (int ct = 0; ct < nct; ct++) {
        uint64_t *o = out + (size_t)(ct0 + ct) * ((K1 - 1) * N + 1);
        for (int i = tid; i < (K1 - 1) * N; i += THREADS) {
            const int p = i / N, j = i - p * N;
            const uint64_t *a = reinterpret_cast<const uint64_t *>(buf + (ct * K1 + p) * BUF_STRIDE);
            o[i] = j == 0 ? a[0] : (0 - a[N - j]);
        }
        if (tid == 0) o[(K1 - 1) * N] = reinterpret_cast<const uint64_t *>(buf + (ct * K1 + K1 - 1) * BUF_STRIDE)[0] + out_add;
    }
    stamp.stop(clk);
}

#define TAE_B1KW_PARAMS                                                                                        \
    const uint64_t *__restrict__, int, const uint64_t *__restrict__, const cplx *__restrict__,               \
        uint64_t *__restrict__, long, uint64_t, uint64_t, const cplx *__restrict__, const double *__restrict__, \
        uint64_t *__restrict__, uint64_t *__restrict__
#ifndef TAE_B1K_INSTANTIATE
extern template __global__ void br_kernel<6, 7>(TAE_B1KW_PARAMS);
#endif

}  // namespace br1024w
}  // namespace tae
