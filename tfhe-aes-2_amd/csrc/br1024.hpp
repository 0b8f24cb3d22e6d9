// Batched blind rotation for N = 1024, k = 2 (the 8-bit model's set, shortint_woppbs_8bit.rs:39-86,
// and params_sqrd_lvl_1/4/256): C = 2 ciphertexts per 512-thread workgroup.
//
// Every FFT job (ciphertext, polynomial) is one wave: lane t runs the radix-8 DFT of each of the
// three passes of the oracle's M = 512 schedule (FftPlan<512>: pass 0 on points t + 64 m, pass 1 on
// 64 (t >> 3) + (t & 7) + 8 m, pass 2 on 8 t + m, twiddles w[u k], w[8 u k], none), exchanging
// through the job's own LDS region (wave-local, no barrier).  The spectra live one decomposition
// level at a time (pbs_l = 6); the MAC runs with thread = Fourier position (512) over the six
// (q, ct) accumulators, each GGSW value loaded once for both ciphertexts.  Operation order per
// output is the oracle's (explicit fma).  The oracle skips the u k == 0 twiddles; here every lane
// multiplies, and W^0 = (1, -0) is exact, so at most the sign of a zero differs, which no later
// operation turns into a different u64 output (from_torus(+-0) = 0): results are bit-exact, and the
// lane-uniform code drops two selects per twiddle (8-bit CBS launch -3.9%).
// LDS (126 KB): ACC [C][k+1][N] u64, spectra [C (k+1)][576] cplx (+1 pad per 8: conflict-free
// b128 accesses at strides 1, 8 and 64), twist / W_512 / untwist tables.
#pragma once
#include "br512.hpp"
#include "lf1k.hpp"

namespace tae {
namespace br1024 {

// progress-based wave priority (see br512x4.hpp): 3 after a barrier, stepping down through a phase
template <int P>
__device__ __forceinline__ void s_setprio_c() {
#ifndef TAE_X4_NORR
    __builtin_amdgcn_s_setprio(P);
#endif
}

constexpr int N = 1024, M = 512, K1 = 3, THREADS = 512;

// TAE_B1K_PROF (debug builds only): per-phase cycle sums of every wave of workgroup 0
#ifdef TAE_B1K_PROF
#define BPROF_DECL uint64_t bprof_[6] = {0}, bprof_t_ = clock64();
#define BPROF(i)                           \
    do {                                   \
        asm volatile("" ::: "memory");     \
        const uint64_t now_ = clock64();   \
        bprof_[i] += now_ - bprof_t_;      \
        bprof_t_ = now_;                   \
    } while (0)
#else
#define BPROF_DECL
#define BPROF(i) \
    do {         \
    } while (0)
#endif

// a job's lanes are one wave and a wave's LDS operations execute in order: hand-offs inside a job
// only need the compiler not to reorder
__device__ __forceinline__ void wave_sync() { asm volatile("" ::: "memory"); }
constexpr int BUF_STRIDE = M + M / 8;  // cplx
constexpr int ACC_STRIDE = N;          // u64

__device__ __forceinline__ int pidx(int q) { return q + (q >> 3); }

// The MAC thread's Fourier position.  Consecutive positions put 2 lanes of some ds_read_b128 groups on
// one bank (pidx's +1 per 8 makes a wave's 64 slots fall unevenly on the 16 bank groups).  Instead each
// half-wave h takes four runs of 8 positions r = s + 8 j with one class s = h mod 8 and j in {0, 2, 1, 3}
// (+4 for h >= 8): slots 9 r + i then hit every bank group once per 16-lane group (scripts/layout/
// b1k_banks.py checks it); a run is one 128-byte line of every GGSW row, so the row loads stay whole
// lines.  A bijection of the 512 positions (the MAC is per position, the results go back by position).
__device__ __forceinline__ int mac_pos(int tid) {
    const int h = tid >> 5, o = (tid >> 3) & 3;
    const int j = (h & 8 ? 4 : 0) + ((o & 1) << 1) + (o >> 1);
    return 8 * ((h & 7) + 8 * j) + (tid & 7);
}

// c ? a : b on the two doubles (a struct select here went through scratch memory)
__device__ __forceinline__ cplx csel(bool c, cplx a, cplx b) { return {c ? a.re : b.re, c ? a.im : b.im}; }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// msk ? b : a for a wave-uniform all-ones / all-zeros msk, as a VOP3 select on an SGPR pair (the compiler's
// own form reads the condition from VCC)
__device__ __forceinline__ uint32_t sel_sgpr(uint32_t a, uint32_t b, bool c) {
    const uint64_t msk = ((uint64_t)__builtin_amdgcn_readfirstlane(c ? ~0u : 0u) << 32) |
                         __builtin_amdgcn_readfirstlane(c ? ~0u : 0u);
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(msk));
    return r;
}

// dft<8, 512, INV> of fft_device.hpp with the W8 factors from the table (w[64] = W8^1, w[192] = W8^3)
template <bool INV>
__device__ __forceinline__ void dft8(cplx *v, cplx w1, cplx w3) {
    cplx y[8];
#pragma unroll
    for (int n1 = 0; n1 < 2; n1++) dft4<INV>(v[n1], v[n1 + 2], v[n1 + 4], v[n1 + 6]);
#pragma unroll
    for (int k1 = 0; k1 < 4; k1++) y[2 * k1] = v[2 * k1];
    y[1] = v[1];
    y[3] = cmul(v[3], INV ? cconj(w1) : w1);
    y[5] = INV ? cplx{-v[5].im, v[5].re} : cplx{v[5].im, -v[5].re};
    y[7] = cmul(v[7], INV ? cconj(w3) : w3);
#pragma unroll
    for (int k1 = 0; k1 < 4; k1++) {
        const cplx a = y[2 * k1], b = y[2 * k1 + 1];
        v[k1] = cadd(a, b);
        v[k1 + 4] = csub(a, b);
    }
}

// Mode: PBS -> GGSW_i = bsk + i * ggsw_sz, per-ciphertext rotation a~_i; steps = n.
//       VP  -> GGSW_t = ggsw_f + (g * n_in + b) * ggsw_sz, rotation X^{-2^t} shared; steps = n_in.
// C ciphertexts per workgroup: 2 (6 FFT jobs on 8 waves, GGSW loads shared by both) for batches that
// fill the chip, 1 (3 jobs, one per SIMD) for small batches -- e.g. the 8-bit model's extract_bits
// rounds of one byte per block, where C = 2 would leave half the CUs idle.  LP levels per pass: with
// C = 1 and an even level count, LP = 2 runs the FFTs of two decomposition levels together (6 jobs on
// 8 waves instead of 3), halving the level passes and their barriers; the MAC still consumes the
// levels in descending order.
// (HIP: the second launch bound is the minimum waves per SIMD.)
// OCC workgroups per CU: 1 (two waves per SIMD, 256 VGPRs) or 2 (C = 1 workgroups, four waves per SIMD,
// <= 128 VGPRs: the lane's fused-DFT8 constants and twiddles read from LDS at each use; the two workgroups'
// barriers are independent, so one's MAC can run beside the other's FFTs).
template <int LEV, bool PBS, int BLOG, int C, int LP, int OCC = 1>
__global__ void __launch_bounds__(THREADS, 2 * OCC)
    br_kernel(const uint64_t *__restrict__ lwe_in, int n, const uint64_t *__restrict__ lut, int n_out,
              const cplx *__restrict__ ggsw_base, int n_in, uint64_t *__restrict__ out, long B,
              uint64_t body_add, uint64_t out_add, const cplx *__restrict__ twist, const cplx *__restrict__ untwist,
              const cplx *__restrict__ wtab, const double *__restrict__ lf, uint64_t *__restrict__ clk) {
    static_assert(LEV % LP == 0, "levels per pass must divide the level count");
    // the 8-bit model's PBS runs the fused-twiddle transform (lf1k.hpp) on a BSK rescaled by conj(E2)
    constexpr bool LFT = PBS && LEV == 6 && BLOG == 7;
    ClockStamp stamp;
    stamp.start(clk);
    constexpr int LOGN = 10, CJ = C * K1, JOBS = CJ * LP;
    extern __shared__ __align__(16) unsigned char smem[];
    uint64_t *acc = reinterpret_cast<uint64_t *>(smem);           // [CJ][ACC_STRIDE]
    cplx *buf = reinterpret_cast<cplx *>(acc + CJ * ACC_STRIDE);  // [JOBS][BUF_STRIDE], job = (lh, ct, p)
    double *s_lf = reinterpret_cast<double *>(buf + JOBS * BUF_STRIDE);  // LFT: lf1k.hpp's table, else:
    const cplx *s_untw = reinterpret_cast<const cplx *>(s_lf + lf1k::UNTW);
    cplx *s_tw = buf + JOBS * BUF_STRIDE;                           // twist
    cplx *s_w = s_tw + M;                                           // W_512 table
    cplx *s_utw = s_w + M;                                          // untwist = conj(twist) / M
    // per-lane twiddles of passes 0 and 1 in lane order: s_w[t k] / s_w[8 (t & 7) k] read straight from
    // the W table put 2-8 lanes of a b128 group on one bank (PMC: conflict cycles ~ all LDS cycles)
    cplx *s_w0 = s_utw + M;                                         // [k - 1][t] = W_512^{t k}, k = 1..7
    cplx *s_w1 = s_w0 + 7 * 64;                                     // [k - 1][uu] = W_512^{8 uu k}
    const int tid = threadIdx.x;
    const int jb = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int t = tid & 63;
    const bool fjob = jb < JOBS;
    const int jcp = fjob ? jb % CJ : 0;  // (ct, p) of the job
    const int jlh = fjob ? jb / CJ : 0;  // level offset inside a pass
    const int jct = jcp / K1;
    const size_t ggsw_sz = (size_t)LEV * K1 * K1 * M;

    long ct0, g = 0;
    int nct;
    if (PBS) {
        ct0 = (long)blockIdx.x * C;
        nct = (int)min((long)C, B - ct0);
    } else {
        // XCD-aware order (br512x4.hpp): a group's workgroups share one XCD's L2
        const int nwg = (int)gridDim.x, q8 = nwg >> 3, r8 = nwg & 7, x8 = (int)blockIdx.x & 7;
        const int lb = x8 * q8 + min(x8, r8) + ((int)blockIdx.x >> 3);
        const int per_group = (n_out + C - 1) / C;
        g = lb / per_group;
        ct0 = (long)(lb - g * per_group) * C;
        nct = min(C, n_out - (int)ct0);
    }
    const bool jvalid = fjob && jct < nct;

    if constexpr (LFT) {
        for (int i = tid; i < lf1k::KERNEL_DOUBLES; i += THREADS) s_lf[i] = lf[i];
    } else {
        for (int i = tid; i < M; i += THREADS) {
            s_tw[i] = twist[i];
            s_w[i] = wtab[i];
            s_utw[i] = untwist[i];
        }
        for (int i = tid; i < 7 * 64; i += THREADS) s_w0[i] = wtab[(i & 63) * ((i >> 6) + 1)];
        if (tid < 7 * 8) s_w1[tid] = wtab[8 * (tid & 7) * ((tid >> 3) + 1)];
    }
    const cplx *gbase = PBS ? ggsw_base : ggsw_base + (size_t)g * n_in * ggsw_sz;
    const uint32_t gbytes = (uint32_t)((size_t)(PBS ? n : n_in) * ggsw_sz * sizeof(cplx));
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc((void *)gbase, (short)0, gbytes, 0x00020000);
    const int pos = mac_pos(tid);  // MAC: Fourier position
    const int gvoff = pos * (int)sizeof(cplx);

    for (int i = tid; i < CJ * N; i += THREADS) {
        const int job = i / N, j = i - job * N;
        const int ct = job / K1, c = job - ct * K1;
        uint64_t v = 0;
        if (ct < nct) {
            if (PBS) {
                const uint64_t *in = lwe_in + (size_t)(ct0 + ct) * (n + 1);
                const int bt = mod_switch(in[n] + body_add, LOGN);
                const int e0 = (2 * N - (bt % (2 * N))) % (2 * N);
                v = rotated_coeff(lut + c * N, j, e0, N);
            } else {
                v = c < K1 - 1 ? 0 : lut[(size_t)(ct0 + ct) * N + j];
            }
        }
        acc[job * ACC_STRIDE + j] = v;
    }
    br512::lds_sync();
    const cplx w81 = LFT ? wtab[64] : s_w[64], w83 = LFT ? wtab[192] : s_w[192];
    // The lane's pass-0 / pass-1 twiddles are the same for every FFT of the launch. With LP = 1 the
    // register budget (two waves per SIMD) holds them, which saves 14 LDS reads per FFT job: the CBS
    // launch (C = 2, 2048 ciphertexts) takes 64.1 ms instead of 70.9, same box. The LP = 2 variant
    // would spill.
    constexpr bool WREG = LP == 1 && OCC == 1;
    cplx w0r[7], w1r[7];
    // LFT: likewise the lane's fused-DFT8 constants of the forward passes 1 / 2 and the inverse passes
    // 1 / 0, and the lane-uniform ones of pass 0
    lf1k::K8 kf1, kf2, ki1, ki0;
    lf1k::P0c k0;
    if constexpr (LFT) {
        k0 = lf1k::p0(lf);
        if constexpr (WREG) {
            kf1 = lf1k::k8(s_lf, lf1k::F1, 8, t >> 3);
            kf2 = lf1k::k8(s_lf, lf1k::F2, 64, t);
            ki1 = lf1k::k8(s_lf, lf1k::I1, 8, t & 7);
            ki0 = lf1k::k8(s_lf, lf1k::I0, 64, t);
        }
    } else if constexpr (WREG) {
#pragma unroll
        for (int kk = 1; kk < 8; kk++) {
            w0r[kk - 1] = s_w0[(kk - 1) * 64 + (tid & 63)];
            w1r[kk - 1] = s_w1[(kk - 1) * 8 + (tid & 7)];
        }
    }
    // likewise the lane's eight twist factors of pass 0, for the 8-bit model's shapes where it was
    // measured (62.2 vs 64.1 ms for the CBS launch, same box, although its PBS instantiation then
    // spills 18 VGPRs outside the FFT passes; the lvl_1/4/256 shapes would spill more, unmeasured)
    constexpr bool TWREG = WREG && BLOG <= 7 && !LFT;
    cplx twr[8];
    if constexpr (TWREG) {
#pragma unroll
        for (int m = 0; m < 8; m++) twr[m] = s_tw[(tid & 63) + 64 * m];
    }
#define TW_AT(m) (TWREG ? twr[m] : s_tw[tt + 64 * (m)])
#define W0_AT(kk) (WREG ? w0r[(kk) - 1] : s_w0[((kk) - 1) * 64 + tt])
#define W1_AT(kk) (WREG ? w1r[(kk) - 1] : s_w1[((kk) - 1) * 8 + uu])
#define KF1 (WREG ? kf1 : lf1k::k8(s_lf, lf1k::F1, 8, gg))
#define KF2 (WREG ? kf2 : lf1k::k8(s_lf, lf1k::F2, 64, tt))
#define KI1 (WREG ? ki1 : lf1k::k8(s_lf, lf1k::I1, 8, uu))
#define KI0 (WREG ? ki0 : lf1k::k8(s_lf, lf1k::I0, 64, tt))

    const int steps = PBS ? n : n_in;
    uint64_t a_next = (PBS && jvalid) ? lwe_in[(size_t)(ct0 + jct) * (n + 1)] : 0;
    cplx accr[K1 * C];
    cplx gv[LP * K1 * K1];
    BPROF_DECL
    for (int step = 0; step < steps; step++) {
        s_setprio_c<2>();
        int e, gstep;
        if (PBS) {
            const uint64_t a = a_next;
            if (step + 1 < steps && jvalid) a_next = lwe_in[(size_t)(ct0 + jct) * (n + 1) + step + 1];
            e = mod_switch(a, LOGN) % (2 * N);
            gstep = step * (int)(ggsw_sz * sizeof(cplx));
        } else {
            const int b = n_in - 1 - step;
            e = 2 * N - (1 << step);
            gstep = b * (int)(ggsw_sz * sizeof(cplx));
        }
        // ---- rotated difference + decomposition of coefficients j = t + 64 m (+ M) ----
        int tt = t;
        asm volatile("" : "+v"(tt));
        // digits: int16 pairs (x_j, x_{j+M}) per level, or for base_log <= 7 (the 8-bit model, up to 6
        // levels) int8 quadruples holding two levels, so that the per-level loop needs no indexed array
        constexpr bool BYTES = BLOG <= 7;
        constexpr int DW = BYTES ? (LEV + 1) / 2 : LEV;
        uint32_t dig[DW][8];
        if (fjob) {
            const uint64_t *poly = acc + jcp * ACC_STRIDE;
            const int bt = tt - e;
#pragma unroll
            for (int m = 0; m < 8; m++) {
                const int j = tt + 64 * m;
                const int ti = (bt + 64 * m) & (2 * N - 1);  // entry of [ACC, -ACC]
                const int ph = ti & (N - 1);
                const uint64_t m0 = (uint64_t)(int64_t)((ti << 21) >> 31);
                const uint64_t m1 = (uint64_t)(int64_t)(((ti + M) << 21) >> 31);
                const uint64_t v0 = poly[ph], v1 = poly[ph ^ M];
                const uint64_t p0 = poly[j], p1 = poly[j + M];
                const uint64_t x0 = (v0 ^ m0) - (p0 + m0), x1 = (v1 ^ m1) - (p1 + m1);
                // both coefficients at once with 16-bit SIMD ops (fft_device.hpp decompose16p: level l's
                // digits of x0 / x1 in the low / high half of dp[l])
                uint32_t dp[LEV];
                decompose16p<LEV, BLOG>(x0, x1, dp);
                if constexpr (BYTES) {
#pragma unroll
                    for (int w = 0; w < DW; w++)  // bytes (x0, x1) of level 2w, then of level 2w + 1
                        dig[w][m] = 2 * w + 1 < LEV ? perm_b32(dp[2 * w + 1], dp[2 * w], 0x06040200u)
                                                    : perm_b32(dp[2 * w], dp[2 * w], 0x00000200u) & 0xFFFFu;
                } else {
#pragma unroll
                    for (int l = 0; l < LEV; l++) dig[l][m] = dp[l];
                }
            }
        }
#pragma unroll
        for (int a = 0; a < K1 * C; a++) accr[a] = cplx{0.0, 0.0};

        BPROF(0);
        for (int lev0 = LEV; lev0 >= 1; lev0 -= LP) {
            // the level's GGSW values at this thread's Fourier position: before the FFTs (their L2 latency
            // hidden behind them), or with OCC = 2 after the barrier (the register budget; the other
            // workgroup of the CU runs meanwhile)
            auto load_gv = [&] {
#pragma unroll
                for (int lh = 0; lh < LP; lh++)
#pragma unroll
                    for (int p = 0; p < K1; p++)
#pragma unroll
                        for (int q = 0; q < K1; q++) {
                            const int soff = gstep + (((lev0 - lh - 1) * K1 + p) * K1 + q) * M * (int)sizeof(cplx);
                            const u32x4 rv = __builtin_amdgcn_raw_buffer_load_b128(grs, gvoff, soff, 0);
                            __builtin_memcpy(&gv[(lh * K1 + p) * K1 + q], &rv, sizeof(cplx));
                        }
            };
            if constexpr (OCC == 1) load_gv();
            const int lev = lev0 - jlh;  // this wave's level
            if (fjob) {
                cplx *X = buf + jb * BUF_STRIDE;
                cplx v[8];
                if constexpr (LFT) {
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
                } else {
                // pass 0: twist, DFT8 over m, w[t kk] -> position t + 64 kk
#pragma unroll
                for (int m = 0; m < 8; m++) {
                    double a0, a1;
                    if constexpr (BYTES) {
                        const int wsel = (lev - 1) >> 1, sh = ((lev - 1) & 1) * 16;
                        uint32_t dw = dig[0][m];
#ifdef TAE_B1K_SGPRSEL
#pragma unroll
                        for (int w = 1; w < DW; w++) dw = sel_sgpr(dw, dig[w][m], wsel == w);
#else
#pragma unroll
                        for (int w = 1; w < DW; w++) {  // mask select (a ternary became a scratch index)
                            const uint32_t msk = 0u - (uint32_t)(wsel == w);
                            dw = (dw & ~msk) | (dig[w][m] & msk);
                        }
#endif
                        a0 = (double)(int32_t)__builtin_amdgcn_sbfe(dw, sh, 8);
                        a1 = (double)(int32_t)__builtin_amdgcn_sbfe(dw, sh + 8, 8);
                    } else {
                        uint32_t dw = dig[0][m];
#pragma unroll
                        for (int l = 1; l < LEV; l++) dw = lev - 1 == l ? dig[l][m] : dw;
                        a0 = br512::lo16(dw);
                        a1 = br512::hi16(dw);
                    }
                    const cplx tw = TW_AT(m);
                    v[m] = {fma(a0, tw.re, -(a1 * tw.im)), fma(a0, tw.im, a1 * tw.re)};
                }
                dft8<false>(v, w81, w83);
                X[pidx(tt)] = v[0];
#pragma unroll
                for (int kk = 1; kk < 8; kk++) {
                    const cplx tv = cmul(v[kk], W0_AT(kk));
                    X[pidx(tt + 64 * kk)] = tv;  // W^0 = 1 exactly: only the sign of a zero can differ from skipping it
                }
                }
                wave_sync();
                if (lev0 == LEV) s_setprio_c<1>(); else s_setprio_c<2>();
                // pass 1: points 64 gg + uu + 8 m, w[8 uu kk]
                {
                    const int gg = tt >> 3, uu = tt & 7;
#pragma unroll
                    for (int m = 0; m < 8; m++) v[m] = X[pidx(64 * gg + uu + 8 * m)];
                    if constexpr (LFT) {
                        lf1k::dft8<false>(v, KF1);
#pragma unroll
                        for (int kk = 0; kk < 8; kk++) X[pidx(64 * gg + uu + 8 * kk)] = v[kk];
                    } else {
                        dft8<false>(v, w81, w83);
                        X[pidx(64 * gg + uu)] = v[0];
#pragma unroll
                        for (int kk = 1; kk < 8; kk++) {
                            const cplx tv = cmul(v[kk], W1_AT(kk));
                            X[pidx(64 * gg + uu + 8 * kk)] = tv;  // W^0 = 1 exactly: only the sign of a zero can differ from skipping it
                        }
                    }
                }
                wave_sync();
                if (lev0 == LEV) s_setprio_c<0>(); else s_setprio_c<1>();
                // pass 2: points 8 t + m, no twiddles
#pragma unroll
                for (int m = 0; m < 8; m++) v[m] = X[pidx(8 * tt + m)];
                if constexpr (LFT) lf1k::dft8<false>(v, KF2);
                else dft8<false>(v, w81, w83);
#pragma unroll
                for (int kk = 0; kk < 8; kk++) X[pidx(8 * tt + kk)] = v[kk];
            }
            BPROF(1);
            br512::lds_sync();
            BPROF(2);
            s_setprio_c<3>();
            if constexpr (OCC == 2) load_gv();
            // MAC at Fourier position pos: accumulator (q, c) = accr[q * C + c]; levels descending, p ascending
#pragma unroll
            for (int lp = 0; lp < LP * K1; lp++) {
                const int lh = lp / K1, p = lp - lh * K1;
                // (no priority step-down inside the MAC: stepping down at 1/3 and 2/3 of it took the
                // CBS launch 61.1 -> 62.3 ms, same box)
                cplx x[C];
#pragma unroll
                for (int c = 0; c < C; c++) x[c] = buf[((lh * C + c) * K1 + p) * BUF_STRIDE + pidx(pos)];
#pragma unroll
                for (int q = 0; q < K1; q++)
#pragma unroll
                    for (int c = 0; c < C; c++) {
                        const cplx gg = gv[lp * K1 + q];
                        double re = accr[q * C + c].re, im = accr[q * C + c].im;
                        re = fma(x[c].re, gg.re, re);
                        re = fma(-x[c].im, gg.im, re);
                        im = fma(x[c].re, gg.im, im);
                        im = fma(x[c].im, gg.re, im);
                        accr[q * C + c] = {re, im};
                    }
            }
            BPROF(3);
            br512::lds_sync();
            BPROF(2);
            s_setprio_c<3>();
        }
        // ---- inverse FFT of the MAC results, accumulated into ACC ----
#pragma unroll
        for (int q = 0; q < K1; q++)
#pragma unroll
            for (int c = 0; c < C; c++) buf[(c * K1 + q) * BUF_STRIDE + pidx(pos)] = accr[q * C + c];
        br512::lds_sync();
        s_setprio_c<3>();
        if (jb < CJ) {
            cplx *Y = buf + jb * BUF_STRIDE;
            cplx v[8];
            // inverse pass 2: points 8 t + kk, no twiddles
#pragma unroll
            for (int kk = 0; kk < 8; kk++) v[kk] = Y[pidx(8 * tt + kk)];
            dft8<true>(v, w81, w83);
#pragma unroll
            for (int m = 0; m < 8; m++) Y[pidx(8 * tt + m)] = v[m];
            wave_sync();
            // inverse pass 1: conj(w[8 uu kk]) on points 64 gg + uu + 8 kk
            {
                const int gg = tt >> 3, uu = tt & 7;
                if constexpr (LFT) {
#pragma unroll
                    for (int kk = 0; kk < 8; kk++) v[kk] = Y[pidx(64 * gg + uu + 8 * kk)];
                    lf1k::dft8<true>(v, KI1);
                } else {
                    v[0] = Y[pidx(64 * gg + uu)];
#pragma unroll
                    for (int kk = 1; kk < 8; kk++) {
                        const cplx y = Y[pidx(64 * gg + uu + 8 * kk)];
                        const cplx tv = cmul(y, cconj(W1_AT(kk)));
                        v[kk] = tv;  // W^0 = 1 exactly: only the sign of a zero can differ from skipping it
                    }
                    dft8<true>(v, w81, w83);
                }
#pragma unroll
                for (int m = 0; m < 8; m++) Y[pidx(64 * gg + uu + 8 * m)] = v[m];
            }
            wave_sync();
            s_setprio_c<2>();
            // inverse pass 0: conj(w[t kk]) on points t + 64 kk, untwist, from_torus, ACC +=
            if constexpr (LFT) {
#pragma unroll
                for (int kk = 0; kk < 8; kk++) v[kk] = Y[pidx(tt + 64 * kk)];
                lf1k::dft8<true>(v, KI0);
            } else {
                v[0] = Y[pidx(tt)];
#pragma unroll
                for (int kk = 1; kk < 8; kk++) {
                    const cplx y = Y[pidx(tt + 64 * kk)];
                    const cplx tv = cmul(y, cconj(W0_AT(kk)));
                    v[kk] = tv;  // W^0 = 1 exactly: only the sign of a zero can differ from skipping it
                }
                dft8<true>(v, w81, w83);
            }
            uint64_t *poly = acc + jb * ACC_STRIDE;
#pragma unroll
            for (int m = 0; m < 8; m++) {
                const int j = tt + 64 * m;
                // untwist; LFT: by conj(twist), the 2^-9 going into the exponent (exact)
                constexpr int SH = LFT ? 9 : 0;
                constexpr double SC = LFT ? 0x1p-9 : 1.0;
                const cplx t = cmul(v[m], LFT ? s_untw[j] : s_utw[j]);
                bool o0, o1;
                uint64_t a0 = torus_add_fast_sh<SH>(t.re, poly[j], o0), a1 = torus_add_fast_sh<SH>(t.im, poly[j + M], o1);
                if (__builtin_amdgcn_ballot_w64(!(o0 && o1))) {  // zeros, out-of-range magnitudes (rare)
                    a0 = poly[j] + from_torus_bits(t.re * SC);
                    a1 = poly[j + M] + from_torus_bits(t.im * SC);
                }
                poly[j] = a0;
                poly[j + M] = a1;
            }
        }
        // LP > 1: the second-level waves decompose polynomials the first-level waves just updated
        if constexpr (LP > 1) br512::lds_sync();
        else wave_sync();
        BPROF(4);
    }
#ifdef TAE_B1K_PROF
    if (blockIdx.x == 0 && (tid & 63) == 0)
        printf("b1kprof wave %d: dec %llu fft %llu bar %llu mac %llu inv %llu\n", jb, (unsigned long long)bprof_[0],
               (unsigned long long)bprof_[1], (unsigned long long)bprof_[2], (unsigned long long)bprof_[3],
               (unsigned long long)bprof_[4]);
#endif
    br512::lds_sync();
    for (int ct = 0; ct < nct; ct++) {
        const uint64_t *a = acc + ct * K1 * ACC_STRIDE;
        uint64_t *o = PBS ? out + (size_t)(ct0 + ct) * (K1 - 1) * N + (size_t)(ct0 + ct)
                          : out + ((size_t)g * n_out + ct0 + ct) * ((K1 - 1) * N + 1);
        for (int i = tid; i < (K1 - 1) * N; i += THREADS) {
            const int p = i / N, j = i - p * N;
            o[i] = j == 0 ? a[p * ACC_STRIDE] : (0 - a[p * ACC_STRIDE + N - j]);
        }
        if (tid == 0) o[(K1 - 1) * N] = a[(K1 - 1) * ACC_STRIDE] + out_add;
    }
    stamp.stop(clk);
}

#undef W0_AT
#undef W1_AT
#undef TW_AT
#undef KF1
#undef KF2
#undef KI1
#undef KI0

// lft: the fused-twiddle transform's table (22 KiB) in place of br1024's twiddle tables (31 KiB)
inline size_t lds_bytes(int C, int LP = 1, bool lft = false) {
    return (size_t)C * K1 * ACC_STRIDE * 8 + (size_t)C * K1 * LP * BUF_STRIDE * 16 +
           (lft ? (size_t)lf1k::KERNEL_DOUBLES * 8 : 3 * (size_t)M * 16 + (7 * 64 + 7 * 8) * 16);
}

// (levels, base_log) combinations of the N=1024 parameter sets: returns the kernel or nullptr
typedef void (*kernel_t)(const uint64_t *, int, const uint64_t *, int, const cplx *, int, uint64_t *, long, uint64_t,
                         uint64_t, const cplx *, const cplx *, const cplx *, const double *, uint64_t *);
// The kernels are instantiated in their own translation unit (br1024_inst.hip, Makefile B1KFLAGS: -O2 there is
// -0.7% per 8192-bootstrap launch, same box); other files reach them through these selectors.
// the 8-bit model's PBS as one ciphertext per workgroup at two workgroups per CU (OCC = 2)
kernel_t pick_occ2(int levels, int base_log);
// LP levels per pass; LP = 2 only for the PBS with at least two passes (nullptr otherwise)
template <int C, int LP = 1>
kernel_t pick(bool pbs, int levels, int base_log);

#ifdef TAE_B1K_INSTANTIATE
kernel_t pick_occ2(int levels, int base_log) {
    if (levels == 6 && base_log == 7) return (kernel_t)br_kernel<6, true, 7, 1, 1, 2>;
    return nullptr;
}

template <int C, int LP>
kernel_t pick(bool pbs, int levels, int base_log) {
#define TAE_BR1024(L, BL)                                                                                  \
    if constexpr (LP == 1)                                                                                 \
        if (levels == L && base_log == BL)                                                                 \
            return pbs ? (kernel_t)br_kernel<L, true, BL, C, LP> : (kernel_t)br_kernel<L, false, BL, C, LP>; \
    if constexpr (LP == 2 && L % 2 == 0 && L >= 4)                                                         \
        if (pbs && levels == L && base_log == BL) return (kernel_t)br_kernel<L, true, BL, C, LP>;
    TAE_BR1024(6, 7)   // 8-bit model PBS (shortint_woppbs_8bit.rs:39-86)
    TAE_BR1024(4, 6)   // 8-bit model CBS GGSW
    TAE_BR1024(2, 15)  // params_sqrd_lvl_1 / _4 PBS
    TAE_BR1024(4, 9)   // params_sqrd_lvl_256 PBS
    TAE_BR1024(1, 10)  // lvl_1 CBS
    TAE_BR1024(1, 11)  // lvl_4 CBS
    TAE_BR1024(1, 14)  // lvl_256 CBS
#undef TAE_BR1024
    return nullptr;
}

template kernel_t pick<2, 1>(bool, int, int);
template kernel_t pick<1, 1>(bool, int, int);
template kernel_t pick<1, 2>(bool, int, int);
#endif

}  // namespace br1024
}  // namespace tae
