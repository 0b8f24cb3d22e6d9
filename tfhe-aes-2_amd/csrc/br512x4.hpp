// Batched blind rotation for N = 512, k = 4 with FOUR waves per SIMD: 1024-thread workgroups, C = 3
// ciphertexts each, ACC and one level of spectra in LDS, every GGSW value loaded from L2 feeding three
// accumulators.  Instantiations: <3, true, 12> the PBS of params_sqrd_lvl_64, <7, true, 6> the
// shortint_1bit bootstrap (a test vector per ciphertext, lut_mod), <1, false, 13> vertical packing.
//
// Every FFT job (ciphertext, polynomial) is one whole wave: lane (u, r) = (lane & 15, lane >> 4)
// holds the four points x[r + 4 i] of column (or row) u of the 16 x 16 FFT.  A DFT16 runs as
//   DFT4 over i in registers -> W16^{r k1} -> 4 x 4 transpose across the lanes u, u+16, u+32, u+48
//   -> DFT4 over r,
// every output getting the oracle's DFT16 operation sequence (tfhe_oracle.c); the W16^0 / W16^4
// factors are generic products with exact (1, 0) / (0, -1) and change nothing but signs of zeros.
// The kernel is bound by VALU issue (scripts/probes/valu_rates.hip: one wave issues a VALU op at
// most every ~14 cycles, four waves keep the SIMD near its ~6-cycle f64 rate): the permlane
// transposes cost ~7% of the launch and moving them to LDS costs more (+15%, the MAC, table and
// pass traffic already keeps LDS about half busy); the torus conversion takes the integer fast path
// (fft_device.hpp torus_add_fast).
// 16 waves (15 jobs + 1 idle) give the SIMDs four waves each; registers are held under 128 per
// lane.  The MAC splits the 15 (q, ct) accumulators of a Fourier position 4/4/4/3 over four
// 256-thread groups (one wave of each group per SIMD).  Lane (u, r) of a job decomposes and
// updates the ACC coefficients j = u + 16 r + 64 i (+ 256), so each LDS access of a wave touches
// 64 consecutive coefficients.
#pragma once
#include "br512.hpp"
#include "lf512.hpp"

namespace tae {
namespace br512x4 {

using br512::K1;
using br512::lds_sync;
using br512::M;
using br512::N;
using br512::swap16;
using br512::swap32;
using br512::u32x4;
using br512::wave_sync;

constexpr int C = 3, JOBS = C * K1, THREADS = 1024;

// Spectrum layout without LDS bank conflicts.  Position q = q0 + 4 q1 + 16 q2 + 64 q3 (base-4 digits) of a
// job's spectrum lives at slot
//   sidx(q) = SF[4 q0 + q2] + SG1[q1] + SG3[q3]          (0 .. 289; BUF_STRIDE 290 complex per job)
// which is affine in q3 for pass A / A^-1 (lane (u, r) = (q0 + 4 q1, q2), register k2 = q3) and in q1 for
// pass B / B^-1 (lane (u, r) = (4 q3 + q2, q0), register i = q1): every access is a per-lane base plus an
// immediate.  The tables come from a search against MI355X_MICROARCH.md's LDS lane groups (ds_read_b128:
// four groups of 16 lanes, 64 banks; ds_write_b128: eight groups of 8 lanes, 32 banks): every group of
// those four passes touches distinct 16-byte bank groups, and so does every group of the MAC reads and
// MAC-result stores with MAC thread t on position t (contiguous GGSW loads).
// The +1-per-16 padding this replaces left 2-way conflicts in every group of the pass-B and A^-1 reads
// (SQ_LDS_BANK_CONFLICT 4.4e9 cycles per launch = 9% of the LDS-array cycles, profiles/r03_*).
constexpr int BUF_STRIDE = 290;
__device__ constexpr int SF[16] = {-36, -45, -39, -38, -37, -30, -44, -31, -22, -55, -29, -20, -47, -28, -14, -53};
constexpr int SG1[4] = {42, 78, 74, 46};
constexpr int SG3[4] = {13, 81, 157, 225};
__host__ __device__ constexpr int sidx(int q) { return SF[4 * (q & 3) + ((q >> 4) & 3)] + SG1[(q >> 2) & 3] + SG3[q >> 6]; }

// Progress-based wave priority: after every barrier a wave starts at priority 3 and steps down as
// it completes parts of the phase, so the SIMD arbiter favours the waves that are behind and the
// four waves of a SIMD reach the next barrier together (oldest-first arbitration otherwise starves
// the youngest wave, whose tail then runs alone with its latencies exposed).
#define PRIO(n) __builtin_amdgcn_s_setprio(n)

// TAE_X4_PROF (debug builds only): per-phase cycle sums (s_memtime) of every wave of one workgroup,
// printed at exit: 0 decomposition, 1 pass A, 2 pass B, 3 barrier after the FFTs, 4 MAC, 5 barrier
// after the MAC, 6 MAC store + barrier, 7 pass B^-1, 8 pass A^-1 + ACC update, 9 end-of-step wait.
#ifdef TAE_X4_PROF
#define PROF_DECL uint64_t prof_[10] = {0}, prof_t_ = clock64();
#define PROF_T(i)                        \
    do {                                 \
        asm volatile("" ::: "memory");   \
        const uint64_t now_ = clock64(); \
        prof_[i] += now_ - prof_t_;      \
        prof_t_ = now_;                  \
    } while (0)
#else
#define PROF_DECL
#define PROF_T(i) \
    do {          \
    } while (0)
#endif

constexpr int ACC_STRIDE = N;

// Timing-only bound builds (garbage results; never the product): TAE_X4_HALFTW computes every twiddle /
// twist product with 2 f64 ops instead of 4; TAE_X4_NOSWAP drops the DFT16 lane transposes entirely.
#ifdef TAE_X4_HALFTW
__device__ __forceinline__ cplx twmul(cplx a, cplx b) { return {fma(a.re, b.re, a.im), fma(a.im, b.im, a.re)}; }
#else
__device__ __forceinline__ cplx twmul(cplx a, cplx b) { return cmul(a, b); }
#endif

// DFT16 over the lanes (u, 0..3) of a row group: in v[i] = x[r + 4 i], out v[k2] = X[r + 4 k2];
// tw[k1 - 1] = W16^{r k1} (forward values).  Stage-1 outputs M[r][k1] are transposed to
// M[0..3][r]: swap32 on k1 bit 1 vs r bit 1, then swap16 on bit 0.  (br512lat's register form.)
template <bool INV>
__device__ __forceinline__ void dft16x4(cplx *v, const cplx *tw) {
    dft4<INV>(v[0], v[1], v[2], v[3]);
    v[1] = twmul(v[1], INV ? cconj(tw[0]) : tw[0]);
    v[2] = twmul(v[2], INV ? cconj(tw[1]) : tw[1]);
    v[3] = twmul(v[3], INV ? cconj(tw[2]) : tw[2]);
#ifndef TAE_X4_NOSWAP
    swap32(v[0], v[2]);
    swap32(v[1], v[3]);
    swap16(v[0], v[1]);
    swap16(v[2], v[3]);
#endif
    dft4<INV>(v[0], v[1], v[2], v[3]);
}

// MAC of one level for group G (accumulators pi = 4G .. min(4G+4, 15), (q, ct) = (pi / 3, pi % 3));
// gv[p * 2 + (q - Q0)], per accumulator p ascending with the oracle's fma chain.
template <int G>
__device__ __forceinline__ void mac_level(const cplx *buf, int pos, cplx *accr, const cplx *gv) {
    constexpr int PI0 = 4 * G, NA = (15 - PI0) < 4 ? (15 - PI0) : 4, Q0 = PI0 / 3;
#pragma unroll
    for (int p = 0; p < K1; p++) {
        if (p == 2) PRIO(2);  // (from row 1 on: 0.2-0.35% slower on two boxes)
        if (p == 3) PRIO(1);
        if (p == 4) PRIO(0);
        cplx x[C];
#pragma unroll
        for (int c = 0; c < C; c++) x[c] = buf[(c * K1 + p) * BUF_STRIDE + pos];
#pragma unroll
        for (int a = 0; a < NA; a++) {
            const int pi = PI0 + a, q = pi / 3, c = pi % 3;
            const cplx gg = gv[p * 2 + (q - Q0)];
            double re = accr[a].re, im = accr[a].im;
            re = fma(x[c].re, gg.re, re);
            re = fma(-x[c].im, gg.im, re);
            im = fma(x[c].re, gg.im, im);
            im = fma(x[c].im, gg.re, im);
            accr[a] = {re, im};
        }
    }
}

template <int G>
__device__ __forceinline__ void mac_store(cplx *buf, int pos, const cplx *accr) {
    constexpr int PI0 = 4 * G, NA = (15 - PI0) < 4 ? (15 - PI0) : 4;
#pragma unroll
    for (int a = 0; a < NA; a++) {
        const int pi = PI0 + a, q = pi / 3, c = pi % 3;
        buf[(c * K1 + q) * BUF_STRIDE + pos] = accr[a];
    }
}

// Mode: PBS -> GGSW_i = bsk + i * ggsw_sz, per-ciphertext rotation a~_i; steps = n.
//       VP  -> GGSW_t = ggsw_f + (g * n_in + b) * ggsw_sz, rotation X^{-2^t} shared; steps = n_in.
template <int LEV, bool PBS, int BLOG>
__global__ void __launch_bounds__(THREADS, 1)
    br_kernel(const uint64_t *__restrict__ lwe_in, int n, const uint64_t *__restrict__ lut, int n_out,
              const cplx *__restrict__ ggsw_base, int n_in, uint64_t *__restrict__ out, long B,
              uint64_t body_add, uint64_t out_add, const cplx *__restrict__ twist, const cplx *__restrict__ wtab,
              const double *__restrict__ lf, uint64_t *__restrict__ clk, long lut_mod = 1) {
    constexpr int LOGN = 9;
    ClockStamp stamp;
    stamp.start(clk);
    extern __shared__ __align__(16) unsigned char smem[];
    uint64_t *acc = reinterpret_cast<uint64_t *>(smem);             // [JOBS][ACC_STRIDE]
    cplx *buf = reinterpret_cast<cplx *>(acc + JOBS * ACC_STRIDE);  // [JOBS][BUF_STRIDE]
    cplx *s_tw = buf + JOBS * BUF_STRIDE;                           // twist e^{i pi j / N}
    cplx *s_twa = s_tw + M;                                         // [16 a + b] = W_M^{a b}
    cplx *s_utw = s_twa + M;                                        // conj(twist) 2^-8 (exact)
    cplx *s_w16 = s_utw + M;                                        // [r][3]: W16^{r k1}, k1 = 1..3
    // PBS mode: the fused-twiddle transform's table (lf512.hpp) in place of the four tables above
    double *s_lf = reinterpret_cast<double *>(s_tw);
    const cplx *s_untw = reinterpret_cast<const cplx *>(s_lf + lf512::UNTW);
    const int tid = threadIdx.x;
    const int jb = __builtin_amdgcn_readfirstlane(tid >> 6);  // job = wave
    const int lane = tid & 63, u = lane & 15, r = lane >> 4;
    const bool fjob = jb < JOBS;
    const int jct = fjob ? jb / K1 : 0;
    const size_t ggsw_sz = (size_t)LEV * K1 * K1 * M;

    long ct0, g = 0;
    int nct;
    if (PBS) {
        ct0 = (long)blockIdx.x * C;
        nct = (int)min((long)C, B - ct0);
    } else {
        // XCD-aware order: blocks b, b + 8, b + 16, ... run on one XCD, so give each XCD a contiguous range of
        // the (group, outputs) order: the workgroups of a group then read its GGSWs from one L2 (round 4: 13.3 GB
        // of L2-miss traffic per launch against 1.7 GB of GGSW, every group's 8 workgroups on 8 XCDs)
        const int nwg = (int)gridDim.x, q8 = nwg >> 3, r8 = nwg & 7, x8 = (int)blockIdx.x & 7;
        const int lb = x8 * q8 + min(x8, r8) + ((int)blockIdx.x >> 3);
        const int per_group = (n_out + C - 1) / C;
        g = lb / per_group;
        ct0 = (long)(lb - g * per_group) * C;
        nct = min(C, n_out - (int)ct0);
    }
    const bool jvalid = fjob && jct < nct;

    if constexpr (PBS) {
        for (int t = tid; t < lf512::KERNEL_DOUBLES; t += THREADS) s_lf[t] = lf[t];
    } else {
        for (int t = tid; t < M; t += THREADS) {
            s_tw[t] = twist[t];
            s_twa[t] = wtab[(t >> 4) * (t & 15)];
            s_utw[t] = cplx{twist[t].re * 0x1p-8, -twist[t].im * 0x1p-8};
        }
    }
    // lane-uniform constants of the fused transform's first stage (scalar registers)
    double lf_s2 = 0, lf_c8 = 0, lf_t8 = 0;
    if constexpr (PBS) {
        lf_s2 = lf[lf512::CONSTS];
        lf_c8 = lf[lf512::CONSTS + 1];
        lf_t8 = lf[lf512::CONSTS + 2];
    }
    if (!PBS && tid < 12) {
        // s_w16[3 r + k1 - 1] = W16^{r k1} = W_M^{16 e}, e = r k1 mod 16; exact 1 and -i for e = 0, 4
        const int rr = tid / 3, k1 = tid - 3 * rr + 1;
        const int e = (rr * k1) & 15;
        const cplx w = wtab[16 * e];
        s_w16[tid] = e == 0 ? cplx{1.0, 0.0} : (e == 4 ? cplx{0.0, -1.0} : w);
    }

    const cplx *gbase = PBS ? ggsw_base : ggsw_base + (size_t)g * n_in * ggsw_sz;
    const uint32_t gbytes = (uint32_t)((size_t)(PBS ? n : n_in) * ggsw_sz * sizeof(cplx));
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc((void *)gbase, (short)0, gbytes, 0x00020000);
    const int grp = jb >> 2;  // MAC group (wave-uniform)
    const int pos = tid & (M - 1);
    const int gvoff = pos * (int)sizeof(cplx);
    const int spos = sidx(pos);
    // per-lane spectrum slots of the FFT passes (see sidx): pass A / A^-1 and pass B / B^-1
    const int baseA = SF[4 * (u & 3) + r] + SG1[u >> 2], baseB = SF[4 * r + (u & 3)] + SG3[u >> 2];
    const int q0 = (4 * grp) / 3;           // first GGSW column of the group
    const int nq = grp == 3 ? 1 : 2;        // columns it needs

    for (int t = tid; t < JOBS * N; t += THREADS) {
        const int job = t / N, j = t - job * N;
        const int ct = job / K1, c = job - ct * K1;
        uint64_t v = 0;
        if (ct < nct) {
            if (PBS) {
                const uint64_t *in = lwe_in + (size_t)(ct0 + ct) * (n + 1);
                const int bt = mod_switch(in[n] + body_add, LOGN);
                const int e0 = (2 * N - (bt % (2 * N))) % (2 * N);
                // PBS: the test vector of ciphertext ct0 + ct (lut_mod > 1: one per ciphertext, shortint_1bit)
                v = rotated_coeff(lut + ((ct0 + ct) % lut_mod) * (K1 * N) + c * N, j, e0, N);
            } else {
                v = c < K1 - 1 ? 0 : lut[(size_t)(ct0 + ct) * N + j];
            }
        }
        acc[job * ACC_STRIDE + j] = v;
    }
    lds_sync();

    const int steps = PBS ? n : n_in;
    uint64_t a_next = (PBS && jvalid) ? lwe_in[(size_t)(ct0 + jct) * (n + 1)] : 0;
    cplx accr[4];
    cplx gv[K1 * 2];
    const cplx *my_w16 = s_w16 + 3 * r;
    cplx *jbuf = buf + jb * BUF_STRIDE;  // this job's spectrum
    PROF_DECL
    for (int step = 0; step < steps; step++) {
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
        // GGSW values (lev, p, q) at this thread's Fourier position, q in this group's columns
        auto load_level = [&](int lev) {
#pragma unroll
            for (int p = 0; p < K1; p++)
#pragma unroll
                for (int qq = 0; qq < 2; qq++) {
                    if (qq < nq) {
                        const int soff = gstep + (((lev - 1) * K1 + p) * K1 + q0 + qq) * M * (int)sizeof(cplx);
                        const u32x4 rv = __builtin_amdgcn_raw_buffer_load_b128(grs, gvoff, soff, 0);
                        __builtin_memcpy(&gv[p * 2 + qq], &rv, sizeof(cplx));
                    }
                }
        };
        PRIO(3);  // (2 here and a step-down in level 3's pass A: +0.5-0.9% time, same box)
        // ---- rotated difference + decomposition of coefficients j = u + 16 r + 64 i (+ M) ----
        int ll = lane;
        asm volatile("" : "+v"(ll));
        // digits of all levels: 16-bit pairs (decompose16p), or for deep decompositions of at most 7-bit
        // digits (shortint_1bit: 7 levels of 2^6) byte pairs, two levels per dword (16 instead of 28 VGPRs)
        constexpr bool DBYTES = PBS && LEV > 3 && BLOG <= 7;
        uint32_t dig[DBYTES ? (LEV + 1) / 2 : LEV][4];
        if (fjob) {
            const uint64_t *poly = acc + jb * ACC_STRIDE;
            // coefficient j of ACC * X^e is entry t = (j - e) mod 2N of [ACC, -ACC]
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
                // both halves at once with 16-bit SIMD ops (fft_device.hpp decompose16p)
                uint32_t dp[LEV];
#ifdef TAE_X4_NODEC  // timing-only bound (garbage results): bit fields instead of the balanced decomposition
#pragma unroll
                for (int l = 0; l < LEV; l++) dp[l] = (uint32_t)(x0 >> (20 * l)) ^ (uint32_t)(x1 >> (20 * l + 8));
#else
                decompose16p<LEV, BLOG>(x0, x1, dp);
#endif
                if constexpr (DBYTES) {
#pragma unroll
                    for (int l = 0; l < LEV; l += 2) {  // bytes 0, 1: level l (j, j + M); bytes 2, 3: level l + 1
                        const uint32_t up = l + 1 < LEV ? dp[(l + 1) % LEV] : 0u;
                        dig[l >> 1][i] = __builtin_amdgcn_perm(up, dp[l], 0x06040200u);
                    }
                } else {
#pragma unroll
                    for (int l = 0; l < LEV; l++) dig[l][i] = dp[l];
                }
            }
        }
#pragma unroll
        for (int a = 0; a < 4; a++) accr[a] = cplx{0.0, 0.0};
        PRIO(2);
        PROF_T(0);

#pragma unroll
        for (int lev = LEV; lev >= 1; lev--) {
            load_level(lev);
            if constexpr (PBS) {
                // fused-twiddle transform (lf512.hpp): pass A = DFT4 of the twisted digits, transpose, fused
                // DFT4 -> LDS position u + 16 k (its W_M^{u k} and psi^u factors ride into pass B)
                if (fjob) {
                    cplx v[4];
                    if constexpr (DBYTES) {
                        const int sh = ((lev - 1) & 1) * 16;  // lev is a compile-time constant (unrolled)
                        int dr[4], di[4];
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            uint32_t dw = dig[0][i];
#pragma unroll
                            for (int w = 1; w < (LEV + 1) / 2; w++)
                                if ((lev - 1) >> 1 == w) dw = dig[w][i];
                            dr[i] = __builtin_amdgcn_sbfe((int)dw, sh, 8);
                            di[i] = __builtin_amdgcn_sbfe((int)dw, sh + 8, 8);
                        }
                        lf512::a1i(dr, di, v, lf_s2, lf_c8, lf_t8);
                    } else {
                        uint32_t dw[4];
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            dw[i] = dig[0][i];
#pragma unroll
                            for (int l = 1; l < LEV; l++)
                                if (lev - 1 == l) dw[i] = dig[l][i];
                        }
                        lf512::a1(dw, v, lf_s2, lf_c8, lf_t8);
                    }
                    br512::transpose4(v);
                    lf512::dft4<false>(v, lf512::k4(s_lf, lf512::FA2, 4, r));
                    if (lev == LEV) PRIO(2);
#pragma unroll
                    for (int k2 = 0; k2 < 4; k2++) jbuf[baseA + SG3[k2]] = v[k2];
                }
                wave_sync();
                PRIO(1);
                PROF_T(1);
                // pass B (row kappa = u): fused DFT4 over the columns r + 4 i, transpose, fused DFT4, in place
                if (fjob) {
                    cplx v[4];
#pragma unroll
                    for (int i = 0; i < 4; i++) v[i] = jbuf[baseB + SG1[i]];
                    lf512::dft4<false>(v, lf512::k4(s_lf, lf512::FB1, 16, u));
                    br512::transpose4(v);
                    lf512::dft4<false>(v, lf512::k4(s_lf, lf512::FB2, 64, lane));
                    PRIO(0);
#pragma unroll
                    for (int k2 = 0; k2 < 4; k2++) jbuf[baseB + SG1[k2]] = v[k2];
                }
            } else {
            // the lane's W16 factors, read once for passes A and B (dead before the MAC, so they do
            // not add to its register peak): 3 of the 11 LDS reads of pass B's LDS-bound phase
            cplx w16[3];
#pragma unroll
            for (int k = 0; k < 3; k++) w16[k] = my_w16[k];
            // pass A (column u): twist, DFT16 over m = r + 4 i, W_M^{u k} -> LDS position u + 16 k
            if (fjob) {
                cplx v[4];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    uint32_t dw = dig[0][i];
#pragma unroll
                    for (int l = 1; l < LEV; l++)
                        if (lev - 1 == l) dw = dig[l][i];
                    const double a0 = br512::lo16(dw), a1 = br512::hi16(dw);
                    const cplx tw = s_tw[ll + 64 * i];
#ifdef TAE_X4_HALFTW
                    v[i] = {fma(a0, tw.re, a1), fma(a1, tw.im, a0)};
#else
                    v[i] = {fma(a0, tw.re, -(a1 * tw.im)), fma(a0, tw.im, a1 * tw.re)};
#endif
                }
                dft16x4<false>(v, w16);
                if (lev == LEV) PRIO(2);  // levels below the first keep 3 through pass A (-0.9%, same box)
#pragma unroll
                for (int k2 = 0; k2 < 4; k2++) {
                    const int k = r + 4 * k2;
                    jbuf[baseA + SG3[k2]] = twmul(v[k2], s_twa[16 * k + u]);
                }
            }
            wave_sync();
            PRIO(1);
            PROF_T(1);
            // pass B (row u): DFT16 over positions 16 u + r + 4 i, in place
            if (fjob) {
                cplx v[4];
#pragma unroll
                for (int i = 0; i < 4; i++) v[i] = jbuf[baseB + SG1[i]];
                dft16x4<false>(v, w16);
                PRIO(0);
#pragma unroll
                for (int k2 = 0; k2 < 4; k2++) jbuf[baseB + SG1[k2]] = v[k2];
            }
            }
            PROF_T(2);
#ifdef TAE_X4_NOBARF  // timing-only bound (garbage): no barrier between the FFTs and the MAC
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#else
            lds_sync();
#endif
            PROF_T(3);
            PRIO(3);
            switch (grp) {
            case 0: mac_level<0>(buf, spos, accr, gv); break;
            case 1: mac_level<1>(buf, spos, accr, gv); break;
            case 2: mac_level<2>(buf, spos, accr, gv); break;
            default: mac_level<3>(buf, spos, accr, gv); break;
            }
            PROF_T(4);
#ifdef TAE_X4_NOBARM  // timing-only bound (garbage): no barrier between a level's MAC and the next level's pass A
            if (lev == 1) lds_sync();
#else
            lds_sync();
#endif
            PROF_T(5);
            PRIO(3);
        }
        // ---- inverse FFT of the MAC results, accumulated into ACC ----
        switch (grp) {
        case 0: mac_store<0>(buf, spos, accr); break;
        case 1: mac_store<1>(buf, spos, accr); break;
        case 2: mac_store<2>(buf, spos, accr); break;
        default: mac_store<3>(buf, spos, accr); break;
        }
        lds_sync();
        PROF_T(6);
        PRIO(3);
        if constexpr (PBS) {
            if (fjob) {  // pass B^-1 (row kappa = u): DFT4 over i, transpose, fused DFT4
                cplx v[4];
#pragma unroll
                for (int i = 0; i < 4; i++) v[i] = jbuf[baseB + SG1[i]];
                dft4<true>(v[0], v[1], v[2], v[3]);
                br512::transpose4(v);
                lf512::dft4<true>(v, lf512::k4(s_lf, lf512::IB2, 4, r));
#pragma unroll
                for (int k2 = 0; k2 < 4; k2++) jbuf[baseB + SG1[k2]] = v[k2];
            }
            wave_sync();
            PROF_T(7);
            PRIO(3);
            if (fjob) {  // pass A^-1 (column u): fused DFT4, transpose, fused DFT4, untwist, from_torus, ACC +=
                cplx v[4];
#pragma unroll
                for (int i = 0; i < 4; i++) v[i] = jbuf[baseA + SG3[i]];
                lf512::dft4<true>(v, lf512::k4(s_lf, lf512::IA1, 16, u));
                br512::transpose4(v);
                lf512::dft4<true>(v, lf512::k4(s_lf, lf512::IA2, 64, lane));
                uint64_t *poly = acc + jb * ACC_STRIDE;
#pragma unroll
                for (int k2 = 0; k2 < 4; k2++) {
                    const int j = ll + 64 * k2;  // m = r + 4 k2 -> j = u + 16 m
                    const cplx t = cmul(v[k2], s_untw[j]);  // x 2^-8 (exact) in the conversion
#ifdef TAE_X4_NOTORUS  // timing-only bound (garbage results): the f64 bit patterns added instead of the conversion
                    uint64_t a0 = poly[j] + f64_bits(t.re), a1 = poly[j + M] + f64_bits(t.im);
#else
                    bool o0, o1;
                    uint64_t a0 = torus_add_fast_sh<8>(t.re, poly[j], o0), a1 = torus_add_fast_sh<8>(t.im, poly[j + M], o1);
                    if (__builtin_amdgcn_ballot_w64(!(o0 && o1))) {  // zeros, out-of-range magnitudes (rare)
                        a0 = poly[j] + from_torus_bits(t.re * 0x1p-8);
                        a1 = poly[j + M] + from_torus_bits(t.im * 0x1p-8);
                    }
#endif
                    poly[j] = a0;
                    poly[j + M] = a1;
                }
            }
        } else {
        cplx w16[3];  // for both inverse passes
#pragma unroll
        for (int k = 0; k < 3; k++) w16[k] = my_w16[k];
        if (fjob) {  // pass B^-1 (row u)
            cplx v[4];
#pragma unroll
            for (int i = 0; i < 4; i++) v[i] = jbuf[baseB + SG1[i]];
            dft16x4<true>(v, w16);
#pragma unroll
            for (int k2 = 0; k2 < 4; k2++) jbuf[baseB + SG1[k2]] = v[k2];
        }
        wave_sync();
        PROF_T(7);
        PRIO(3);
        if (fjob) {  // pass A^-1 (column u): conj(W_M^{u kk}), DFT16^-1 over kk, untwist, from_torus, ACC +=
            cplx v[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int kk = r + 4 * i;
                v[i] = twmul(jbuf[baseA + SG3[i]], cconj(s_twa[16 * kk + u]));
            }
            dft16x4<true>(v, w16);
            uint64_t *poly = acc + jb * ACC_STRIDE;
#pragma unroll
            for (int k2 = 0; k2 < 4; k2++) {
                const int j = ll + 64 * k2;  // m = r + 4 k2 -> j = u + 16 m
                const cplx t = twmul(v[k2], s_utw[j]);
                bool o0, o1;
                uint64_t a0 = torus_add_fast(t.re, poly[j], o0), a1 = torus_add_fast(t.im, poly[j + M], o1);
                if (__builtin_amdgcn_ballot_w64(!(o0 && o1))) {  // zeros, out-of-range magnitudes (rare)
                    a0 = poly[j] + from_torus_bits(t.re);
                    a1 = poly[j + M] + from_torus_bits(t.im);
                }
                poly[j] = a0;
                poly[j + M] = a1;
            }
        }
        }
        wave_sync();  // the next step's decomposition reads this wave's ACC writes (in-order LDS)
        PROF_T(8);
#ifdef TAE_X4_PROF
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
        PROF_T(9);
    }
#ifdef TAE_X4_PROF
    if (blockIdx.x == 100 && lane == 0)
        printf("x4prof wave %2d: dec %llu passA %llu passB %llu barF %llu mac %llu barM %llu store %llu invB %llu invA %llu end %llu\n",
               jb, (unsigned long long)prof_[0], (unsigned long long)prof_[1], (unsigned long long)prof_[2],
               (unsigned long long)prof_[3], (unsigned long long)prof_[4], (unsigned long long)prof_[5],
               (unsigned long long)prof_[6], (unsigned long long)prof_[7], (unsigned long long)prof_[8],
               (unsigned long long)prof_[9]);
#endif
    lds_sync();  // sample extraction reads every job's ACC
    for (int ct = 0; ct < nct; ct++) {
        const uint64_t *a = acc + ct * K1 * ACC_STRIDE;
        uint64_t *o = PBS ? out + (size_t)(ct0 + ct) * (K1 - 1) * N + (size_t)(ct0 + ct)
                          : out + ((size_t)g * n_out + ct0 + ct) * ((K1 - 1) * N + 1);
        for (int t = tid; t < (K1 - 1) * N; t += THREADS) {
            const int p = t / N, j = t - p * N;
            o[t] = j == 0 ? a[p * ACC_STRIDE] : (0 - a[p * ACC_STRIDE + N - j]);
        }
        if (tid == 0) o[(K1 - 1) * N] = a[(K1 - 1) * ACC_STRIDE] + out_add;
    }
    stamp.stop(clk);
}

inline size_t lds_bytes() {
    return (size_t)JOBS * ACC_STRIDE * 8 + (size_t)JOBS * BUF_STRIDE * 16 + 3 * (size_t)M * 16 + 12 * 16;
}

// The instantiations are compiled in their own translation unit (br512x4_inst.hip) with the post-RA machine
// scheduler off (-mllvm --enable-post-misched=false: -0.7 to -1.1% per launch, same box; the other kernels
// lose 2-4% with it); every other file sees them through these extern declarations.
#define TAE_X4_PARAMS                                                                                         \
    const uint64_t *__restrict__, int, const uint64_t *__restrict__, int, const cplx *__restrict__, int,    \
        uint64_t *__restrict__, long, uint64_t, uint64_t, const cplx *__restrict__, const cplx *__restrict__, \
        const double *__restrict__, uint64_t *__restrict__, long
#ifndef TAE_X4_INSTANTIATE
extern template __global__ void br_kernel<3, true, 12>(TAE_X4_PARAMS);
extern template __global__ void br_kernel<7, true, 6>(TAE_X4_PARAMS);
extern template __global__ void br_kernel<1, false, 13>(TAE_X4_PARAMS);
#endif

}  // namespace br512x4
}  // namespace tae
