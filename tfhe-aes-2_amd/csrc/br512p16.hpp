// Batched blind rotation for N = 512, k = 4 (params_sqrd_lvl_64's PBS, 3 levels of 2^12) with SIXTEEN points
// per lane in the forward transforms: the DFT16s of the fused-twiddle transform (lf512.hpp) run wholly in one
// lane's registers, with no cross-lane permutes.
//
// Why: br512x4 holds four points per lane, so every DFT16 needs a 4 x 4 transpose over four
// lanes (16 v_permlane*_swap per job wave and pass, ~19% of its VALU issue).  Sixteen points per lane need no
// transpose, but a wave then carries four FFT jobs (one per 16 lanes), so the CU needs about twice br512x4's
// 15 jobs in flight to keep its SIMDs issuing.  This kernel gets 30 by running ALL three levels of C = 2
// ciphertexts at once (2 ct x 5 polynomials x 3 levels), which fits 160 KiB of LDS as
//     ACC          [2 ct][5 poly][512] u64                      40960 B
//     job area     30 forward jobs x 4096 B (256 spectrum slots) 122880 B   = 163840 B
// with the transform's constant table read from global memory (L1 / L2) instead of LDS.
//
// Per CMux step (ct0 += GGSW [x] (ct0 X^e - ct0), fft64 add_external_product_assign), four barriers:
//   D  waves IW0.. (one per polynomial (ct, p)): rotated difference + balanced digits of all three levels
//      (br512x4's code), written to the digit slots of jobs (ct, p, lev)            | barrier
//   F  waves 0..7 (four jobs each, lane u of a job = column / row u): pass A = DFT4s of the digits (lf512 a1)
//      and the fused DFT4s over the lane's own 16 points -> job region -> pass B (in place, wave-local) | barrier
//   M  all 16 waves: thread (slot group s, Fourier position): the oracle's fma chain over (level desc, row asc)
//      for 2 or 4 of the 10 (ct, q) accumulators (group 2 holds q = 2 and q = 4, so each GGSW value is loaded
//      once per workgroup)                                                           | barrier
//      accumulators -> inverse regions (br512x4's sidx layout)                       | barrier
//   I  waves IW0..: br512x4's PBS-mode inverse (pass B^-1, pass A^-1, untwist, torus, ACC +=) on job (ct, q),
//      then straight into the next step's D (same wave, same polynomial: no barrier).
// Every output sees the same f64 / integer operation sequence as br512x4 and the oracle (tfhe_oracle.c
// or_lf_fwd / or_lf_bwd_add, ext_product_add): bit-exact.  LDS layouts are conflict-free under the lane-group
// model (scripts/layout/p16_banks.py, tests/test_lds_layouts.py).
#pragma once
#include "br512.hpp"
#include "br512x4.hpp"
#include "lf512.hpp"

namespace tae {
namespace br512p16 {

using br512::K1;
using br512::lds_sync;
using br512::M;
using br512::N;
using br512::u32x4;
using br512::wave_sync;

constexpr int C = 2, LEV = 3, THREADS = 1024;
constexpr int JOBS = C * K1 * LEV;        // 30 forward FFT jobs (ct, p, lev) per step
constexpr int FWAVES = (JOBS + 3) / 4;    // 8 waves of four 16-lane jobs
constexpr int POLYS = C * K1;             // 10 inverse jobs / ACC polynomials
constexpr int IW0 = 6;                    // inverse / decomposition waves IW0 .. IW0 + POLYS - 1
constexpr int ACC_BYTES = POLYS * N * 8;  // 40960
constexpr int JOB_BYTES = 4096, GROUP_BYTES = 4 * JOB_BYTES, DIG_BYTES = 1024;
constexpr int INV_OFF = JOB_BYTES, INV_BYTES = br512x4::BUF_STRIDE * 16;  // 4640: two per group after the digits
constexpr int LDS_BYTES = ACC_BYTES + JOBS * JOB_BYTES;                  // 163840 = 160 KiB
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
static_assert(INV_OFF + 2 * INV_BYTES <= GROUP_BYTES, "two inverse regions per job group");
static_assert((POLYS + 1) / 2 <= JOBS / 4, "inverse regions live in whole job groups");
static_assert(IW0 + POLYS <= THREADS / 64, "inverse waves");

// job (ct, p, lev): index (ct K1 + p) LEV + lev - 1; wave w runs jobs 4w .. 4w + 3
__host__ __device__ constexpr int job_of(int ct, int p, int lev) { return (ct * K1 + p) * LEV + lev - 1; }
// spectrum slot of Fourier position P = a + 16 b inside a job region (16-byte slots): an XOR swizzle, so that
// every forward-pass access is a lane base XOR a compile-time constant (one VALU op) plus an immediate offset
__host__ __device__ constexpr int slot16(int P) { return 16 * (P >> 4) + ((P & 15) ^ (P >> 4)); }
// MAC thread (t mod 256) -> Fourier position: slot16(mac_pos(t)) = t (contiguous, conflict-free LDS reads)
__host__ __device__ constexpr int mac_pos(int t) { return 16 * (t >> 4) + ((t & 15) ^ (t >> 4)); }
// byte offsets inside the job area
__host__ __device__ constexpr int job_off(int J) { return J * JOB_BYTES; }
__host__ __device__ constexpr int dig_off(int J) { return (J >> 2) * GROUP_BYTES + (J & 3) * DIG_BYTES; }
__host__ __device__ constexpr int inv_off(int k) { return (k >> 1) * GROUP_BYTES + INV_OFF + (k & 1) * INV_BYTES; }

using lf512::K4;

// TAE_P16_PROF (debug builds only, never the product): per-phase cycle sums (clock64) of every wave of one
// workgroup, printed at exit: 0 decomposition, 1 barrier after it, 2 forward transforms, 3 GGSW prefetch +
// barrier, 4 MAC, 5 barrier after it, 6 accumulator stores + barrier, 7 inverse + ACC update.
#ifdef TAE_P16_PROF
#define P16_PROF_ARGS , uint64_t *prof_, uint64_t &prof_t_
#define P16_PROF_PASS , prof_, prof_t_
#define P16_PROF_DECL uint64_t prof_[8] = {0}, prof_t_ = clock64();
#define P16_T(i)                         \
    do {                                 \
        asm volatile("" ::: "memory");   \
        const uint64_t now_ = clock64(); \
        prof_[i] += now_ - prof_t_;      \
        prof_t_ = now_;                  \
    } while (0)
#else
#define P16_PROF_ARGS
#define P16_PROF_PASS
#define P16_PROF_DECL
#define P16_T(i) \
    do {         \
    } while (0)
#endif

// MAC thread groups (waves 4 G .. 4 G + 3, one per SIMD): accumulators (q, ct) for both ct and q = QA, plus q = 4
// in group 2 (NQ = 2), so that each GGSW value is loaded once per workgroup: 2 / 2 / 4 / 2 accumulators.
template <int G>
struct MacGroup {
    static constexpr int NQ = G == 2 ? 2 : 1;
    static constexpr int q(int qi) { return qi ? 4 : G; }
};

// GGSW values (lev, p, q) at the thread's Fourier position, one level
template <int G>
__device__ __forceinline__ void mac_load(cplx *gv, int lev, __amdgpu_buffer_rsrc_t grs, int gvoff, int gstep) {
    constexpr int NQ = MacGroup<G>::NQ;
#pragma unroll
    for (int p = 0; p < K1; p++)
#pragma unroll
        for (int qi = 0; qi < NQ; qi++) {
            const int soff = gstep + (((lev - 1) * K1 + p) * K1 + MacGroup<G>::q(qi)) * M * (int)sizeof(cplx);
            const u32x4 rv = __builtin_amdgcn_raw_buffer_load_b128(grs, gvoff, soff, 0);
            __builtin_memcpy(&gv[p * NQ + qi], &rv, sizeof(cplx));
        }
}

// one level of the oracle's fma chain (rows p ascending) into accr[qi C + ct]
template <int G>
__device__ __forceinline__ void mac_level(const unsigned char *mrow, int lev, const cplx *gv, cplx *accr) {
    constexpr int NQ = MacGroup<G>::NQ;
#pragma unroll
    for (int p = 0; p < K1; p++) {
        cplx x[C];
#pragma unroll
        for (int ct = 0; ct < C; ct++) x[ct] = *reinterpret_cast<const cplx *>(mrow + job_off(job_of(ct, p, lev)));
#pragma unroll
        for (int qi = 0; qi < NQ; qi++) {
            const cplx gg = gv[p * NQ + qi];
#pragma unroll
            for (int ct = 0; ct < C; ct++) {
                cplx &o = accr[qi * C + ct];
                double re = o.re, im = o.im;
                re = fma(x[ct].re, gg.re, re);
                re = fma(-x[ct].im, gg.im, re);
                im = fma(x[ct].re, gg.im, im);
                im = fma(x[ct].im, gg.re, im);
                o = {re, im};
            }
        }
    }
}

// the MAC of one step for group G: levels 3, 2 of GGSW values issued before the barrier that ends the forward
// transforms (waves without a forward job issue them at once), level 1 after level 3's chain; the accumulators
// go to the inverse regions after a second barrier (the job regions they overlap are read until then).  Three
// barriers on every path.
template <int G>
__device__ __forceinline__ void mac_step(unsigned char *jarea, int mslot, int spos, __amdgpu_buffer_rsrc_t grs,
                                         int gvoff, int gstep P16_PROF_ARGS) {
    constexpr int NQ = MacGroup<G>::NQ;
    cplx g3[K1 * NQ], g2[K1 * NQ], g1[K1 * NQ], accr[NQ * C];
    mac_load<G>(g3, 3, grs, gvoff, gstep);
    mac_load<G>(g2, 2, grs, gvoff, gstep);
    lds_sync();
    P16_T(3);
    const unsigned char *mrow = jarea + mslot * 16;
#pragma unroll
    for (int a = 0; a < NQ * C; a++) accr[a] = cplx{0.0, 0.0};
    mac_level<G>(mrow, 3, g3, accr);
    mac_load<G>(g1, 1, grs, gvoff, gstep);
    mac_level<G>(mrow, 2, g2, accr);
    mac_level<G>(mrow, 1, g1, accr);
    P16_T(4);
    lds_sync();
    P16_T(5);
#pragma unroll
    for (int qi = 0; qi < NQ; qi++)
#pragma unroll
        for (int ct = 0; ct < C; ct++)
            *reinterpret_cast<cplx *>(jarea + inv_off(ct * K1 + MacGroup<G>::q(qi)) + spos * 16) = accr[qi * C + ct];
    lds_sync();
    P16_T(6);
}

// PBS: lwe_in [B][n+1] (small key), lut the test vector GLWE [(k+1) N], bsk the Fourier BSK (conj(E2)-rescaled),
// out [B][k N + 1]; body_add / out_add as br512x4 (homomorphic_shift_boolean); lf the lf512 table.
template <int LEV_, int BLOG>
__global__ void __launch_bounds__(THREADS, 1)
    br_kernel(const uint64_t *__restrict__ lwe_in, int n, const uint64_t *__restrict__ lut,
              const cplx *__restrict__ bsk, uint64_t *__restrict__ out, long B, uint64_t body_add, uint64_t out_add,
              const double *__restrict__ lf, uint64_t *__restrict__ clk) {
    static_assert(LEV_ == LEV, "br512p16 is laid out for three levels");
    constexpr int LOGN = 9;
    ClockStamp stamp;
    stamp.start(clk);
    extern __shared__ __align__(16) unsigned char smem[];
    uint64_t *acc = reinterpret_cast<uint64_t *>(smem);
    unsigned char *jarea = smem + ACC_BYTES;
    const int tid = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63, u = lane & 15, r = lane >> 4;
    const long ct0 = (long)blockIdx.x * C;
    const int nct = (int)min((long)C, B - ct0);
    const size_t ggsw_sz = (size_t)LEV * K1 * K1 * M;

    // roles (wave-uniform): F waves run four forward jobs each; I waves own one polynomial (ct, p) = wv - IW0
    const bool fw = wv < FWAVES;
    const int fjob = wv * 4 + r;  // this lane's forward job (r = 16-lane group)
    const bool fvalid = fw && fjob < JOBS;
    const bool iw = wv >= IW0 && wv < IW0 + POLYS;
    const int kp = iw ? wv - IW0 : 0;
    const int ict = kp / K1;

    for (int t = tid; t < POLYS * N; t += THREADS) {
        const int poly = t / N, j = t - poly * N;
        const int ct = poly / K1, c = poly - ct * K1;
        uint64_t v = 0;
        if (ct < nct) {
            const uint64_t *in = lwe_in + (size_t)(ct0 + ct) * (n + 1);
            const int bt = mod_switch(in[n] + body_add, LOGN);
            const int e0 = (2 * N - (bt % (2 * N))) % (2 * N);
            v = rotated_coeff(lut + c * N, j, e0, N);
        }
        acc[t] = v;
    }
    // lane-uniform constants: pass A's integer DFT4 and its four fused stage-2 DFT4s (k1 = 0..3)
    const double lf_s2 = lf[lf512::CONSTS], lf_c8 = lf[lf512::CONSTS + 1], lf_t8 = lf[lf512::CONSTS + 2];
    K4 fa2[4];
#pragma unroll
    for (int k1 = 0; k1 < 4; k1++) fa2[k1] = lf512::k4(lf, lf512::FA2, 4, k1);
    lds_sync();

    const __amdgpu_buffer_rsrc_t grs =
        __builtin_amdgcn_make_buffer_rsrc((void *)bsk, (short)0, (uint32_t)((size_t)n * ggsw_sz * sizeof(cplx)), 0x00020000);
    const int mslot = tid & 255;        // MAC thread: spectrum slot (contiguous) ...
    const int mpos = mac_pos(mslot);    // ... of Fourier position mpos
    const int gvoff = mpos * (int)sizeof(cplx);
    const int spos = br512x4::sidx(mpos);  // its slot in the inverse regions
    const int grp = wv >> 2;  // MAC thread group
    // inverse waves' per-lane slots (br512x4's sidx layout): pass A / A^-1 and pass B / B^-1
    const int baseA = br512x4::SF[4 * (u & 3) + r] + br512x4::SG1[u >> 2];
    const int baseB = br512x4::SF[4 * r + (u & 3)] + br512x4::SG3[u >> 2];

    uint64_t a_next = (iw && ict < nct) ? lwe_in[(size_t)(ct0 + ict) * (n + 1)] : 0;
    P16_PROF_DECL
    for (int step = 0; step < n; step++) {
        const int gstep = step * (int)(ggsw_sz * sizeof(cplx));
        // ---- D: rotated difference and digits of polynomial kp, all levels -> digit slots ----
        if (iw) {
            const uint64_t a = a_next;
            if (step + 1 < n && ict < nct) a_next = lwe_in[(size_t)(ct0 + ict) * (n + 1) + step + 1];
            const int e = mod_switch(a, LOGN) % (2 * N);
            int ll = lane;
            asm volatile("" : "+v"(ll));
            const uint64_t *poly = acc + kp * N;
            uint32_t dig[LEV][4];
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
#pragma unroll
                for (int l = 0; l < LEV; l++) dig[l][i] = dp[l];
            }
            // digit slot layout [r][u][i]: lane (u, r) holds m = r + 4 i of column u
#pragma unroll
            for (int l = 0; l < LEV; l++) {
                const u32x4 w = {dig[l][0], dig[l][1], dig[l][2], dig[l][3]};
                *reinterpret_cast<u32x4 *>(jarea + dig_off(kp * LEV + l) + (16 * r + u) * 16) = w;
            }
        }
        P16_T(0);
        lds_sync();
        P16_T(1);
        // ---- F: forward transforms, 16 points per lane ----
        if (fvalid) {
            const unsigned char *ds = jarea + dig_off(fjob);
            uint32_t dw[4][4];
#pragma unroll
            for (int rr = 0; rr < 4; rr++) {
                const u32x4 w = *reinterpret_cast<const u32x4 *>(ds + (16 * rr + u) * 16);
#pragma unroll
                for (int i = 0; i < 4; i++) dw[rr][i] = w[i];
            }
            cplx s[4][4];  // pass A stage 1: s[rr][k1], DFT4 over i of the digits m = rr + 4 i
#pragma unroll
            for (int rr = 0; rr < 4; rr++) lf512::a1(dw[rr], s[rr], lf_s2, lf_c8, lf_t8);
            // LDS byte addresses (job regions are 256-B aligned): pass A lane u writes P = u + 16 k at
            // (A ^ 16 k) + 256 k, pass B lane kappa = u reads / writes P = lam + 16 kappa at Bk ^ 16 lam
            int A = ACC_BYTES + JOB_BYTES * fjob + 16 * u;
            asm volatile("" : "+v"(A));  // per step: keep the 16 XORs in the loop (not 16 hoisted registers)
            // stage 2 per k1 over rr, outputs k2 -> position u + 16 (k1 + 4 k2)
#pragma unroll
            for (int k1 = 0; k1 < 4; k1++) {
                cplx v[4] = {s[0][k1], s[1][k1], s[2][k1], s[3][k1]};
                lf512::dft4<false>(v, fa2[k1]);
#pragma unroll
                for (int k2 = 0; k2 < 4; k2++) {
                    const int k = k1 + 4 * k2;
                    *reinterpret_cast<cplx *>(smem + ((A ^ (16 * k)) + 256 * k)) = v[k2];
                }
            }
            wave_sync();
            // pass B (row kappa = u): stage 1 over i for each rr (points lam = rr + 4 i), stage 2 over rr
            const K4 fb1 = lf512::k4(lf, lf512::FB1, 16, u);
            K4 fb2[4];
#pragma unroll
            for (int l1 = 0; l1 < 4; l1++) fb2[l1] = lf512::k4(lf, lf512::FB2, 64, u + 16 * l1);
            int Bk = ACC_BYTES + JOB_BYTES * fjob + 272 * u;
            asm volatile("" : "+v"(Bk));
#pragma unroll
            for (int rr = 0; rr < 4; rr++) {
#pragma unroll
                for (int i = 0; i < 4; i++) s[rr][i] = *reinterpret_cast<const cplx *>(smem + (Bk ^ (16 * (rr + 4 * i))));
                lf512::dft4<false>(s[rr], fb1);
            }
            asm volatile("" : "+v"(Bk));  // recompute the store addresses (one XOR each) instead of holding 16
#pragma unroll
            for (int l1 = 0; l1 < 4; l1++) {
                cplx v[4] = {s[0][l1], s[1][l1], s[2][l1], s[3][l1]};
                lf512::dft4<false>(v, fb2[l1]);
#pragma unroll
                for (int k2 = 0; k2 < 4; k2++)
                    *reinterpret_cast<cplx *>(smem + (Bk ^ (16 * (l1 + 4 * k2)))) = v[k2];
            }
        }
        P16_T(2);
        // ---- M: the external product's MAC (three barriers) ----
        switch (grp) {
        case 0: mac_step<0>(jarea, mslot, spos, grs, gvoff, gstep P16_PROF_PASS); break;
        case 1: mac_step<1>(jarea, mslot, spos, grs, gvoff, gstep P16_PROF_PASS); break;
        case 2: mac_step<2>(jarea, mslot, spos, grs, gvoff, gstep P16_PROF_PASS); break;
        default: mac_step<3>(jarea, mslot, spos, grs, gvoff, gstep P16_PROF_PASS); break;
        }
        // ---- I: inverse transform of (ct, q) = kp, accumulated into its ACC polynomial ----
        if (iw) {
            cplx *jbuf = reinterpret_cast<cplx *>(jarea + inv_off(kp));
            {  // pass B^-1 (row kappa = u): DFT4 over i, transpose, fused DFT4
                cplx v[4];
#pragma unroll
                for (int i = 0; i < 4; i++) v[i] = jbuf[baseB + br512x4::SG1[i]];
                dft4<true>(v[0], v[1], v[2], v[3]);
                br512::transpose4(v);
                lf512::dft4<true>(v, lf512::k4(lf, lf512::IB2, 4, r));
#pragma unroll
                for (int k2 = 0; k2 < 4; k2++) jbuf[baseB + br512x4::SG1[k2]] = v[k2];
            }
            wave_sync();
            {  // pass A^-1 (column u): fused DFT4, transpose, fused DFT4, untwist, from_torus, ACC +=
                cplx v[4];
#pragma unroll
                for (int i = 0; i < 4; i++) v[i] = jbuf[baseA + br512x4::SG3[i]];
                lf512::dft4<true>(v, lf512::k4(lf, lf512::IA1, 16, u));
                br512::transpose4(v);
                lf512::dft4<true>(v, lf512::k4(lf, lf512::IA2, 64, lane));
                uint64_t *poly = acc + kp * N;
                const cplx *untw = reinterpret_cast<const cplx *>(lf + lf512::UNTW);
                int ll = lane;
                asm volatile("" : "+v"(ll));
#pragma unroll
                for (int k2 = 0; k2 < 4; k2++) {
                    const int j = ll + 64 * k2;
                    const cplx t = cmul(v[k2], untw[j]);  // x 2^-8 (exact) in the conversion
                    bool o0, o1;
                    uint64_t a0 = torus_add_fast_sh<8>(t.re, poly[j], o0), a1 = torus_add_fast_sh<8>(t.im, poly[j + M], o1);
                    if (__builtin_amdgcn_ballot_w64(!(o0 && o1))) {  // zeros, out-of-range magnitudes (rare)
                        a0 = poly[j] + from_torus_bits(t.re * 0x1p-8);
                        a1 = poly[j + M] + from_torus_bits(t.im * 0x1p-8);
                    }
                    poly[j] = a0;
                    poly[j + M] = a1;
                }
            }
            wave_sync();  // the next step's decomposition (this wave) reads these ACC writes (in-order LDS)
        }
#ifdef TAE_P16_PROF
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
        P16_T(7);
    }
#ifdef TAE_P16_PROF
    if (blockIdx.x == 100 && lane == 0)
        printf("p16prof wave %2d: dec %llu barD %llu fwd %llu pre+barF %llu mac %llu barM %llu store %llu inv %llu\n", wv,
               (unsigned long long)prof_[0], (unsigned long long)prof_[1], (unsigned long long)prof_[2],
               (unsigned long long)prof_[3], (unsigned long long)prof_[4], (unsigned long long)prof_[5],
               (unsigned long long)prof_[6], (unsigned long long)prof_[7]);
#endif
    lds_sync();  // sample extraction reads every polynomial's ACC
    for (int ct = 0; ct < nct; ct++) {
        const uint64_t *a = acc + ct * K1 * N;
        uint64_t *o = out + (size_t)(ct0 + ct) * ((K1 - 1) * N + 1);
        for (int t = tid; t < (K1 - 1) * N; t += THREADS) {
            const int p = t / N, j = t - p * N;
            o[t] = j == 0 ? a[p * N] : (0 - a[p * N + N - j]);
        }
        if (tid == 0) o[(K1 - 1) * N] = a[(K1 - 1) * N] + out_add;
    }
    stamp.stop(clk);
}

inline size_t lds_bytes() { return LDS_BYTES; }

#define TAE_P16_PARAMS                                                                                        \
    const uint64_t *__restrict__, int, const uint64_t *__restrict__, const cplx *__restrict__,              \
        uint64_t *__restrict__, long, uint64_t, uint64_t, const double *__restrict__, uint64_t *__restrict__
#ifndef TAE_P16_INSTANTIATE
extern template __global__ void br_kernel<3, 12>(TAE_P16_PARAMS);
#endif

}  // namespace br512p16
}  // namespace tae
