// Batched blind rotation for N = 512, k = 4 with TWO waves per SIMD: 512-thread workgroups.
//
// Same work split as br512.hpp (C = 3 ciphertexts per workgroup, ACC and one level of spectra in
// LDS, GGSW values shared by the three accumulators of a Fourier position), but every FFT job
// (ciphertext, polynomial) runs on 32 lanes instead of 16: a lane pair (rows 2r, 2r + 1 of a wave,
// lanes l and l + 16) splits each radix-16 DFT of the 16 x 16 FFT.  Lane h of the pair runs the
// first-stage DFT4s of inputs a in {2h, 2h+1}, the pair trades half of the results with one
// v_permlane16_swap per dword (gfx950; semantics probed by scripts/probes/permlane_swap.hip),
// and lane h runs the second-stage DFT4s of outputs b in {2h, 2h+1}.  Each output value gets the
// same f64 operation sequence as the CPU oracle's DFT16 (tfhe_oracle.c), so results stay
// bit-exact; W16^0 / W16^4 factors become generic products with exact (1, 0) / (0, -1) factors
// and change nothing but the sign of zeros.
//
// With 8 waves per workgroup (137 KB LDS, one workgroup per CU) each SIMD holds two waves: the
// second wave issues while the first waits on LDS, the GGSW stream or an f64 dependency.
// The MAC splits the 15 (q, ct) accumulators of a Fourier position 8 / 7 over the two halves of
// the workgroup (wave-uniform), each half loading only the GGSW columns q it needs.
#pragma once
#include "br512.hpp"

namespace tae {
namespace br512x2 {

using br512::BUF_STRIDE;
using br512::K1;
using br512::lds_sync;
using br512::M;
using br512::N;
using br512::pidx;
using br512::u32x4;
using br512::W16;

constexpr int C = 3, JOBS = C * K1, THREADS = 512;

// A job's 32 lanes live in one wave and LDS operations of a wave execute in order, so hand-offs
// inside a job (pass A -> pass B, pass B^-1 -> pass A^-1, ACC update -> next decomposition) only
// need the compiler not to reorder the accesses; workgroup barriers remain where data crosses jobs
// (spectra -> MAC -> next level / inverse).
__device__ __forceinline__ void wave_sync() { asm volatile("" ::: "memory"); }
constexpr int ACC_STRIDE = N;
#ifdef TAE_DBG_NOBAR
#define DBG_SYNC() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
#else
#define DBG_SYNC() lds_sync()
#endif  // u64 per ACC polynomial (no padding: see acc_phys)

// ACC coefficient j lives at acc_phys(j): bit 5 of j flips bit 4.  The two lanes of a pair touch
// coefficients 32 apart (same ds_read_b64 bank otherwise); after the swizzle they are 16 u64 =
// 32 banks apart, and any 16 consecutive coefficients still cover 16 distinct bank pairs.
__device__ __forceinline__ int acc_phys(int j) { return j ^ ((j & 32) >> 1); }

// coefficient j of poly * X^e (e in [0, 2N)) on a swizzled ACC polynomial
__device__ __forceinline__ uint64_t rotated_acc(const uint64_t *poly, int j, int e) {
    int src = j - e;
    bool neg = false;
    if (src < 0) {
        src += N;
        neg = !neg;
    }
    if (src < 0) {
        src += N;
        neg = !neg;
    }
    const uint64_t v = poly[acc_phys(src)];
    return neg ? (0 - v) : v;
}

// MAC thread -> Fourier position: odd 16-blocks rotated by one so that, with the +1-per-16 buffer
// padding, the 16 lanes of every ds_read_b128 lane group hit 16 distinct 4-bank groups.
__device__ __forceinline__ int mac_pos(int t) { return (t & 0xF0) | ((t - ((t >> 4) & 1)) & 15); }

__device__ __forceinline__ void swap16(cplx &x, cplx &y) {
    // v_permlane16_swap: lanes of even rows keep x and receive the odd-row partner's x in y;
    // lanes of odd rows receive the even-row partner's y in x and keep y.
    u32x4 a, b;
    __builtin_memcpy(&a, &x, 16);
    __builtin_memcpy(&b, &y, 16);
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const auto r = __builtin_amdgcn_permlane16_swap(a[w], b[w], false, false);
        a[w] = r[0];
        b[w] = r[1];
    }
    __builtin_memcpy(&x, &a, 16);
    __builtin_memcpy(&y, &b, 16);
}

// Half of a DFT16 on lane h of a pair.  In:  v[al + 2 i] = x[2h + al + 4 i]  (al < 2, i < 4).
// Out: v[S(bl, k2)] = X[2h + bl + 4 k2] with S(bl, 0) = 2bl, S(bl, 1) = 2bl + 1, S(bl, 2) = 4 + 2bl,
// S(bl, 3) = 5 + 2bl.  tw[0..5] = W16^{a b} for (a, b) = (2h, 1..3), (2h+1, 1..3) (forward values).
template <bool INV>
__device__ __forceinline__ void half_dft16(cplx *v, const cplx *tw) {
    dft4<INV>(v[0], v[2], v[4], v[6]);  // a = 2h      : v[2 b]     = Y(a, b)
    dft4<INV>(v[1], v[3], v[5], v[7]);  // a = 2h + 1  : v[1 + 2 b] = Y(a, b)
    v[2] = cmul(v[2], INV ? cconj(tw[0]) : tw[0]);
    v[4] = cmul(v[4], INV ? cconj(tw[1]) : tw[1]);
    v[6] = cmul(v[6], INV ? cconj(tw[2]) : tw[2]);
    v[3] = cmul(v[3], INV ? cconj(tw[3]) : tw[3]);
    v[5] = cmul(v[5], INV ? cconj(tw[4]) : tw[4]);
    v[7] = cmul(v[7], INV ? cconj(tw[5]) : tw[5]);
    // P = slots of b in {0, 1} (v[0..3]), Q = slots of b in {2, 3} (v[4..7]); after the swaps both
    // lanes hold v[al + 2 bl] = Y(al, 2h + bl) and v[4 + al + 2 bl] = Y(2 + al, 2h + bl)
    swap16(v[0], v[4]);
    swap16(v[1], v[5]);
    swap16(v[2], v[6]);
    swap16(v[3], v[7]);
    dft4<INV>(v[0], v[1], v[4], v[5]);  // b = 2h
    dft4<INV>(v[2], v[3], v[6], v[7]);  // b = 2h + 1
}

// slot of input index (al, i) and output index (bl, k2)
__device__ __forceinline__ constexpr int in_slot(int al, int i) { return al + 2 * i; }
__device__ __forceinline__ constexpr int out_slot(int bl, int k2) { return (k2 < 2 ? 0 : 4) + 2 * bl + (k2 & 1); }
// digit (relative to 2h) of input slot L and of output slot S
__device__ __forceinline__ constexpr int in_idx(int L) { return (L & 1) + 4 * (L >> 1); }
__device__ __forceinline__ constexpr int out_idx(int S) { return ((S >> 1) & 1) + 4 * ((S & 1) + ((S >> 2) << 1)); }

template <int HALF, int LEV>
__device__ __forceinline__ void mac_level(const cplx *buf, int pos, cplx *accr, const cplx *gv) {
    // accumulator pi (HALF 0: pi = 0..7, HALF 1: pi = 8..14) is (q, ct) = (pi / 3, pi % 3);
    // gv[p * 3 + (q - q0)] with q0 = 0 / 2.  Per accumulator: p ascending, the oracle's fma chain.
    constexpr int NA = HALF ? 7 : 8, PI0 = HALF ? 8 : 0, Q0 = HALF ? 2 : 0;
#pragma unroll
    for (int p = 0; p < K1; p++) {
        cplx x[C];
#pragma unroll
        for (int c = 0; c < C; c++) x[c] = buf[(c * K1 + p) * BUF_STRIDE + pos];
#pragma unroll
        for (int a = 0; a < NA; a++) {
            const int pi = PI0 + a, q = pi / 3, c = pi % 3;
            const cplx gg = gv[p * 3 + (q - Q0)];
            double re = accr[a].re, im = accr[a].im;
            re = fma(x[c].re, gg.re, re);
            re = fma(-x[c].im, gg.im, re);
            im = fma(x[c].re, gg.im, im);
            im = fma(x[c].im, gg.re, im);
            accr[a] = {re, im};
        }
    }
}

// Mode: PBS -> GGSW_i = bsk + i * ggsw_sz, per-ciphertext rotation a~_i; steps = n.
//       VP  -> GGSW_t = ggsw_f + (g * n_in + b) * ggsw_sz, rotation X^{-2^t} shared; steps = n_in.
// BLOG: decomposition base log (12 for the PBS, 13 for the CBS GGSW of params_sqrd_lvl_64), a
// template parameter so the digit extraction compiles to constant shifts.
template <int LEV, bool PBS, int BLOG>
__global__ void __launch_bounds__(THREADS, 1)
    br_kernel(const uint64_t *__restrict__ lwe_in, int n, const uint64_t *__restrict__ lut, int n_out,
              const cplx *__restrict__ ggsw_base, int n_in, uint64_t *__restrict__ out, long B, int base_log,
              uint64_t body_add, uint64_t out_add, const cplx *__restrict__ twist, const cplx *__restrict__ wtab,
              W16 W) {
    constexpr int LOGN = 9;
    extern __shared__ __align__(16) unsigned char smem[];
    uint64_t *acc = reinterpret_cast<uint64_t *>(smem);             // [JOBS][ACC_STRIDE]
    cplx *buf = reinterpret_cast<cplx *>(acc + JOBS * ACC_STRIDE);  // [JOBS][BUF_STRIDE]
    cplx *s_tw = buf + JOBS * BUF_STRIDE;                           // twist e^{i pi j / N}
    cplx *s_twa = s_tw + M;                                         // [16 a + b] = W_M^{a b}
    cplx *s_utw = s_twa + M;                                        // conj(twist) 2^-8 (exact)
    cplx *s_w16 = s_utw + M;                                        // [h][6] stage-1 factors
    const int tid = threadIdx.x;
    const int jb = tid >> 5, t32 = tid & 31;
    const int h = t32 >> 4, u = t32 & 15;  // lane pair (u, u + 16) of a job
    const bool fjob = jb < JOBS;
    const int jct = fjob ? jb / K1 : 0;
    const size_t ggsw_sz = (size_t)LEV * K1 * K1 * M;

    long ct0, g = 0;
    int nct;
    if (PBS) {
        ct0 = (long)blockIdx.x * C;
        nct = (int)min((long)C, B - ct0);
    } else {
        const int per_group = (n_out + C - 1) / C;
        g = blockIdx.x / per_group;
        ct0 = (long)(blockIdx.x - g * per_group) * C;
        nct = min(C, n_out - (int)ct0);
    }
    const bool jvalid = fjob && jct < nct;

    for (int t = tid; t < M; t += THREADS) {
        s_tw[t] = twist[t];
        s_twa[t] = wtab[(t >> 4) * (t & 15)];
        s_utw[t] = cplx{twist[t].re * 0x1p-8, -twist[t].im * 0x1p-8};
    }
    if (tid < 12) {
        // s_w16[6 h + 3 al + b - 1] = W16^{(2h + al) b} = W_M^{16 e}; exact 1 and -i for e = 0, 4.
        // (Straight-line selects: a switch on tid here compiled to a divergent branch tree that
        //  produced wrong entries on gfx950.)
        const int hh = tid / 6, r = tid - 6 * hh, al = r / 3, b = r - 3 * al + 1;
        const int e = ((2 * hh + al) * b) & 15;
        const cplx w = wtab[16 * e];
        s_w16[tid] = e == 0 ? cplx{1.0, 0.0} : (e == 4 ? cplx{0.0, -1.0} : w);
    }
    const cplx *my_w16 = s_w16 + 6 * h;

    const cplx *gbase = PBS ? ggsw_base : ggsw_base + (size_t)g * n_in * ggsw_sz;
    const uint32_t gbytes = (uint32_t)((size_t)(PBS ? n : n_in) * ggsw_sz * sizeof(cplx));
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc((void *)gbase, (short)0, gbytes, 0x00020000);
    const int pos = mac_pos(tid & (M - 1));
    const int half = __builtin_amdgcn_readfirstlane(tid >> 8);  // wave-uniform MAC half
    const int gvoff = pos * (int)sizeof(cplx);

    for (int t = tid; t < JOBS * N; t += THREADS) {
        const int job = t / N, j = t - job * N;
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
        acc[job * ACC_STRIDE + acc_phys(j)] = v;
    }
    lds_sync();

    const int steps = PBS ? n : n_in;
    uint64_t a_next = (PBS && jvalid) ? lwe_in[(size_t)(ct0 + jct) * (n + 1)] : 0;
#if defined(TAE_DBG_PRIO1)
    if (half) __builtin_amdgcn_s_setprio(1);
#elif defined(TAE_DBG_PRIO0)
    if (!half) __builtin_amdgcn_s_setprio(1);
#endif
    cplx accr[8];
    cplx gv[K1 * 3];
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
        // GGSW values (lev, p, q) at this thread's Fourier position, q in this half's three columns
        auto load_level = [&](int lev) {
            const int q0 = half ? 2 : 0;
#pragma unroll
            for (int p = 0; p < K1; p++)
#pragma unroll
                for (int qq = 0; qq < 3; qq++) {
                    const int soff = gstep + (((lev - 1) * K1 + p) * K1 + q0 + qq) * M * (int)sizeof(cplx);
                    const u32x4 r = __builtin_amdgcn_raw_buffer_load_b128(grs, gvoff, soff, 0);
                    __builtin_memcpy(&gv[p * 3 + qq], &r, sizeof(cplx));
                }
        };
        // ---- rotated difference + decomposition of this lane's 8 x 2 coefficients ----
        int uu = u;
        asm volatile("" : "+v"(uu));
        uint32_t dig[LEV][8];
#ifdef TAE_DBG_NODEC
        if (fjob) {
            const uint64_t *poly = acc + jb * ACC_STRIDE;
#pragma unroll
            for (int L = 0; L < 8; L++)
#pragma unroll
                for (int l = 0; l < LEV; l++) dig[l][L] = (uint32_t)poly[acc_phys(uu + 16 * L + l)] ^ e;
        }
        if (false) {
#else
        if (fjob) {
#endif
            const uint64_t *poly = acc + jb * ACC_STRIDE;
            // coefficient j of ACC * X^e is entry t = (j - e) mod 2N of the negacyclic extension
            // [ACC, -ACC]: ACC[t mod N], negated when t >= N; coefficient j + M is entry t + M,
            // stored at phys(t mod N) ^ M (the swizzle leaves bit 8 alone)
            const int bt = uu + 32 * h - e;
#pragma unroll
            for (int L = 0; L < 8; L++) {
                const int j = uu + 16 * (2 * h + in_idx(L));
                const int t = (bt + 16 * in_idx(L)) & (2 * N - 1);
                const int ph = acc_phys(t & (N - 1));
                const uint64_t m0 = (uint64_t)(int64_t)((t << 22) >> 31);
                const uint64_t m1 = (uint64_t)(int64_t)(((t + M) << 22) >> 31);
                const uint64_t v0 = poly[ph], v1 = poly[ph ^ M];
                const uint64_t p0 = poly[acc_phys(j)], p1 = poly[acc_phys(j) + M];
                // (v ^ m) - (p + m) = v - p, or -v - p when m = -1
                const uint64_t x0 = (v0 ^ m0) - (p0 + m0), x1 = (v1 ^ m1) - (p1 + m1);
                uint32_t d0[LEV], d1[LEV];
                decompose16<LEV>(x0, BLOG, d0);
                decompose16<LEV>(x1, BLOG, d1);
#pragma unroll
                for (int l = 0; l < LEV; l++) dig[l][L] = d0[l] | (d1[l] << 16);
                if ((L & 3) == 3) __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int a = 0; a < 8; a++) accr[a] = cplx{0.0, 0.0};

#pragma unroll
        for (int lev = LEV; lev >= 1; lev--) {
#ifndef TAE_DBG_NOGLOAD
            load_level(lev);
#else
            if (lev == LEV) load_level(lev);
#endif
            // pass A: twist, half DFT16 over n2, W_M^{u k}, -> LDS position u + 16 k
            if (fjob) {
                cplx v[8];
#pragma unroll
                for (int L = 0; L < 8; L++) {
                    uint32_t dw = dig[0][L];
#pragma unroll
                    for (int l = 1; l < LEV; l++)
                        if (lev - 1 == l) dw = dig[l][L];
                    const double a0 = br512::lo16(dw), a1 = br512::hi16(dw);
                    const cplx tw = (s_tw + uu)[16 * (2 * h + in_idx(L))];
                    v[L] = {fma(a0, tw.re, -(a1 * tw.im)), fma(a0, tw.im, a1 * tw.re)};
                }
                half_dft16<false>(v, my_w16);
                cplx *dst = buf + jb * BUF_STRIDE;
#pragma unroll
                for (int S = 0; S < 8; S++) {
                    const int k = 2 * h + out_idx(S);
                    dst[pidx(uu + 16 * k)] = cmul(v[S], (s_twa + uu)[16 * k]);
                }
            }
            wave_sync();
            // pass B: half DFT16 over positions 16 u + m, in place
            if (fjob) {
                cplx *base = buf + jb * BUF_STRIDE;
                cplx v[8];
#pragma unroll
                for (int L = 0; L < 8; L++) v[L] = base[pidx(16 * uu + 2 * h + in_idx(L))];
                half_dft16<false>(v, my_w16);
#pragma unroll
                for (int S = 0; S < 8; S++) base[pidx(16 * uu + 2 * h + out_idx(S))] = v[S];
            }
            DBG_SYNC();
#ifndef TAE_DBG_NOMAC
            if (half == 0)
                mac_level<0, LEV>(buf, pidx(pos), accr, gv);
            else
                mac_level<1, LEV>(buf, pidx(pos), accr, gv);
#endif
            DBG_SYNC();
        }
        // ---- inverse FFT of the MAC results, accumulated into ACC ----
        {
            const int pp = pidx(pos);
            if (half == 0) {
#pragma unroll
                for (int a = 0; a < 8; a++) buf[((a % 3) * K1 + a / 3) * BUF_STRIDE + pp] = accr[a];
            } else {
#pragma unroll
                for (int a = 0; a < 7; a++) buf[(((a + 8) % 3) * K1 + (a + 8) / 3) * BUF_STRIDE + pp] = accr[a];
            }
        }
        DBG_SYNC();
        if (fjob) {  // pass B^-1
            cplx *base = buf + jb * BUF_STRIDE;
            cplx v[8];
#pragma unroll
            for (int L = 0; L < 8; L++) v[L] = base[pidx(16 * uu + 2 * h + in_idx(L))];
            half_dft16<true>(v, my_w16);
#pragma unroll
            for (int S = 0; S < 8; S++) base[pidx(16 * uu + 2 * h + out_idx(S))] = v[S];
        }
        wave_sync();
        if (fjob) {  // pass A^-1: conj(W_M^{u kk}), half DFT16, untwist, from_torus, ACC +=
            const cplx *src = buf + jb * BUF_STRIDE;
            cplx v[8];
#pragma unroll
            for (int L = 0; L < 8; L++) {
                const int kk = 2 * h + in_idx(L);
                v[L] = cmul(src[pidx(uu + 16 * kk)], cconj((s_twa + uu)[16 * kk]));
            }
            half_dft16<true>(v, my_w16);
            uint64_t *poly = acc + jb * ACC_STRIDE;
            const cplx *utp = s_utw + uu;
#pragma unroll
            for (int S = 0; S < 8; S++) {
                const int m = 2 * h + out_idx(S);
                const cplx t = cmul(v[S], utp[16 * m]);
                const int jp = acc_phys(uu + 16 * m);
#ifdef TAE_DBG_NOTAIL
                poly[jp] += (uint64_t)__double_as_longlong(t.re);
                poly[jp + M] += (uint64_t)__double_as_longlong(t.im);
#else
                poly[jp] += from_torus_bits(t.re);
                poly[jp + M] += from_torus_bits(t.im);
#endif
            }
        }
        wave_sync();
    }
    lds_sync();  // sample extraction reads every job's ACC
    for (int ct = 0; ct < nct; ct++) {
        const uint64_t *a = acc + ct * K1 * ACC_STRIDE;
        uint64_t *o = PBS ? out + (size_t)(ct0 + ct) * (K1 - 1) * N + (size_t)(ct0 + ct)
                          : out + ((size_t)g * n_out + ct0 + ct) * ((K1 - 1) * N + 1);
        for (int t = tid; t < (K1 - 1) * N; t += THREADS) {
            const int p = t / N, j = t - p * N;
            o[t] = j == 0 ? a[p * ACC_STRIDE] : (0 - a[p * ACC_STRIDE + acc_phys(N - j)]);
        }
        if (tid == 0) o[(K1 - 1) * N] = a[(K1 - 1) * ACC_STRIDE] + out_add;
    }
}

inline size_t lds_bytes() {
    return (size_t)JOBS * ACC_STRIDE * 8 + (size_t)JOBS * BUF_STRIDE * 16 + 3 * (size_t)M * 16 + 12 * 16;
}

}  // namespace br512x2
}  // namespace tae
