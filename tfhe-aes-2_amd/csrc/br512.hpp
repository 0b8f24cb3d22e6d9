// Batched blind rotation for N = 512, k = 4 (params_sqrd_lvl_64): C ciphertexts per 256-thread
// workgroup run the whole CMux chain together so that every Fourier-GGSW value loaded from L2
// feeds C accumulators (the BSK stream is the bandwidth term), while the f64 work
// (FFTs + MAC) stays on the VALU.
//
// Per CMux step (ct0 += GGSW [x] (ct0 * X^e - ct0), fft64 add_external_product_assign):
//   decompose   240 threads = (ct, poly p) x 16 lanes; each lane owns coefficients j = u + 16 m and
//               j + 256 (m < 16), decomposes them ONCE for all levels (packed int16 in registers)
//   per level   pass A (DFT16 + twiddles, registers) -> LDS -> pass B (DFT16, in place) ->
//   (finest     MAC: thread s = Fourier position, C x (k+1) accumulators, the (k+1)^2 GGSW values of
//    first)     the level prefetched into registers before the FFT passes
//   inverse     MAC results -> LDS -> pass B^-1 -> pass A^-1 -> untwist, from_torus, ACC += (LDS)
// The arithmetic is the same fixed f64 sequence as the CPU oracle (tfhe_oracle.c): radix-16 DIF,
// MAC over (level desc, row asc) with the same fma chain, untwist = conj(twist) * 2^-8 (exact).
// LDS: ACC [C][k+1][N + 16] u64 (padded: two jobs of one 32-lane group hit disjoint banks) and
// FFT buffers [C (k+1)][17 x 16] cplx (one pad slot per 16: conflict-free 16 x 16 transposes).
#pragma once
#include "fft_device.hpp"

namespace tae {
namespace br512 {

constexpr int N = 512, M = 256, R = 16, TPJ = 16, K1 = 5;
constexpr int ACC_STRIDE = N + 16;  // u64
constexpr int BUF_STRIDE = 17 * 16; // cplx

struct W16 {  // W_16^e for e in {1, 2, 3, 6, 9} (table values, passed as kernel arguments -> SGPRs)
    cplx w1, w2, w3, w6, w9;
};

__device__ __forceinline__ int pidx(int q) { return q + (q >> 4); }  // padded FFT-buffer index

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <bool INV>
__device__ __forceinline__ cplx tw16(cplx x, int e, const W16 &W) {
    // e in 0..9; e == 4 is the exact -i (+i inverse); others generic cmul with table values
    cplx t;
    switch (e) {
    case 0: return x;
    case 4: return INV ? cplx{-x.im, x.re} : cplx{x.im, -x.re};
    case 1: t = W.w1; break;
    case 2: t = W.w2; break;
    case 3: t = W.w3; break;
    case 6: t = W.w6; break;
    default: t = W.w9; break;
    }
    return cmul(x, INV ? cconj(t) : t);
}

template <bool INV>
__device__ __forceinline__ void dft16(cplx *v, const W16 &W) {
    cplx y[16];
#pragma unroll
    for (int n1 = 0; n1 < 4; n1++) dft4<INV>(v[n1], v[n1 + 4], v[n1 + 8], v[n1 + 12]);
#pragma unroll
    for (int n1 = 0; n1 < 4; n1++)
#pragma unroll
        for (int k1 = 0; k1 < 4; k1++) y[4 * k1 + n1] = tw16<INV>(v[n1 + 4 * k1], n1 * k1, W);
#pragma unroll
    for (int k1 = 0; k1 < 4; k1++) dft4<INV>(y[4 * k1], y[4 * k1 + 1], y[4 * k1 + 2], y[4 * k1 + 3]);
#pragma unroll
    for (int k1 = 0; k1 < 4; k1++)
#pragma unroll
        for (int k2 = 0; k2 < 4; k2++) v[k1 + 4 * k2] = y[4 * k1 + k2];
}

// all LEV digits of the balanced base-2^B decomposition (d[l-1] = level l, 1 = most significant)
template <int LEV>
__device__ __forceinline__ void decompose_all(uint64_t x, int base_log, int32_t *d) {
    const int nrb = 64 - base_log * LEV;
    uint64_t s = x >> (nrb - 1);
    s += s & 1;
    s >>= 1;
    const uint32_t mask = (1u << base_log) - 1;
    // after the first level the state fits 32 bits (base_log * (LEV - 1) <= 32 for these params)
    uint64_t res = s & mask;
    uint64_t st = s >> base_log;
    uint64_t carry = (((res - 1) | st) & res) >> (base_log - 1);
    st += carry;
    d[LEV - 1] = (int32_t)(res - (carry << base_log));
    uint32_t st32 = (uint32_t)st;
#pragma unroll
    for (int l = LEV - 1; l >= 1; l--) {
        const uint32_t r = st32 & mask;
        st32 >>= base_log;
        const uint32_t c = (((r - 1) | st32) & r) >> (base_log - 1);
        st32 += c;
        d[l - 1] = (int32_t)(r - (c << base_log));
    }
}

__device__ __forceinline__ double lo16(uint32_t w) { return (double)((int32_t)(w << 16) >> 16); }
__device__ __forceinline__ double hi16(uint32_t w) { return (double)((int32_t)w >> 16); }

// Mode: PBS -> GGSW_i = bsk + i * ggsw_sz, per-ciphertext rotation a~_i; steps = n.
//       VP  -> GGSW_t = ggsw_f + (g * n_in + b) * ggsw_sz, rotation X^{-2^t} shared; steps = n_in.
template <int C, int LEV, bool PBS>
__global__ void __launch_bounds__(256, 1)
    br_kernel(const uint64_t *__restrict__ lwe_in, int n, const uint64_t *__restrict__ lut, int n_out,
              const cplx *__restrict__ ggsw_base, int n_in, uint64_t *__restrict__ out, long B, int base_log,
              uint64_t body_add, uint64_t out_add, const cplx *__restrict__ twist, const cplx *__restrict__ wtab,
              W16 W) {
    constexpr int JOBS = C * K1;
    static_assert(JOBS * TPJ <= 256, "jobs");
    constexpr int LOGN = 9;
    extern __shared__ __align__(16) unsigned char smem[];
    uint64_t *acc = reinterpret_cast<uint64_t *>(smem);                  // [JOBS][ACC_STRIDE]
    cplx *buf = reinterpret_cast<cplx *>(acc + JOBS * ACC_STRIDE);       // [JOBS][BUF_STRIDE]
    const int tid = threadIdx.x;
    const int jb = tid / TPJ, u = tid - jb * TPJ;
    const bool fjob = jb < JOBS;
    const int jct = fjob ? jb / K1 : 0, jp = fjob ? jb - (jb / K1) * K1 : 0;
    const size_t ggsw_sz = (size_t)LEV * K1 * K1 * M;

    // ---- work assignment ----
    long ct0;            // first ciphertext (PBS) / first LUT output (VP) of this workgroup
    long g = 0;          // VP group
    int nct;             // valid ciphertexts in this workgroup
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

    // ---- twiddle tables in LDS: twist e^{i pi j/N}; pass-A twiddles s_twa[16 a + b] = W_M^{a b}
    //      (symmetric), read by lane u at s_twa[16 k + u]: constant offsets, and the 16 lanes of a
    //      job hit 16 distinct 4-bank groups (the u-major read was a 16-way ds_read_b128 conflict) ----
    cplx *s_tw = buf + JOBS * BUF_STRIDE;
    cplx *s_twa = s_tw + M;
    for (int t = tid; t < M; t += 256) {
        s_tw[t] = twist[t];
        s_twa[t] = wtab[(t >> 4) * (t & 15)];
    }
    const cplx *my_twa = s_twa + u;

    // ---- GGSW stream through a buffer descriptor: per-lane voffset, uniform soffset ----
    const cplx *gbase = PBS ? ggsw_base : ggsw_base + (size_t)g * n_in * ggsw_sz;
    const uint32_t gbytes = (uint32_t)((size_t)(PBS ? n : n_in) * ggsw_sz * sizeof(cplx));
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc((void *)gbase, (short)0, gbytes, 0x00020000);
    const int gvoff = tid * (int)sizeof(cplx);

    // ---- ACC init: PBS: LUT * X^{-b~} ; VP: trivial GLWE with body = LUT_j ----
    for (int t = tid; t < JOBS * N; t += 256) {
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
        acc[job * ACC_STRIDE + j] = v;
    }
    lds_sync();

    const int steps = PBS ? n : n_in;
    uint64_t a_next = (PBS && jvalid) ? lwe_in[(size_t)(ct0 + jct) * (n + 1)] : 0;
    cplx accr[C][K1];
    constexpr int PF = 2;  // GGSW rows prefetched before the FFT passes (register budget)
    cplx gv[PF][K1];
    for (int step = 0; step < steps; step++) {
        // rotation exponent for this lane's ciphertext and the GGSW of this step
        int e;
        int gstep;  // byte offset of this step's GGSW in the descriptor
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
        // GGSW row (lev, p) at this lane's Fourier position: K1 values
        auto load_row = [&](int lev, int p, cplx *dst) {
#pragma unroll
            for (int c = 0; c < K1; c++) {
                const int soff = gstep + (((lev - 1) * K1 + p) * K1 + c) * M * (int)sizeof(cplx);
                const u32x4 r = __builtin_amdgcn_raw_buffer_load_b128(grs, gvoff, soff, 0);
                __builtin_memcpy(&dst[c], &r, sizeof(cplx));
            }
        };
        // ---- rotated difference + decomposition (all levels at once) ----
        // (uu: an opaque copy of u, so the 16 per-m indices are recomputed each step instead of
        //  being hoisted out of the step loop and spilled)
        int uu = u;
        asm volatile("" : "+v"(uu));
        uint32_t dig[LEV][R];
        if (fjob) {
            const uint64_t *poly = acc + jb * ACC_STRIDE;
#pragma unroll
            for (int m = 0; m < R; m++) {
                const int j = uu + TPJ * m;
                const uint64_t x0 = rotated_coeff(poly, j, e, N) - poly[j];
                const uint64_t x1 = rotated_coeff(poly, j + M, e, N) - poly[j + M];
                int32_t d0[LEV], d1[LEV];
                decompose_all<LEV>(x0, base_log, d0);
                decompose_all<LEV>(x1, base_log, d1);
#pragma unroll
                for (int l = 0; l < LEV; l++) dig[l][m] = ((uint32_t)d0[l] & 0xFFFFu) | ((uint32_t)d1[l] << 16);
                // bound the compiler's LDS-load hoisting (register pressure: 4 u64 loads per m)
                if ((m & 3) == 3) __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int c = 0; c < C; c++)
#pragma unroll
            for (int q = 0; q < K1; q++) accr[c][q] = cplx{0.0, 0.0};

#pragma unroll
        for (int lev = LEV; lev >= 1; lev--) {
            // prefetch the first PF GGSW rows of this level (the rest is issued at the MAC start)
#pragma unroll
            for (int p = 0; p < PF; p++) load_row(lev, p, gv[p]);
            // pass A: twist, DFT16, W_M^{u k}
            if (fjob) {
                cplx v[R];
#pragma unroll
                for (int m = 0; m < R; m++) {
                    // select this level's packed digits with constant indices (dig stays in VGPRs)
                    uint32_t dw = dig[0][m];
#pragma unroll
                    for (int l = 1; l < LEV; l++)
                        if (lev - 1 == l) dw = dig[l][m];
                    const double a0 = lo16(dw), a1 = hi16(dw);
                    const cplx tw = (s_tw + uu)[TPJ * m];
                    v[m] = {fma(a0, tw.re, -(a1 * tw.im)), fma(a0, tw.im, a1 * tw.re)};
                }
                dft16<false>(v, W);
                if (u != 0) {
#pragma unroll
                    for (int kk = 1; kk < R; kk++) v[kk] = cmul(v[kk], my_twa[TPJ * kk]);
                }
                cplx *dst = buf + jb * BUF_STRIDE;
#pragma unroll
                for (int kk = 0; kk < R; kk++) dst[pidx(u + TPJ * kk)] = v[kk];
            }
            lds_sync();
            // pass B: DFT16 over positions 16 u + m, in place
            if (fjob) {
                cplx *base = buf + jb * BUF_STRIDE + pidx(TPJ * u);
                cplx v[R];
#pragma unroll
                for (int m = 0; m < R; m++) v[m] = base[m];
                dft16<false>(v, W);
#pragma unroll
                for (int kk = 0; kk < R; kk++) base[kk] = v[kk];
            }
            lds_sync();
            // MAC at Fourier position tid
            {
                const int pos = pidx(tid);
                cplx gv2[K1 - PF][K1];
#pragma unroll
                for (int p = PF; p < K1; p++) load_row(lev, p, gv2[p - PF]);
#pragma unroll
                for (int p = 0; p < K1; p++) {
#pragma unroll
                    for (int c = 0; c < C; c++) {
                        const cplx x = buf[(c * K1 + p) * BUF_STRIDE + pos];
#pragma unroll
                        for (int q = 0; q < K1; q++) {
                            const cplx gg = p < PF ? gv[p][q] : gv2[p - PF][q];
                            double re = accr[c][q].re, im = accr[c][q].im;
                            re = fma(x.re, gg.re, re);
                            re = fma(-x.im, gg.im, re);
                            im = fma(x.re, gg.im, im);
                            im = fma(x.im, gg.re, im);
                            accr[c][q] = {re, im};
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            lds_sync();
        }
        // ---- inverse FFT of the MAC results, accumulated into ACC ----
        {
            const int pos = pidx(tid);
#pragma unroll
            for (int c = 0; c < C; c++)
#pragma unroll
                for (int q = 0; q < K1; q++) buf[(c * K1 + q) * BUF_STRIDE + pos] = accr[c][q];
        }
        lds_sync();
        if (fjob) {  // pass B^-1 (stride 1, no twiddles)
            cplx *base = buf + jb * BUF_STRIDE + pidx(TPJ * u);
            cplx v[R];
#pragma unroll
            for (int m = 0; m < R; m++) v[m] = base[m];
            dft16<true>(v, W);
#pragma unroll
            for (int kk = 0; kk < R; kk++) base[kk] = v[kk];
        }
        lds_sync();
        if (fjob) {  // pass A^-1, untwist (= conj(twist) * 2^-8, exact), from_torus, ACC +=
            const cplx *src = buf + jb * BUF_STRIDE;
            cplx v[R];
#pragma unroll
            for (int kk = 0; kk < R; kk++) v[kk] = src[pidx(u + TPJ * kk)];
            if (u != 0) {
#pragma unroll
                for (int kk = 1; kk < R; kk++) v[kk] = cmul(v[kk], cconj(my_twa[TPJ * kk]));
            }
            dft16<true>(v, W);
            uint64_t *poly = acc + jb * ACC_STRIDE + uu;  // coefficient j = u + 16 m
            const cplx *twp = s_tw + uu;
#pragma unroll
            for (int m = 0; m < R; m++) {
                const cplx tw = twp[TPJ * m];
                const cplx ut = {tw.re * 0x1p-8, -tw.im * 0x1p-8};
                const cplx t = cmul(v[m], ut);
                poly[TPJ * m] += from_torus(t.re);
                poly[TPJ * m + M] += from_torus(t.im);
            }
        }
        lds_sync();
    }
    // ---- sample extraction (coefficient 0) ----
    for (int ct = 0; ct < nct; ct++) {
        const uint64_t *a = acc + ct * K1 * ACC_STRIDE;
        uint64_t *o = PBS ? out + (size_t)(ct0 + ct) * (K1 - 1) * N + (size_t)(ct0 + ct)
                          : out + ((size_t)g * n_out + ct0 + ct) * ((K1 - 1) * N + 1);
        for (int t = tid; t < (K1 - 1) * N; t += 256) {
            const int p = t / N, j = t - p * N;
            o[t] = j == 0 ? a[p * ACC_STRIDE] : (0 - a[p * ACC_STRIDE + N - j]);
        }
        if (tid == 0) o[(K1 - 1) * N] = a[(K1 - 1) * ACC_STRIDE] + out_add;
    }
}

inline size_t lds_bytes(int C) {
    return (size_t)C * K1 * ACC_STRIDE * 8 + (size_t)C * K1 * BUF_STRIDE * 16 + 2 * (size_t)M * 16;
}

}  // namespace br512
}  // namespace tae
