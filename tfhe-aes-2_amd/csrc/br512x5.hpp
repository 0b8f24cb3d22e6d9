// Batched blind rotation for N = 512, k = 4: the br512x4.hpp work split (1024 threads, C = 3
// ciphertexts, job = wave, 4-lane DFT16s) with the accumulators in registers and two spectrum
// buffers in LDS, so a wave's FFT of level l+1 and its MAC share of level l run between the same
// pair of barriers:
//
//   phase 0:      FFT(level L)          -> S0            | barrier
//   phase k:      FFT(level L-k)        -> S[k & 1]      (k < LEV)
//                 MAC(level L-k+1)      <- S[(k-1) & 1]  | barrier
//   phase LEV:    MAC(level 1), MAC results -> S[LEV & 1] | barrier
//   next step:    inverse FFT of the own job in S[LEV & 1], ACC += (registers); the own slot of
//                 S[LEV & 1] then stages ACC for the rotated read of the decomposition.
//
// LEV + 1 barriers per step instead of 2 LEV + 1, and every interval mixes VALU-heavy FFT passes
// with the LDS-read-heavy MAC.  Lane (u, r) owns ACC coefficients j = lane + 64 i and j + 256
// (i < 4): exactly the coefficients its decomposition consumes and its inverse pass produces, so
// ACC (8 u64) never leaves the lane except through the staging copy.  Same fixed operation
// sequence as br512x4 / the oracle: bit-identical results.
#pragma once
#include "br512.hpp"
#include "br512x2.hpp"
#include "br512x4.hpp"

namespace tae {
namespace br512x5 {

using br512::BUF_STRIDE;
using br512::K1;
using br512::lds_sync;
using br512::M;
using br512::N;
using br512::pidx;
using br512::u32x4;
using br512x2::mac_pos;
using br512x2::wave_sync;
using br512x4::dft16x4;
using br512x4::mac_level;
using br512x4::mac_store;

constexpr int C = 3, JOBS = C * K1, THREADS = 1024;

__device__ __forceinline__ void barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int LEV, bool PBS, int BLOG>
__global__ void __launch_bounds__(THREADS, 1)
    br_kernel(const uint64_t *__restrict__ lwe_in, int n, const uint64_t *__restrict__ lut, int n_out,
              const cplx *__restrict__ ggsw_base, int n_in, uint64_t *__restrict__ out, long B,
              uint64_t body_add, uint64_t out_add, const cplx *__restrict__ twist, const cplx *__restrict__ wtab) {
    constexpr int LOGN = 9;
    extern __shared__ __align__(16) unsigned char smem[];
    cplx *sbuf = reinterpret_cast<cplx *>(smem);  // [2][JOBS][BUF_STRIDE]
    cplx *s_tw = sbuf + 2 * JOBS * BUF_STRIDE;    // twist e^{i pi j / N}
    cplx *s_twa = s_tw + M;                       // [16 a + b] = W_M^{a b}
    cplx *s_utw = s_twa + M;                      // conj(twist) 2^-8 (exact)
    cplx *s_w16 = s_utw + M;                      // [r][3]: W16^{r k1}, k1 = 1..3
    const int tid = threadIdx.x;
    const int jb = __builtin_amdgcn_readfirstlane(tid >> 6);  // job = wave
    const int lane = tid & 63, u = lane & 15, r = lane >> 4;
    const bool fjob = jb < JOBS;
    const int jct = fjob ? jb / K1 : 0;
    const int jpoly = fjob ? jb - jct * K1 : 0;
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
        const int rr = tid / 3, k1 = tid - 3 * rr + 1;
        const int e = (rr * k1) & 15;
        const cplx w = wtab[16 * e];
        s_w16[tid] = e == 0 ? cplx{1.0, 0.0} : (e == 4 ? cplx{0.0, -1.0} : w);
    }

    const cplx *gbase = PBS ? ggsw_base : ggsw_base + (size_t)g * n_in * ggsw_sz;
    const uint32_t gbytes = (uint32_t)((size_t)(PBS ? n : n_in) * ggsw_sz * sizeof(cplx));
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc((void *)gbase, (short)0, gbytes, 0x00020000);
    const int grp = jb >> 2;
    const int pos = mac_pos(tid & (M - 1));
    const int gvoff = pos * (int)sizeof(cplx);
    const int q0 = (4 * grp) / 3;
    const int nq = grp == 3 ? 1 : 2;

    int ll = lane;
    asm volatile("" : "+v"(ll));
    // ACC coefficients j = ll + 64 i (lo) and j + M (hi) of the own job, initial = LUT * X^{-b~}
    uint64_t accl[4], acch[4];
    {
        int e0 = 0;
        if (PBS && jvalid) {
            const uint64_t *in = lwe_in + (size_t)(ct0 + jct) * (n + 1);
            const int bt = mod_switch(in[n] + body_add, LOGN);
            e0 = (2 * N - (bt % (2 * N))) % (2 * N);
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int j = ll + 64 * i;
            uint64_t lo = 0, hi = 0;
            if (jvalid) {
                if (PBS) {
                    lo = rotated_coeff(lut + jpoly * N, j, e0, N);
                    hi = rotated_coeff(lut + jpoly * N, j + M, e0, N);
                } else if (jpoly == K1 - 1) {
                    lo = lut[(size_t)(ct0 + jct) * N + j];
                    hi = lut[(size_t)(ct0 + jct) * N + j + M];
                }
            }
            accl[i] = lo;
            acch[i] = hi;
        }
    }
    lds_sync();  // tables

    const int steps = PBS ? n : n_in;
    uint64_t a_next = (PBS && jvalid) ? lwe_in[(size_t)(ct0 + jct) * (n + 1)] : 0;
    cplx accr[4];
    cplx gv[K1 * 2];
    const cplx *my_w16 = s_w16 + 3 * r;
    cplx *own[2] = {sbuf + jb * BUF_STRIDE, sbuf + (JOBS + jb) * BUF_STRIDE};

    // inverse FFT of the own job's MAC results (in S[LEV & 1]) and ACC += from_torus(.)
    auto inverse_into_acc = [&]() {
        cplx *base = own[LEV & 1];
        {  // pass B^-1 (row u)
            cplx v[4];
#pragma unroll
            for (int i = 0; i < 4; i++) v[i] = base[pidx(16 * u + r + 4 * i)];
            dft16x4<true>(v, my_w16);
#pragma unroll
            for (int k2 = 0; k2 < 4; k2++) base[pidx(16 * u + r + 4 * k2)] = v[k2];
        }
        wave_sync();
        {  // pass A^-1 (column u), untwist, from_torus
            cplx v[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int kk = r + 4 * i;
                v[i] = cmul(base[pidx(u + 16 * kk)], cconj(s_twa[16 * kk + u]));
            }
            dft16x4<true>(v, my_w16);
#pragma unroll
            for (int k2 = 0; k2 < 4; k2++) {
                const cplx t = cmul(v[k2], s_utw[ll + 64 * k2]);
                accl[k2] += from_torus_bits(t.re);
                acch[k2] += from_torus_bits(t.im);
            }
        }
        wave_sync();
    };

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
        uint32_t dig[LEV][4];
        if (fjob) {
            if (step > 0) inverse_into_acc();
            // stage ACC in the own slot of S[LEV & 1]; coefficient j of ACC * X^e is entry
            // t = (j - e) mod 2N of [ACC, -ACC]
            uint64_t *stg = reinterpret_cast<uint64_t *>(own[LEV & 1]);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                stg[ll + 64 * i] = accl[i];
                stg[ll + 64 * i + M] = acch[i];
            }
            wave_sync();
            const int bt = ll - e;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int t = (bt + 64 * i) & (2 * N - 1);
                const int ph = t & (N - 1);
                const uint64_t m0 = (uint64_t)(int64_t)((t << 22) >> 31);
                const uint64_t m1 = (uint64_t)(int64_t)(((t + M) << 22) >> 31);
                const uint64_t v0 = stg[ph], v1 = stg[ph ^ M];
                const uint64_t x0 = (v0 ^ m0) - (accl[i] + m0), x1 = (v1 ^ m1) - (acch[i] + m1);
                uint32_t d0[LEV], d1[LEV];
                decompose16<LEV>(x0, BLOG, d0);
                decompose16<LEV>(x1, BLOG, d1);
#pragma unroll
                for (int l = 0; l < LEV; l++) dig[l][i] = d0[l] | (d1[l] << 16);
            }
            wave_sync();
        }
#pragma unroll
        for (int a = 0; a < 4; a++) accr[a] = cplx{0.0, 0.0};

#pragma unroll
        for (int k = 0; k <= LEV; k++) {
            const int lev = LEV - k;  // FFT level of this phase (k < LEV)
#ifndef TAE_X5_LATE_G
            if (k >= 1) load_level(lev + 1);
#endif
            if (k < LEV && fjob) {
                // pass A (column u): twist, DFT16 over m = r + 4 i, W_M^{u k} -> position u + 16 k
                cplx *dst = own[k & 1];
                cplx v[4];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const uint32_t dw = dig[(lev > 0 ? lev : 1) - 1][i];
                    const double a0 = br512::lo16(dw), a1 = br512::hi16(dw);
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
                // pass B (row u): DFT16 over positions 16 u + r + 4 i, in place
#pragma unroll
                for (int i = 0; i < 4; i++) v[i] = dst[pidx(16 * u + r + 4 * i)];
                dft16x4<false>(v, my_w16);
#pragma unroll
                for (int k2 = 0; k2 < 4; k2++) dst[pidx(16 * u + r + 4 * k2)] = v[k2];
            }
            wave_sync();  // keep the MAC's loads below the FFT (register pressure)
            if (k >= 1) {
#ifdef TAE_X5_LATE_G
                load_level(lev + 1);
#endif
                const cplx *src = sbuf + ((k - 1) & 1) * JOBS * BUF_STRIDE;
                switch (grp) {
                case 0: mac_level<0>(src, pidx(pos), accr, gv); break;
                case 1: mac_level<1>(src, pidx(pos), accr, gv); break;
                case 2: mac_level<2>(src, pidx(pos), accr, gv); break;
                default: mac_level<3>(src, pidx(pos), accr, gv); break;
                }
            }
            if (k == LEV) {
                cplx *dstm = sbuf + (LEV & 1) * JOBS * BUF_STRIDE;
                switch (grp) {
                case 0: mac_store<0>(dstm, pidx(pos), accr); break;
                case 1: mac_store<1>(dstm, pidx(pos), accr); break;
                case 2: mac_store<2>(dstm, pidx(pos), accr); break;
                default: mac_store<3>(dstm, pidx(pos), accr); break;
                }
            }
            barrier();
        }
    }
    if (fjob && steps > 0) inverse_into_acc();
    lds_sync();
    // sample extraction reads every job's ACC: copy to S0
    uint64_t *accs = reinterpret_cast<uint64_t *>(sbuf);  // [JOBS][N]
    if (fjob) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            accs[jb * N + ll + 64 * i] = accl[i];
            accs[jb * N + ll + 64 * i + M] = acch[i];
        }
    }
    lds_sync();
    for (int ct = 0; ct < nct; ct++) {
        const uint64_t *a = accs + ct * K1 * N;
        uint64_t *o = PBS ? out + (size_t)(ct0 + ct) * (K1 - 1) * N + (size_t)(ct0 + ct)
                          : out + ((size_t)g * n_out + ct0 + ct) * ((K1 - 1) * N + 1);
        for (int t = tid; t < (K1 - 1) * N; t += THREADS) {
            const int p = t / N, j = t - p * N;
            o[t] = j == 0 ? a[p * N] : (0 - a[p * N + N - j]);
        }
        if (tid == 0) o[(K1 - 1) * N] = a[(K1 - 1) * N] + out_add;
    }
}

inline size_t lds_bytes() { return 2 * (size_t)JOBS * BUF_STRIDE * 16 + 3 * (size_t)M * 16 + 12 * 16; }

}  // namespace br512x5
}  // namespace tae
