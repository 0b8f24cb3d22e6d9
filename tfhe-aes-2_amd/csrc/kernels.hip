// HIP kernels for gfx950 (CDNA4) and the Engine that drives them.
//
// Hot path, batched over every input bit of every SBOX of a round:
//   keyswitch_kernel      tfhe keyswitch_lwe_ciphertext            (extract_dual_bit_from_bit,
//                                                                   shortint_woppbs_1bit.rs:339-363)
//   blind_rotate_kernel   tfhe FourierLweBootstrapKey::bootstrap   (homomorphic_shift_boolean)
//                         tfhe wop_pbs::vertical_packing           (blind_rotate_assign, VP flavour)
//   pfks_kernel           tfhe private_functional_keyswitch_lwe_ciphertext_into_glwe_ciphertext
//   fft_torus_kernel      tfhe FourierGgswCiphertext::fill_with_forward_fourier (and the BSK)
//   aes_*_kernel          ShiftRows / MixColumns / AddRoundKey as LWE additions
//                         (fhe_sbox_gal_mul_pbs.rs:61-132, data_model.rs:270-281)
#include <hip/hip_runtime.h>

#include <cerrno>

#include <algorithm>
#include <cstdio>
#include <climits>
#include <cstring>
#include <stdexcept>

#include "aes.hpp"
#include "br512.hpp"
#include "br512x4.hpp"
#include "br512p16.hpp"
#include "br512lat.hpp"
#include "br1024.hpp"
#include "br1024w.hpp"
#include "br1024lat.hpp"
#include "ksgemm.hpp"
#include "engine.hpp"
#include "fft_device.hpp"

namespace tae {

void hip_check(hipError_t e, const char *what) {
    if (e != hipSuccess) throw HipError{std::string(what) + ": " + hipGetErrorString(e)};
}
#define HIPC(x) hip_check((x), #x)

namespace {

constexpr int kThreads = 256;
#ifndef TAE_G6_WM
constexpr int kG6WM = 4;  // PFKS GEMM: 96 x WM ciphertexts per workgroup tile, 256 x WM threads
#else
constexpr int kG6WM = TAE_G6_WM;
#endif
constexpr size_t kS1Rows = 16384;  // shortint_1bit selector trees: level-0 bootstraps per chunk (at least)

// ---------------------------------------------------------------------------------------------
// External product on an LDS-resident GLWE accumulator:
//   acc += GGSW [x] (acc * X^e - acc)          (cmux(ct0 = acc, ct1 = acc * X^e, ggsw))
// or, with ct1 given (the CMux tree of vertical packing), acc += GGSW [x] (ct1 - acc).
// GGSW Fourier layout [lev-1][row p][col c][M]; rows consumed finest level first, p ascending
// (fft64 add_external_product_assign: ggsw.into_levels().rev() zipped with the decomposition).
// ---------------------------------------------------------------------------------------------
template <int N>
__device__ void ext_product_step(uint64_t *__restrict__ acc, cplx *__restrict__ X, cplx *__restrict__ Y,
                                 int e, const cplx *__restrict__ ggsw, int k, int levels, int base_log,
                                 const cplx *__restrict__ twist, const cplx *__restrict__ untwist,
                                 const cplx *__restrict__ w, const uint64_t *__restrict__ ct1 = nullptr) {
    constexpr int M = N / 2;
    constexpr int R = FftPlan<M>::R, P = FftPlan<M>::P, TPJ = M / R;
    const int tid = threadIdx.x;
    // One decomposition level at a time (finest first): X holds that level's k+1 spectra and Y the
    // running MAC, so LDS does not grow with the level count (pbs_l = 6 for the 8-bit model).
    for (int lev = levels; lev >= 1; lev--) {
        // ---- forward pass 0: rotated difference, decomposition, twist, DFT_R, twiddles ----
        for (int jt = tid; jt < (k + 1) * TPJ; jt += blockDim.x) {
            const int p = jt / TPJ, u = jt - p * TPJ;
            const uint64_t *poly = acc + p * N;
            cplx v[R];
#pragma unroll
            for (int m = 0; m < R; m++) {
                const int j = u + m * TPJ;
                const uint64_t *c1 = ct1 ? ct1 + p * N : nullptr;
                const uint64_t d0 = (c1 ? c1[j] : rotated_coeff(poly, j, e, N)) - poly[j];
                const uint64_t d1 = (c1 ? c1[j + M] : rotated_coeff(poly, j + M, e, N)) - poly[j + M];
                const double x0 = (double)decomp_digit(d0, base_log, levels, lev);
                const double x1 = (double)decomp_digit(d1, base_log, levels, lev);
                const cplx t = twist[j];
                v[m] = {fma(x0, t.re, -(x1 * t.im)), fma(x0, t.im, x1 * t.re)};
            }
            dft<R, M, false>(v, w);
            cplx *dst = X + p * M;
#pragma unroll
            for (int kk = 0; kk < R; kk++) dst[u + kk * TPJ] = (u * kk) ? cmul(v[kk], w[u * kk]) : v[kk];
        }
        __syncthreads();
        // ---- forward passes 1..P-1 ----
        int L = TPJ / R;
#pragma unroll
        for (int s = 1; s < P; s++, L /= R) {
            for (int jt = tid; jt < (k + 1) * TPJ; jt += blockDim.x) {
                const int r = jt / TPJ, t = jt - r * TPJ;
                const int g = t / L, u = t - g * L;
                cplx *base = X + r * M + g * R * L + u;
                cplx v[R];
#pragma unroll
                for (int m = 0; m < R; m++) v[m] = base[m * L];
                dft<R, M, false>(v, w);
                const int step = M / (R * L);
#pragma unroll
                for (int kk = 0; kk < R; kk++) base[kk * L] = (u * kk) ? cmul(v[kk], w[u * kk * step]) : v[kk];
            }
            __syncthreads();
        }
        // ---- pointwise multiply-accumulate with this level's GGSW rows (fixed fma order:
        //      level descending, row ascending, as in the oracle) ----
        for (int idx = tid; idx < (k + 1) * M; idx += blockDim.x) {
            const int c = idx / M, f = idx - c * M;
            double re = 0.0, im = 0.0;
            if (lev != levels) {
                re = Y[c * M + f].re;
                im = Y[c * M + f].im;
            }
            for (int p = 0; p <= k; p++) {
                const int r = (lev - 1) * (k + 1) + p;
                const cplx x = X[p * M + f];
                const cplx g = ggsw[((size_t)r * (k + 1) + c) * M + f];
                re = fma(x.re, g.re, re);
                re = fma(-x.im, g.im, re);
                im = fma(x.re, g.im, im);
                im = fma(x.im, g.re, im);
            }
            Y[c * M + f] = {re, im};
        }
        __syncthreads();
    }
    int L;
    // ---- inverse passes P-1..1 (DIT) ----
    L = 1;
#pragma unroll
    for (int s = P - 1; s >= 1; s--, L *= R) {
        for (int jt = tid; jt < (k + 1) * TPJ; jt += blockDim.x) {
            const int c = jt / TPJ, t = jt - c * TPJ;
            const int g = t / L, u = t - g * L;
            cplx *base = Y + c * M + g * R * L + u;
            const int step = M / (R * L);
            cplx v[R];
#pragma unroll
            for (int kk = 0; kk < R; kk++) v[kk] = (u * kk) ? cmul(base[kk * L], cconj(w[u * kk * step])) : base[kk * L];
            dft<R, M, true>(v, w);
#pragma unroll
            for (int m = 0; m < R; m++) base[m * L] = v[m];
        }
        __syncthreads();
    }
    // ---- inverse pass 0 + untwist + torus rounding, accumulated into acc ----
    for (int jt = tid; jt < (k + 1) * TPJ; jt += blockDim.x) {
        const int c = jt / TPJ, u = jt - c * TPJ;
        const cplx *base = Y + c * M + u;
        cplx v[R];
#pragma unroll
        for (int kk = 0; kk < R; kk++) v[kk] = (u * kk) ? cmul(base[kk * TPJ], cconj(w[u * kk])) : base[kk * TPJ];
        dft<R, M, true>(v, w);
        uint64_t *out = acc + c * N;
#pragma unroll
        for (int m = 0; m < R; m++) {
            const int j = u + m * TPJ;
            const cplx t = cmul(v[m], untwist[j]);
            out[j] += from_torus(t.re);
            out[j + M] += from_torus(t.im);
        }
    }
    __syncthreads();
}

template <int N>
__device__ void sample_extract_store(const uint64_t *acc, int k, uint64_t body_add, uint64_t *out) {
    for (int t = threadIdx.x; t < k * N; t += blockDim.x) {
        const int p = t / N, j = t - p * N;
        out[t] = j == 0 ? acc[p * N] : (0 - acc[p * N + N - j]);
    }
    if (threadIdx.x == 0) out[k * N] = acc[k * N] + body_add;
}

// ---------------------------------------------------------------------------------------------
// PBS: one workgroup per ciphertext; ACC = LUT * X^{-b~}; for i < n with a_i != 0:
// cmux(ACC, ACC * X^{a~_i}, BSK_i); extract coefficient 0.  (fft64 bootstrap.rs blind_rotate_assign)
// ---------------------------------------------------------------------------------------------
template <int N>
__global__ void __launch_bounds__(kThreads) pbs_kernel(const uint64_t *__restrict__ lwe_in, uint64_t *__restrict__ lwe_out,
                                                    const uint64_t *__restrict__ lut, const cplx *__restrict__ bsk,
                                                    const cplx *__restrict__ twist, const cplx *__restrict__ untwist,
                                                    const cplx *__restrict__ w, int n, int k, int levels, int base_log,
                                                    uint64_t body_add, uint64_t out_add, size_t lut_mod, size_t ct_off) {
    constexpr int M = N / 2;
    constexpr int logN = (N == 512) ? 9 : 10;
    extern __shared__ __align__(16) unsigned char smem[];
    uint64_t *acc = reinterpret_cast<uint64_t *>(smem);
    cplx *X = reinterpret_cast<cplx *>(acc + (k + 1) * N);
    cplx *Y = X + (k + 1) * M;
    const uint64_t *in = lwe_in + (size_t)blockIdx.x * (n + 1);
    lut += ((ct_off + blockIdx.x) % lut_mod) * (size_t)(k + 1) * N;  // this ciphertext's test vector
    const int bt = mod_switch(in[n] + body_add, logN);
    const int e0 = (2 * N - (bt % (2 * N))) % (2 * N);  // X^{-b~}
    for (int t = threadIdx.x; t < (k + 1) * N; t += blockDim.x) {
        const int c = t / N, j = t - c * N;
        acc[t] = rotated_coeff(lut + c * N, j, e0, N);
    }
    __syncthreads();
    const size_t ggsw_sz = (size_t)levels * (k + 1) * (k + 1) * M;
    for (int i = 0; i < n; i++) {
        const uint64_t a = in[i];
        if (a == 0) continue;
        const int e = mod_switch(a, logN) % (2 * N);
        ext_product_step<N>(acc, X, Y, e, bsk + (size_t)i * ggsw_sz, k, levels, base_log, twist, untwist, w);
    }
    sample_extract_store<N>(acc, k, out_add, lwe_out + (size_t)blockIdx.x * (k * N + 1));
}

// ---------------------------------------------------------------------------------------------
// Vertical packing: workgroup (group g, output j): ACC = trivial(LUT_j), or the CMux tree's GLWE
// init[g][j] when the LUT has more than one polynomial; for the GGSWs n_in-1 .. b_stop,
// cmux(ACC, ACC * X^{-2^t}, GGSW); extract coefficient 0.  (wop_pbs::vertical_packing ->
// blind_rotate_assign)
// ---------------------------------------------------------------------------------------------
template <int N>
__global__ void __launch_bounds__(kThreads) vp_kernel(const cplx *__restrict__ ggsw_f, int n_in, const uint64_t *__restrict__ lut,
                                                   int n_out, uint64_t *__restrict__ out, const cplx *__restrict__ twist,
                                                   const cplx *__restrict__ untwist, const cplx *__restrict__ w, int k,
                                                   int levels, int base_log, const uint64_t *__restrict__ init = nullptr,
                                                   int b_stop = 0) {
    constexpr int M = N / 2;
    extern __shared__ __align__(16) unsigned char smem[];
    uint64_t *acc = reinterpret_cast<uint64_t *>(smem);
    cplx *X = reinterpret_cast<cplx *>(acc + (k + 1) * N);
    cplx *Y = X + (k + 1) * M;
    const int g = blockIdx.x / n_out, jout = blockIdx.x - g * n_out;
    if (init) {
        const uint64_t *src = init + (size_t)blockIdx.x * (k + 1) * N;
        for (int t = threadIdx.x; t < (k + 1) * N; t += blockDim.x) acc[t] = src[t];
    } else {
        for (int t = threadIdx.x; t < (k + 1) * N; t += blockDim.x)
            acc[t] = t < k * N ? 0 : lut[(size_t)jout * N + (t - k * N)];
    }
    __syncthreads();
    const size_t ggsw_sz = (size_t)levels * (k + 1) * (k + 1) * M;
    int deg = 1;
    for (int b = n_in - 1; b >= b_stop; b--, deg <<= 1) {
        const int e = 2 * N - deg;
        ext_product_step<N>(acc, X, Y, e, ggsw_f + ((size_t)g * n_in + b) * ggsw_sz, k, levels, base_log, twist,
                            untwist, w);
    }
    sample_extract_store<N>(acc, k, 0, out + ((size_t)g * n_out + jout) * (k * N + 1));
}

// ---------------------------------------------------------------------------------------------
// CMux tree of vertical packing (wop_pbs cmux_tree_memory_optimized) for LUTs of 2^tree
// polynomials (input_bits > log2 N).  Leaves: trivial GLWEs of the LUT polynomials,
// [n_out][2^tree][(k+1)N], shared by every group.  One tree level: workgroup (g, j, i) computes
// node i = cmux(c0 = src[g][j][2i], c1 = src[g][j][2i+1], GGSW_{g, t}) = c0 + GGSW [x] (c1 - c0).
// ---------------------------------------------------------------------------------------------
__global__ void vp_leaves_kernel(const uint64_t *__restrict__ lut, size_t small_len, int n_out, int cnt, int k, int N,
                                 uint64_t *__restrict__ leaves) {
    const size_t glwe = (size_t)(k + 1) * N;
    const size_t total = (size_t)n_out * cnt * glwe;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        const size_t row = t / glwe, c = t - row * glwe;
        const size_t j = row / cnt, i = row - j * cnt;
        leaves[t] = c < (size_t)k * N ? 0 : lut[j * small_len + i * N + (c - (size_t)k * N)];
    }
}

template <int N>
__global__ void __launch_bounds__(kThreads) cmux_tree_kernel(const cplx *__restrict__ ggsw_f, int n_in, int t,
                                                          const uint64_t *__restrict__ src, long src_gstride, int cnt,
                                                          int n_out, uint64_t *__restrict__ dst,
                                                          const cplx *__restrict__ twist, const cplx *__restrict__ untwist,
                                                          const cplx *__restrict__ w, int k, int levels, int base_log) {
    constexpr int M = N / 2;
    extern __shared__ __align__(16) unsigned char smem[];
    uint64_t *acc = reinterpret_cast<uint64_t *>(smem);
    cplx *X = reinterpret_cast<cplx *>(acc + (k + 1) * N);
    cplx *Y = X + (k + 1) * M;
    const size_t glwe = (size_t)(k + 1) * N;
    const int half = cnt / 2;
    const size_t gj = blockIdx.x / half;
    const int i = (int)(blockIdx.x - gj * half);
    const size_t g = gj / n_out, j = gj - g * n_out;
    const uint64_t *c0 = src + g * src_gstride + (j * cnt + 2 * i) * glwe;
    for (int x = threadIdx.x; x < (int)glwe; x += blockDim.x) acc[x] = c0[x];
    __syncthreads();
    const size_t ggsw_sz = (size_t)levels * (k + 1) * (k + 1) * M;
    ext_product_step<N>(acc, X, Y, 0, ggsw_f + (g * n_in + t) * ggsw_sz, k, levels, base_log, twist, untwist, w,
                        c0 + glwe);
    uint64_t *o = dst + (gj * half + i) * glwe;
    for (int x = threadIdx.x; x < (int)glwe; x += blockDim.x) o[x] = acc[x];
}

// ---------------------------------------------------------------------------------------------
// Forward torus FFT of many polynomials (GGSW / BSK to the Fourier domain).  TPJ threads per
// polynomial, 256/TPJ polynomials per workgroup.
// ---------------------------------------------------------------------------------------------
// N = 512 (R = 16, 16 threads per polynomial, four polynomials per wave): the spectrum sits in LDS with
// one pad slot per 16 (fft_pidx) and a polynomial stride of 272 slots (= 0 mod 16), so that every
// ds_read_b128 lane group (MI355X_MICROARCH.md: lanes {0-3, 12-15, 20-27}, ... of two polynomials) of
// pass 1's stride-16 reads and of the final reads hits 16 distinct 16-byte bank groups; the old stride 273
// put two lanes of those groups on one (PMC SQ_LDS_BANK_CONFLICT 65% of the LDS cycles, round 4).
// N = 1024 (R = 8, one polynomial per wave): one pad slot per 8 (slot 9 u + m in pass 2, where the
// unpadded stride-8 reads and writes were 8-way conflicts: 356% conflict cycles, round 4).
template <int M>
__device__ __forceinline__ int fft_pidx(int f) { return M == 256 ? f + (f >> 4) : f + (f >> 3); }
template <int M>
constexpr int fft_poly_stride() { return M == 256 ? 272 : M + M / 8; }
// lane -> offset inside a pair of 64-value output chunks for the N = 1024 final reads (see fft_torus_kernel)
__constant__ unsigned char kFftTau1k[64] = {0,  1,  2,  3,  8,  9,  10, 11, 12, 13, 14, 15, 4,  5,  6,  7,
                                            72, 73, 74, 75, 64, 65, 66, 67, 68, 69, 70, 71, 76, 77, 78, 79,
                                            16, 17, 18, 19, 24, 25, 26, 27, 28, 29, 30, 31, 20, 21, 22, 23,
                                            88, 89, 90, 91, 80, 81, 82, 83, 84, 85, 86, 87, 92, 93, 94, 95};

template <int N>
__global__ void __launch_bounds__(kThreads) fft_torus_kernel(const uint64_t *__restrict__ in, cplx *__restrict__ out,
                                                          size_t count, const cplx *__restrict__ twist,
                                                          const cplx *__restrict__ w) {
    constexpr int M = N / 2;
    constexpr int R = FftPlan<M>::R, P = FftPlan<M>::P, TPJ = M / R, JPB = kThreads / TPJ;
    extern __shared__ __align__(16) unsigned char smem[];
    cplx *buf = reinterpret_cast<cplx *>(smem);
    const int local = threadIdx.x / TPJ, u = threadIdx.x - local * TPJ;
    const size_t poly = (size_t)blockIdx.x * JPB + local;
    const bool active = poly < count;
    cplx *X = buf + local * fft_poly_stride<M>();
    if (active) {
        const uint64_t *src = in + poly * N;
        cplx v[R];
#pragma unroll
        for (int m = 0; m < R; m++) {
            const int j = u + m * TPJ;
            const double x0 = (double)(int64_t)src[j] * 0x1p-64, x1 = (double)(int64_t)src[j + M] * 0x1p-64;
            const cplx t = twist[j];
            v[m] = {fma(x0, t.re, -(x1 * t.im)), fma(x0, t.im, x1 * t.re)};
        }
        dft<R, M, false>(v, w);
#pragma unroll
        for (int kk = 0; kk < R; kk++) X[fft_pidx<M>(u + kk * TPJ)] = (u * kk) ? cmul(v[kk], w[u * kk]) : v[kk];
    }
    __syncthreads();
    int L = TPJ / R;
#pragma unroll
    for (int s = 1; s < P; s++, L /= R) {
        if (active) {
            const int gg = u / L, uu = u - gg * L;
            const int b0 = gg * R * L + uu;
            cplx v[R];
#pragma unroll
            for (int m = 0; m < R; m++) v[m] = X[fft_pidx<M>(b0 + m * L)];
            dft<R, M, false>(v, w);
            const int step = M / (R * L);
#pragma unroll
            for (int kk = 0; kk < R; kk++)
                X[fft_pidx<M>(b0 + kk * L)] = (uu * kk) ? cmul(v[kk], w[uu * kk * step]) : v[kk];
        }
        __syncthreads();
    }
    if (active) {
        cplx *dst = out + poly * M;
        if constexpr (M == 512) {
            // final reads of N = 1024 by lane permutation: read c (0..7) of lane u takes f = 128 (c >> 1) + 32 (c & 1)
            // + kFftTau1k[u], which gives each ds_read_b128 lane group the two 8-blocks a, a + 8 of f, whose slots
            // 9 a + b cover all 16 bank groups (the lane-ordered f = u + 64 c were 2-way conflicts in every group;
            // scripts/layout/fft1k_banks.py); every read still stores whole 128-byte lines
#pragma unroll
            for (int c = 0; c < 8; c++) {
                const int f = 128 * (c >> 1) + 32 * (c & 1) + kFftTau1k[u];
                dst[f] = X[fft_pidx<M>(f)];
            }
        } else {
            for (int f = u; f < M; f += TPJ) dst[f] = X[fft_pidx<M>(f)];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Keyswitch: out[b] = (0, .., 0, body) - sum_i sum_l d_{b,i,l} * KSK[i][l].  Thread = output
// coefficient j, CT ciphertexts per workgroup; digits staged in LDS per chunk of inputs.
// ---------------------------------------------------------------------------------------------
constexpr int KS_CT = 16, KS_CHUNK = 64;

__global__ void __launch_bounds__(kThreads) keyswitch_kernel(const uint64_t *__restrict__ in, uint64_t *__restrict__ out,
                                                          const uint64_t *__restrict__ ksk, size_t B, int K, int n,
                                                          int ks_l, int ks_b) {
    __shared__ int8_t dig[KS_CT][KS_CHUNK][8];
    const int j = blockIdx.x * kThreads + threadIdx.x;
    const size_t b0 = (size_t)blockIdx.y * KS_CT;
    uint64_t acc[KS_CT];
#pragma unroll
    for (int c = 0; c < KS_CT; c++) acc[c] = 0;
    for (int i0 = 0; i0 < K; i0 += KS_CHUNK) {
        for (int idx = threadIdx.x; idx < KS_CT * KS_CHUNK; idx += kThreads) {
            const int c = idx / KS_CHUNK, ii = idx - c * KS_CHUNK;
            const int i = i0 + ii;
            const bool ok = (b0 + c < B) && i < K;
            const uint64_t x = ok ? in[(b0 + c) * (K + 1) + i] : 0;
            for (int l = 1; l <= ks_l; l++) dig[c][ii][l - 1] = ok ? (int8_t)decomp_digit(x, ks_b, ks_l, l) : 0;
        }
        __syncthreads();
        if (j <= n) {
            const int iend = min(KS_CHUNK, K - i0);
            for (int ii = 0; ii < iend; ii++)
                for (int l = 0; l < ks_l; l++) {
                    const uint64_t key = ksk[((size_t)(i0 + ii) * ks_l + l) * (n + 1) + j];
#pragma unroll
                    for (int c = 0; c < KS_CT; c++) acc[c] -= mul_i32_u64(dig[c][ii][l], key);
                }
        }
        __syncthreads();
    }
    if (j <= n)
        for (int c = 0; c < KS_CT; c++)
            if (b0 + c < B) out[(b0 + c) * (n + 1) + j] = acc[c] + (j == n ? in[(b0 + c) * (K + 1) + K] : 0);
}

// ---------------------------------------------------------------------------------------------
// PFKS: GGSW row q of ciphertext b = - sum_{i<=K} sum_l d_{b,i,l} * PFPKSK[q][i][l]
// ---------------------------------------------------------------------------------------------
constexpr int PF_CT = 32, PF_CHUNK = 32;

__global__ void __launch_bounds__(kThreads) pfks_kernel(const uint64_t *__restrict__ in, uint64_t *__restrict__ ggsw,
                                                     const uint64_t *__restrict__ pfpksk, size_t B, int K, int glwe,
                                                     int pf_l, int pf_b, int cbs_l, int level, int k) {
    __shared__ int32_t dig[PF_CT][PF_CHUNK][4];
    const int col = blockIdx.x * kThreads + threadIdx.x;
    const int q = blockIdx.y;
    const size_t b0 = (size_t)blockIdx.z * PF_CT;
    uint64_t acc[PF_CT];
#pragma unroll
    for (int c = 0; c < PF_CT; c++) acc[c] = 0;
    const uint64_t *key = pfpksk + (size_t)q * (K + 1) * pf_l * glwe;
    for (int i0 = 0; i0 <= K; i0 += PF_CHUNK) {
        for (int idx = threadIdx.x; idx < PF_CT * PF_CHUNK; idx += kThreads) {
            const int c = idx / PF_CHUNK, ii = idx - c * PF_CHUNK;
            const int i = i0 + ii;
            const bool ok = (b0 + c < B) && i <= K;
            const uint64_t x = ok ? in[(b0 + c) * (K + 1) + i] : 0;
            for (int l = 1; l <= pf_l; l++) dig[c][ii][l - 1] = ok ? (int32_t)decomp_digit(x, pf_b, pf_l, l) : 0;
        }
        __syncthreads();
        if (col < glwe) {
            const int iend = min(PF_CHUNK, K + 1 - i0);
            for (int ii = 0; ii < iend; ii++)
                for (int l = 0; l < pf_l; l++) {
                    const uint64_t kv = key[((size_t)(i0 + ii) * pf_l + l) * glwe + col];
#pragma unroll
                    for (int c = 0; c < PF_CT; c++) acc[c] -= mul_i32_u64(dig[c][ii][l], kv);
                }
        }
        __syncthreads();
    }
    if (col < glwe)
        for (int c = 0; c < PF_CT; c++)
            if (b0 + c < B) ggsw[(((b0 + c) * cbs_l + (level - 1)) * (k + 1) + q) * (size_t)glwe + col] = acc[c];
}

// ---------------------------------------------------------------------------------------------
// AES linear layer as LWE additions (state = [blk][16 bytes][8 bits][K+1])
// ---------------------------------------------------------------------------------------------
// state = blocks + rk[round 0]   (xor_state, data_model.rs:270-274)
__global__ void aes_ark0_kernel(const uint64_t *__restrict__ blocks, const uint64_t *__restrict__ rk,
                                uint64_t *__restrict__ state, size_t nb, int L) {
    const size_t total = nb * 128 * (size_t)L;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        const size_t within = t % (128 * (size_t)L);
        state[t] = blocks[t] + rk[within];
    }
}

// ShiftRows on the three SubBytes*{1,2,3} states, MixColumns, AddRoundKey:
// out[r][c] = 2s[r][c'] + s[r+3][.] + s[r+2][.] + 3s[r+1][.]  (fhe_sbox_gal_mul_pbs.rs:61-82)
__global__ void aes_mix_kernel(const uint64_t *__restrict__ muls, const uint64_t *__restrict__ rk_round,
                               uint64_t *__restrict__ state, size_t nb, int L) {
    const size_t total = nb * 128 * (size_t)L;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        const size_t coef = t % L;
        const size_t ct = t / L;  // blk*128 + pos*8 + bit
        const int bit = (int)(ct & 7);
        const int pos = (int)((ct >> 3) & 15);
        const size_t blk = ct >> 7;
        const int c = pos >> 2, row = pos & 3;
        // after ShiftRows, element (rr, c) comes from SubBytes output byte 4*((c+rr)%4) + rr
        auto src = [&](int rr, int m) {
            const int byte = 4 * ((c + rr) & 3) + rr;
            return muls[(((blk * 16 + byte) * 24) + 8 * m + bit) * (size_t)L + coef];
        };
        state[t] = src(row, 1) + src((row + 3) & 3, 0) + src((row + 2) & 3, 0) + src((row + 1) & 3, 2) +
                   rk_round[(size_t)(pos * 8 + bit) * L + coef];
    }
}

// last round: SubBytes (8->8), ShiftRows, AddRoundKey(rk[40..44])
__global__ void aes_final_kernel(const uint64_t *__restrict__ sb, const uint64_t *__restrict__ rk_round,
                                 uint64_t *__restrict__ out, size_t nb, int L) {
    const size_t total = nb * 128 * (size_t)L;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        const size_t coef = t % L;
        const size_t ct = t / L;
        const int bit = (int)(ct & 7);
        const int pos = (int)((ct >> 3) & 15);
        const size_t blk = ct >> 7;
        const int c = pos >> 2, row = pos & 3;
        const int byte = 4 * ((c + row) & 3) + row;
        out[t] = sb[((blk * 16 + byte) * 8 + bit) * (size_t)L + coef] + rk_round[(size_t)(pos * 8 + bit) * L + coef];
    }
}

__global__ void lwe_add_kernel(uint64_t *__restrict__ a, const uint64_t *__restrict__ b, size_t count) {
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < count; t += (size_t)gridDim.x * blockDim.x)
        a[t] += b[t];
}

// ---------------------------------------------------------------------------------------------
// 8-bit model helpers (shortint_woppbs_8bit.rs / fhe_sbox_pbs.rs)
// ---------------------------------------------------------------------------------------------
__global__ void lwe_shl_kernel(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, size_t count, int shift) {
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < count; t += (size_t)gridDim.x * blockDim.x)
        out[t] = in[t] << shift;
}

__global__ void lwe_sub_kernel(uint64_t *__restrict__ a, const uint64_t *__restrict__ b, size_t count) {
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < count; t += (size_t)gridDim.x * blockDim.x)
        a[t] -= b[t];
}

// dst[r * dst_stride + j] = src[r * len + j]
__global__ void copy_rows_kernel(const uint64_t *__restrict__ src, uint64_t *__restrict__ dst, size_t rows, int len,
                                 size_t dst_stride) {
    const size_t total = rows * (size_t)len;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        const size_t r = t / len, j = t - r * len;
        dst[r * dst_stride + j] = src[t];
    }
}

// ShiftRows + MixColumns (fhe_sbox_pbs.rs:33-73: gf_256_mul as shifts and XORs of bits, i.e. LWE
// additions) + AddRoundKey on small-key bits.  sb = SubBytes output [blk][16 bytes][8 bits][L];
// T.idx[o][*] = the input bits (column-local, byte-major, MSB-first, -1 terminated) summed into
// output bit o of a column (or_mix_column_terms in the oracle).
struct MixTerms {
    int8_t idx[32][8];
};

__global__ void aes8_mix_kernel(const uint64_t *__restrict__ sb, const uint64_t *__restrict__ rk_round,
                                uint64_t *__restrict__ state, size_t nb, int L, MixTerms T) {
    const size_t total = nb * 128 * (size_t)L;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        const size_t coef = t % L;
        const size_t ct = t / L;
        const int bit = (int)(ct & 7);
        const int pos = (int)((ct >> 3) & 15);
        const size_t blk = ct >> 7;
        const int c = pos >> 2, row = pos & 3, o = 8 * row + bit;
        uint64_t acc = rk_round[(size_t)(pos * 8 + bit) * L + coef];
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const int i = T.idx[o][q];
            if (i < 0) break;
            const int ri = i >> 3, bi = i & 7;
            const int byte = 4 * ((c + ri) & 3) + ri;  // ShiftRows: state[ri][c] = sb[ri][(c + ri) % 4]
            acc += sb[((blk * 16 + byte) * 8 + bi) * (size_t)L + coef];
        }
        state[t] = acc;
    }
}

// ---- shortint_1bit model (src/tfhe/shortint_1bit.rs) ----
// test_vector_from_ciphertexts (shortint_1bit.rs:392-492) for pair p: with P0 / P1 the packing keyswitches of the two
// ciphertexts, tv = sum_{i in [0, N/4) u [3N/4, N)} X^i P0 + sum_{i in [N/4, 3N/4)} X^i P1 (negacyclic,
// wrapping u64: the reference's add-then-rotate loops in closed form).  One workgroup per (pair, polynomial).
// The term of shift i is E[t + N - i] of the negacyclic extension E = [-P, P] (length 2N), so each run of
// shifts with one source is a window of E: tv[t] = sum over the three runs of Pre[t + N - i0 + 1] -
// Pre[t + N - i1 + 1], Pre the exclusive prefix sums of E (mod 2^64, hence exact): O(N) per polynomial.
template <int N>
__global__ void __launch_bounds__(kThreads) s1_tv_kernel(const uint64_t *__restrict__ pks, uint64_t *__restrict__ tv, int k) {
    constexpr int PER = 2 * N / kThreads;
    static_assert(PER * kThreads == 2 * N, "s1_tv_kernel shape");
    __shared__ uint64_t pa[2 * N + 1], pb[2 * N + 1], part[2][kThreads];
    const size_t pair = blockIdx.x / (k + 1);
    const int c = blockIdx.x - (int)pair * (k + 1);
    const size_t glwe = (size_t)(k + 1) * N;
    const uint64_t *p0 = pks + 2 * pair * glwe + (size_t)c * N, *p1 = p0 + glwe;
    const int tid = threadIdx.x, y0 = tid * PER;
    uint64_t xa[PER], xb[PER], sa = 0, sb = 0;
#pragma unroll
    for (int j = 0; j < PER; j++) {
        const int y = y0 + j;
        xa[j] = y < N ? 0 - p0[y] : p0[y - N];
        xb[j] = y < N ? 0 - p1[y] : p1[y - N];
        sa += xa[j];
        sb += xb[j];
    }
    part[0][tid] = sa;
    part[1][tid] = sb;
    __syncthreads();
    for (int off = 1; off < kThreads; off <<= 1) {  // inclusive scan of the per-thread sums
        const uint64_t ua = tid >= off ? part[0][tid - off] : 0, ub = tid >= off ? part[1][tid - off] : 0;
        __syncthreads();
        part[0][tid] += ua;
        part[1][tid] += ub;
        __syncthreads();
    }
    uint64_t ea = tid ? part[0][tid - 1] : 0, eb = tid ? part[1][tid - 1] : 0;
#pragma unroll
    for (int j = 0; j < PER; j++) {
        pa[y0 + j] = ea;
        pb[y0 + j] = eb;
        ea += xa[j];
        eb += xb[j];
    }
    if (tid == kThreads - 1) {
        pa[2 * N] = ea;
        pb[2 * N] = eb;
    }
    __syncthreads();
    for (int t = tid; t < N; t += kThreads) {
        const int z = t + N + 1;  // window of the run [i0, i1): Pre[z - i0] - Pre[z - i1]
        const uint64_t acc = (pa[z] - pa[z - N / 4]) + (pb[z - N / 4] - pb[z - 3 * N / 4]) + (pa[z - 3 * N / 4] - pa[z - N]);
        tv[pair * glwe + (size_t)c * N + t] = acc;
    }
}

// keyswitch_lwe_ciphertext_list_and_pack_in_glwe_ciphertext: out = sum_j X^j P_j over count keyswitched
// GLWEs P_j (one workgroup per polynomial)
template <int N>
__global__ void __launch_bounds__(kThreads) s1_pack_kernel(const uint64_t *__restrict__ pks, int count, uint64_t *__restrict__ out,
                                                        int k) {
    const int c = blockIdx.x;
    const size_t glwe = (size_t)(k + 1) * N;
    for (int t = threadIdx.x; t < N; t += blockDim.x) {
        uint64_t acc = 0;
        for (int j = 0; j < count; j++) {
            const int src = t - j;
            const uint64_t v = pks[(size_t)j * glwe + (size_t)c * N + (src < 0 ? src + N : src)];
            acc += src < 0 ? (0 - v) : v;
        }
        out[(size_t)c * N + t] = acc;
    }
}

// row b of out = row (b / reps) * stride + sel of in (the selector bit of each bootstrap of a tree level)
__global__ void s1_gather_kernel(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, size_t rows, size_t reps,
                                 int stride, int sel, int L) {
    const size_t total = rows * (size_t)L;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        const size_t r = t / L, j = t - r * L;
        out[t] = in[((r / reps) * stride + sel) * (size_t)L + j];
    }
}

// the Fourier BSK the fused-twiddle transforms multiply with (lf512.hpp, lf1k.hpp): G * conj(E2(pos)) per
// position (M = 256 or 512 positions), the oracle's lf_rescale (same cmul)
__global__ void __launch_bounds__(kThreads) lf_rescale_kernel(cplx *__restrict__ g, size_t polys, int M,
                                                              const cplx *__restrict__ e2) {
    const size_t total = polys * M;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x)
        g[t] = cmul(g[t], e2[t & (M - 1)]);
}

unsigned grid_for(size_t total) { return (unsigned)std::min<size_t>((total + kThreads - 1) / kThreads, 65536); }

constexpr int kBrC = 3;  // ciphertexts per workgroup in the batched N=512 blind rotation

template <int N>
size_t br_lds_bytes(int k, int levels) {
    (void)levels;  // ext_product_step works one level at a time
    return (size_t)(k + 1) * N * 8 + 2 * (size_t)(k + 1) * (N / 2) * 16;
}

}  // namespace

// =============================================================================================
// Engine
// =============================================================================================

void *Engine::alloc(size_t bytes) {
    void *p = nullptr;
    HIPC(hipMalloc(&p, std::max<size_t>(bytes, 16)));
    return p;
}

template <class T>
T *Engine::grow(T *&ptr, size_t &cap, size_t count) {
    if (count > cap) {
        if (ptr) HIPC(hipFree(ptr));
        ptr = nullptr;  // a failing alloc below must not leave a freed pointer for ~Engine
        cap = 0;
        ptr = static_cast<T *>(alloc(count * sizeof(T)));
        cap = count;
    }
    return ptr;
}

void Engine::init_common() {
    HIPC(hipSetDevice(device_));
    // TAE_CU_MASK (probe / A-B knob, scripts/probes/stage_overlap.py): "lo:N" or "hi:N" restricts the engine
    // stream to the first / last N CUs of the device's CU mask (hipExtStreamCreateWithCUMask); batch rounds
    // are then sized for N CUs
    int mask_cus = 0;
    if (const char *cm = getenv("TAE_CU_MASK")) {
        int total = 0;
        HIPC(hipDeviceGetAttribute(&total, hipDeviceAttributeMultiprocessorCount, device_));
        const bool hi = !strncmp(cm, "hi:", 3);
        if (!hi && strncmp(cm, "lo:", 3)) throw std::runtime_error("TAE_CU_MASK must be lo:N or hi:N");
        char *end = nullptr;
        const long nc = strtol(cm + 3, &end, 10);
        if (end == cm + 3 || *end || nc < 1 || nc > total || total > 256)
            throw std::runtime_error(std::string("TAE_CU_MASK: bad CU count in '") + cm + "'");
        uint32_t mask[8] = {0};
        for (int c = 0; c < nc; c++) {
            const int b = hi ? total - 1 - c : c;
            mask[b >> 5] |= 1u << (b & 31);
        }
        HIPC(hipExtStreamCreateWithCUMask(&stream_, 8, mask));
        mask_cus = (int)nc;
    } else {
        HIPC(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    }
    if (p_.N != 512 && p_.N != 1024) throw std::runtime_error("unsupported polynomial size");
    const FftTables t = make_fft_tables(p_.N);
    const size_t tb = sizeof(double) * 2 * t.M;
    d_twist_ = static_cast<cplx *>(alloc(tb));
    d_untwist_ = static_cast<cplx *>(alloc(tb));
    d_w_ = static_cast<cplx *>(alloc(tb));
    HIPC(hipMemcpy(d_twist_, t.twist.data(), tb, hipMemcpyHostToDevice));
    HIPC(hipMemcpy(d_untwist_, t.untwist.data(), tb, hipMemcpyHostToDevice));
    HIPC(hipMemcpy(d_w_, t.w.data(), tb, hipMemcpyHostToDevice));
    // homomorphic_shift_boolean accumulators: body = -alpha, alpha = 2^(63 - cbs_b * level)
    std::vector<uint64_t> luts((size_t)std::max(p_.cbs_l, 1) * p_.glwe_len(), 0);
    for (int lev = 1; lev <= p_.cbs_l; lev++) {
        const uint64_t alpha = 1ull << (63 - p_.cbs_b * lev);
        for (int j = 0; j < p_.N; j++) luts[(size_t)(lev - 1) * p_.glwe_len() + (size_t)p_.k * p_.N + j] = 0 - alpha;
    }
    d_lut_shift_ = static_cast<uint64_t *>(alloc(luts.size() * 8));
    HIPC(hipMemcpy(d_lut_shift_, luts.data(), luts.size() * 8, hipMemcpyHostToDevice));
    // AES LUTs (fhe_impls/shortint_woppbs_1bit.rs:32-45, :94-128) -- built host-side once
    std::vector<uint64_t> f24(256), f8(256);
    for (int x = 0; x < 256; x++) {
        const uint8_t s = kSbox[x];
        f24[x] = ((uint64_t)gf_256_mul(s, 1) << 16) | ((uint64_t)gf_256_mul(s, 2) << 8) | gf_256_mul(s, 3);
        f8[x] = s;
    }
    std::vector<uint64_t> l24(24 * lut_small_len(p_.N, 8)), l8(8 * lut_small_len(p_.N, 8));
    generate_lut(p_.N, 8, 24, f24.data(), l24.data());
    generate_lut(p_.N, 8, 8, f8.data(), l8.data());
    d_lut24_ = static_cast<uint64_t *>(alloc(l24.size() * 8));
    d_lut8_ = static_cast<uint64_t *>(alloc(l8.size() * 8));
    HIPC(hipMemcpy(d_lut24_, l24.data(), l24.size() * 8, hipMemcpyHostToDevice));
    HIPC(hipMemcpy(d_lut8_, l8.data(), l8.size() * 8, hipMemcpyHostToDevice));
    if (p_.model == 2) {
        // shortint_1bit ByteT (fhe_impls/shortint_1bit.rs:17-50): bootstrap_assign's identity test vector
        // and sbox_substitute's 8 multivariate test vectors (one per output bit, MSB first), each the
        // 128 cleartext test vectors of generate_multivariate_test_vector (shortint_1bit.rs:519-536)
        const size_t glwe = p_.glwe_len(), V = 128;
        std::vector<uint64_t> tvs(8 * V * glwe), id(glwe);
        for (int f = 0; f < 8; f++)
            for (size_t v = 0; v < V; v++) {
                const uint8_t s0 = kSbox[2 * v], s1 = kSbox[2 * v + 1];
                s1_test_vector(p_, (s0 >> (7 - f)) & 1, (s1 >> (7 - f)) & 1, &tvs[(f * V + v) * glwe]);
            }
        s1_test_vector(p_, 0, 1, id.data());
        d_s1_sbox_tv_ = static_cast<uint64_t *>(alloc(tvs.size() * 8));
        d_s1_id_tv_ = static_cast<uint64_t *>(alloc(id.size() * 8));
        HIPC(hipMemcpy(d_s1_sbox_tv_, tvs.data(), tvs.size() * 8, hipMemcpyHostToDevice));
        HIPC(hipMemcpy(d_s1_id_tv_, id.data(), id.size() * 8, hipMemcpyHostToDevice));
    }
    if (p_.model == 8 || p_.model == 2) {
        int terms[32][32];
        mix_column_terms(terms);
        for (int o = 0; o < 32; o++) {
            int q = 0;
            for (int i = 0; i < 32; i++)
                for (int c = 0; c < terms[o][i]; c++) {
                    if (q >= 8) throw std::runtime_error("MixColumns network: more than 8 terms per bit");
                    mix_idx_[o][q++] = (int8_t)i;
                }
            for (; q < 8; q++) mix_idx_[o][q] = -1;
        }
    }
    if (p_.model == 8) {
        // 8-bit model: SBOX / identity LUTs without padding (fhe_impls/shortint_woppbs_8bit.rs:17-35)
        std::vector<uint64_t> fs(256), fi(256), ws(std::max(p_.N, 256)), wi(std::max(p_.N, 256));
        for (int x = 0; x < 256; x++) {
            fs[x] = kSbox[x];
            fi[x] = (uint64_t)x;
        }
        generate_lut_without_padding(p_.N, fs.data(), ws.data());
        generate_lut_without_padding(p_.N, fi.data(), wi.data());
        d_wlut_sbox_ = static_cast<uint64_t *>(alloc(ws.size() * 8));
        d_wlut_id_ = static_cast<uint64_t *>(alloc(wi.size() * 8));
        HIPC(hipMemcpy(d_wlut_sbox_, ws.data(), ws.size() * 8, hipMemcpyHostToDevice));
        HIPC(hipMemcpy(d_wlut_id_, wi.data(), wi.size() * 8, hipMemcpyHostToDevice));
    }
    // batched N=512, k=4 blind rotation (params_sqrd_lvl_64): br512x4 for large batches, br512lat for
    // small ones.  TAE_BR_LAT_MAX (a tuning knob, both sides pinned by tests) is the batch size up
    // to which br512lat runs (0: never).
    // The fused transform and its conj(E2)-rescaled BSK go with the blind rotation's N = 512, k = 4 shape,
    // exactly as the oracle's lf_set (tfhe_oracle.c): params_sqrd_lvl_64 (3 x 2^12: br512x4 / br512lat) and
    // the shortint_1bit set (7 x 2^6, per-ciphertext test vectors: br512x4 only); the vertical-packing
    // instantiation br512x4<1, false, 13> also needs cbs 1 x 2^13.
    lf512_ = p_.N == 512 && p_.k == 4;
    x4_512_ = lf512_ && p_.pbs_l == 3 && p_.pbs_b == 12;
    x4_s1_ = lf512_ && p_.pbs_l == 7 && p_.pbs_b == 6;
    if (lf512_ && !x4_512_ && !x4_s1_) throw std::runtime_error("N = 512, k = 4 set without a blind rotation kernel");
    x4_vp_ = x4_512_ && p_.cbs_l == 1 && p_.cbs_b == 13;
    // the 8-bit model's set: its PBS blind rotations run the N = 1024 fused-twiddle transform (lf1k.hpp)
    lf1k_ = p_.N == 1024 && p_.k == 2 && p_.pbs_l == 6 && p_.pbs_b == 7;
    if (lf512_ || lf1k_) {  // the blind rotations' fused-twiddle transform (lf512.hpp / lf1k.hpp)
        const std::vector<double> lf = lf512_ ? make_lf512_table() : make_lf1k_table();
        d_lf_ = static_cast<double *>(alloc(lf.size() * 8));
        HIPC(hipMemcpy(d_lf_, lf.data(), lf.size() * 8, hipMemcpyHostToDevice));
    }
    const char *blat = getenv("TAE_BR_LAT_MAX");
    lat_max_ = blat ? atol(blat) : 256;
    HIPC(hipDeviceGetAttribute(&num_cu_, hipDeviceAttributeMultiprocessorCount, device_));
    if (mask_cus) num_cu_ = mask_cus;
    // the lvl_64 PBS throughput kernel: br512p16 (sixteen points per lane, two ciphertexts per workgroup) or
    // br512x4 (four points per lane, three per workgroup); TAE_PBS_KERNEL = p16 / x4 (A/B knob, both pinned by tests)
    if (const char *pk = getenv("TAE_PBS_KERNEL")) {
        if (!strcmp(pk, "p16")) p16_ = true;
        else if (!strcmp(pk, "x4")) p16_ = false;
        else throw std::runtime_error(std::string("TAE_PBS_KERNEL must be p16 or x4, got '") + pk + "'");
    }
    if (x4_512_) {
        HIPC(hipFuncSetAttribute((const void *)br512p16::br_kernel<3, 12>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)br512p16::lds_bytes()));
        HIPC(hipFuncSetAttribute((const void *)br512lat::br_kernel<3, 12>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)br512lat::lds_bytes(3)));
        HIPC(hipFuncSetAttribute((const void *)br512x4::br_kernel<3, true, 12>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    }
    if (x4_vp_)
        HIPC(hipFuncSetAttribute((const void *)br512x4::br_kernel<1, false, 13>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    if (x4_s1_)
        HIPC(hipFuncSetAttribute((const void *)br512x4::br_kernel<7, true, 6>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    // batched N=1024, k=2 blind rotation (br1024.hpp); other shapes run the generic kernels
    if (p_.N == 1024 && p_.k == 2) {
        br1024_pbs_ = br1024::pick<2>(true, p_.pbs_l, p_.pbs_b);
        // one ciphertext per workgroup: two levels per pass where the level count allows (TAE_B1K_PAIR=0: one)
        const char *pair = getenv("TAE_B1K_PAIR");
        br1024_pbs1_lp_ = (pair && pair[0] == '0') ? 1 : 2;
        br1024_pbs1_ = br1024_pbs1_lp_ == 2 ? br1024::pick<1, 2>(true, p_.pbs_l, p_.pbs_b) : nullptr;
        if (!br1024_pbs1_) {
            br1024_pbs1_lp_ = 1;
            br1024_pbs1_ = br1024::pick<1>(true, p_.pbs_l, p_.pbs_b);
        }
        br1024_vp_ = br1024::pick<2>(false, p_.cbs_l, p_.cbs_b);
        // TAE_B1K_OCC2=1 (A/B knob): large PBS batches as one ciphertext per workgroup, two per CU
        const char *occ2 = getenv("TAE_B1K_OCC2");
        if (occ2 && occ2[0] == '1' && lf1k_) {
            br1024_occ2_ = br1024::pick_occ2(p_.pbs_l, p_.pbs_b);
            if (br1024_occ2_)
                HIPC(hipFuncSetAttribute((const void *)br1024_occ2_, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)br1024::lds_bytes(1, 1, true)));
        }
        for (auto kf : {br1024_pbs_, br1024_vp_})
            if (kf)
                HIPC(hipFuncSetAttribute((const void *)kf, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)br1024::lds_bytes(2)));
        // the 8-bit model's PBS at large batches: four ciphertexts per 768-thread workgroup (br1024w.hpp;
        // TAE_B1K_WIDE=0: br1024's two-ciphertext kernel instead)
        const char *wide = getenv("TAE_B1K_WIDE");
        b1kw_ = lf1k_ && p_.pbs_l == 6 && p_.pbs_b == 7 && !(wide && wide[0] == '0');
        if (b1kw_)
            HIPC(hipFuncSetAttribute((const void *)br1024w::br_kernel<6, 7>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)br1024w::lds_bytes()));
        // one ciphertext per 1024-thread workgroup, three levels per pass (the 8-bit model's PBS;
        // TAE_B1K_LAT=0: br1024's one-ciphertext kernel instead)
        const char *blat = getenv("TAE_B1K_LAT");
        if (lf1k_ && !(blat && blat[0] == '0')) {
            br1024lat_ = br1024lat::br_kernel<6, 7, 3>;
            br1024lat_lds_ = br1024lat::lds_bytes<6, 7, 3>();
            HIPC(hipFuncSetAttribute((const void *)br1024lat_, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)br1024lat_lds_));
        }
        if (br1024_pbs1_)
            HIPC(hipFuncSetAttribute((const void *)br1024_pbs1_, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)br1024::lds_bytes(1, br1024_pbs1_lp_)));
    }
    // opt-in to >64 KiB dynamic LDS for the blind-rotation kernels
    if (p_.N == 512) {
        HIPC(hipFuncSetAttribute((const void *)pbs_kernel<512>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        HIPC(hipFuncSetAttribute((const void *)vp_kernel<512>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        HIPC(hipFuncSetAttribute((const void *)cmux_tree_kernel<512>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    } else {
        HIPC(hipFuncSetAttribute((const void *)pbs_kernel<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        HIPC(hipFuncSetAttribute((const void *)vp_kernel<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        HIPC(hipFuncSetAttribute((const void *)cmux_tree_kernel<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    }
}

void Engine::bsk_to_fourier(const uint64_t *d_bsk_std) {
    d_bsk_f_ = static_cast<cplx *>(alloc(p_.bsk_fourier_len() * sizeof(cplx)));
    const size_t polys = (size_t)p_.n * p_.pbs_l * (p_.k + 1) * (p_.k + 1);
    const int M = p_.M();
    if (p_.N == 512) {
        constexpr int JPB = kThreads / (256 / 16);
        fft_torus_kernel<512><<<(unsigned)((polys + JPB - 1) / JPB), kThreads, JPB * fft_poly_stride<256>() * sizeof(cplx), stream_>>>(
            d_bsk_std, d_bsk_f_, polys, d_twist_, d_w_);
    } else {
        constexpr int JPB = kThreads / (512 / 8);
        fft_torus_kernel<1024><<<(unsigned)((polys + JPB - 1) / JPB), kThreads, JPB * fft_poly_stride<512>() * sizeof(cplx), stream_>>>(
            d_bsk_std, d_bsk_f_, polys, d_twist_, d_w_);
    }
    HIPC(hipGetLastError());
    if (lf512_ || lf1k_) {  // the blind rotations run the fused-twiddle transform: its BSK carries conj(E2)
        const cplx *e2 = reinterpret_cast<const cplx *>(d_lf_ + (lf512_ ? lf512::E2 : lf1k::E2));
        lf_rescale_kernel<<<grid_for(polys * M), kThreads, 0, stream_>>>(d_bsk_f_, polys, M, e2);
        HIPC(hipGetLastError());
    }
    HIPC(hipStreamSynchronize(stream_));
}

Engine::Engine(const ServerKeyRaw &keys, int device) : p_(keys.p), device_(device) {
    init_common();
    owns_keys_ = true;
    d_ksk_ = static_cast<uint64_t *>(alloc(keys.ksk.size() * 8));
    d_pfpksk_ = static_cast<uint64_t *>(alloc(keys.pfpksk.size() * 8));
    HIPC(hipMemcpy(d_ksk_, keys.ksk.data(), keys.ksk.size() * 8, hipMemcpyHostToDevice));
    HIPC(hipMemcpy(d_pfpksk_, keys.pfpksk.data(), keys.pfpksk.size() * 8, hipMemcpyHostToDevice));
    uint64_t *d_bsk = static_cast<uint64_t *>(alloc(keys.bsk.size() * 8));
    HIPC(hipMemcpy(d_bsk, keys.bsk.data(), keys.bsk.size() * 8, hipMemcpyHostToDevice));
    bsk_to_fourier(d_bsk);
    HIPC(hipFree(d_bsk));
    prepare_mfma_keys();
}

// Key limb matrices for the int8-MFMA keyswitches (ksgemm.hpp), built once on device.
void Engine::prepare_mfma_keys() {
    HIPC(hipFuncSetAttribute((const void *)ksgemm::gemm_g6<6, 4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)ksgemm::gemm_g6_lds<4>()));
    HIPC(hipFuncSetAttribute((const void *)ksgemm::gemm_g6<6, kG6WM, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)ksgemm::gemm_g6_lds<kG6WM>()));
    // int8-MFMA keyswitches when the digits fit their limbs (PFKS 17-bit digits as 3 x 6-bit limbs,
    // KS digits as one byte); otherwise (params_sqrd_lvl_1: pfks base 2^24) the u64 VALU kernels
    mfma_ks_ = p_.pfks_b <= 16 && p_.ks_b <= 7;
    if (!mfma_ks_) return;
    const int glwe = (int)p_.glwe_len();
    if (p_.model == 2) {
        // packing keyswitch (keyswitch_lwe_ciphertext_into_glwe_ciphertext) = the KS GEMM with the packing
        // key: kd = (i, l) over n x pfks_l, col over the GLWE, the LWE body added at column kN
        const int kd = p_.n * p_.pfks_l, nc = (p_.k + 1) * p_.N, kd_ks = p_.K() * p_.ks_l, nc_ks = p_.n + 1;
        if (p_.pfks_b > 7) throw std::runtime_error("packing keyswitch digits must fit one byte");
        kp_pf_ = (kd + ksgemm::TK - 1) / ksgemm::TK * ksgemm::TK;
        kp_ks_ = (kd_ks + ksgemm::TK - 1) / ksgemm::TK * ksgemm::TK;
        d_pf_bt_ = static_cast<int8_t *>(alloc((size_t)nc * 8 * kp_pf_));
        d_ks_bt_ = static_cast<int8_t *>(alloc((size_t)nc_ks * 8 * kp_ks_));
        dim3 gp((kp_pf_ + 63) / 64, (nc + 63) / 64), gks((kp_ks_ + 63) / 64, (nc_ks + 63) / 64);
        ksgemm::prep_key<<<gp, kThreads, 0, stream_>>>(d_pfpksk_, d_pf_bt_, kd, kp_pf_, nc, nc, nc, 0);
        ksgemm::prep_key<<<gks, kThreads, 0, stream_>>>(d_ksk_, d_ks_bt_, kd_ks, kp_ks_, nc_ks, nc_ks, nc_ks, 0);
        HIPC(hipGetLastError());
        HIPC(hipStreamSynchronize(stream_));
        return;
    }
    const int kd_pf = (p_.K() + 1) * p_.pfks_l, kd_ks = p_.K() * p_.ks_l;
    kp_pf_ = (kd_pf + ksgemm::TK - 1) / ksgemm::TK * ksgemm::TK;
    kp_ks_ = (kd_ks + ksgemm::TK - 1) / ksgemm::TK * ksgemm::TK;
    const int nc_pf = (p_.k + 1) * glwe, nc_ks = p_.n + 1;
    const long pf_blk = (long)(p_.K() + 1) * p_.pfks_l * glwe;
    d_pf_bt_ = static_cast<int8_t *>(alloc((size_t)nc_pf * 8 * kp_pf_));
    d_ks_bt_ = static_cast<int8_t *>(alloc((size_t)nc_ks * 8 * kp_ks_));
    dim3 gpf((kp_pf_ + 63) / 64, (nc_pf + 63) / 64), gks((kp_ks_ + 63) / 64, (nc_ks + 63) / 64);
    // the LDS-DMA GEMM reads both operands row-pair interleaved (ksgemm::op_off; Kp % 128 == 0)
    ksgemm::prep_key<<<gpf, kThreads, 0, stream_>>>(d_pfpksk_, d_pf_bt_, kd_pf, kp_pf_, nc_pf, glwe, glwe, pf_blk, true);
    // TAE_PFKS_LAYOUT (a tuning knob, every value pinned by tests/test_gpu_parity.py): "rows" = 6-bit
    // row-tile limbs always, "k" = K layout always, "k5" = K layout always and without clamped digits
    const char *lay = getenv("TAE_PFKS_LAYOUT");
    const bool k5 = lay && !strcmp(lay, "k5");
    pf_kl_ = ksgemm::kslots_build(p_.pfks_b, p_.pfks_l, pf_slots_, !k5);
    if (lay) {
        if (!strcmp(lay, "rows")) pf_kl_min_ = LONG_MAX;
        if (!strcmp(lay, "k") || k5) pf_kl_min_ = 0;
    }
    if (pf_kl_) {  // K-layout key rows (limbs in K) and the per-column offset correction
        kp_pf_kl_ = ((p_.K() + 1) * pf_slots_.S + ksgemm::TK - 1) / ksgemm::TK * ksgemm::TK;
        d_pf_bt_kl_ = static_cast<int8_t *>(alloc((size_t)nc_pf * 8 * kp_pf_kl_));
        dim3 gkl((kp_pf_kl_ + 63) / 64, (nc_pf + 63) / 64);
        ksgemm::prep_key_kl<<<gkl, kThreads, 0, stream_>>>(d_pfpksk_, d_pf_bt_kl_, p_.K() + 1, p_.pfks_l, kp_pf_kl_,
                                                           nc_pf, glwe, glwe, pf_blk, pf_slots_);
        d_pf_corr_ = static_cast<uint64_t *>(alloc((size_t)nc_pf * 8));
        ksgemm::key_offset_corr<<<(nc_pf + 255) / 256, 256, 0, stream_>>>(d_pfpksk_, d_pf_corr_, p_.K() + 1, p_.pfks_l,
                                                                          nc_pf, glwe, glwe, pf_blk, pf_slots_);
    }
    ksgemm::prep_key<<<gks, kThreads, 0, stream_>>>(d_ksk_, d_ks_bt_, kd_ks, kp_ks_, nc_ks, nc_ks, nc_ks, 0);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(stream_));
}

// digit scratch for B ciphertexts x rows_per_ct rows of Kp bytes (padding columns zeroed)
static void ensure_digits(int8_t *&buf, size_t &cap, size_t rows, int Kd, int Kp, hipStream_t s, bool il = false) {
    const size_t need = rows * (size_t)Kp;
    if (need > cap) {
        if (buf) hip_check(hipFree(buf), "hipFree");
        hip_check(hipMalloc(&buf, need), "hipMalloc digits");
        cap = need;
    }
    if (Kp > Kd) {
        const size_t total = rows * (size_t)(Kp - Kd);
        ksgemm::zero_pad<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(buf, (long)rows, Kd, Kp, il);
        hip_check(hipGetLastError(), "zero_pad");
    }
}

Engine::Engine(const Params &p, int device, const uint64_t *d_ksk, const uint64_t *d_bsk,
               const uint64_t *d_pfpksk)
    : p_(p), device_(device) {
    init_common();
    owns_keys_ = false;
    order_after_caller();  // the key buffers may still be in flight on the caller's stream (RCCL broadcast)
    d_ksk_ = const_cast<uint64_t *>(d_ksk);
    d_pfpksk_ = const_cast<uint64_t *>(d_pfpksk);
    bsk_to_fourier(d_bsk);
    prepare_mfma_keys();
}

Engine::~Engine() {
    hipSetDevice(device_);
    hipStreamSynchronize(stream_);
    if (owns_keys_) {
        hipFree(d_ksk_);
        hipFree(d_pfpksk_);
    }
    for (void *q : {(void *)d_bsk_f_, (void *)d_twist_, (void *)d_untwist_, (void *)d_w_, (void *)d_lut_shift_,
                    (void *)d_lut24_, (void *)d_lut8_, (void *)d_small_, (void *)d_big_, (void *)d_ggsw_,
                    (void *)d_ggsw_f_, (void *)d_state_, (void *)d_muls_, (void *)d_pf_bt_, (void *)d_ks_bt_, (void *)d_pf_corr_, (void *)d_pf_bt_kl_,
                    (void *)d_digits_, (void *)d_wlut_sbox_, (void *)d_wlut_id_, (void *)d_lut_x_, (void *)d_xbuf_,
                    (void *)d_xsh_, (void *)d_xks_, (void *)d_xpbs_, (void *)d_ints_, (void *)d_s1_sbox_tv_,
                    (void *)d_s1_id_tv_, (void *)d_s1_in_, (void *)d_s1_out_, (void *)d_s1_pks_, (void *)d_s1_tv_, (void *)d_pf_flags_, (void *)d_clk_, (void *)d_lf_, (void *)d_acc_w_})
        if (q) hipFree(q);
    for (auto &e : ev_pool_) hipEventDestroy(e);
    if (caller_ev_) hipEventDestroy(caller_ev_);
    hipStreamDestroy(stream_);
}

void Engine::synchronize() { HIPC(hipStreamSynchronize(stream_)); }

void Engine::order_after_caller() {
    HIPC(hipSetDevice(device_));
    if (!caller_stream_) {
        HIPC(hipDeviceSynchronize());
        return;
    }
    if (!caller_ev_) HIPC(hipEventCreateWithFlags(&caller_ev_, hipEventDisableTiming));
    HIPC(hipEventRecord(caller_ev_, caller_stream_));
    HIPC(hipStreamWaitEvent(stream_, caller_ev_, 0));
}

void Engine::reserve(size_t bits, size_t outputs) {
    grow(d_small_, cap_small_, bits * p_.small_len());
    grow(d_big_, cap_big_, bits * p_.big_len());
    grow(d_ggsw_, cap_ggsw_, bits * p_.cbs_ggsw_len());
    grow(d_ggsw_f_, cap_ggsw_f_, bits * p_.cbs_ggsw_fourier_len());
    (void)outputs;
}

void Engine::keyswitch(const uint64_t *d_in, uint64_t *d_out, size_t B) {
    if (!B) return;
    if (mfma_ks_) {
        const int K = p_.K(), kd = K * p_.ks_l;
        ensure_digits(d_digits_, cap_digits_, B, kd, kp_ks_, stream_);
        const size_t thr = B * (size_t)K;
        ksgemm::prep_digits<1, 8><<<(unsigned)((thr + 255) / 256), 256, 0, stream_>>>(
            d_in, K + 1, d_digits_, (long)B, K, kp_ks_, p_.ks_b, p_.ks_l);
        const long mtiles = (long)((B + ksgemm::TM - 1) / ksgemm::TM);
        const long ntiles = ((long)(p_.n + 1) * 8 + ksgemm::TN - 1) / ksgemm::TN;
        ksgemm::gemm<1, 8><<<(unsigned)(mtiles * ntiles), 256, 0, stream_>>>(
            d_digits_, d_ks_bt_, kp_ks_, (long)B, mtiles, p_.n + 1, d_out, p_.n + 1, (long)B, d_in + K, K + 1, p_.n);
        HIPC(hipGetLastError());
        return;
    }
    dim3 grid((unsigned)((p_.n + 1 + kThreads - 1) / kThreads), (unsigned)((B + KS_CT - 1) / KS_CT));
    keyswitch_kernel<<<grid, kThreads, 0, stream_>>>(d_in, d_out, d_ksk_, B, p_.K(), p_.n, p_.ks_l, p_.ks_b);
    HIPC(hipGetLastError());
}

void Engine::bootstrap(const uint64_t *d_small, const uint64_t *d_lut_glwe, uint64_t *d_big, size_t B,
                       uint64_t body_add, uint64_t out_add, size_t lut_mod) {
    if (!B) return;
    if (lut_mod == 0) throw std::runtime_error("bootstrap: lut_mod must be >= 1");
    if (lut_mod > 1 && (x4_512_ || br1024_pbs_ || br1024lat_))
        throw std::runtime_error("per-ciphertext test vectors run on br512x4<7, true, 6> or the generic blind rotation");
    if (x4_s1_) {
        // shortint_1bit (7 levels of 2^6, per-ciphertext test vectors): three ciphertexts per workgroup at any
        // batch size (br512lat runs the three levels of params_sqrd_lvl_64 in parallel and has no 7-level form)
        const unsigned wgs = (unsigned)((B + 2) / 3);
        br512x4::br_kernel<7, true, 6><<<wgs, br512x4::THREADS, br512x4::lds_bytes(), stream_>>>(
            d_small, p_.n, d_lut_glwe, 0, d_bsk_f_, 0, d_big, (long)B, body_add, out_add, d_twist_, d_w_, d_lf_, nullptr,
            (long)lut_mod);
        HIPC(hipGetLastError());
        return;
    }
    if (x4_512_) {
        if ((long)B <= lat_max_) {
            br512lat::br_kernel<3, 12><<<(unsigned)B, br512lat::THREADS, br512lat::lds_bytes(3), stream_>>>(
                d_small, p_.n, d_lut_glwe, d_bsk_f_, d_big, (long)B, body_add, out_add, d_lf_);
            HIPC(hipGetLastError());
            return;
        }
        // whole rounds of C ciphertexts per CU on the throughput kernel (br512p16: C = 2, br512x4: C = 3); a
        // remainder that would leave most CUs idle in a last round goes to br512lat (one ciphertext per CU)
        long bx = (long)B;
        const long cpw = p16_ ? br512p16::C : br512x4::C;
        const long per_round = cpw * num_cu_, rest = (long)B % per_round;
        if ((long)B > per_round && rest > 0 && rest <= std::min<long>(lat_max_, num_cu_)) bx -= rest;
        const unsigned wgs = (unsigned)((bx + cpw - 1) / cpw);
        uint64_t *clk = clock_buffer(wgs);
        timed(ST_PBS_MAIN, [&] {
            if (p16_)
                br512p16::br_kernel<3, 12><<<wgs, br512p16::THREADS, br512p16::lds_bytes(), stream_>>>(
                    d_small, p_.n, d_lut_glwe, d_bsk_f_, d_big, bx, body_add, out_add, d_lf_, clk);
            else
                br512x4::br_kernel<3, true, 12><<<wgs, br512x4::THREADS, br512x4::lds_bytes(), stream_>>>(
                    d_small, p_.n, d_lut_glwe, 0, d_bsk_f_, 0, d_big, bx, body_add, out_add, d_twist_, d_w_, d_lf_, clk);
            HIPC(hipGetLastError());
        });
        record_clock(clk, wgs);
        if (timing_) times_.pbs_main_cts += (double)bx;
        if (bx < (long)B) {
            br512lat::br_kernel<3, 12><<<(unsigned)(B - bx), br512lat::THREADS, br512lat::lds_bytes(3), stream_>>>(
                d_small + (size_t)bx * (p_.n + 1), p_.n, d_lut_glwe, d_bsk_f_, d_big + (size_t)bx * p_.big_len(),
                (long)B - bx, body_add, out_add, d_lf_);
            HIPC(hipGetLastError());
        }
        return;
    }
    if (br1024lat_ && (long)B <= (long)num_cu_) {
        br1024lat_<<<(unsigned)B, br1024lat::THREADS, br1024lat_lds_, stream_>>>(
            d_small, p_.n, d_lut_glwe, d_bsk_f_, d_big, (long)B, body_add, out_add, d_w_, d_lf_);
        HIPC(hipGetLastError());
        return;
    }
    if (br1024_occ2_ && (long)B > (long)num_cu_) {
        uint64_t *clk = clock_buffer(B);
        br1024_occ2_<<<(unsigned)B, br1024::THREADS, br1024::lds_bytes(1, 1, true), stream_>>>(
            d_small, p_.n, d_lut_glwe, 0, d_bsk_f_, 0, d_big, (long)B, body_add, out_add, d_twist_, d_untwist_, d_w_,
            d_lf_, clk);
        HIPC(hipGetLastError());
        record_clock(clk, B);
        return;
    }
    if (b1kw_ && lut_mod == 1 && (long)B >= (long)br1024w::C * num_cu_) {
        // four ciphertexts per workgroup (every CU busy from 4 x CUs ciphertexts on)
        const size_t wgs = (B + br1024w::C - 1) / br1024w::C;
        grow(d_acc_w_, cap_acc_w_, B * (size_t)(p_.k + 1) * p_.N);
        uint64_t *clk = clock_buffer(wgs);
        br1024w::br_kernel<6, 7><<<(unsigned)wgs, br1024w::THREADS, br1024w::lds_bytes(), stream_>>>(
            d_small, p_.n, d_lut_glwe, d_bsk_f_, d_big, (long)B, body_add, out_add, d_w_, d_lf_, d_acc_w_, clk);
        HIPC(hipGetLastError());
        record_clock(clk, wgs);
        return;
    }
    if (br1024_pbs_) {
        // two ciphertexts per workgroup share its GGSW loads, but below one per CU they leave CUs idle
        const int C = (long)B <= (long)num_cu_ ? 1 : 2;
        const size_t wgs = (B + C - 1) / C;
        uint64_t *clk = C == 2 ? clock_buffer(wgs) : nullptr;  // the throughput instantiation only
        (C == 1 ? br1024_pbs1_ : br1024_pbs_)<<<(unsigned)wgs, br1024::THREADS,
                                                 br1024::lds_bytes(C, C == 1 ? br1024_pbs1_lp_ : 1, lf1k_), stream_>>>(
            d_small, p_.n, d_lut_glwe, 0, d_bsk_f_, 0, d_big, (long)B, body_add, out_add, d_twist_, d_untwist_, d_w_,
            d_lf_, clk);
        HIPC(hipGetLastError());
        record_clock(clk, wgs);
        return;
    }
    for (size_t off = 0; off < B; off += 65535) {
        const unsigned g = (unsigned)std::min<size_t>(65535, B - off);
        if (p_.N == 512) {
            pbs_kernel<512><<<g, kThreads, br_lds_bytes<512>(p_.k, p_.pbs_l), stream_>>>(
                d_small + off * p_.small_len(), d_big + off * p_.big_len(), d_lut_glwe, d_bsk_f_, d_twist_, d_untwist_,
                d_w_, p_.n, p_.k, p_.pbs_l, p_.pbs_b, body_add, out_add, lut_mod, off);
        } else {
            pbs_kernel<1024><<<g, kThreads, br_lds_bytes<1024>(p_.k, p_.pbs_l), stream_>>>(
                d_small + off * p_.small_len(), d_big + off * p_.big_len(), d_lut_glwe, d_bsk_f_, d_twist_, d_untwist_,
                d_w_, p_.n, p_.k, p_.pbs_l, p_.pbs_b, body_add, out_add, lut_mod, off);
        }
        HIPC(hipGetLastError());
    }
}

void Engine::pbs_shift_boolean(const uint64_t *d_small, uint64_t *d_big, size_t B, int level) {
    const uint64_t alpha = 1ull << (63 - p_.cbs_b * level);
    bootstrap(d_small, d_lut_shift_ + (size_t)(level - 1) * p_.glwe_len(), d_big, B, 1ull << 62, alpha);
}

void Engine::pfks_into_ggsw(const uint64_t *d_big, uint64_t *d_ggsw, size_t B, int level) {
    if (!B) return;
    const int glwe = (int)p_.glwe_len();
    if (mfma_ks_ && pf_kl_ && (long)B >= pf_kl_min_) {
        // K layout: rows = ciphertexts, K = (K+1) x S limb slots (ksgemm.hpp KSlots)
        const int K = p_.K(), kd = (K + 1) * pf_slots_.S;
        constexpr long TMR = 96 * kG6WM;  // ciphertexts per tile (384)
        const long mt = (long)((B + TMR - 1) / TMR);
        ensure_digits(d_digits_, cap_digits_, (size_t)mt * TMR, kd, kp_pf_kl_, stream_, true);
        const size_t thr = B * (size_t)(K + 1);
        bool clamp = false;
        for (int l = 0; l < p_.pfks_l; l++) clamp = clamp || pf_slots_.clamp[l];
        const int fw = (int)(((size_t)(K + 1) * p_.pfks_l + 31) / 32);  // flag words per ciphertext
        if (clamp) {
            const size_t need = B * (size_t)fw;
            grow(d_pf_flags_, cap_pf_flags_, need);
            HIPC(hipMemsetAsync(d_pf_flags_, 0, need * 4, stream_));
        }
        ksgemm::prep_digits_kl<<<(unsigned)((thr + 255) / 256), 256, 0, stream_>>>(
            d_big, K + 1, d_digits_, (long)B, K + 1, kp_pf_kl_, p_.pfks_b, p_.pfks_l, pf_slots_, d_pf_flags_, fw);
        const int ncols = (p_.k + 1) * glwe;
        const long out_stride = (long)p_.cbs_l * ncols;
        const long ntiles = ((long)ncols * 8 + ksgemm::BTN - 1) / ksgemm::BTN;
        uint64_t *dst = d_ggsw + (size_t)(level - 1) * ncols;
        ksgemm::gemm_g6<6, kG6WM, true><<<(unsigned)(mt * ntiles), 256 * kG6WM, ksgemm::gemm_g6_lds<kG6WM>(), stream_>>>(
            d_digits_, d_pf_bt_kl_, kp_pf_kl_, mt, ncols, dst, out_stride, (long)B, d_pf_corr_);
        if (clamp) {
            const long pf_blk = (long)(K + 1) * p_.pfks_l * glwe;
            ksgemm::pfks_clamp_fixup<<<(unsigned)((B + 3) / 4), 256, 0, stream_>>>(
                d_pf_flags_, fw, (long)B, p_.pfks_l, p_.pfks_b, d_pfpksk_, ncols, glwe, glwe, pf_blk, dst, out_stride);
        }
        HIPC(hipGetLastError());
        return;
    }
    if (mfma_ks_) {
        // digits as 3 balanced 6-bit limbs, limb index in the MFMA row tile (ksgemm.hpp gemm_g6)
        const int K = p_.K(), kd = (K + 1) * p_.pfks_l;
        const long mt4 = (long)((B + 127) / 128);  // 384-row tiles (128 ciphertexts x 3 limbs)
        ensure_digits(d_digits_, cap_digits_, (size_t)mt4 * 384, kd, kp_pf_, stream_, true);
        const size_t thr = B * (size_t)(K + 1);
        ksgemm::prep_digits3<6><<<(unsigned)((thr + 255) / 256), 256, 0, stream_>>>(
            d_big, K + 1, d_digits_, (long)B, K + 1, kp_pf_, p_.pfks_b, p_.pfks_l, true);
        const int ncols = (p_.k + 1) * glwe;
        const long out_stride = (long)p_.cbs_l * ncols;
        const long ntiles = ((long)ncols * 8 + ksgemm::BTN - 1) / ksgemm::BTN;
        uint64_t *dst = d_ggsw + (size_t)(level - 1) * ncols;
        ksgemm::gemm_g6<6, 4><<<(unsigned)(mt4 * ntiles), 1024, ksgemm::gemm_g6_lds<4>(), stream_>>>(
            d_digits_, d_pf_bt_, kp_pf_, mt4, ncols, dst, out_stride, (long)B);
        HIPC(hipGetLastError());
        return;
    }
    dim3 grid((unsigned)((glwe + kThreads - 1) / kThreads), (unsigned)(p_.k + 1), (unsigned)((B + PF_CT - 1) / PF_CT));
    pfks_kernel<<<grid, kThreads, 0, stream_>>>(d_big, d_ggsw, d_pfpksk_, B, p_.K(), glwe, p_.pfks_l, p_.pfks_b,
                                                p_.cbs_l, level, p_.k);
    HIPC(hipGetLastError());
}

void Engine::ggsw_to_fourier(const uint64_t *d_ggsw, cplx *d_ggsw_f, size_t B) {
    if (!B) return;
    const size_t polys = B * p_.cbs_l * (p_.k + 1) * (p_.k + 1);
    if (p_.N == 512) {
        constexpr int JPB = kThreads / 16;
        fft_torus_kernel<512><<<(unsigned)((polys + JPB - 1) / JPB), kThreads, JPB * fft_poly_stride<256>() * sizeof(cplx), stream_>>>(
            d_ggsw, d_ggsw_f, polys, d_twist_, d_w_);
    } else {
        constexpr int JPB = kThreads / 64;
        fft_torus_kernel<1024><<<(unsigned)((polys + JPB - 1) / JPB), kThreads, JPB * fft_poly_stride<512>() * sizeof(cplx), stream_>>>(
            d_ggsw, d_ggsw_f, polys, d_twist_, d_w_);
    }
    HIPC(hipGetLastError());
}

// LUTs with 2^tree polynomials: the CMux tree over GGSWs tree-1 .. 0 (tfhe-rs order: the first
// `tree` GGSWs select the polynomial), then the blind rotation over GGSWs n_in-1 .. tree on the
// generic kernels (oracle: or_vertical_packing).
void Engine::vertical_packing_tree(const cplx *d_ggsw_f, size_t G, int n_in, int tree, const uint64_t *d_lut,
                                   int n_out, uint64_t *d_out) {
    const size_t glwe = p_.glwe_len(), cnt0 = (size_t)1 << tree, small_len = (size_t)p_.N << tree;
    uint64_t *leaves = nullptr, *lv[2] = {nullptr, nullptr};
    HIPC(hipMallocAsync((void **)&leaves, (size_t)n_out * cnt0 * glwe * 8, stream_));
    HIPC(hipMallocAsync((void **)&lv[0], G * n_out * (cnt0 / 2) * glwe * 8, stream_));
    if (cnt0 >= 4) HIPC(hipMallocAsync((void **)&lv[1], G * n_out * (cnt0 / 4) * glwe * 8, stream_));
    vp_leaves_kernel<<<1024, 256, 0, stream_>>>(d_lut, small_len, n_out, (int)cnt0, p_.k, p_.N, leaves);
    HIPC(hipGetLastError());
    const uint64_t *src = leaves;
    long gstride = 0;
    int cnt = (int)cnt0, buf = 0;
    for (int t = tree - 1; t >= 0; t--, cnt /= 2, buf ^= 1) {
        const unsigned wgs = (unsigned)(G * n_out * (size_t)(cnt / 2));
        if (p_.N == 512)
            cmux_tree_kernel<512><<<wgs, kThreads, br_lds_bytes<512>(p_.k, p_.cbs_l), stream_>>>(
                d_ggsw_f, n_in, t, src, gstride, cnt, n_out, lv[buf], d_twist_, d_untwist_, d_w_, p_.k, p_.cbs_l,
                p_.cbs_b);
        else
            cmux_tree_kernel<1024><<<wgs, kThreads, br_lds_bytes<1024>(p_.k, p_.cbs_l), stream_>>>(
                d_ggsw_f, n_in, t, src, gstride, cnt, n_out, lv[buf], d_twist_, d_untwist_, d_w_, p_.k, p_.cbs_l,
                p_.cbs_b);
        HIPC(hipGetLastError());
        src = lv[buf];
        gstride = (long)(n_out * (size_t)(cnt / 2) * glwe);
    }
    const unsigned wgs = (unsigned)(G * (size_t)n_out);
    if (p_.N == 512)
        vp_kernel<512><<<wgs, kThreads, br_lds_bytes<512>(p_.k, p_.cbs_l), stream_>>>(
            d_ggsw_f, n_in, d_lut, n_out, d_out, d_twist_, d_untwist_, d_w_, p_.k, p_.cbs_l, p_.cbs_b, src, tree);
    else
        vp_kernel<1024><<<wgs, kThreads, br_lds_bytes<1024>(p_.k, p_.cbs_l), stream_>>>(
            d_ggsw_f, n_in, d_lut, n_out, d_out, d_twist_, d_untwist_, d_w_, p_.k, p_.cbs_l, p_.cbs_b, src, tree);
    HIPC(hipGetLastError());
    HIPC(hipFreeAsync(leaves, stream_));
    HIPC(hipFreeAsync(lv[0], stream_));
    if (lv[1]) HIPC(hipFreeAsync(lv[1], stream_));
}

void Engine::vertical_packing(const cplx *d_ggsw_f, size_t G, int n_in, const uint64_t *d_lut, int n_out,
                              uint64_t *d_out) {
    if (!G) return;
    int logN = 0;
    while ((1 << logN) < p_.N) logN++;
    if (n_in > logN) {
        vertical_packing_tree(d_ggsw_f, G, n_in, n_in - logN, d_lut, n_out, d_out);
        return;
    }
    if (x4_vp_) {
        const size_t wgs = G * (size_t)((n_out + kBrC - 1) / kBrC);
        br512x4::br_kernel<1, false, 13><<<(unsigned)wgs, br512x4::THREADS, br512x4::lds_bytes(), stream_>>>(
            nullptr, 0, d_lut, n_out, d_ggsw_f, n_in, d_out, (long)G, 0, 0, d_twist_, d_w_, nullptr, nullptr);
        HIPC(hipGetLastError());
        return;
    }
    if (br1024_vp_) {
        const size_t wgs = G * (size_t)((n_out + 1) / 2);
        br1024_vp_<<<(unsigned)wgs, br1024::THREADS, br1024::lds_bytes(2), stream_>>>(
            nullptr, 0, d_lut, n_out, d_ggsw_f, n_in, d_out, (long)G, 0, 0, d_twist_, d_untwist_, d_w_, nullptr,
            nullptr);
        HIPC(hipGetLastError());
        return;
    }
    const size_t total = G * (size_t)n_out;
    for (size_t off = 0; off < total; off += 65535 - (65535 % n_out)) {
        const size_t chunk = std::min<size_t>(65535 - (65535 % n_out), total - off);
        const size_t g0 = off / n_out;
        if (p_.N == 512)
            vp_kernel<512><<<(unsigned)chunk, kThreads, br_lds_bytes<512>(p_.k, p_.cbs_l), stream_>>>(
                d_ggsw_f + g0 * n_in * p_.cbs_ggsw_fourier_len(), n_in, d_lut, n_out, d_out + g0 * n_out * p_.big_len(),
                d_twist_, d_untwist_, d_w_, p_.k, p_.cbs_l, p_.cbs_b);
        else
            vp_kernel<1024><<<(unsigned)chunk, kThreads, br_lds_bytes<1024>(p_.k, p_.cbs_l), stream_>>>(
                d_ggsw_f + g0 * n_in * p_.cbs_ggsw_fourier_len(), n_in, d_lut, n_out, d_out + g0 * n_out * p_.big_len(),
                d_twist_, d_untwist_, d_w_, p_.k, p_.cbs_l, p_.cbs_b);
        HIPC(hipGetLastError());
    }
}

hipEvent_t Engine::next_event() {
    if (ev_used_ == ev_pool_.size()) {
        hipEvent_t e;
        HIPC(hipEventCreate(&e));
        ev_pool_.push_back(e);
    }
    return ev_pool_[ev_used_++];
}

template <class F>
void Engine::timed(int stage, F fn) {
    if (!timing_) {
        fn();
        return;
    }
    Span sp{next_event(), next_event(), stage};
    HIPC(hipEventRecord(sp.a, stream_));
    fn();
    HIPC(hipEventRecord(sp.b, stream_));
    spans_.push_back(sp);
}

uint64_t *Engine::clock_buffer(size_t wgs) {
    if (!clock_) return nullptr;
    grow(d_clk_, cap_clk_, 2 * wgs);
    HIPC(hipMemsetAsync(d_clk_, 0, 2 * wgs * 8, stream_));
    return d_clk_;
}

void Engine::record_clock(const uint64_t *clk, size_t wgs) {
    if (!clk) return;
    std::vector<uint64_t> h(2 * wgs);
    HIPC(hipMemcpyAsync(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost, stream_));
    HIPC(hipStreamSynchronize(stream_));
    std::vector<double> ghz;
    ghz.reserve(wgs);
    for (size_t w = 0; w < wgs; w++)
        if (h[2 * w + 1] > 0) ghz.push_back((double)h[2 * w] / (double)h[2 * w + 1] * 0.1);  // 100 MHz reference
    if (ghz.empty()) return;
    std::nth_element(ghz.begin(), ghz.begin() + ghz.size() / 2, ghz.end());
    times_.pbs_clock_ghz_sum += ghz[ghz.size() / 2];
    times_.pbs_clock_launches += 1;
}

void Engine::collect_times() {
    if (spans_.empty()) return;
    HIPC(hipEventSynchronize(spans_.back().b));
    for (const Span &sp : spans_) {
        float ms = 0;
        HIPC(hipEventElapsedTime(&ms, sp.a, sp.b));
        float *dst[] = {&times_.keyswitch, &times_.pbs, &times_.pfks, &times_.ggsw_fft, &times_.vertical_packing,
                        &times_.extract, &times_.linear, &times_.pbs_main};
        *dst[sp.stage] += ms;
    }
    spans_.clear();
    ev_used_ = 0;
}

void Engine::circuit_bootstrap(const uint64_t *d_bits, size_t G, int n_in, const uint64_t *d_lut, int n_out,
                               uint64_t *d_out) {
    const size_t bits = G * n_in;
    reserve(bits, G * n_out);
    timed(ST_KS, [&] { keyswitch(d_bits, d_small_, bits); });
    cbs_vp_stages(d_small_, G, n_in, d_lut, n_out, d_out);
}

void Engine::cbs_vp(const uint64_t *d_small_bits, size_t G, int n_in, const uint64_t *d_lut, int n_out,
                    uint64_t *d_out) {
    reserve(G * n_in, G * n_out);
    cbs_vp_stages(d_small_bits, G, n_in, d_lut, n_out, d_out);
}

// circuit_bootstrap_boolean per bit and level (homomorphic_shift_boolean PBS + k+1 PFKS into the
// GGSW rows of that level), GGSW to the Fourier domain, vertical packing
void Engine::cbs_vp_stages(const uint64_t *d_small_bits, size_t G, int n_in, const uint64_t *d_lut, int n_out,
                           uint64_t *d_out) {
    const size_t bits = G * n_in;
    for (int lev = 1; lev <= p_.cbs_l; lev++) {
        timed(ST_PBS, [&] { pbs_shift_boolean(d_small_bits, d_big_, bits, lev); });
        if (timing_) times_.pbs_launches++;
        timed(ST_PFKS, [&] { pfks_into_ggsw(d_big_, d_ggsw_, bits, lev); });
    }
    timed(ST_FFT, [&] { ggsw_to_fourier(d_ggsw_, d_ggsw_f_, bits); });
    timed(ST_VP, [&] { vertical_packing(d_ggsw_f_, G, n_in, d_lut, n_out, d_out); });
    collect_times();
}

void Engine::extract_bits(const uint64_t *d_in, size_t B, int delta_log, int nbits, uint64_t *d_out) {
    if (!B) return;
    if (nbits < 1 || delta_log < 1 || delta_log + nbits > 64) throw std::runtime_error("extract_bits: bad bit range");
    const size_t L = p_.big_len(), S = p_.small_len(), glwe = p_.glwe_len();
    if (lut_x_delta_ != delta_log || lut_x_bits_ < nbits) {
        // accumulators: trivial GLWE with body -alpha, alpha = 2^(delta_log - 1 + bit_idx)
        std::vector<uint64_t> luts((size_t)nbits * glwe, 0);
        for (int b = 0; b < nbits; b++) {
            const uint64_t alpha = 1ull << (delta_log - 1 + b);
            for (int j = 0; j < p_.N; j++) luts[(size_t)b * glwe + (size_t)p_.k * p_.N + j] = 0 - alpha;
        }
        if (d_lut_x_) HIPC(hipFree(d_lut_x_));
        d_lut_x_ = static_cast<uint64_t *>(alloc(luts.size() * 8));
        HIPC(hipMemcpy(d_lut_x_, luts.data(), luts.size() * 8, hipMemcpyHostToDevice));
        lut_x_delta_ = delta_log;
        lut_x_bits_ = nbits;
    }
    grow(d_xbuf_, cap_xbuf_, B * L);
    grow(d_xsh_, cap_xsh_, B * L);
    grow(d_xks_, cap_xks_, B * S);
    grow(d_xpbs_, cap_xpbs_, B * L);
    HIPC(hipMemcpyAsync(d_xbuf_, d_in, B * L * 8, hipMemcpyDeviceToDevice, stream_));
    for (int bit_idx = 0; bit_idx < nbits; bit_idx++) {
        // shift the extracted bit to the MSB, keyswitch: that is the output bit (LSB first, stored
        // from the end so that the list is MSB first)
        lwe_shl_kernel<<<grid_for(B * L), kThreads, 0, stream_>>>(d_xbuf_, d_xsh_, B * L, 64 - delta_log - bit_idx - 1);
        HIPC(hipGetLastError());
        keyswitch(d_xsh_, d_xks_, B);
        copy_rows_kernel<<<grid_for(B * S), kThreads, 0, stream_>>>(d_xks_, d_out + (size_t)(nbits - 1 - bit_idx) * S, B,
                                                                  (int)S, (size_t)nbits * S);
        HIPC(hipGetLastError());
        if (bit_idx == nbits - 1) break;
        // PBS of (ks + q/4) with accumulator -alpha, + alpha: an encryption of the bit at alpha * 2;
        // subtract it from the input to clear that bit
        const uint64_t alpha = 1ull << (delta_log - 1 + bit_idx);
        bootstrap(d_xks_, d_lut_x_ + (size_t)bit_idx * glwe, d_xpbs_, B, 1ull << 62, alpha);
        lwe_sub_kernel<<<grid_for(B * L), kThreads, 0, stream_>>>(d_xbuf_, d_xpbs_, B * L);
        HIPC(hipGetLastError());
    }
}

void Engine::bootstrap_bytes8(const uint64_t *d_bytes, size_t G, const uint64_t *d_lut, uint64_t *d_out) {
    if (!G) return;
    grow(d_ints_, cap_ints_, G * p_.big_len());
    cbs_vp(d_bytes, G, 8, d_lut, 1, d_ints_);
    timed(ST_EXTRACT, [&] { extract_bits(d_ints_, G, 56, 8, d_out); });
    collect_times();
}

void Engine::aes8_encrypt_blocks(const uint64_t *d_rk, const uint64_t *d_blocks, size_t nb, int rounds,
                                 uint64_t *d_out) {
    if (!nb) return;
    if (p_.model != 8) throw std::runtime_error("aes8_encrypt_blocks needs the 8-bit model parameters");
    if (rounds < 1 || rounds > 10) throw std::runtime_error("rounds must be in 1..=10");
    const int L = (int)p_.small_len();
    const size_t state_len = nb * 128 * (size_t)L;
    times_ = StageTimes{};
    grow(d_state_, cap_state_, state_len);
    grow(d_muls_, cap_muls_, state_len);
    const size_t byte_stride = 8 * (size_t)L;
    MixTerms T;
    std::memcpy(T.idx, mix_idx_, sizeof(T.idx));
    aes_ark0_kernel<<<grid_for(state_len), kThreads, 0, stream_>>>(d_blocks, d_rk, d_state_, nb, L);
    HIPC(hipGetLastError());
    for (int r = 1; r < rounds; r++) {
        bootstrap_bytes8(d_state_, nb * 16, d_wlut_sbox_, d_muls_);
        aes8_mix_kernel<<<grid_for(state_len), kThreads, 0, stream_>>>(d_muls_, d_rk + (size_t)16 * r * byte_stride,
                                                                        d_state_, nb, L, T);
        HIPC(hipGetLastError());
    }
    bootstrap_bytes8(d_state_, nb * 16, d_wlut_sbox_, d_muls_);
    aes_final_kernel<<<grid_for(state_len), kThreads, 0, stream_>>>(d_muls_, d_rk + (size_t)160 * byte_stride, d_out,
                                                                     nb, L);
    HIPC(hipGetLastError());
}

void Engine::aes_encrypt_blocks(const uint64_t *d_rk, const uint64_t *d_blocks, size_t nb, int rounds,
                                uint64_t *d_out) {
    if (!nb) return;
    if (rounds < 1 || rounds > 10) throw std::runtime_error("rounds must be in 1..=10");
    const int L = (int)p_.big_len();
    const size_t state_len = nb * 128 * (size_t)L;
    times_ = StageTimes{};
    grow(d_state_, cap_state_, state_len);
    grow(d_muls_, cap_muls_, nb * 16 * 24 * (size_t)L);
    const size_t byte_stride = 8 * (size_t)L;
    aes_ark0_kernel<<<grid_for(state_len), kThreads, 0, stream_>>>(d_blocks, d_rk, d_state_, nb, L);
    HIPC(hipGetLastError());
    for (int r = 1; r < rounds; r++) {
        circuit_bootstrap(d_state_, nb * 16, 8, d_lut24_, 24, d_muls_);
        aes_mix_kernel<<<grid_for(state_len), kThreads, 0, stream_>>>(d_muls_, d_rk + (size_t)16 * r * byte_stride,
                                                                       d_state_, nb, L);
        HIPC(hipGetLastError());
    }
    circuit_bootstrap(d_state_, nb * 16, 8, d_lut8_, 8, d_muls_);
    aes_final_kernel<<<grid_for(state_len), kThreads, 0, stream_>>>(d_muls_, d_rk + (size_t)160 * byte_stride, d_out,
                                                                     nb, L);
    HIPC(hipGetLastError());
}

// ---- shortint_1bit model ----
void Engine::require_s1() const {
    if (p_.model != 2) throw std::runtime_error("this stage belongs to the shortint_1bit parameter set");
}

void Engine::s1_bootstrap(const uint64_t *d_in, const uint64_t *d_tvs, size_t lut_mod, uint64_t *d_out, size_t B) {
    require_s1();
    if (!B) return;
    grow(d_big_, cap_big_, B * p_.big_len());
    timed(ST_PBS, [&] { bootstrap(d_in, d_tvs, d_big_, B, 0, 0, lut_mod); });
    timed(ST_KS, [&] { keyswitch(d_big_, d_out, B); });
}

void Engine::s1_pks(const uint64_t *d_in, size_t B, uint64_t *d_out) {
    require_s1();
    if (!B) return;
    const int L = p_.n + 1, kd = p_.n * p_.pfks_l, nc = (p_.k + 1) * p_.N;
    ensure_digits(d_digits_, cap_digits_, B, kd, kp_pf_, stream_);
    const size_t thr = B * (size_t)p_.n;
    ksgemm::prep_digits<1, 8><<<(unsigned)((thr + 255) / 256), 256, 0, stream_>>>(d_in, L, d_digits_, (long)B, p_.n,
                                                                                  kp_pf_, p_.pfks_b, p_.pfks_l);
    const long mtiles = (long)((B + ksgemm::TM - 1) / ksgemm::TM);
    const long ntiles = ((long)nc * 8 + ksgemm::TN - 1) / ksgemm::TN;
    ksgemm::gemm<1, 8><<<(unsigned)(mtiles * ntiles), 256, 0, stream_>>>(d_digits_, d_pf_bt_, kp_pf_, (long)B, mtiles, nc,
                                                                          d_out, nc, (long)B, d_in + p_.n, L, p_.k * p_.N);
    HIPC(hipGetLastError());
}

void Engine::s1_tv_from_pks(const uint64_t *d_pks, size_t P, uint64_t *d_tv) {
    require_s1();
    if (!P) return;
    s1_tv_kernel<512><<<(unsigned)(P * (p_.k + 1)), kThreads, 0, stream_>>>(d_pks, d_tv, p_.k);
    HIPC(hipGetLastError());
}

void Engine::s1_pack(const uint64_t *d_in, int count, uint64_t *d_out) {
    require_s1();
    if (count < 1 || count > p_.N) throw std::runtime_error("packing keyswitch: 1..N ciphertexts");
    grow(d_s1_pks_, cap_s1_pks_, (size_t)count * p_.glwe_len());
    s1_pks(d_in, (size_t)count, d_s1_pks_);
    s1_pack_kernel<512><<<(unsigned)(p_.k + 1), kThreads, 0, stream_>>>(d_s1_pks_, count, d_out, p_.k);
    HIPC(hipGetLastError());
}

void Engine::s1_multivariate(const uint64_t *d_bits, size_t G, int nbits, const uint64_t *d_tvs, int n_fn,
                             uint64_t *d_out) {
    require_s1();
    if (!G) return;
    if (nbits < 1 || nbits > 8) throw std::runtime_error("multivariate functions take 1..8 bits");
    // groups are independent: run them in chunks of about `rows` level-0 bootstraps, so the scratch (~60 KB
    // per row: inputs, outputs, big LWEs, packing keyswitches, test vectors) is bounded whatever the batch.
    // Each selector level halves the batch; at 128 rows per CU the last level of an 8-bit tree still has a
    // bootstrap per CU (the AES S-box: 8 x 128 rows per group, 32 groups per chunk on 256 CUs, 2 GB).
    // TAE_S1_ROWS overrides the row budget (tests, A/B).
    // The value must be a positive integer; anything else throws.  The budget is clamped so that the chunk's
    // scratch fits in half of the free device memory.
    size_t rows = std::max<size_t>(kS1Rows, 128 * (size_t)num_cu_);
    if (const char *rows_env = getenv("TAE_S1_ROWS")) {
        char *end = nullptr;
        errno = 0;
        const long long v = strtoll(rows_env, &end, 10);
        if (errno != 0 || end == rows_env || *end != '\0' || v <= 0)
            throw std::runtime_error(std::string("TAE_S1_ROWS must be a positive integer, got '") + rows_env + "'");
        rows = (size_t)v;
    }
    {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0) {
            // per level-0 row: gathered input and output shortints, a packing-keyswitch GLWE, half a test vector,
            // and the bootstrap's big-LWE output
            const size_t per_row = sizeof(uint64_t) * (2 * p_.small_len() + p_.glwe_len() + p_.glwe_len() / 2 +
                                                       (size_t)p_.k * p_.N + 1);
            const size_t cap = std::max<size_t>(1, free_b / 2 / per_row);
            rows = std::min(rows, cap);
        }
    }
    const size_t rows_per_group = (size_t)n_fn << (nbits - 1);
    const size_t gc = std::max<size_t>(1, rows / rows_per_group);
    const size_t L = p_.small_len();
    for (size_t g0 = 0; g0 < G; g0 += gc)
        s1_multivariate_chunk(d_bits + g0 * nbits * L, std::min(gc, G - g0), nbits, d_tvs, n_fn,
                              d_out + g0 * n_fn * L);
}

void Engine::s1_multivariate_chunk(const uint64_t *d_bits, size_t G, int nbits, const uint64_t *d_tvs, int n_fn,
                                   uint64_t *d_out) {
    const int L = p_.n + 1;
    const size_t glwe = p_.glwe_len();
    size_t V = (size_t)1 << (nbits - 1), B = G * n_fn * V;
    grow(d_s1_in_, cap_s1_in_, B * L);
    grow(d_s1_out_, cap_s1_out_, B * L);
    grow(d_s1_pks_, cap_s1_pks_, B * glwe);
    grow(d_s1_tv_, cap_s1_tv_, std::max<size_t>(B / 2, 1) * glwe);
    const uint64_t *tvs = d_tvs;
    size_t lut_mod = (size_t)n_fn * V;  // level 0: the cleartext test vectors, shared by every group
    for (int sel = nbits - 1;; sel--) {
        // apply_selectors_rec (shortint_1bit.rs:549-576): bootstrap every test vector of (group, fn) with
        // the group's selector bit sel, then pack the results pairwise into the next level's vectors
        s1_gather_kernel<<<grid_for(B * L), kThreads, 0, stream_>>>(d_bits, d_s1_in_, B, (size_t)n_fn * V, nbits, sel, L);
        HIPC(hipGetLastError());
        s1_bootstrap(d_s1_in_, tvs, lut_mod, V == 1 ? d_out : d_s1_out_, B);
        if (V == 1) break;
        timed(ST_PFKS, [&] {
            s1_pks(d_s1_out_, B, d_s1_pks_);
            s1_tv_from_pks(d_s1_pks_, B / 2, d_s1_tv_);
        });
        V /= 2;
        B /= 2;
        tvs = d_s1_tv_;
        lut_mod = B;
    }
}

// fhe_sbox_pbs::encrypt_block_for_rounds (fhe_sbox_pbs.rs:75-121) over nb blocks of shortint_1bit bits with
// ByteT::sbox_substitute = 8 multivariate functions per byte (fhe_impls/shortint_1bit.rs:32-50); MixColumns
// and AddRoundKey are the same LWE-addition network as the 8-bit model's (shortint unchecked_add,
// shortint_1bit.rs:109-120)
void Engine::s1_aes_encrypt_blocks(const uint64_t *d_rk, const uint64_t *d_blocks, size_t nb, int rounds,
                                   uint64_t *d_out) {
    require_s1();
    if (!nb) return;
    if (rounds < 1 || rounds > 10) throw std::runtime_error("rounds must be in 1..=10");
    const int L = (int)p_.small_len();
    const size_t state_len = nb * 128 * (size_t)L;
    times_ = StageTimes{};
    grow(d_state_, cap_state_, state_len);
    grow(d_muls_, cap_muls_, state_len);
    const size_t byte_stride = 8 * (size_t)L;
    MixTerms T;
    std::memcpy(T.idx, mix_idx_, sizeof(T.idx));
    aes_ark0_kernel<<<grid_for(state_len), kThreads, 0, stream_>>>(d_blocks, d_rk, d_state_, nb, L);
    HIPC(hipGetLastError());
    for (int r = 1; r < rounds; r++) {
        s1_multivariate(d_state_, nb * 16, 8, d_s1_sbox_tv_, 8, d_muls_);
        aes8_mix_kernel<<<grid_for(state_len), kThreads, 0, stream_>>>(d_muls_, d_rk + (size_t)16 * r * byte_stride,
                                                                        d_state_, nb, L, T);
        HIPC(hipGetLastError());
    }
    s1_multivariate(d_state_, nb * 16, 8, d_s1_sbox_tv_, 8, d_muls_);
    aes_final_kernel<<<grid_for(state_len), kThreads, 0, stream_>>>(d_muls_, d_rk + (size_t)160 * byte_stride, d_out,
                                                                     nb, L);
    HIPC(hipGetLastError());
    collect_times();
}

void Engine::lwe_add(uint64_t *d_a, const uint64_t *d_b, size_t count) {
    lwe_add_kernel<<<grid_for(count), kThreads, 0, stream_>>>(d_a, d_b, count);
    HIPC(hipGetLastError());
}

}  // namespace tae
