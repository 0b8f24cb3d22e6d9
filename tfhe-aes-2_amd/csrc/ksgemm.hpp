// Integer keyswitch as an int8 MFMA GEMM (exact mod 2^64).
//
// Both keyswitches of the hot path are   out[b][col] = body - sum_{kd} d[b][kd] * KEY[kd][col]
//   PFKS  (private_functional_keyswitch_lwe_ciphertext_into_glwe_ciphertext, all k+1 keys at once):
//         kd = (i, l) over the K+1 big-LWE coefficients x pfks_l levels, col = (q, t) over the
//         (k+1) x (k+1)N GGSW row coefficients, d = signed 2^16-base digits (17-bit range)
//   KS    (keyswitch_lwe_ciphertext): kd = (i, l) over K x ks_l, col over n+1, |d| <= 4
// With u64 keys and small signed digits this is a GEMM of (B x Kd) by (Kd x C) modulo 2^64.  It
// runs on the i8 matrix cores:
//   KEY = sum_j k_j 256^j      with balanced signed bytes k_j (8 limbs, wraps mod 2^64)
//   d   = sum_m d_m 2^(LB m)   with balanced signed LB-bit limbs (MA limbs; MA = 1 for KS)
//   d * KEY = sum_{m,j} 2^(LB m + 8 j) (d_m k_j)  (mod 2^64)
// The GEMM rows are (b, m) and the columns (col, j); every i32 partial sum is exact
// (|d_m k_j| <= 2^(LB-1) * 128, summed over <= 2^13 terms), and the epilogue recombines the
// MA x 8 partial sums of each (b, col): shift, sum over m in-lane, sum over j across 8 lanes.
// Integer results are therefore bit-identical to the u64 loop of the CPU oracle.
//
// Tiling: 256 threads = 4 waves (2 x 2), workgroup tile 128 rows x 128 cols, K tile 128 bytes,
// v_mfma_i32_32x32x32_i8 (lane l: A[l & 31][16 (l >> 5) + t], B[16 (l >> 5) + t][l & 31];
// verified by scripts/probes/mfma_i8_layout.hip).  LDS rows padded to 144 B (conflict-free
// ds_read_b128), double-buffered; grouped tile order (see gemm) bounds the HBM re-reads.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kslots.hpp"

namespace tae {
namespace ksgemm {

constexpr int TM = 128, TN = 128, TK = 128, LROW = TK + 16;
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// balanced signed byte limbs of a u64 (k = sum_j limb_j 256^j mod 2^64)
__device__ __forceinline__ void key_limbs(uint64_t k, int8_t *lb) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const int8_t s = (int8_t)(uint8_t)(k & 0xFF);
        lb[j] = s;
        k = (k - (uint64_t)(int64_t)s) >> 8;
    }
}

// Operand layouts in HBM.  Row-major: element (row, k) at row * Kp + k.  Row-pair interleaved
// (the LDS-DMA GEMMs gemm_g4 / gemm_g5): rows 2i and 2i + 1 share each 128-byte line, 64 K bytes of
// each, so one 64-byte K step of a row pair is one whole cache line (one L2 request instead of two
// half-line requests issued a K step apart).  Needs Kp % 64 == 0 and an even row count.
__host__ __device__ __forceinline__ long op_off(long row, long k, int Kp, bool il) {
    return il ? (row >> 1) * 2 * Kp + (k >> 6) * 128 + (row & 1) * 64 + (k & 63) : row * Kp + k;
}

// ---- key preparation: u64 key rows -> Bt[(col * 8 + j) * Kp + kd] (int8) ----
// key element for (kd, col) at key[kd * key_kd_stride + (col / cols_per_block) * key_blk_stride +
// col % cols_per_block]; used for both PFPKSK ([q][i][l][glwe]) and KSK ([i][l][n+1]).
__global__ void __launch_bounds__(256) prep_key(const uint64_t *__restrict__ key, int8_t *__restrict__ Bt, int Kd, int Kp,
                                                int ncols, int cols_per_block, long key_kd_stride,
                                                long key_blk_stride, bool il = false) {
    __shared__ int8_t tile[64][8][65];
    const int kd0 = blockIdx.x * 64, col0 = blockIdx.y * 64;
    // load 64 kd x 64 cols (col fastest, coalesced), split into limbs
    for (int t = threadIdx.x; t < 64 * 64; t += 256) {
        const int kk = t >> 6, cc = t & 63;
        const int kd = kd0 + kk, col = col0 + cc;
        int8_t lb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (kd < Kd && col < ncols) {
            const uint64_t v = key[(long)kd * key_kd_stride + (long)(col / cols_per_block) * key_blk_stride +
                                   col % cols_per_block];
            key_limbs(v, lb);
        }
#pragma unroll
        for (int j = 0; j < 8; j++) tile[cc][j][kk] = lb[j];
    }
    __syncthreads();
    // write rows (col, j) with 64 contiguous kd bytes
    for (int t = threadIdx.x; t < 64 * 8 * 64; t += 256) {
        const int kk = t & 63, row = t >> 6;  // row = cc * 8 + j
        const int cc = row >> 3, j = row & 7;
        const int col = col0 + cc, kd = kd0 + kk;
        if (col < ncols && kd < Kp) Bt[op_off((long)col * 8 + j, kd, Kp, il)] = tile[cc][j][kk];
    }
}

// ---- digits: big LWE [B][K+1] -> A[(b * MA + m) * Kp + i * L + (lev - 1)] ----
template <int MA, int LB>
__global__ void __launch_bounds__(256) prep_digits(const uint64_t *__restrict__ in, long in_stride, int8_t *__restrict__ A,
                                                   long B, int n_in, int Kp, int base_log, int levels) {
    const long t = (long)blockIdx.x * 256 + threadIdx.x;
    const long b = t / n_in;
    const int i = (int)(t - b * n_in);
    if (b >= B) return;
    const uint64_t x = in[b * in_stride + i];
    // tfhe-rs SignedDecomposer: closest representable, balanced digits (finest first)
    const int nrb = 64 - base_log * levels;
    uint64_t s = x >> (nrb - 1);
    s += s & 1;
    s >>= 1;
    const uint64_t mask = (1ull << base_log) - 1;
    for (int lev = levels; lev >= 1; lev--) {
        const uint64_t res = s & mask;
        s >>= base_log;
        uint64_t carry = ((res - 1) | s) & res;
        carry >>= (base_log - 1);
        s += carry;
        int32_t d = (int32_t)(res - (carry << base_log));
        const long kd = (long)i * levels + (lev - 1);
#pragma unroll
        for (int m = 0; m < MA; m++) {
            int32_t limb;
            if (m == MA - 1) {
                limb = d;
            } else {
                limb = ((d + (1 << (LB - 1))) & ((1 << LB) - 1)) - (1 << (LB - 1));
                d = (d - limb) >> LB;
            }
            A[(b * MA + m) * Kp + kd] = (int8_t)limb;
        }
    }
}

// zero the padding columns kd in [Kd, Kp) of every row (done once per buffer size change)
__global__ void zero_pad(int8_t *A, long rows, int Kd, int Kp, bool il = false) {
    const long t = (long)blockIdx.x * 256 + threadIdx.x;
    const int w = Kp - Kd;
    const long r = t / w;
    if (r < rows) A[op_off(r, Kd + (t - r * w), Kp, il)] = 0;
}

// ---- the GEMM ----
template <int MA, int LB>
__global__ void __launch_bounds__(256, 2)
    gemm(const int8_t *__restrict__ A, const int8_t *__restrict__ Bt, int Kp, long Mrows, long mtiles, int ncols,
         uint64_t *__restrict__ out, long out_stride, long B, const uint64_t *__restrict__ body_in, long body_stride,
         int body_col) {
    __shared__ __align__(16) int8_t sA[2][TM * LROW];
    __shared__ __align__(16) int8_t sB[2][TN * LROW];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave >> 1, wn = wave & 1;
    // grouped tile order: GN n-tiles per group, n fastest inside it.  The ~512 co-resident WGs
    // cover 16 m-tiles x GN n-tiles, and with round-robin XCD dispatch each XCD keeps GN/8 key
    // tiles in its L2 while the digits are re-read once per group instead of once per n-tile.
    constexpr long GN = 32;
    const long ntiles = (((long)ncols * 8) + TN - 1) / TN;
    const long gsz = GN * mtiles;
    const long ng = blockIdx.x / gsz, rr = blockIdx.x - ng * gsz;
    const long gw = min(GN, ntiles - ng * GN);
    const long mt = rr / gw, nt = ng * GN + (rr - (rr / gw) * gw);
    const long row0 = mt * TM;
    const long col8_0 = nt * TN;  // first (col, j) column of the tile
    const long N8 = (long)ncols * 8;

    // loader mapping: chunk c = tid + 256 t (t < 4): row = c >> 3, 16-byte column kc = c & 7
    v4i ra[4], rb[4];
    auto gload = [&](int k0) {
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const int c = tid + 256 * t, r = c >> 3, kc = c & 7;
            const long ar = row0 + r, br = col8_0 + r;
            ra[t] = ar < Mrows ? *reinterpret_cast<const v4i *>(A + ar * Kp + k0 + kc * 16) : v4i{0, 0, 0, 0};
            rb[t] = br < N8 ? *reinterpret_cast<const v4i *>(Bt + br * Kp + k0 + kc * 16) : v4i{0, 0, 0, 0};
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const int c = tid + 256 * t, r = c >> 3, kc = c & 7;
            *reinterpret_cast<v4i *>(&sA[buf][r * LROW + kc * 16]) = ra[t];
            *reinterpret_cast<v4i *>(&sB[buf][r * LROW + kc * 16]) = rb[t];
        }
    };

    v16i acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = v16i{0};

    const int r = lane & 31, h = lane >> 5;
    gload(0);
    lstore(0);
    __syncthreads();
    const int nk = Kp / TK;
    for (int ks = 0; ks < nk; ks++) {
        const int cur = ks & 1;
        if (ks + 1 < nk) gload((ks + 1) * TK);
#pragma unroll
        for (int kk = 0; kk < TK / 32; kk++) {
            v4i fa[2], fb[2];
#pragma unroll
            for (int ti = 0; ti < 2; ti++)
                fa[ti] = *reinterpret_cast<const v4i *>(&sA[cur][(wm * 64 + ti * 32 + r) * LROW + kk * 32 + h * 16]);
#pragma unroll
            for (int tj = 0; tj < 2; tj++)
                fb[tj] = *reinterpret_cast<const v4i *>(&sB[cur][(wn * 64 + tj * 32 + r) * LROW + kk * 32 + h * 16]);
#pragma unroll
            for (int ti = 0; ti < 2; ti++)
#pragma unroll
                for (int tj = 0; tj < 2; tj++)
                    acc[ti][tj] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[ti], fb[tj], acc[ti][tj], 0, 0, 0);
        }
        if (ks + 1 < nk) {
            lstore(cur ^ 1);
            __syncthreads();
        }
    }

    // ---- epilogue: recombine limbs, reduce over the 8 key limbs, store ----
    const int j = r & 7;  // key limb of this lane's column
#pragma unroll
    for (int ti = 0; ti < 2; ti++)
#pragma unroll
        for (int tj = 0; tj < 2; tj++) {
            const long col = (col8_0 + wn * 64 + tj * 32 + r) >> 3;
            // rows of reg q: (q & 3) + 8 (q >> 2) + 4 h  within the 32-row tile
#pragma unroll
            for (int g = 0; g < 16 / MA; g++) {
                uint64_t v = 0;
#pragma unroll
                for (int m = 0; m < MA; m++) {
                    const int q = g * MA + m;
                    const int sh = LB * m + 8 * j;
                    const uint64_t p = (uint64_t)(int64_t)acc[ti][tj][q];
                    v += sh < 64 ? (p << sh) : 0;
                }
                // sum over the 8 lanes (j = 0..7) that hold the same column
#pragma unroll
                for (int x = 1; x < 8; x <<= 1) {
                    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
                    const uint32_t olo = __shfl_xor((int)lo, x, 64), ohi = __shfl_xor((int)hi, x, 64);
                    v += ((uint64_t)ohi << 32) | olo;
                }
                const int q0 = g * MA;
                const int row = (q0 & 3) + 8 * (q0 >> 2) + 4 * h;
                const long grow = row0 + wm * 64 + ti * 32 + row;  // (b, m=0) row
                const long b = grow / MA;
                if (j == 0 && col < ncols && b < B) {
                    uint64_t o = 0 - v;
                    if (col == body_col) o += body_in[b * body_stride];
                    out[b * out_stride + col] = o;
                }
            }
        }
}

constexpr int BTN = 256;  // key columns (col, limb) per PFKS workgroup tile

// ---- PFKS with 3 balanced 6-bit digit limbs (|d| <= 2^16 fits [-133152, 128991]; every i32 partial
// sum stays exact: 32 * 128 * 4224 < 2^31), 25% fewer MFMAs than 4 x 5 bits.  The limb index sits in
// the MFMA row-tile: A row (b, m) = (b / 32) * 96 + 32 m + b % 32, so the 32 x 32 tiles ti = m of a
// wave hold the three limbs of the same 32 ciphertexts in the same lanes and the epilogue combines
// them in-lane. ----
template <int LB3>
__global__ void __launch_bounds__(256) prep_digits3(const uint64_t *__restrict__ in, long in_stride,
                                                    int8_t *__restrict__ A, long B, int n_in, int Kp, int base_log,
                                                    int levels, bool il = false) {
    const long t = (long)blockIdx.x * 256 + threadIdx.x;
    const long b = t / n_in;
    const int i = (int)(t - b * n_in);
    if (b >= B) return;
    const uint64_t x = in[b * in_stride + i];
    const int nrb = 64 - base_log * levels;
    uint64_t s = x >> (nrb - 1);
    s += s & 1;
    s >>= 1;
    const uint64_t mask = (1ull << base_log) - 1;
    const long rbase = (b >> 5) * 96 + (b & 31);
    for (int lev = levels; lev >= 1; lev--) {
        const uint64_t res = s & mask;
        s >>= base_log;
        uint64_t carry = ((res - 1) | s) & res;
        carry >>= (base_log - 1);
        s += carry;
        int32_t d = (int32_t)(res - (carry << base_log));
        const long kd = (long)i * levels + (lev - 1);
#pragma unroll
        for (int m = 0; m < 3; m++) {
            int32_t limb;
            if (m == 2) {
                limb = d;
            } else {
                limb = ((d + (1 << (LB3 - 1))) & ((1 << LB3) - 1)) - (1 << (LB3 - 1));
                d = (d - limb) >> LB3;
            }
            A[op_off(rbase + 32 * m, kd, Kp, il)] = (int8_t)limb;
        }
    }
}

// ---- PFKS in the K layout: the digit limbs go into the K dimension instead of the row tile ----
// Slot s of big-LWE coefficient i (K index i * S + s) holds limb limb(s) of the level-lev(s) digit,
// and the key rows are pre-shifted to match:
//   A[b][i S + s]       = limb_{limb(s)}(d_{lev(s)}[b][i] - c_{lev(s)})      (balanced signed bytes)
//   B[(col, j)][i S + s] = byte j of (KEY[i][lev(s)][col] << 8 limb(s))
// so sum_s A B recombines as sum_j 256^j P[b][(col, j)] = sum_{i,l} (d_l - c_l) KEY[i][l][col]
// (mod 2^64), and the offsets come back through corr[col] = sum_{i,l} c_l KEY[i][l][col].  Each level
// gets the fewest 8-bit limbs that hold its digit range after an offset: params_sqrd_lvl_64 (base
// 2^16, 2 levels) has the top digit in [-32767, 32768] (2 limbs with c = 129: [-32896, 32639] + 129)
// and the lower one in [-32768, 32768] (3 limbs) -- 5 slots per coefficient against 2 x 3 rows of the
// 6-bit row-tile layout, 17% fewer MFMAs; base 2^12 (8-bit model, lvl_256) needs 2 limbs per level
// instead of 3.  i32 sums stay exact: 128 * 128 * S (K+1) < 2^31 for every set here.
// digits in the K layout, row-pair interleaved rows b (op_off): one thread per (b, i)
// clamp_flags (levels with ks.clamp): bit (i levels + l) of row b's flag words marks a digit +2^(B-1)
// stored as -2^(B-1); the words of the rows must be zero on entry.
__global__ void __launch_bounds__(256) prep_digits_kl(const uint64_t *__restrict__ in, long in_stride,
                                                      int8_t *__restrict__ A, long B, int n_in, int Kp, int base_log,
                                                      int levels, KSlots ks, uint32_t *__restrict__ clamp_flags = nullptr,
                                                      int flag_words = 0) {
    const long t = (long)blockIdx.x * 256 + threadIdx.x;
    const long b = t / n_in;
    const int i = (int)(t - b * n_in);
    if (b >= B) return;
    const int64_t half = 1ll << (base_log - 1);
    kl_for_each_digit(in[b * in_stride + i], base_log, levels, [&](int lev, int64_t digit) {
        if (ks.clamp[lev - 1] && digit == half) {
            digit = -half;
            const int bit = i * levels + lev - 1;
            atomicOr(clamp_flags + b * flag_words + (bit >> 5), 1u << (bit & 31));
        }
        int64_t d = digit - ks.off[lev - 1];
        const int n = ks.nlimb[lev - 1];
        const long k0 = (long)i * ks.S + ks.first[lev - 1];
        for (int m = 0; m < n; m++) A[op_off(b, k0 + m, Kp, true)] = (int8_t)kl_next_limb(d, m == n - 1);
    });
}

// key rows in the K layout (prep_key with the slot shift): element (kd = i * L + l, col) of the u64
// key at key[kd * key_kd_stride + (col / cols_per_block) * key_blk_stride + col % cols_per_block]
__global__ void __launch_bounds__(256) prep_key_kl(const uint64_t *__restrict__ key, int8_t *__restrict__ Bt, int n_coef,
                                                   int levels, int Kp, int ncols, int cols_per_block, long key_kd_stride,
                                                   long key_blk_stride, KSlots ks) {
    __shared__ int8_t tile[64][8][65];
    const int k0 = blockIdx.x * 64, col0 = blockIdx.y * 64;
    for (int t = threadIdx.x; t < 64 * 64; t += 256) {
        const int kk = t >> 6, cc = t & 63;
        const int k = k0 + kk, col = col0 + cc;
        int8_t lb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const int i = k / ks.S, sl = k - i * ks.S;
        if (i < n_coef && col < ncols) {
            const long kd = (long)i * levels + ks.lev[sl];
            const uint64_t v = key[kd * key_kd_stride + (long)(col / cols_per_block) * key_blk_stride + col % cols_per_block];
            key_limbs(v << (8 * ks.limb[sl]), lb);
        }
#pragma unroll
        for (int j = 0; j < 8; j++) tile[cc][j][kk] = lb[j];
    }
    __syncthreads();
    for (int t = threadIdx.x; t < 64 * 8 * 64; t += 256) {
        const int kk = t & 63, row = t >> 6;
        const int cc = row >> 3, j = row & 7;
        const int col = col0 + cc, k = k0 + kk;
        if (col < ncols && k < Kp) Bt[op_off((long)col * 8 + j, k, Kp, true)] = tile[cc][j][kk];
    }
}

// corr[col] = sum_{i, l} c_l KEY[i][l][col] (mod 2^64)
__global__ void __launch_bounds__(256) key_offset_corr(const uint64_t *__restrict__ key, uint64_t *__restrict__ corr,
                                                       int n_coef, int levels, int ncols, int cols_per_block,
                                                       long key_kd_stride, long key_blk_stride, KSlots ks) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    if (col >= ncols) return;
    const uint64_t *kc = key + (long)(col / cols_per_block) * key_blk_stride + col % cols_per_block;
    uint64_t acc = 0;
    for (int l = 0; l < levels; l++) {
        if (!ks.off[l]) continue;
        uint64_t sum = 0;
        for (int i = 0; i < n_coef; i++) sum += kc[((long)i * levels + l) * key_kd_stride];
        acc += (uint64_t)ks.off[l] * sum;
    }
    corr[col] = acc;
}

// Correction of the clamped digits (kslots_build): out[b][col] -= KEY[i][l][col] << base_log for every
// flag set in row b.  One wave per row; rows without flags (all but ~1-2% at 16-bit digits) cost the
// read of their flag words.  Every (row, col) belongs to one wave: no atomics.
__global__ void __launch_bounds__(256) pfks_clamp_fixup(const uint32_t *__restrict__ clamp_flags, int flag_words,
                                                        long B, int levels, int base_log, const uint64_t *__restrict__ key,
                                                        int ncols, int cols_per_block, long key_kd_stride,
                                                        long key_blk_stride, uint64_t *__restrict__ out, long out_stride) {
    const long b = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (b >= B) return;
    const uint32_t *fl = clamp_flags + b * flag_words;
    for (int w0 = 0; w0 < flag_words; w0 += 64) {
        const uint32_t mine = w0 + lane < flag_words ? fl[w0 + lane] : 0u;
        uint64_t any = __builtin_amdgcn_ballot_w64(mine != 0);
        while (any) {
            const int src = (int)__builtin_ctzll(any);
            any &= any - 1;
            uint32_t word = (uint32_t)__builtin_amdgcn_readlane((int)mine, src);
            while (word) {
                const int bit = (w0 + src) * 32 + (int)__builtin_ctz(word);
                word &= word - 1;
                const long kd = bit;  // = i * levels + l, the key row of (i, l)
                for (int col = lane; col < ncols; col += 64) {
                    const uint64_t kv =
                        key[kd * key_kd_stride + (long)(col / cols_per_block) * key_blk_stride + col % cols_per_block];
                    out[b * out_stride + col] -= kv << base_log;
                }
            }
        }
    }
}

// ---- gemm_g6: the PFKS GEMM (3-limb digits, LDS-DMA staging) ----
// - Staging: global_load_lds (16 B per lane, no VGPR staging, no ds_write) into a ring of G4S stages
//   of 64-byte K steps; two steps stay in flight across the per-step barrier by a counted vmcnt
//   (cdna_hip_programming.md section 5: "Async global->LDS copy", "Pipelining across barriers").
// - The LDS image is lane-linear (rows of 64 B, no padding), so the bank-conflict swizzle (16-byte
//   chunk c of row r stored at c ^ ((r >> 2) & 3)) goes on the per-lane global source address and
//   on the fragment reads.
// - Operands row-pair interleaved in HBM (op_off): one K step of two rows is one 128-byte line.
// - WM x 4 waves of 96 x 64 (3 limbs x 32 ciphertexts by 64 key columns), workgroup tile
//   96 WM x 256.  WM = 4 (1024 threads, 384 x 256, 160 KiB ring) moves 30% fewer operand bytes per
//   MFMA than WM = 2 (192 x 256) and runs four MFMA streams per SIMD: 22.5 -> 20.1 ms per
//   16384-ciphertext launch (WM = 3: 21.0).  The 6 WM + 16 pieces of 16 rows per stage are dealt
//   round-robin over the waves.
// - Epilogue: the three limb partial sums of a (ciphertext, key limb j) combine in-lane with shifts,
//   the 8 key limbs across 8 lanes: bit-identical to the u64 loop.
#ifndef TAE_G4S
constexpr int G4K = 64, G4S = 4;                      // K bytes per step, ring stages
#else
constexpr int G4K = 64, G4S = TAE_G4S;
#endif
__device__ __forceinline__ int g4_swz(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }

// global_load_lds_dwordx4: 16 bytes per lane from src to lds_base + 16 * lane (lds_base wave-uniform).
// The target builtin exists only in the device pass of the single-source compile.
__device__ __forceinline__ void g4_glds(const int8_t *src, int8_t *lds_base) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_global_load_lds(src, lds_base, 16, 0, 0);
#else
    (void)src;
    (void)lds_base;
#endif
}

template <int WM>
inline size_t gemm_g6_lds() { return (size_t)G4S * (96 * WM + BTN) * G4K; }

// KL: K-layout operands (prep_digits_kl / prep_key_kl): tile rows are ciphertexts, the epilogue only
// recombines the 8 key limbs and adds corr[col].
template <int LB3, int WM, bool KL = false>
__global__ void __launch_bounds__(256 * WM, 1)
    gemm_g6(const int8_t *__restrict__ A, const int8_t *__restrict__ Bt, int Kp, long mtiles, int ncols,
            uint64_t *__restrict__ out, long out_stride, long B, const uint64_t *__restrict__ corr = nullptr) {
    constexpr int TMR = 96 * WM, NW = 4 * WM;              // tile rows, waves
    constexpr int SA = TMR * G4K, SAB = (TMR + BTN) * G4K;  // stage bytes
    constexpr int NPA = TMR / 16, NP = NPA + BTN / 16;      // 16-row pieces per stage
    extern __shared__ __align__(16) int8_t smem_g[];
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int wm = wave >> 2, wn = wave & 3;
    const long ntiles = (((long)ncols * 8) + BTN - 1) / BTN;
#ifndef TAE_G6_GN
    constexpr long GN = 8;
#else
    constexpr long GN = TAE_G6_GN;
#endif
#ifndef TAE_G6_NOXCD
    // XCD-aware order (cdna_hip_programming.md T1, bijective form): blocks b, b + 8, b + 16, ... run
    // on one XCD, so give them a contiguous range of the grouped tile order; its ~32 co-resident
    // tiles are then 4 M tiles x GN (= 8) N tiles sharing their operand K slices in that XCD's L2
    const long nwg = (long)gridDim.x, q8 = nwg >> 3, r8 = nwg & 7, x8 = blockIdx.x & 7;
    const long bid = x8 * q8 + min(x8, r8) + (blockIdx.x >> 3);
#else
    const long bid = blockIdx.x;
#endif
    const long gsz = GN * mtiles;
    const long ng = bid / gsz, rr = bid - ng * gsz;
    const long gw = min(GN, ntiles - ng * GN);
    const long mt = rr / gw, nt = ng * GN + (rr - (rr / gw) * gw);
    const long row0 = mt * TMR;
    const long col8_0 = nt * BTN;
    const long N8 = (long)ncols * 8;

    const int lrow = lane >> 2, lch = lane & 3;
    const int nk = Kp / G4K;
    auto stage = [&](int st, int ks) {
        const int k0 = ks * G4K;
        int8_t *base = smem_g + st * SAB;
#pragma unroll
        for (int p = wave; p < NP; p += NW) {  // piece p: rows 16 p .. 16 p + 15 of the stage image
            const int row = 16 * p + lrow;
            const int8_t *src;
            if (p < NPA) {
                src = A + op_off(row0 + row, k0, Kp, true) + 16 * g4_swz(row, lch);
            } else {
                const int rb = row - TMR;
                const long br = min(col8_0 + rb, N8 - 1);  // rows past the last column feed unstored outputs
                src = Bt + op_off(br, k0, Kp, true) + 16 * g4_swz(rb, lch);
            }
            g4_glds(src, base + 16 * p * G4K);
        }
    };
#ifdef TAE_G6_PF
    // L2 prefetch TAE_G6_PF steps beyond the ring (A/B knob): before each step's stage DMA, wave 0 loads one
    // dword of 56 operand lines of step ks + G4S - 1 + TAE_G6_PF (this tile's share of the lines its XCD's
    // co-resident tiles stream: A lines (nt mod 8) x 24 .. + 23 of its 192, B lines (mt mod 4) x 32 .. + 31 of its
    // 128) into the first 256 bytes of the stage that its own DMA then overwrites (vector-memory returns are
    // in issue order), so the ring's loads of that step find their lines in L2.
    const bool pf_wave = wave == 0;
    auto prefetch = [&](int st, int ks) {
        if (!pf_wave) return;
        const int kp = min(ks, nk - 1) * G4K;
        const int8_t *src;
        if (lane < 24 || lane >= 56) {
            const int a = (int)(nt & 7) * 24 + (lane < 24 ? lane : lane - 56);
            src = A + op_off(row0 + 2 * a, kp, Kp, true);
        } else {
            const int b = (int)(mt & 3) * 32 + lane - 24;
            src = Bt + op_off(min(col8_0 + 2 * b, N8 - 2), kp, Kp, true);
        }
#if defined(__HIP_DEVICE_COMPILE__)
        __builtin_amdgcn_global_load_lds(src, smem_g + st * SAB, 4, 0, 0);
#else
        (void)src;
        (void)st;
#endif
    };
    const int per_wave = (NP / NW) + (wave < NP % NW ? 1 : 0) + (pf_wave ? 1 : 0);
#else
    const int per_wave = (NP / NW) + (wave < NP % NW ? 1 : 0);
#endif
    auto wait_steps = [&](int keep) {  // retire all but this wave's loads of `keep` later steps
        switch (per_wave * keep) {
        case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
        case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        }
    };

    v16i acc[3][2];
#pragma unroll
    for (int a = 0; a < 3; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = v16i{0};

    const int r = lane & 31, h = lane >> 5;
    for (int ks = 0; ks < G4S - 1 && ks < nk; ks++) {
#ifdef TAE_G6_PF
        prefetch(ks, ks + G4S - 1 + TAE_G6_PF);
#endif
        stage(ks, ks);
    }
    for (int ks = 0; ks < nk; ks++) {
        wait_steps(min(G4S - 2, nk - 1 - ks));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#ifndef TAE_G6_NOBAR  // timing-only bound (racy): no per-step barrier
        __builtin_amdgcn_s_barrier();
#endif
        __builtin_amdgcn_sched_barrier(0);
#ifndef TAE_G6_NODMA  // timing-only bound (stale tiles): no operand stream after the prologue
        if (ks + G4S - 1 < nk) {
#ifdef TAE_G6_PF
            prefetch((ks + G4S - 1) % G4S, ks + 2 * (G4S - 1) + TAE_G6_PF);
#endif
            stage((ks + G4S - 1) % G4S, ks + G4S - 1);
        }
#endif
        const int8_t *a_s = smem_g + (ks % G4S) * SAB, *b_s = a_s + SA;
        v4i fa[2][3], fb[2][2];
#pragma unroll
        for (int kk = 0; kk < G4K / 32; kk++) {
#pragma unroll
            for (int m = 0; m < 3; m++) {
                const int row = wm * 96 + m * 32 + r;
                fa[kk][m] = *reinterpret_cast<const v4i *>(a_s + row * G4K + 16 * g4_swz(row, 2 * kk + h));
            }
#pragma unroll
            for (int tj = 0; tj < 2; tj++) {
                const int row = wn * 64 + tj * 32 + r;
                fb[kk][tj] = *reinterpret_cast<const v4i *>(b_s + row * G4K + 16 * g4_swz(row, 2 * kk + h));
            }
        }
#pragma unroll
        for (int kk = 0; kk < G4K / 32; kk++)
#pragma unroll
            for (int m = 0; m < 3; m++)
#pragma unroll
                for (int tj = 0; tj < 2; tj++)
                    acc[m][tj] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[kk][m], fb[kk][tj], acc[m][tj], 0, 0, 0);
    }

    const int j = r & 7;
    if constexpr (KL) {
        // The 8 key-limb sums of an output sit in 8 lanes; instead of shuffling, each m-tile goes
        // through this wave's part of the (now idle) staging ring: E[row][tj 32 + r] (rows padded to 68
        // dwords: the 16 lanes of a ds_read_b128 group read 16 rows on distinct banks), then every lane
        // reads whole outputs' limbs (2 x b128) and stores them -- no spills, all lanes storing.
        static_assert(16 * 32 * 68 * 4 * WM / 4 <= G4S * (96 * WM + BTN) * G4K, "epilogue fits the ring");
        __syncthreads();  // every wave is done with the ring
        int *E = reinterpret_cast<int *>(smem_g) + wave * 32 * 68;
        const long b0 = row0 + wm * 96;
        const long colb = (col8_0 + wn * 64) >> 3;  // first key column of this wave
#pragma unroll
        for (int m = 0; m < 3; m++) {
#pragma unroll
            for (int tj = 0; tj < 2; tj++)
#pragma unroll
                for (int q = 0; q < 16; q++) E[((q & 3) + 8 * (q >> 2) + 4 * h) * 68 + tj * 32 + r] = acc[m][tj][q];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-local hand-off
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int row = lane & 31, g = (lane >> 5) + 2 * k;  // g: 8-column group = key column
                const v4i lo = *reinterpret_cast<const v4i *>(E + row * 68 + 8 * g);
                const v4i hi = *reinterpret_cast<const v4i *>(E + row * 68 + 8 * g + 4);
                uint64_t v = 0;
#pragma unroll
                for (int jj = 0; jj < 4; jj++) {
                    v += (uint64_t)(int64_t)lo[jj] << (8 * jj);
                    v += (uint64_t)(int64_t)hi[jj] << (8 * (jj + 4));
                }
                const long b = b0 + 32 * m + row, col = colb + g;
                if (col < ncols && b < B) out[b * out_stride + col] = 0 - (v + corr[col]);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next m overwrites
        }
        return;
    }
    const long b0 = (mt * WM + wm) * 32;
#pragma unroll
    for (int tj = 0; tj < 2; tj++) {
        const long col = (col8_0 + wn * 64 + tj * 32 + r) >> 3;
#pragma unroll
        for (int q = 0; q < 16; q++) {
            uint64_t v = 0;
#pragma unroll
            for (int m = 0; m < 3; m++) {
                const int sh = LB3 * m + 8 * j;
                const uint64_t p = (uint64_t)(int64_t)acc[m][tj][q];
                v += sh < 64 ? (p << sh) : 0;
            }
#pragma unroll
            for (int x = 1; x < 8; x <<= 1) {
                const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
                const uint32_t olo = __shfl_xor((int)lo, x, 64), ohi = __shfl_xor((int)hi, x, 64);
                v += ((uint64_t)ohi << 32) | olo;
            }
            const long b = b0 + (q & 3) + 8 * (q >> 2) + 4 * h;
            if (j == 0 && col < ncols && b < B) out[b * out_stride + col] = 0 - v;
        }
    }
}

}  // namespace ksgemm
}  // namespace tae
