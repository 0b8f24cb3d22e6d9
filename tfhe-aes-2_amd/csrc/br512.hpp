// Shared pieces of the batched N = 512, k = 4 blind rotations (params_sqrd_lvl_64): br512x4.hpp
// (large batches, three ciphertexts per 1024-thread workgroup) and br512lat.hpp (small batches,
// one ciphertext per workgroup).
//
// Per CMux step (ct0 += GGSW [x] (ct0 * X^e - ct0), fft64 add_external_product_assign):
//   decompose   rotated difference and its balanced digits for every level at once (packed int16)
//   per level   pass A (twist, DFT16, W_256 twiddles) -> LDS -> pass B (DFT16)
//   (finest     MAC: Fourier position x (q, ct) accumulators against the level's GGSW rows
//    first)
//   inverse     MAC results -> LDS -> pass B^-1 -> pass A^-1 -> untwist, from_torus, ACC += (LDS)
// The arithmetic is the same fixed f64 sequence as the CPU oracle (tfhe_oracle.c): radix-16 DIF,
// MAC over (level desc, row asc) with the same fma chain, untwist = conj(twist) * 2^-8 (exact).
// FFT buffers hold [job][17 x 16] cplx (one pad slot per 16: conflict-free 16 x 16 transposes).
#pragma once
#include "fft_device.hpp"

namespace tae {
namespace br512 {

constexpr int N = 512, M = 256, K1 = 5;
constexpr int BUF_STRIDE = 17 * 16;  // cplx

__device__ __forceinline__ int pidx(int q) { return q + (q >> 4); }  // padded FFT-buffer index

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// A job's lanes live in one wave and the LDS operations of a wave execute in order, so hand-offs
// inside a job (pass A -> pass B, pass B^-1 -> pass A^-1, ACC update -> next decomposition) only
// need the compiler not to reorder the accesses; workgroup barriers remain where data crosses jobs.
__device__ __forceinline__ void wave_sync() { asm volatile("" ::: "memory"); }

// MAC thread -> Fourier position: odd 16-blocks rotated by one so that, with the +1-per-16 buffer
// padding, the 16 lanes of every ds_read_b128 lane group hit 16 distinct 4-bank groups.
__device__ __forceinline__ int mac_pos(int t) { return (t & 0xF0) | ((t - ((t >> 4) & 1)) & 15); }

// v_permlane16_swap: lanes of even rows keep x and receive the odd-row partner's x in y; lanes of
// odd rows receive the even-row partner's y in x and keep y (scripts/probes/permlane_swap.hip).
__device__ __forceinline__ void swap16(cplx &x, cplx &y) {
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

__device__ __forceinline__ void swap32(cplx &x, cplx &y) {
    // v_permlane32_swap: lanes 0-31 keep x and receive the partner's (lane + 32) x in y; lanes 32-63
    // receive the partner's y in x and keep y
    u32x4 a, b;
    __builtin_memcpy(&a, &x, 16);
    __builtin_memcpy(&b, &y, 16);
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const auto r = __builtin_amdgcn_permlane32_swap(a[w], b[w], false, false);
        a[w] = r[0];
        b[w] = r[1];
    }
    __builtin_memcpy(&x, &a, 16);
    __builtin_memcpy(&y, &b, 16);
}

// 4 x 4 transpose over the lane rows (lanes u, u+16, u+32, u+48) of a DFT16 job: register k of lane
// row r moves to register r of lane row k
__device__ __forceinline__ void transpose4(cplx *v) {
#ifndef TAE_X4_NOSWAP  // timing-only bound (garbage results): no lane transposes
    swap32(v[0], v[2]);
    swap32(v[1], v[3]);
    swap16(v[0], v[1]);
    swap16(v[2], v[3]);
#endif
}

__device__ __forceinline__ double lo16(uint32_t w) { return (double)((int32_t)(w << 16) >> 16); }
__device__ __forceinline__ double hi16(uint32_t w) { return (double)((int32_t)w >> 16); }

}  // namespace br512
}  // namespace tae
