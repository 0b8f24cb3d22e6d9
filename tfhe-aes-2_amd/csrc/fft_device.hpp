// Negacyclic f64 FFT building blocks for CDNA4 (gfx950).
//
// Math (tfhe-fft 0.7 as used by tfhe-rs fft64, Cargo.lock:773): a real polynomial p of size N is
// folded to z_j = (p_j + i p_{j+M}) * e^{i pi j / N}, M = N/2, and transformed with an M-point
// DFT; the backward path runs the inverse DFT, multiplies by conj(twist)/M and takes the
// fractional part of the torus value (UnsignedTorus::from_torus).
//
// Schedule: decimation-in-frequency, radix R (R=16 for M=256, R=8 for M=512), P passes, so the
// spectrum lives in digit-reversed order; the inverse is the mirrored decimation-in-time.  Every
// f64 operation is fixed (explicit fma, -ffp-contract=off), so the CPU oracle can restate the
// schedule and compare ciphertexts bit-exactly.  A pass is done by M/R threads ("TPJ" threads per
// polynomial), each holding R complex values in registers; passes exchange through LDS.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "cplx.hpp"

namespace tae {

__device__ __forceinline__ cplx cmul(cplx a, cplx b) {
    return {fma(a.re, b.re, -(a.im * b.im)), fma(a.re, b.im, a.im * b.re)};
}
__device__ __forceinline__ cplx cconj(cplx a) { return {a.re, -a.im}; }
__device__ __forceinline__ cplx cadd(cplx a, cplx b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cplx csub(cplx a, cplx b) { return {a.re - b.re, a.im - b.im}; }

template <int M>
struct FftPlan;
template <>
struct FftPlan<256> {
    static constexpr int R = 16, P = 2;
};
template <>
struct FftPlan<512> {
    static constexpr int R = 8, P = 3;
};

template <bool INV>
__device__ __forceinline__ void dft4(cplx &a, cplx &b, cplx &c, cplx &d) {
    const cplx t0 = cadd(a, c), t1 = csub(a, c), t2 = cadd(b, d), t3 = csub(b, d);
    a = cadd(t0, t2);
    c = csub(t0, t2);
    if (!INV) {
        b = {t1.re + t3.im, t1.im - t3.re};
        d = {t1.re - t3.im, t1.im + t3.re};
    } else {
        b = {t1.re - t3.im, t1.im + t3.re};
        d = {t1.re + t3.im, t1.im - t3.re};
    }
}

// x * W_R^e (W_R = e^{-2 pi i / R}, conjugated for the inverse); e == R/4 is the exact -i / +i
template <int R, int M, bool INV>
__device__ __forceinline__ cplx tw_small(cplx x, int e, const cplx *__restrict__ w) {
    if (e == 0) return x;
    if (4 * e == R) return INV ? cplx{-x.im, x.re} : cplx{x.im, -x.re};
    const cplx t = w[e * (M / R)];
    return cmul(x, INV ? cconj(t) : t);
}

// In-register R-point DFT in natural order.  DFT16 = 4x4 (x[n1 + 4 n2] -> X[k1 + 4 k2]),
// DFT8 = 2x4 (x[n1 + 2 n2] -> X[k1 + 4 k2]).
template <int R, int M, bool INV>
__device__ __forceinline__ void dft(cplx *v, const cplx *__restrict__ w) {
    if constexpr (R == 16) {
        cplx y[16];
#pragma unroll
        for (int n1 = 0; n1 < 4; n1++) dft4<INV>(v[n1], v[n1 + 4], v[n1 + 8], v[n1 + 12]);
#pragma unroll
        for (int n1 = 0; n1 < 4; n1++)
#pragma unroll
            for (int k1 = 0; k1 < 4; k1++) y[4 * k1 + n1] = tw_small<16, M, INV>(v[n1 + 4 * k1], n1 * k1, w);
#pragma unroll
        for (int k1 = 0; k1 < 4; k1++) dft4<INV>(y[4 * k1], y[4 * k1 + 1], y[4 * k1 + 2], y[4 * k1 + 3]);
#pragma unroll
        for (int k1 = 0; k1 < 4; k1++)
#pragma unroll
            for (int k2 = 0; k2 < 4; k2++) v[k1 + 4 * k2] = y[4 * k1 + k2];
    } else {
        static_assert(R == 8, "radix");
        cplx y[8];
#pragma unroll
        for (int n1 = 0; n1 < 2; n1++) dft4<INV>(v[n1], v[n1 + 2], v[n1 + 4], v[n1 + 6]);
#pragma unroll
        for (int n1 = 0; n1 < 2; n1++)
#pragma unroll
            for (int k1 = 0; k1 < 4; k1++) y[2 * k1 + n1] = tw_small<8, M, INV>(v[n1 + 2 * k1], n1 * k1, w);
#pragma unroll
        for (int k1 = 0; k1 < 4; k1++) {
            const cplx a = y[2 * k1], b = y[2 * k1 + 1];
            v[k1] = cadd(a, b);
            v[k1 + 4] = csub(a, b);
        }
    }
}

// ---- torus helpers (tfhe-rs SignedDecomposer, UnsignedTorus::from_torus) ----

// digit of level `lev` (1 = most significant) of the balanced base-2^B decomposition
__device__ __forceinline__ int64_t decomp_digit(uint64_t x, int base_log, int levels, int lev) {
    const int nrb = 64 - base_log * levels;
    uint64_t r = x >> (nrb - 1);
    r += r & 1;
    r >>= 1;  // = closest_representable(x) >> nrb
    uint64_t state = r;
    const uint64_t mask = (1ull << base_log) - 1;
    int64_t digit = 0;
    for (int l = levels; l >= lev; l--) {
        const uint64_t res = state & mask;
        state >>= base_log;
        uint64_t carry = ((res - 1) | state) & res;
        carry >>= (base_log - 1);
        state += carry;
        digit = (int64_t)(res - (carry << base_log));
    }
    return digit;
}

__device__ __forceinline__ uint64_t from_torus(double x) {
    const double f = x - round(x);
    const double v = round(f * 0x1p64);
    const int64_t iv = v >= 0x1p63 ? INT64_MAX : (int64_t)v;
    return (uint64_t)iv;
}

__host__ __device__ __forceinline__ uint64_t f64_bits(double x) {
#ifdef __HIP_DEVICE_COMPILE__
    return (uint64_t)__double_as_longlong(x);
#else
    uint64_t b;
    __builtin_memcpy(&b, &x, 8);
    return b;
#endif
}

// from_torus on the bits of x, integer ops only; equal to from_torus(x) for every finite x.
// |x| 2^64 = m 2^s (m the 53-bit significand, s = biased exponent - 1011).
//   s >= 0: x 2^64 is an integer, f = x - round(x) is exact and f 2^64 == x 2^64 (mod 2^64);
//   s <  0: |x| < 2^-12 so round(x) = 0 and round(x 2^64) = (m + 2^(k-1)) >> k, k = -s
//           (half away from zero on the magnitude).
// The i64 saturation of f 2^64 = +2^63 (x = -(n + 1/2)) gives INT64_MAX instead of 2^63.
__host__ __device__ __forceinline__ uint64_t from_torus_bits(double x) {
    const uint64_t b = f64_bits(x);
    const uint32_t hi = (uint32_t)(b >> 32);
    const int s = (int)((hi >> 20) & 0x7ff) - 1011;
    const uint64_t m = (b & 0xFFFFFFFFFFFFFull) | (1ull << 52);
    uint64_t mag;
    if (__builtin_expect(s >= 0, 1)) {
        mag = s < 64 ? m << s : 0;
    } else {
        const int k = -s;
        mag = k < 64 ? (m + (1ull << (k - 1))) >> k : 0;
    }
    const uint64_t sg = (uint64_t)(int64_t)((int32_t)hi >> 31);
    const uint64_t r = (mag ^ sg) - sg;
    return r - (uint64_t)((sg != 0) & (r == 0x8000000000000000ull));
}

// acc + from_torus_bits(x) on the common path, branch-free: when the scaled exponent s = biased
// exponent - 1011 is in [0, 63] (|x| in [2^-12, 2^52): every inverse-FFT output of the blind rotations
// except exact zeros), x 2^64 = m 2^s is an integer, the magnitude is m << s (mod 2^64) and the sign is
// applied as
//   acc + r = acc + (mag ^ sg) + (neg && mag != 2^63)       (sg = 0 or ~0)
// i.e. acc - mag for negative x, and acc + 2^63 - 1 for the saturated case mag = 2^63 (x = -(n+1/2)).
// `ok` is false when s is outside [0, 63] (the returned value is then garbage): the caller takes
// from_torus_bits for the whole wave behind one wave-uniform branch (12 VALU ops per value here, no exec
// masking or copies of acc; the per-value branch cost ~17 VALU + 4 SALU).
__host__ __device__ __forceinline__ uint64_t torus_add_fast(double x, uint64_t acc, bool &ok) {
    const uint64_t b = f64_bits(x);
    const uint32_t hi = (uint32_t)(b >> 32);
    const uint32_t s = ((hi >> 20) & 0x7ff) - 1011u;
    ok = s <= 63u;
    const uint64_t m = (b & 0xFFFFFFFFFFFFFull) | (1ull << 52);
    const uint64_t mag = m << (s & 63);
    const uint64_t sg = (uint64_t)(int64_t)((int32_t)hi >> 31);
    const uint64_t carry = (uint64_t)((hi >> 31) & (uint32_t)(mag != 0x8000000000000000ull));
    return acc + (mag ^ sg) + carry;
}

// torus_add_fast of x * 2^-SH (exact power-of-two scaling folded into the exponent): the untwist
// conj(twist) / M of the inverse FFT is conj(twist) times an exact 2^-log2(M), so a kernel holding the twist
// factors can multiply by conj(twist) and let the conversion apply the 2^-log2(M) (same result bit for bit
// as the product with the untwist table, outside the subnormal range, which no value here reaches).
template <int SH>
__host__ __device__ __forceinline__ uint64_t torus_add_fast_sh(double x, uint64_t acc, bool &ok) {
    const uint64_t b = f64_bits(x);
    const uint32_t hi = (uint32_t)(b >> 32);
    const uint32_t s = ((hi >> 20) & 0x7ff) - (1011u + SH);
    ok = s <= 63u;
    const uint64_t m = (b & 0xFFFFFFFFFFFFFull) | (1ull << 52);
    const uint64_t mag = m << (s & 63);
    const uint64_t sg = (uint64_t)(int64_t)((int32_t)hi >> 31);
    const uint64_t carry = (uint64_t)((hi >> 31) & (uint32_t)(mag != 0x8000000000000000ull));
    return acc + (mag ^ sg) + carry;
}

// tfhe-rs SignedDecomposer (closest_representable + balanced digits, the carry rule of
// decompose_one_level) for LEV levels of B bits with B * (LEV - 1) < 32: d[l] = the 16-bit two's
// complement pattern of the digit of level l + 1 (1 = most significant), upper half zero.
// x + 2^(nrb-1) >> nrb is closest_representable >> nrb (mod 2^(B LEV)), which is all the digits see.
template <int LEV>
__host__ __device__ __forceinline__ void decompose16(uint64_t x, int B, uint32_t *d) {
    const int nrb = 64 - B * LEV;
    const uint64_t X = x + (1ull << (nrb - 1));
    const uint32_t mask = (1u << B) - 1, neg = 0x10000u - (1u << B);
    uint32_t res = (uint32_t)(X >> nrb) & mask;
    uint32_t st = nrb + B >= 64 ? 0u : (uint32_t)(X >> (nrb + B));
#pragma unroll
    for (int l = LEV - 1; l >= 0; l--) {
        const uint32_t c = (((res - 1) | st) & res) >> (B - 1);
        d[l] = res + c * neg;  // c in {0, 1}: one v_mad_u32_u24
        if (l > 0) {
            st += c;
            res = st & mask;
            st >>= B;
        }
    }
}

// decompose16 for compile-time B (any LEV with B * LEV < 64): the state after the first level is
// kept in 64 bits when B * (LEV - 1) >= 32 (the 8-bit model's PBS: 6 levels of 7 bits).
template <int LEV, int B>
__host__ __device__ __forceinline__ void decompose16t(uint64_t x, uint32_t *d) {
    if constexpr (B * (LEV - 1) < 32) {
        decompose16<LEV>(x, B, d);
    } else {
        constexpr int nrb = 64 - B * LEV;
        const uint64_t X = x + (1ull << (nrb - 1));
        constexpr uint64_t mask = (1ull << B) - 1;
        constexpr uint32_t neg = 0x10000u - (1u << B);
        uint64_t res = (X >> nrb) & mask;
        uint64_t st = X >> (nrb + B);
#pragma unroll
        for (int l = LEV - 1; l >= 0; l--) {
            const uint64_t c = (((res - 1) | st) & res) >> (B - 1);
            d[l] = (uint32_t)res + (uint32_t)c * neg;
            if (l > 0) {
                st += c;
                res = st & mask;
                st >>= B;
            }
        }
    }
}

// ---- packed two-coefficient decomposition (v_pk_* 16-bit SIMD) ----
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__host__ __device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__host__ __device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
// v_perm_b32 / v_alignbit_b32 (host emulation for the native tests); perm selectors < 8 only
__host__ __device__ __forceinline__ uint32_t perm_b32(uint32_t s0, uint32_t s1, uint32_t sel) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_perm(s0, s1, sel);
#else
    const uint64_t v = ((uint64_t)s0 << 32) | s1;
    uint32_t r = 0;
    for (int k = 0; k < 4; k++) r |= (uint32_t)((v >> (8 * ((sel >> (8 * k)) & 7))) & 0xff) << (8 * k);
    return r;
#endif
}
__host__ __device__ __forceinline__ uint32_t alignbit_b32(uint32_t hi, uint32_t lo, int s) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_alignbit(hi, lo, s);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> s);
#endif
}

// decompose16 of two coefficients at once, d[l] = digit of x0 | digit of x1 << 16 (the packed
// layout the FFT passes read), with 16-bit SIMD ops on both halves.  Same digits as decompose16:
// with F_i the B-bit fields of X = x + 2^(nrb-1) above bit nrb (F_0 lowest), the state at field i
// is G_i = F_i + k_i (k_0 = 0), res_i = G_i mod 2^B, ovf_i = G_i >> B, and the carry rule reads bit
// B-1 of the state above, i.e. of F_{i+1} + ovf_i; then k_{i+1} = ovf_i + c_i <= 1 (ovf_i = 1
// forces res_i = 0, so c_i = 0).  The top state above the last field is ovf <= 1: bit B-1 clear.
template <int LEV, int B>
__host__ __device__ __forceinline__ void decompose16p(uint64_t x0, uint64_t x1, uint32_t *d) {
    static_assert(B <= 15 && B * LEV <= 64 && B >= 2, "decompose16p shape");
    constexpr int nrb = 64 - B * LEV;
    const uint64_t X0 = x0 + (1ull << (nrb - 1)), X1 = x1 + (1ull << (nrb - 1));
    constexpr uint32_t MASK = ((1u << B) - 1) * 0x10001u;
    uint32_t F[LEV];
    if constexpr (LEV == 3 && B == 12) {
        // fields at bits 28..39, 40..51, 52..63: F0 straddles the dwords, F1 / F2 are bytes 1-2 / 2-3
        const uint32_t h0 = (uint32_t)(X0 >> 32), h1 = (uint32_t)(X1 >> 32);
        const uint32_t a0 = alignbit_b32(h0, (uint32_t)X0, 28), a1 = alignbit_b32(h1, (uint32_t)X1, 28);
        F[0] = perm_b32(a1, a0, 0x05040100u) & MASK;
        F[1] = perm_b32(h1, h0, 0x06050201u) & MASK;
        F[2] = as_u32(as_u16x2(perm_b32(h1, h0, 0x07060302u)) >> (unsigned short)4);
    } else if constexpr (LEV == 6 && B == 7) {
        // the 8-bit model's PBS: fields at bits 22 + 7 i; F0 in the low dwords, F1 straddles them, F2..F5
        // from the high dwords' 16-bit windows at bits 0, 8 and 16 (v_perm), no 64-bit shifts
        const uint32_t l0 = (uint32_t)X0, l1 = (uint32_t)X1, h0 = (uint32_t)(X0 >> 32), h1 = (uint32_t)(X1 >> 32);
        const u16x2 s7 = {0x7F, 0x7F};
        F[0] = as_u32((as_u16x2(perm_b32(l1, l0, 0x07060302u)) >> (unsigned short)6) & s7);
        F[1] = perm_b32(alignbit_b32(h1, l1, 29), alignbit_b32(h0, l0, 29), 0x05040100u) & MASK;
        const u16x2 w0 = as_u16x2(perm_b32(h1, h0, 0x05040100u)), w8 = as_u16x2(perm_b32(h1, h0, 0x06050201u)),
                    w16 = as_u16x2(perm_b32(h1, h0, 0x07060302u));
        F[2] = as_u32((w0 >> (unsigned short)4) & s7);
        F[3] = as_u32((w8 >> (unsigned short)3) & s7);
        F[4] = as_u32((w16 >> (unsigned short)2) & s7);
        F[5] = as_u32(w16 >> (unsigned short)9);
    } else {
#pragma unroll
        for (int i = 0; i < LEV; i++)
            F[i] = ((uint32_t)(X0 >> (nrb + B * i)) & ((1u << B) - 1)) |
                   (((uint32_t)(X1 >> (nrb + B * i)) & ((1u << B) - 1)) << 16);
    }
    const u16x2 one = {1, 1}, sh = {B, B}, shm = {B - 1, B - 1};
    const u16x2 neg = {(unsigned short)(0x10000u - (1u << B)), (unsigned short)(0x10000u - (1u << B))};
    u16x2 k = {0, 0};
#pragma unroll
    for (int i = 0; i < LEV; i++) {
        u16x2 res, nxt;
        if (i == 0) {
            res = as_u16x2(F[0]);
            nxt = LEV > 1 ? as_u16x2(F[1]) : u16x2{0, 0};
        } else {
            const u16x2 g = as_u16x2(F[i]) + k;
            res = as_u16x2(as_u32(g) & MASK);
            const u16x2 ovf = g >> sh;
            nxt = i + 1 < LEV ? as_u16x2(F[i + 1]) + ovf : u16x2{0, 0};
            k = ovf;
        }
        const u16x2 c = as_u16x2(((as_u32(res - one) | as_u32(nxt)) & as_u32(res))) >> shm;
        d[LEV - 1 - i] = as_u32(res + c * neg);
        if (i == 0) k = c; else k = k + c;
    }
}

// The same digits one level at a time, least significant level first, as signed 32-bit values (what
// v_cvt_f64_i32 takes): digit_first returns the digit of the finest level (LEV) of x and leaves the
// 32-bit state of the fields above it (carry included) in st; each digit_next returns the digit of the
// next coarser level and advances st.  Unpacked 32-bit ops cost half a v_pk_*_u16 op each on gfx950,
// and the state (one register per coefficient) replaces the packed digits of every level.
template <int LEV, int B>
__host__ __device__ __forceinline__ int32_t digit_first(uint64_t x, uint32_t &st) {
    static_assert(B * (LEV - 1) < 32 && B >= 2 && B <= 16, "digit_first shape");
    constexpr int nrb = 64 - B * LEV;
    const uint64_t X = x + (1ull << (nrb - 1));
    const uint32_t res = (uint32_t)(X >> nrb) & ((1u << B) - 1);
    if constexpr (nrb + B >= 64) st = 0u;
    else st = (uint32_t)(X >> (nrb + B));
    const uint32_t c = (((res - 1) | st) & res) >> (B - 1);
    st += c;
    return (int32_t)res - (int32_t)(c << B);
}
template <int B>
__host__ __device__ __forceinline__ int32_t digit_next(uint32_t &st) {
    const uint32_t res = st & ((1u << B) - 1);
    st >>= B;
    const uint32_t c = (((res - 1) | st) & res) >> (B - 1);
    st += c;
    return (int32_t)res - (int32_t)(c << B);
}

// Effective-clock stamps of a blind-rotation launch (diagnostic launches only; every other launch passes
// clk == nullptr and no stamp executes): the workgroup's shader cycles (s_memtime) and 100 MHz reference
// ticks (s_memrealtime) from kernel entry to exit, written by thread 0 to clk[2 wg] / clk[2 wg + 1], a
// buffer nothing else reads (MI355X_MICROARCH.md "DVFS give-back" item 6).  The stamps are wave-uniform
// (SGPRs, no VGPR held across the kernel); lgkmcnt is drained after the first pair.
struct ClockStamp {
    uint64_t c0 = 0, r0 = 0;
    __device__ __forceinline__ void start(const uint64_t *clk) {
        if (clk) {
            c0 = __builtin_amdgcn_s_memtime();
            r0 = __builtin_amdgcn_s_memrealtime();
            __builtin_amdgcn_s_waitcnt(0xC07F);
        }
    }
    __device__ __forceinline__ void stop(uint64_t *clk) {
        if (clk) {
            const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
            __builtin_amdgcn_s_waitcnt(0xC07F);
            if (threadIdx.x == 0) {
                clk[2 * (size_t)blockIdx.x] = c1 - c0;
                clk[2 * (size_t)blockIdx.x + 1] = r1 - r0;
            }
        }
    }
};

// pbs_modulus_switch: round(x * 2N / 2^64) in [0, 2N]
__device__ __forceinline__ int mod_switch(uint64_t x, int logN) {
    uint64_t o = x >> (64 - logN - 2);
    o += o & 1;
    return (int)(o >> 1);
}

// coefficient j of poly * X^e (e in [0, 2N)): poly[src] with sign
__device__ __forceinline__ uint64_t rotated_coeff(const uint64_t *poly, int j, int e, int N) {
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
    const uint64_t v = poly[src];
    return neg ? (0 - v) : v;
}

// (uint64)(int64)d * key mod 2^64 with 32-bit multiplies
__device__ __forceinline__ uint64_t mul_i32_u64(int32_t d, uint64_t key) {
    const uint32_t lo = (uint32_t)key, hi = (uint32_t)(key >> 32);
    const uint32_t du = (uint32_t)d;
    const uint64_t p = (uint64_t)lo * du;
    const uint32_t h = hi * du - (d < 0 ? lo : 0u);
    return p + ((uint64_t)h << 32);
}

}  // namespace tae
