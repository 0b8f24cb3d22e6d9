// The blind rotation's fused-twiddle transform for N = 512 (params_sqrd_lvl_64; br512x4 PBS mode and
// br512lat).  Restated in the oracle as or_lf_fwd / or_lf_bwd_add (oracle/tfhe_oracle.c), which is the
// definition; DESIGN.md §5.1 derives it.
//
// Same 16 x 16 negacyclic DFT, same LDS positions (16 kappa + lambda) and the same lane transposes as the
// radix-16 schedule, but no twiddle or twist is a separate complex product:
//  - every radix-4 stage whose inputs carry unit factors w, w g, w g^2, w g^3 runs relative to w with
//    fused butterflies x + g^2 y = x + c (y + i t y), g^2 = c (1 + i t): 24 fma per DFT4 (dft4), instead of
//    3-4 complex products + 16 adds; w rides into the next stage's ratios, and the last stage of each
//    pass has w = 1;
//  - the forward twist becomes lane-uniform factors inside the first DFT4 (psi^64 = e^{i pi/8}; its
//    e^{i pi/4} products act on the integer digits exactly, a1) plus factors of later ratios;
//  - the inverse input carries E2(pos) = psi^(kappa + (lambda mod 4)), divided out of the Fourier BSK
//    once (lf_rescale_kernel), which keeps every ratio off the imaginary axis.
// Per CMux step and job wave that is 92 instead of 120 f64 operations per forward level and 104 instead
// of 120 for the inverse.
#pragma once
#include "br512.hpp"

namespace tae {
namespace lf512 {

// table (doubles): per-lane (cos, tan) pairs of g^2 and g for each fused stage, the lane-uniform
// constants, conj(twist), conj(E2).  The per-lane tables are chunk-major, [2][n entries][2 doubles] (chunk
// 0: g^2, chunk 1: g), and the (kappa, l1) / (u, m1) ones are indexed by the lane u + 16 r itself, so that
// every wave's ds_read_b128 of them is lane-contiguous (conflict-free) or a broadcast.
constexpr int FA2 = 0;     // [2][4]  forward pass A stage 2, entry = lane row r (k1)
constexpr int FB1 = 16;    // [2][16] forward pass B stage 1, entry = lane column u (kappa)
constexpr int FB2 = 80;    // [2][64] forward pass B stage 2, entry = lane u + 16 r (kappa, l1)
constexpr int IB2 = 336;   // [2][4]  inverse pass B stage 2, entry = r (u1)
constexpr int IA1 = 352;   // [2][16] inverse pass A stage 1, entry = u
constexpr int IA2 = 416;   // [2][64] inverse pass A stage 2, entry = lane u + 16 r (u, m1)
constexpr int CONSTS = 672;  // 1/sqrt 2, cos pi/8, tan pi/8, 0
constexpr int UNTW = 676;  // [256] cplx conj(twist[j])
constexpr int E2 = 1188;   // [256] cplx conj(E2(pos))
constexpr int TOTAL = 1700;
constexpr int KERNEL_DOUBLES = E2;  // what the blind rotations stage in LDS

struct K4 {
    double c2, t2, c1, t1;
};
typedef double d2 __attribute__((ext_vector_type(2)));
// entry idx of the [2][n] chunk-major table at off
__device__ __forceinline__ K4 k4(const double *tab, int off, int n, int idx) {
    const d2 a = *reinterpret_cast<const d2 *>(tab + off + 2 * idx);
    const d2 b = *reinterpret_cast<const d2 *>(tab + off + 2 * (n + idx));
    return {a.x, a.y, b.x, b.y};
}

// x (1 + i t) and a + c t
__device__ __forceinline__ cplx rot(cplx x, double t) { return {fma(-t, x.im, x.re), fma(t, x.re, x.im)}; }
__device__ __forceinline__ cplx addc(cplx a, double c, cplx t) { return {fma(c, t.re, a.re), fma(c, t.im, a.im)}; }

// DFT4 (W4 = -i forward, +i inverse) of x0, g x1, g^2 x2, g^3 x3 relative to x0's factor, in place
template <bool INV>
__device__ __forceinline__ void dft4(cplx *x, const K4 &K) {
    const cplx t = rot(x[2], K.t2), s = rot(x[3], K.t2);
    const cplx u0 = addc(x[0], K.c2, t), u1 = addc(x[0], -K.c2, t);
    const cplx v0 = addc(x[1], K.c2, s), v1 = addc(x[1], -K.c2, s);
    const cplx p = rot(v0, K.t1), q = rot(v1, K.t1);
    x[0] = addc(u0, K.c1, p);
    x[2] = addc(u0, -K.c1, p);
    const double c = INV ? -K.c1 : K.c1;
    x[1] = {fma(c, q.im, u1.re), fma(-c, q.re, u1.im)};
    x[3] = {fma(-c, q.im, u1.re), fma(c, q.re, u1.im)};
}

// forward pass A stage 1: DFT4 over i of d_i psi^(64 i) for the packed digit pairs dw[i] (low half: the
// coefficient j, high half: j + 256), outputs k1 = 0..3 in natural order
// (digits as ints: dr[i] of the coefficient j, di[i] of j + 256)
__device__ __forceinline__ void a1i(const int *dr, const int *di, cplx *q, double s2, double c8, double t8) {
    const int d0r = dr[0], d0i = di[0], d1r = dr[1], d1i = di[1];
    const int d2r = dr[2], d2i = di[2], d3r = dr[3], d3i = di[3];
    const double D0r = d0r, D0i = d0i, D1r = d1r, D1i = d1i;
    const double P2r = d2r - d2i, P2i = d2r + d2i, P3r = d3r - d3i, P3i = d3r + d3i;  // e^{i pi/4} sqrt 2 d
    const cplx ep = {fma(s2, P2r, D0r), fma(s2, P2i, D0i)}, em = {fma(-s2, P2r, D0r), fma(-s2, P2i, D0i)};
    const cplx op = {fma(s2, P3r, D1r), fma(s2, P3i, D1i)}, om = {fma(-s2, P3r, D1r), fma(-s2, P3i, D1i)};
    const cplx a = rot(op, t8), b = rot(om, t8);
    q[0] = addc(ep, c8, a);
    q[2] = addc(ep, -c8, a);
    q[1] = {fma(c8, b.im, em.re), fma(-c8, b.re, em.im)};
    q[3] = {fma(-c8, b.im, em.re), fma(c8, b.re, em.im)};
}
__device__ __forceinline__ void a1(const uint32_t *dw, cplx *q, double s2, double c8, double t8) {
    int dr[4], di[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        dr[i] = (int32_t)(dw[i] << 16) >> 16;
        di[i] = (int32_t)dw[i] >> 16;
    }
    a1i(dr, di, q, s2, c8, t8);
}

}  // namespace lf512
}  // namespace tae
