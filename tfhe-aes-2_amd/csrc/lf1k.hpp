// The blind rotation's fused-twiddle transform for N = 1024 (the 8-bit model's PBS: k = 2, 6 levels of
// 2^7; br1024 / br1024lat PBS mode).  Restated in the oracle as or_lf1k_fwd / or_lf1k_bwd_add
// (oracle/tfhe_oracle.c), which is the definition; DESIGN.md §5.2 derives it.
//
// Same three radix-8 passes, lane programs and LDS positions as br1024's M = 512 schedule, but every
// DFT8 runs on inputs with geometric unit factors x_m g^m (dft8): fused DFT4s of ratio g^2 over the even
// and the odd m (lf512::dft4), then fused butterflies a +- rho b, rho = g W8^k1 = c (1 + i t) -- 72 fma
// per DFT8 instead of 56 flops plus 7 twiddle products (28):
//  - forward pass 0: the twist psi^(t + 64 m) makes its DFT4s the N = 512 transform's integer DFT4
//    (ratio psi^128 = e^{i pi/8}, a1i) and its butterflies lane-uniform (P0); psi^t and the twiddles
//    W^{t kk} become the ratios of pass 1 (per lane group gg, F1) and the rest those of pass 2 (per lane,
//    F2); the forward output is the exact DFT;
//  - inverse: the input carries E2(pos) = psi^((pos >> 6) + ((pos >> 3) & 7)), divided out of the
//    Fourier BSK once (lf_rescale_kernel); pass 2 stays br1024's plain inverse DFT8, passes 1 and 0 are
//    fused (I1 per lane column uu, I0 per lane), then the untwist conj(twist) and the exact 2^-9.
// Per CMux step and FFT job: 208 instead of 256 f64 operations per forward level, 232 instead of 256
// (+ the untwist) for the inverse.
#pragma once
#include "lf512.hpp"

namespace tae {
namespace lf1k {

using lf512::addc;
using lf512::K4;
using lf512::rot;

// table (doubles).  A fused DFT8 is 12 doubles, (cos, tan) of g^4, g^2 and of g W8^-+k1 (k1 = 0..3); the
// per-lane tables hold them as 6 chunks of 2 doubles, chunk-major ([chunk][entry][2]), so that a wave's
// b128 reads are lane-contiguous.
constexpr int P0 = 0;        // 1/sqrt 2, cos pi/8, tan pi/8, 0, then (cos, tan) of psi^64 W8^k1, k1 = 0..3
constexpr int F1 = 12;       // [6][8]  forward pass 1, lane group gg = t >> 3
constexpr int F2 = 108;      // [6][64] forward pass 2, lane t
constexpr int I1 = 876;      // [6][8]  inverse pass 1, lane column uu = t & 7
constexpr int I0 = 972;      // [6][64] inverse pass 0, lane t
constexpr int UNTW = 1740;   // [512] cplx conj(twist[j])
constexpr int E2 = 2764;     // [512] cplx conj(E2(pos))
constexpr int TOTAL = 3788;
constexpr int KERNEL_DOUBLES = E2;  // what the blind rotations stage in LDS

struct K8 {
    double c2, t2, c1, t1;  // the DFT4s: (cos, tan) of g^4 and g^2
    double c[4], t[4];      // the butterflies: rho_k1 = g W8^-+k1
};

using lf512::d2;

// entry idx of the [6][n] chunk-major table at off
__device__ __forceinline__ K8 k8(const double *tab, int off, int n, int idx) {
    d2 ch[6];
#pragma unroll
    for (int q = 0; q < 6; q++) ch[q] = *reinterpret_cast<const d2 *>(tab + off + 2 * (q * n + idx));
    K8 k;
    k.c2 = ch[0].x;
    k.t2 = ch[0].y;
    k.c1 = ch[1].x;
    k.t1 = ch[1].y;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        k.c[q] = ch[2 + q].x;
        k.t[q] = ch[2 + q].y;
    }
    return k;
}

// DFT8 (W8 forward, conj inverse) of x_m g^m relative to x_0's factor, in place, natural order
template <bool INV>
__device__ __forceinline__ void dft8(cplx *v, const K8 &K) {
    const K4 k4 = {K.c2, K.t2, K.c1, K.t1};
    cplx a[4] = {v[0], v[2], v[4], v[6]}, b[4] = {v[1], v[3], v[5], v[7]};
    lf512::dft4<INV>(a, k4);
    lf512::dft4<INV>(b, k4);
#pragma unroll
    for (int k1 = 0; k1 < 4; k1++) {
        const cplx r = rot(b[k1], K.t[k1]);
        v[k1] = addc(a[k1], K.c[k1], r);
        v[k1 + 4] = addc(a[k1], -K.c[k1], r);
    }
}

// forward pass 0's DFT4 over i of the integer pairs (dr[i], di[i]) times (e^{i pi/8})^i (the oracle's
// lf_int_dft4; lf512::a1 on unpacked digits), outputs k1 = 0..3 in natural order
__device__ __forceinline__ void a1i(const int *dr, const int *di, cplx *q, double s2, double c8, double t8) {
    const double D0r = dr[0], D0i = di[0], D1r = dr[1], D1i = di[1];
    const double P2r = dr[2] - di[2], P2i = dr[2] + di[2], P3r = dr[3] - di[3], P3i = dr[3] + di[3];
    const cplx ep = {fma(s2, P2r, D0r), fma(s2, P2i, D0i)}, em = {fma(-s2, P2r, D0r), fma(-s2, P2i, D0i)};
    const cplx op = {fma(s2, P3r, D1r), fma(s2, P3i, D1i)}, om = {fma(-s2, P3r, D1r), fma(-s2, P3i, D1i)};
    const cplx a = rot(op, t8), b = rot(om, t8);
    q[0] = addc(ep, c8, a);
    q[2] = addc(ep, -c8, a);
    q[1] = {fma(c8, b.im, em.re), fma(-c8, b.re, em.im)};
    q[3] = {fma(-c8, b.im, em.re), fma(c8, b.re, em.im)};
}

// the lane-uniform constants of forward pass 0
struct P0c {
    double s2, c8, t8, c[4], t[4];
};
__device__ __forceinline__ P0c p0(const double *tab) {
    P0c k;
    k.s2 = tab[P0];
    k.c8 = tab[P0 + 1];
    k.t8 = tab[P0 + 2];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        k.c[q] = tab[P0 + 4 + 2 * q];
        k.t[q] = tab[P0 + 5 + 2 * q];
    }
    return k;
}

// forward pass 0 of digits (dr[m], di[m]) of coefficients t + 64 m and t + 64 m + 512: v[kk] is position
// t + 64 kk
__device__ __forceinline__ void pass0(const int *dr, const int *di, cplx *v, const P0c &k) {
    cplx A[2][4];
#pragma unroll
    for (int n1 = 0; n1 < 2; n1++) {
        const int er[4] = {dr[n1], dr[n1 + 2], dr[n1 + 4], dr[n1 + 6]};
        const int ei[4] = {di[n1], di[n1 + 2], di[n1 + 4], di[n1 + 6]};
        a1i(er, ei, A[n1], k.s2, k.c8, k.t8);
    }
#pragma unroll
    for (int k1 = 0; k1 < 4; k1++) {
        const cplx r = rot(A[1][k1], k.t[k1]);
        v[k1] = addc(A[0][k1], k.c[k1], r);
        v[k1 + 4] = addc(A[0][k1], -k.c[k1], r);
    }
}

}  // namespace lf1k
}  // namespace tae
