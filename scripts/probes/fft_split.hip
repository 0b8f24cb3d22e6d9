// Probe: the 32-lane (lane-pair) forward/inverse 256-point FFT passes of br512x2.hpp against the
// 16-lane passes of br512.hpp on the same input; prints the number of differing words.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include "../../tfhe-aes-2_amd/csrc/br512x2.hpp"
using namespace tae;
using br512::pidx;

__global__ void old_fft(const cplx *x, const cplx *wtab, br512::W16 W, cplx *out, cplx *inv) {
    __shared__ cplx buf[272], tw[256];
    const int u = threadIdx.x;
    for (int t = u; t < 256; t += 16) tw[t] = wtab[(t >> 4) * (t & 15)];
    __syncthreads();
    cplx v[16];
    for (int m = 0; m < 16; m++) v[m] = x[u + 16 * m];
    br512::dft16<false>(v, W);
    if (u) for (int k = 1; k < 16; k++) v[k] = cmul(v[k], tw[16 * k + u]);
    for (int k = 0; k < 16; k++) buf[pidx(u + 16 * k)] = v[k];
    __syncthreads();
    for (int m = 0; m < 16; m++) v[m] = buf[pidx(16 * u + m)];
    br512::dft16<false>(v, W);
    for (int k = 0; k < 16; k++) buf[pidx(16 * u + k)] = v[k];
    __syncthreads();
    for (int t = u; t < 256; t += 16) out[t] = buf[pidx(t)];
    __syncthreads();
    for (int m = 0; m < 16; m++) v[m] = buf[pidx(16 * u + m)];
    br512::dft16<true>(v, W);
    for (int k = 0; k < 16; k++) buf[pidx(16 * u + k)] = v[k];
    __syncthreads();
    for (int k = 0; k < 16; k++) v[k] = buf[pidx(u + 16 * k)];
    if (u) for (int k = 1; k < 16; k++) v[k] = cmul(v[k], cconj(tw[16 * k + u]));
    br512::dft16<true>(v, W);
    for (int m = 0; m < 16; m++) inv[u + 16 * m] = v[m];
}

__global__ void new_fft(const cplx *x, const cplx *wtab, br512::W16 W, cplx *out, cplx *inv) {
    __shared__ cplx buf[272], tw[256], w16[12];
    const int t32 = threadIdx.x, h = t32 >> 4, u = t32 & 15;
    for (int t = t32; t < 256; t += 32) tw[t] = wtab[(t >> 4) * (t & 15)];
    if (t32 < 12) {
        cplx v = {1.0, 0.0};
        switch (t32) {
        case 3: v = W.w1; break;
        case 4: case 6: v = W.w2; break;
        case 5: case 9: v = W.w3; break;
        case 7: v = {0.0, -1.0}; break;
        case 8: case 10: v = W.w6; break;
        case 11: v = W.w9; break;
        default: break;
        }
        w16[t32] = v;
    }
    __syncthreads();
    const cplx *my = w16 + 6 * h;
    cplx v[8];
    using namespace br512x2;
    for (int L = 0; L < 8; L++) v[L] = x[u + 16 * (2 * h + in_idx(L))];
    half_dft16<false>(v, my);
    for (int S = 0; S < 8; S++) { const int k = 2 * h + out_idx(S); buf[pidx(u + 16 * k)] = cmul(v[S], tw[16 * k + u]); }
    __syncthreads();
    for (int L = 0; L < 8; L++) v[L] = buf[pidx(16 * u + 2 * h + in_idx(L))];
    half_dft16<false>(v, my);
    for (int S = 0; S < 8; S++) buf[pidx(16 * u + 2 * h + out_idx(S))] = v[S];
    __syncthreads();
    for (int t = t32; t < 256; t += 32) out[t] = buf[pidx(t)];
    __syncthreads();
    for (int L = 0; L < 8; L++) v[L] = buf[pidx(16 * u + 2 * h + in_idx(L))];
    half_dft16<true>(v, my);
    for (int S = 0; S < 8; S++) buf[pidx(16 * u + 2 * h + out_idx(S))] = v[S];
    __syncthreads();
    for (int L = 0; L < 8; L++) { const int kk = 2 * h + in_idx(L); v[L] = cmul(buf[pidx(u + 16 * kk)], cconj(tw[16 * kk + u])); }
    half_dft16<true>(v, my);
    for (int S = 0; S < 8; S++) inv[u + 16 * (2 * h + out_idx(S))] = v[S];
}

int main() {
    cplx hx[256], hw[256];
    for (int i = 0; i < 256; i++) {
        hx[i] = {std::sin(0.37 * i + 0.1) * 1000, std::cos(1.3 * i) * 1000};
        hw[i] = {std::cos(2 * M_PI * i / 256), -std::sin(2 * M_PI * i / 256)};
    }
    hw[64] = {0.0, -1.0};
    br512::W16 W{hw[16], hw[32], hw[48], hw[96], hw[144]};
    cplx *dx, *dw, *o1, *o2, *i1, *i2;
    hipMalloc(&dx, 4096); hipMalloc(&dw, 4096); hipMalloc(&o1, 4096); hipMalloc(&o2, 4096); hipMalloc(&i1, 4096); hipMalloc(&i2, 4096);
    hipMemcpy(dx, hx, 4096, hipMemcpyHostToDevice); hipMemcpy(dw, hw, 4096, hipMemcpyHostToDevice);
    old_fft<<<1, 16>>>(dx, dw, W, o1, i1);
    new_fft<<<1, 32>>>(dx, dw, W, o2, i2);
    cplx a[256], b[256], c[256], d[256];
    hipMemcpy(a, o1, 4096, hipMemcpyDeviceToHost); hipMemcpy(b, o2, 4096, hipMemcpyDeviceToHost);
    hipMemcpy(c, i1, 4096, hipMemcpyDeviceToHost); hipMemcpy(d, i2, 4096, hipMemcpyDeviceToHost);
    int nf = 0, ni = 0;
    for (int i = 0; i < 256; i++) {
        if (a[i].re != b[i].re || a[i].im != b[i].im) { if (nf < 6) printf("fwd %3d old (%g,%g) new (%g,%g)\n", i, a[i].re, a[i].im, b[i].re, b[i].im); nf++; }
        if (c[i].re != d[i].re || c[i].im != d[i].im) { if (ni < 6) printf("inv %3d old (%g,%g) new (%g,%g)\n", i, c[i].re, c[i].im, d[i].re, d[i].im); ni++; }
    }
    printf("forward: %d/256 differ, inverse: %d/256 differ; roundtrip old[5] = (%g,%g) vs x*256 (%g,%g)\n", nf, ni, c[5].re, c[5].im, hx[5].re * 256, hx[5].im * 256);
    return 0;
}
