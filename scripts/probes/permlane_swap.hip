// Probe: semantics of v_permlane16_swap_b32 / v_permlane32_swap_b32 on gfx950.
// Each lane passes x = lane, y = 100 + lane; prints what every lane gets back in (r0, r1).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *o) {
    const unsigned l = threadIdx.x;
    auto r = __builtin_amdgcn_permlane16_swap(l, 100 + l, false, false);
    auto s = __builtin_amdgcn_permlane32_swap(l, 100 + l, false, false);
    o[4 * l + 0] = r[0]; o[4 * l + 1] = r[1];
    o[4 * l + 2] = s[0]; o[4 * l + 3] = s[1];
}
int main() {
    unsigned *d, h[256];
    if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
    k<<<1, 64>>>(d);
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    for (int l = 0; l < 64; l++) printf("lane %2d: p16 (%3u,%3u)  p32 (%3u,%3u)\n", l, h[4*l], h[4*l+1], h[4*l+2], h[4*l+3]);
    return 0;
}
