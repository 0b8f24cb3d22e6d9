// Probe: how fast can one 1024-thread workgroup per CU stream a blind-rotation step's GGSW rows
// (params_sqrd_lvl_64: 3 levels x 5 x 5 x 256 cplx = 307200 B) through its vector L1, when every
// workgroup reads the same rows (the latency kernel br512lat: one ciphertext per workgroup)?
// Each step: every thread loads its share with 16-byte buffer loads (coalesced, 1 KiB per wave
// instruction), xors the words into a register, workgroup barrier.  Grid = 128 or 256 workgroups.
//   mode 0: step s reads rows s of a 677-step key (HBM once, then L2 for the other workgroups)
//   mode 1: every step re-reads step 0's rows (L2-resident)
// Output: microseconds per step.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int STEP_BYTES = 307200, STEPS = 677, THREADS = 1024;

template <int MODE>
__global__ void __launch_bounds__(THREADS, 1) stream(const u32x4 *__restrict__ key, unsigned *out) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)key, (short)0, (unsigned)(STEP_BYTES * (size_t)STEPS > 0x7fffffff ? 0x7fffffff : STEP_BYTES * (size_t)STEPS), 0x00020000);
    unsigned x = 0;
    for (int s = 0; s < STEPS; s++) {
        const int soff = MODE == 0 ? s * STEP_BYTES : 0;
        u32x4 v[19];
#pragma unroll
        for (int k = 0; k < 19; k++) {
            const int off = (k * THREADS + (int)threadIdx.x) * 16;
            v[k] = off < STEP_BYTES ? __builtin_amdgcn_raw_buffer_load_b128(rs, off, soff, 0) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int k = 0; k < 19; k++) x ^= v[k][0] ^ v[k][1] ^ v[k][2] ^ v[k][3];
        __syncthreads();
    }
    out[blockIdx.x * THREADS + threadIdx.x] = x;
}

int main() {
    u32x4 *key;
    unsigned *out;
    hipMalloc(&key, (size_t)STEP_BYTES * STEPS);
    hipMemset(key, 1, (size_t)STEP_BYTES * STEPS);
    hipMalloc(&out, 256 * THREADS * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int mode = 0; mode < 2; mode++)
        for (int g : {1, 32, 128, 256}) {
            float best = 1e9f;
            for (int it = 0; it < 4; it++) {
                hipEventRecord(a);
                if (mode == 0) stream<0><<<g, THREADS>>>(key, out);
                else stream<1><<<g, THREADS>>>(key, out);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                if (ms < best) best = ms;
            }
            printf("mode %d grid %3d: %.3f us/step  (%.1f GB/s per WG)\n", mode, g, best * 1e3 / STEPS,
                   STEP_BYTES / (best * 1e-3 / STEPS) / 1e9);
        }
    return 0;
}
