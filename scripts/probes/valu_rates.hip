// Probe: issue cost of the VALU instruction classes the blind rotation uses, at 16 waves per CU
// (4 per SIMD, the br512x4 occupancy), alone and mixed with v_fma_f64 from other waves of the SIMD.
// Each wave runs ITERS x 16 instructions of its class on 8 independent registers (no memory).
// Output: cycles per wave-instruction per SIMD (= kernel time x clock / (instructions per SIMD)).
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int CLS>
__device__ __forceinline__ void body(double *d, unsigned *u, unsigned long long *q) {
    if constexpr (CLS == 0) {  // v_fma_f64
#define F(i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[i]) : "v"(d[(i + 1) & 7]), "v"(d[(i + 2) & 7]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 1) {  // v_add_u32
#define F(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 2) {  // v_lshlrev_b64
#define F(i) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(q[i]) : "v"(u[i]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 3) {  // v_permlane32_swap
#define F(i) { const auto r_ = __builtin_amdgcn_permlane32_swap(u[i], u[(i + 4) & 7], false, false); u[i] = r_[0]; u[(i + 4) & 7] = r_[1]; }
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 4) {  // v_add_f64
#define F(i) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(d[(i + 1) & 7]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 5) {  // v_pk_add_u16
#define F(i) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 6) {  // v_cvt_f64_i32
#define F(i) asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(d[i]) : "v"(u[i]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 7) {  // v_mul_lo_u32 (quarter rate?)
#define F(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 8) {  // v_lshl_add_u64 (gfx950 64-bit add)
#define F(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(q[i]) : "v"(q[(i + 1) & 7]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 9) {  // v_cndmask_b32 with vcc
#define F(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 10) {  // v_mov_b32 (dpp-free)
#define F(i) asm volatile("v_mov_b32 %0, %1" : "=v"(u[i]) : "v"(u[(i + 3) & 7]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 12) {  // v_fma_f64, each depends on the previous (latency)
#define F(i) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[0]) : "v"(d[1]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 13) {  // v_mov_b32 dpp quad_perm
#define F(i) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(u[i]) : "v"(u[(i + 3) & 7]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 14) {  // v_cndmask_b32 with an SGPR pair condition
#define F(i) asm volatile("v_cndmask_b32 %0, %0, %1, s[20:21]" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 15) {  // v_fma_f64 with dependency distance 2 (two chains)
#define F(i) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[(i) & 1]) : "v"(d[2]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 16) {  // v_cndmask_b32 with a DPP quad_perm source (the 2-lane exchange)
#define F(i) asm volatile("v_cndmask_b32_dpp %0, %1, %0, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(u[i]) : "v"(u[(i + 3) & 7]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 17) {  // v_permlane16_swap
#define F(i) { const auto r_ = __builtin_amdgcn_permlane16_swap(u[i], u[(i + 4) & 7], false, false); u[i] = r_[0]; u[(i + 4) & 7] = r_[1]; }
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 18) {  // v_mul_f64
#define F(i) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[i]) : "v"(d[(i + 1) & 7]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 19) {  // v_fma_f64, each followed by one SALU op (counted: the f64 ops only)
#define F(i) asm volatile("v_fma_f64 %0, %0, %1, %2\n\ts_add_u32 s20, s20, 1" : "+v"(d[i]) : "v"(d[(i + 1) & 7]), "v"(d[(i + 2) & 7]) : "s20", "scc");
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 20) {  // v_fma_f64, each followed by two SALU ops
#define F(i) asm volatile("v_fma_f64 %0, %0, %1, %2\n\ts_add_u32 s20, s20, 1\n\ts_add_u32 s21, s21, 1" : "+v"(d[i]) : "v"(d[(i + 1) & 7]), "v"(d[(i + 2) & 7]) : "s20", "s21", "scc");
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 21) {  // v_fma_f64, each followed by one s_waitcnt (nothing outstanding)
#define F(i) asm volatile("v_fma_f64 %0, %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "+v"(d[i]) : "v"(d[(i + 1) & 7]), "v"(d[(i + 2) & 7]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 22) {  // v_fma_f64, each followed by one s_setprio
#define F(i) asm volatile("v_fma_f64 %0, %0, %1, %2\n\ts_setprio 1" : "+v"(d[i]) : "v"(d[(i + 1) & 7]), "v"(d[(i + 2) & 7]));
        REP8(F) REP8(F)
#undef F
    } else if constexpr (CLS == 11) {  // v_pk_fma_f32
#define F(i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(q[i]) : "v"(q[(i + 1) & 7]), "v"(q[(i + 2) & 7]));
        REP8(F) REP8(F)
#undef F
    }
}

// MIX: class A on waves 0..7, class B on waves 8..15 (two of each per SIMD)
template <int A, int B, int T = 1024>
__global__ void __launch_bounds__(T, 1) k(double *out, int iters) {
    __shared__ double sm[2048];  // 16 KiB: the LDS class reads addresses below 0x4000
    if (iters < 0) sm[threadIdx.x & 2047] = 1.0;
    if (iters < -1) out[0] = sm[5];
    double d[8];
    unsigned u[8];
    unsigned long long q[8];
    for (int i = 0; i < 8; i++) {
        d[i] = threadIdx.x * 1e-3 + i;
        u[i] = threadIdx.x * 7 + i;
        q[i] = (unsigned long long)threadIdx.x * 13 + i;
    }
    const bool first = (threadIdx.x >> 6) < (T / 128 > 0 ? T / 128 : 1) || T == 64;
    for (int it = 0; it < iters; it++) {
        if (first)
            body<A>(d, u, q);
        else
            body<B>(d, u, q);
    }
    double s = 0;
    for (int i = 0; i < 8; i++) s += d[i] + (double)u[i] + (double)q[i];
    out[blockIdx.x * T + threadIdx.x] = s;
}

template <int A, int B, int T = 1024>
float run(double *d, int blocks, int iters) {
    k<A, B, T><<<blocks, T>>>(d, 4);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    k<A, B, T><<<blocks, T>>>(d, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

static const char *names[] = {"v_fma_f64", "v_add_u32", "v_lshlrev_b64", "v_permlane32_swap", "v_add_f64",
                              "v_pk_add_u16", "v_cvt_f64_i32", "v_mul_lo_u32", "v_lshl_add_u64", "v_cndmask_b32",
                              "v_mov_b32", "v_pk_fma_f32", "fma_f64 dep1", "v_mov_dpp", "cndmask_sgpr", "fma_f64 dep2",
                              "v_cndmask_dpp", "v_permlane16_swap", "v_mul_f64", "fma_f64+salu", "fma_f64+2salu",
                              "fma_f64+s_waitcnt", "fma_f64+s_setprio"};

template <int A, int B, int T = 1024>
void report(double *d, int blocks, int iters, double ghz) {
    const float ms = run<A, B, T>(d, blocks, iters);
    // per SIMD: T/256 waves x iters x 16 instructions; one block per CU, blocks = CUs
    const double instr_per_simd = (T / 256.0) * iters * 16.0;
    const double cyc = ms * 1e-3 * ghz * 1e9 / instr_per_simd;
    printf("T=%4d %-18s + %-18s: %8.3f ms  %.2f cycles per wave-instruction per SIMD (at %.2f GHz)\n", T, names[A], names[B], ms, cyc, ghz);
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int clk = 0;
    (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    const double ghz = clk / 1e6;
    double *d;
    (void)hipMalloc(&d, sizeof(double) * cus * 1024);
    const int iters = 20000;
    printf("CUs %d, clock attribute %.3f GHz\n", cus, ghz);
    report<0, 0>(d, cus, iters, ghz);
    report<4, 4>(d, cus, iters, ghz);
    report<1, 1>(d, cus, iters, ghz);
    report<2, 2>(d, cus, iters, ghz);
    report<3, 3>(d, cus, iters, ghz);
    report<5, 5>(d, cus, iters, ghz);
    report<6, 6>(d, cus, iters, ghz);
    report<7, 7>(d, cus, iters, ghz);
    report<8, 8>(d, cus, iters, ghz);
    report<9, 9>(d, cus, iters, ghz);
    report<10, 10>(d, cus, iters, ghz);
    report<11, 11>(d, cus, iters, ghz);
    // mixes: f64 fma on half the waves, the other class on the other half
    report<0, 1>(d, cus, iters, ghz);
    report<0, 2>(d, cus, iters, ghz);
    report<0, 3>(d, cus, iters, ghz);
    report<0, 5>(d, cus, iters, ghz);
    report<0, 8>(d, cus, iters, ghz);
    report<0, 10>(d, cus, iters, ghz);
    report<0, 11>(d, cus, iters, ghz);
    // one and two waves per SIMD (T = 256, 512)
    report<0, 0, 256>(d, cus, iters, ghz);
    report<0, 0, 512>(d, cus, iters, ghz);
    report<4, 4, 256>(d, cus, iters, ghz);
    report<1, 1, 256>(d, cus, iters, ghz);
    report<1, 1, 512>(d, cus, iters, ghz);
    report<10, 10, 256>(d, cus, iters, ghz);
    report<3, 3, 256>(d, cus, iters, ghz);
    report<12, 12, 1024>(d, cus, iters, ghz);
    report<12, 12, 256>(d, cus, iters, ghz);
    report<13, 13, 1024>(d, cus, iters, ghz);
    report<13, 13, 256>(d, cus, iters, ghz);
    report<0, 13, 1024>(d, cus, iters, ghz);
    report<14, 14, 1024>(d, cus, iters, ghz);
    report<15, 15, 1024>(d, cus, iters, ghz);
    report<15, 15, 256>(d, cus, iters, ghz);
    report<16, 16, 1024>(d, cus, iters, ghz);
    report<17, 17, 1024>(d, cus, iters, ghz);
    report<18, 18, 1024>(d, cus, iters, ghz);
    report<0, 16, 1024>(d, cus, iters, ghz);
    report<0, 17, 1024>(d, cus, iters, ghz);
    // does a wave's non-VALU instruction cost VALU issue? (cycles per f64 instruction)
    report<19, 19, 1024>(d, cus, iters, ghz);
    report<20, 20, 1024>(d, cus, iters, ghz);
    report<21, 21, 1024>(d, cus, iters, ghz);
    report<22, 22, 1024>(d, cus, iters, ghz);
    report<19, 19, 256>(d, cus, iters, ghz);
    return 0;
}
