// Probe: price of the per-CMux-step hand-off a two-CU split of one ciphertext's blind rotation would need
// (br512lat, one AES block = 128 ciphertexts on 256 CUs).  256 workgroups of 1024 threads, one per CU
// (LDS-sized), in pairs (b, b ^ 8: same XCD).  Every step each workgroup publishes PAY bytes of partial
// spectra and reads its partner's, in the cheapest valid form of MI355X_MICROARCH.md's hand-off table
// (row 1): 8-byte `sc1` stores (relaxed agent-scope atomic stores), every storing wave's vmcnt drain,
// a workgroup barrier, one lane's `sc1` flag store; the partner's lane 0 polls the flag with `sc1` loads
// and s_sleep (bounded, so a missing partner cannot hang the kernel), a barrier, then `sc1` loads of the
// payload.  work_iters of FP64 work per step stand for the halved FFT / MAC phases.  Reports µs per step
// for PAY in {0 (flag only), 4 KB, 10 KB, 20 KB}, with and without the work, and the work alone.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int THREADS = 1024, STEPS = 677;

__global__ void __launch_bounds__(THREADS, 1)
    k(unsigned long long *pay, unsigned *flags, int pay8, int work_iters, int do_sync, unsigned *err, double *sink) {
    extern __shared__ unsigned long long lds[];
    const int b = blockIdx.x, partner = b ^ 8, tid = threadIdx.x;
    double acc = tid * 1e-3, x = 1.0 + tid * 1e-9;
    unsigned long long in = 0;
    for (int s = 1; s <= STEPS; s++) {
        // stand-in for the phase work (dependent FMAs, four chains per thread)
        double a0 = acc, a1 = acc + 1, a2 = acc + 2, a3 = acc + 3;
        for (int i = 0; i < work_iters; i++) {
            a0 = fma(a0, x, 1e-9);
            a1 = fma(a1, x, 1e-9);
            a2 = fma(a2, x, 1e-9);
            a3 = fma(a3, x, 1e-9);
        }
        acc = a0 + a1 + a2 + a3 + (double)(in & 1);
        if (!do_sync) continue;
        // publish this step's payload (parity of s selects the buffer half: the partner may still read s-1)
        unsigned long long *mine = pay + ((size_t)b * 2 + (s & 1)) * pay8;
        for (int t = tid; t < pay8; t += THREADS)
            __hip_atomic_store(&mine[t], (unsigned long long)s * 1000 + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store(&flags[b], (unsigned)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // wait for the partner's step s (bounded spin)
        if (tid == 0) {
            int spins = 0;
            while (__hip_atomic_load(&flags[partner], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)s) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1 << 16)) {
                    atomicAdd(err, 1u);
                    break;
                }
            }
        }
        __syncthreads();
        unsigned long long *theirs = pay + ((size_t)partner * 2 + (s & 1)) * pay8;
        for (int t = tid; t < pay8; t += THREADS) {
            in = __hip_atomic_load(&theirs[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (in != (unsigned long long)s * 1000 + t) atomicAdd(err + 1, 1u);  // stale word
            lds[t] = in;
        }
        __syncthreads();
    }
    sink[b * THREADS + tid] = acc + (double)in;
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = 256;
    if (cus < blocks) {
        printf("needs %d CUs, found %d\n", blocks, cus);
        return 1;
    }
    unsigned long long *pay;
    unsigned *flags, *err;
    double *sink;
    const int max8 = 20480 / 8;
    (void)hipMalloc(&pay, sizeof(unsigned long long) * blocks * 2 * max8);
    (void)hipMalloc(&flags, sizeof(unsigned) * blocks);
    (void)hipMalloc(&err, 2 * sizeof(unsigned));
    (void)hipMalloc(&sink, sizeof(double) * blocks * THREADS);
    const size_t lds = 100 * 1024;  // one workgroup per CU
    (void)hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int pays[] = {0, 4096, 10240, 20480};
    for (int work : {0, 64}) {
        for (int sync = 0; sync <= 1; sync++) {
            for (int pi = 0; pi < 4; pi++) {
                if (!sync && pi) break;
                const int p8 = pays[pi] / 8;
                (void)hipMemset(flags, 0, sizeof(unsigned) * blocks);
                (void)hipMemset(err, 0, 2 * sizeof(unsigned));
                (void)hipDeviceSynchronize();
                (void)hipEventRecord(e0);
                k<<<blocks, THREADS, lds>>>(pay, flags, p8, work, sync, err, sink);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                float ms;
                (void)hipEventElapsedTime(&ms, e0, e1);
                unsigned herr[2] = {0, 0};
                (void)hipMemcpy(herr, err, sizeof herr, hipMemcpyDeviceToHost);
                printf("work_iters %3d  hand-off %s  payload %5d B: %7.3f us per step  (timeouts %u, stale words %u)\n",
                       work, sync ? "yes" : "no ", sync ? pays[pi] : 0, ms * 1e3 / STEPS, herr[0], herr[1]);
            }
        }
    }
    return 0;
}
