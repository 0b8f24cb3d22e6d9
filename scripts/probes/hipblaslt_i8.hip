// Probe: hipBLASLt int8 GEMM (int32 accumulate) on the PFKS shape, to price a library GEMM + separate
// limb-recombination epilogue against the hand-written ksgemm::gemm_g6 (15.9 ms per launch).
// C[M][N] = A[M][K] . B[N][K]^T, M = 16384 ciphertexts, N = 102400 (5 keys x 2560 columns x 8 limbs),
// K = 10304 (2049 coefficients x 5 digit-limb slots, padded).  Timing only: random operands.
// build: hipcc -O2 --offload-arch=gfx950 -x hip scripts/probes/hipblaslt_i8.hip -lhipblaslt -o scripts/probes/hblt
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        auto e_ = (x);                                                                     \
        if ((int)e_ != 0) {                                                                \
            std::printf("error %d at %s:%d\n", (int)e_, __FILE__, __LINE__);               \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

int main(int argc, char **argv) {
    const long M = argc > 1 ? atol(argv[1]) : 16384, N = argc > 2 ? atol(argv[2]) : 102400,
               K = argc > 3 ? atol(argv[3]) : 10304;
    int8_t *A, *B;
    int32_t *C;
    CK(hipMalloc(&A, M * K));
    CK(hipMalloc(&B, N * K));
    CK(hipMalloc(&C, M * N * 4));
    CK(hipMemset(A, 1, M * K));
    CK(hipMemset(B, 3, N * K));
    hipblasLtHandle_t h;
    CK(hipblasLtCreate(&h));
    // column-major view: C^T[N][M] = B[N][K] . A^T  ->  op(A)=T on B (K x N col-major), op(B)=N on A
    hipblasLtMatmulDesc_t desc;
    CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32I, HIP_R_32I));
    hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
    hipblasLtMatrixLayout_t la, lb, lc;
    CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_8I, K, N, K));  // B stored N rows of K -> K x N col-major
    CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_8I, K, M, K));  // A stored M rows of K -> K x M col-major
    CK(hipblasLtMatrixLayoutCreate(&lc, HIP_R_32I, N, M, N));
    hipblasLtMatmulPreference_t pref;
    CK(hipblasLtMatmulPreferenceCreate(&pref));
    size_t ws = 256ull << 20;
    void *wsp;
    CK(hipMalloc(&wsp, ws));
    CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws)));
    std::vector<hipblasLtMatmulHeuristicResult_t> res(16);
    int nres = 0;
    CK(hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, lc, lc, pref, 16, res.data(), &nres));
    std::printf("M %ld N %ld K %ld: %d algorithms\n", M, N, K, nres);
    int32_t alpha = 1, beta = 0;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int a = 0; a < nres; a++) {
        float best = 1e30f;
        bool ok = true;
        for (int it = 0; it < 4 && ok; it++) {
            CK(hipEventRecord(e0, 0));
            if (hipblasLtMatmul(h, desc, &alpha, B, la, A, lb, &beta, C, lc, C, lc, &res[a].algo, wsp, ws, 0) != 0)
                ok = false;
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it > 0 && ms < best) best = ms;
        }
        if (!ok) {
            std::printf("algo %d: failed\n", a);
            continue;
        }
        std::printf("algo %d: %.3f ms  %.2f POP/s\n", a, best, 2.0 * M * N * K / best / 1e9 / 1e3);
    }
    int32_t probe;
    CK(hipMemcpy(&probe, C, 4, hipMemcpyDeviceToHost));
    std::printf("C[0] = %d (expect %ld)\n", probe, 3L * K);
    return 0;
}
