// Stand-alone A/B timing of GEMM kernel variants (no torch): hipEvent timing of two
// builds of csrc/kernels/gemm_big.hip linked side by side (the second compiled with
// -Dddl_gemm_big2=ddl_gemm_big3 and different -D switches), plus an older object as
// ddl_gemm_big.  Build: see profiles/README.md (gemm_ab_*.log).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstring>
#include <cstdint>

extern "C" int ddl_gemm_big2(int mode, const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M,
                             int N, int K, const void* bias, int bias_bf16, int act, void* aux, int out_f32,
                             int splits, void* ws, long ws_elems, const int* conv, int row_remap, const void* res,
                             int accumulate, const void* zero, float* colstats, hipStream_t st);
extern "C" int ddl_gemm_big3(int mode, const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M,
                             int N, int K, const void* bias, int bias_bf16, int act, void* aux, int out_f32,
                             int splits, void* ws, long ws_elems, const int* conv, int row_remap, const void* res,
                             int accumulate, const void* zero, float* colstats, hipStream_t st);
extern "C" int ddl_gemm_big(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                            const void* bias, int bias_bf16, int act, void* aux, int accumulate, hipStream_t st);

int main() {
    const int shapes[][3] = {{16384, 2304, 768}, {16384, 768, 768}, {16384, 3072, 768}, {16384, 768, 3072},
                             {4096, 4096, 4096}, {8192, 8192, 8192}};
    void *A, *B, *C, *Z;
    (void)ddl_gemm_big;
    hipMalloc(&A, 8192L * 8192 * 2);
    hipMalloc(&B, 8192L * 8192 * 2);
    hipMalloc(&C, 8192L * 8192 * 2);
    hipMalloc(&Z, 256);
    {   // uniform random bf16 in [-1, 1) (constant operands read high)
        std::vector<uint16_t> h(8192L * 8192);
        uint32_t s = 12345;
        for (auto& v : h) {
            s = s * 1664525u + 1013904223u;
            const float f = ((s >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;
            uint32_t u;
            memcpy(&u, &f, 4);
            v = (uint16_t)(u >> 16);
        }
        hipMemcpy(A, h.data(), h.size() * 2, hipMemcpyHostToDevice);
        hipMemcpy(B, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    }
    hipMemset(Z, 0, 256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // mode 0 NT: C[M,N] = A[M,K] B[N,K]^T; mode 1 NN: A[M,K], B[K,N] (KO); mode 2 TN: A[K,M] (KO), B[K,N] (KO)
    struct Case { int mode, M, N, K, splits; };
    const Case cases[] = {
        {0, 16384, 2304, 768, 1}, {0, 16384, 768, 768, 1}, {0, 16384, 3072, 768, 1}, {0, 16384, 768, 3072, 1},
        {0, 4096, 4096, 4096, 1}, {0, 8192, 8192, 8192, 1},
        {1, 16384, 768, 2304, 1}, {1, 16384, 768, 768, 1}, {1, 16384, 3072, 768, 1}, {1, 16384, 768, 3072, 1},
        {1, 4096, 4096, 4096, 1},
        {2, 2304, 768, 16384, 4}, {2, 768, 768, 16384, 8}, {2, 3072, 768, 16384, 4}, {2, 768, 3072, 16384, 4},
        {2, 4096, 4096, 4096, 1}};
    float* ws;
    hipMalloc(&ws, 8L * 4096 * 4096 * 4);
    for (const Case& c : cases) {
        const int M = c.M, N = c.N, K = c.K;
        const long lda = c.mode == 2 ? M : K;
        const long ldb = c.mode == 0 ? K : N;
        for (int v = 1; v < 3; ++v) {
            auto run = [&] {
                auto f = v == 1 ? ddl_gemm_big2 : ddl_gemm_big3;
                f(c.mode, A, lda, B, ldb, C, N, M, N, K, nullptr, 0, 0, nullptr, 0, c.splits, ws, 8L * 4096 * 4096,
                  nullptr, 0, nullptr, 0, Z, nullptr, 0);
            };
            for (int i = 0; i < 5; ++i) run();
            hipEventRecord(e0, 0);
            const int it = 50;
            for (int i = 0; i < it; ++i) run();
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            ms /= it;
            printf("%s mode=%d M=%d N=%d K=%d splits=%d  %.4f ms  %.1f TF\n", v == 1 ? "old" : "new", c.mode, M, N, K,
                   c.splits, ms, 2.0 * M * N * K / ms / 1e9);
        }
    }
    return 0;
}
