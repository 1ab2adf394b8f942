// Diagnostics kernels (not on the training path).
//
// ddl_occupy: a stand-in for a concurrent RCCL collective.  RCCL's channel blocks
// stay resident on their CUs for the whole collective; this kernel parks `nblocks`
// 256-thread workgroups (96 KB of LDS each, so at most one per CU) for `usec`
// microseconds, measured on the constant 100 MHz real-time counter.  Timing a GEMM
// beside it on another stream shows what a persistent kernel loses when some CUs
// are taken (benchmarks/comm_overlap.py).
#include "ddl_common.h"

namespace {

__global__ __launch_bounds__(256) void occupy_k(float usec, int* sink) {
    __shared__ float pad[96 * 1024 / 4];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t ticks = (uint64_t)(usec * 100.f);      // 100 MHz
    float acc = 0.f;
    for (int i = threadIdx.x; i < 96 * 1024 / 4; i += 256) pad[i] = (float)i;
    __syncthreads();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
        __builtin_amdgcn_s_sleep(8);
        acc += pad[(threadIdx.x * 37) & (96 * 1024 / 4 - 1)];
    }
    if (acc == -1.f) sink[threadIdx.x] = 1;   // never true: keeps the loop body
}

}  // namespace

DDL_API int ddl_occupy(int nblocks, float usec, int* sink, hipStream_t st) {
    if (nblocks <= 0) return 0;
    occupy_k<<<nblocks, 256, 0, st>>>(usec, sink);
    DDL_RETURN_LAUNCH();
}
