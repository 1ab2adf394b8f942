// MFMA shape study for the GEMM main loop: v_mfma_f32_16x16x32_bf16 (what every
// kernel of this library issues) against v_mfma_f32_32x32x16_bf16, in the GEMM main loop's regime --
// each wave owns a 64 x 64 output tile and re-reads its A / B fragments from an LDS image every k-step
// with ds_read_b128 (8 per 32-deep k-step for BOTH shapes: the same LDS bytes per FLOP, since those
// are set by the wave tile, not by the instruction), two waves per SIMD as in the 8-phase kernels,
// uniform random [-1, 1) operands (zero operands let the chip hold a higher clock: rule 25).
//
//   hipcc -O3 --offload-arch=gfx950 csrc/bench/mfma_shape_bench.cpp -o build/mfma_shape_bench
//   ./build/mfma_shape_bench            (stand-alone: no torch, hipEvent timing, interleaved rounds)
//
// Per variant: TFLOP/s over the whole grid (one 8-wave workgroup per CU) and the
// in-kernel clock (s_memtime / s_memrealtime ratio, stamped by lane 0 of wave 0 of each workgroup into a
// buffer of its own -- never into an output).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

constexpr int NT = 512;            // 8 waves: two per SIMD
constexpr int IMG = 64 * 1024;     // LDS operand image (bytes), filled once from global memory
constexpr int KSTEPS = 4096;       // 32-deep k-steps per wave

// fragment read: 16 bytes per lane, lane l at l * 16 of a 1 KB block (a conflict-free ds_read_b128
// for both variants: what a swizzled GEMM image gives; which k / row a lane's bytes stand for does
// not change the timing, only the bit patterns, and both variants read the same random image).
// A first version used the unswizzled fragment offsets (row * 64 + chunk * 16): 2-4-way conflicts
// made BOTH variants LDS-bound (16x16x32 3255, 32x32x16 1998 flop/cycle/CU) -- a layout artefact.
__device__ __forceinline__ bf16x8 rd(const char* img, int off) {
    return *reinterpret_cast<const bf16x8*>(img + (off & (IMG - 16)));
}

template <int SHAPE>
__global__ __launch_bounds__(NT, 1) void mfma_loop_k(const uint4* __restrict__ src, float* __restrict__ out,
                                                     unsigned long long* __restrict__ stamps) {
    __shared__ __attribute__((aligned(16))) char img[IMG];
    for (int i = threadIdx.x; i < IMG / 16; i += NT) reinterpret_cast<uint4*>(img)[i] = src[i];
    __syncthreads();
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    if (SHAPE == 16) {
        f32x4 acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
        const int base = w * 4096 + l * 16;
#pragma unroll 1
        for (int k = 0; k < KSTEPS; ++k) {
            const int o = base + (k & 7) * 1024;
            bf16x8 a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = rd(img, o + i * 1024);
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = rd(img, o + 32768 + j * 1024);
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
        }
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
        out[blockIdx.x * NT + threadIdx.x] = s;
    } else {
        f32x16 acc[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
        const int base = w * 4096 + l * 16;
#pragma unroll 1
        for (int k = 0; k < KSTEPS; ++k) {
            const int o = base + (k & 7) * 1024;
            bf16x8 a[2][2], b[2][2];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) {
                    a[i][kk] = rd(img, o + (2 * i + kk) * 1024);
                    b[i][kk] = rd(img, o + 32768 + (2 * i + kk) * 1024);
                }
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][kk], a[i][kk], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
        }
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) s += acc[i][j][e];
        out[blockIdx.x * NT + threadIdx.x] = s;
    }
    if (threadIdx.x == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
}

int main() {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = ncu;                       // one 8-wave workgroup per CU (64 KB LDS)
    std::vector<uint16_t> h(IMG / 2);
    uint32_t s = 12345;
    for (auto& v : h) {                         // uniform random bf16 in [-1, 1)
        s = s * 1664525u + 1013904223u;
        const float f = ((s >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;
        uint32_t u;
        memcpy(&u, &f, 4);
        v = (uint16_t)(u >> 16);
    }
    uint4* src;
    float* out;
    unsigned long long* st;
    CK(hipMalloc(&src, IMG));
    CK(hipMalloc(&out, (size_t)grid * NT * 4));
    CK(hipMalloc(&st, (size_t)grid * 16));
    CK(hipMemcpy(src, h.data(), IMG, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double flop = 2.0 * 64 * 64 * 32 * KSTEPS * 8 * grid;   // per launch: 8 waves x 64x64 x 32 per k-step
    auto run = [&](int shape, int reps) {
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) {
            if (shape == 16) mfma_loop_k<16><<<grid, NT>>>(src, out, st);
            else mfma_loop_k<32><<<grid, NT>>>(src, out, st);
        }
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<unsigned long long> hs((size_t)grid * 2);
        CK(hipMemcpy(hs.data(), st, hs.size() * 8, hipMemcpyDeviceToHost));
        std::vector<double> clk;
        for (int b = 0; b < grid; ++b)
            if (hs[2 * b + 1]) clk.push_back((double)hs[2 * b] / (double)hs[2 * b + 1] * 0.1);   // GHz (100 MHz ref)
        std::sort(clk.begin(), clk.end());
        return std::make_pair(flop * reps / (ms * 1e-3) / 1e12, clk.empty() ? 0.0 : clk[clk.size() / 2]);
    };
    run(16, 20);
    run(32, 20);                                // warm both, then interleave (rule 24)
    std::vector<double> t16, t32, c16, c32;
    for (int round = 0; round < 7; ++round) {
        auto a = run(16, 40);
        auto b = run(32, 40);
        t16.push_back(a.first); c16.push_back(a.second);
        t32.push_back(b.first); c32.push_back(b.second);
        printf("round %d: 16x16x32 %.0f TF/s (clock %.2f GHz) | 32x32x16 %.0f TF/s (clock %.2f GHz)\n", round, a.first,
               a.second, b.first, b.second);
    }
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    printf("median: 16x16x32 %.0f TF/s @ %.2f GHz, 32x32x16 %.0f TF/s @ %.2f GHz, ratio 16/32 = %.3f\n", med(t16),
           med(c16), med(t32), med(c32), med(t16) / med(t32));
    printf("flop/cycle/CU: 16x16x32 %.0f, 32x32x16 %.0f (peak 4096)\n", med(t16) * 1e12 / (med(c16) * 1e9) / grid,
           med(t32) * 1e12 / (med(c32) * 1e9) / grid);
    return 0;
}
