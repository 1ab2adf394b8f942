// Common device helpers for the gfx950 (MI355X, CDNA4) kernels.
//
// Conventions: wave64 everywhere (hard-coded 64, never 32), bf16 stored as raw
// 16-bit payloads, every memory-bound kernel moves 16 bytes per lane.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

#define DDL_API extern "C" __attribute__((visibility("default")))
#define DDL_WAVE 64

typedef uint16_t bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// Launch-error helper: every C entry point returns the HIP error code (0 = ok).
#define DDL_RETURN_LAUNCH() return (int)hipGetLastError()

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// Round-to-nearest-even; NaN stays NaN.  hipcc lowers the __bf16 cast to
// v_cvt_pk_bf16_f32 on gfx950.
__device__ __forceinline__ bf16_t f2bf(float f) {
    __bf16 h = (__bf16)f;
    return __builtin_bit_cast(bf16_t, h);
}

__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
    return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

// 8 bf16 <-> 8 floats through one 16-byte access.
__device__ __forceinline__ void load8(const bf16_t* p, float* v) {
    uint4 u = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}
// the same load with the non-temporal cache policy: for a pass that is the LAST reader of a tensor
// too large for the caches to keep anyway
__device__ __forceinline__ void load8_nt(const bf16_t* p, float* v) {
    typedef uint32_t u32v4 __attribute__((ext_vector_type(4)));
    const u32v4 u = __builtin_nontemporal_load(reinterpret_cast<const u32v4*>(p));
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}
__device__ __forceinline__ void load8_nt(const float* p, float* v) {
    typedef float f32v4 __attribute__((ext_vector_type(4)));
    const f32v4 a = __builtin_nontemporal_load(reinterpret_cast<const f32v4*>(p));
    const f32v4 b = __builtin_nontemporal_load(reinterpret_cast<const f32v4*>(p) + 1);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void store8(bf16_t* p, const float* v) {
    uint4 u;
    u.x = pack2bf(v[0], v[1]);
    u.y = pack2bf(v[2], v[3]);
    u.z = pack2bf(v[4], v[5]);
    u.w = pack2bf(v[6], v[7]);
    *reinterpret_cast<uint4*>(p) = u;
}
__device__ __forceinline__ void load8(const float* p, float* v) {
    float4 a = reinterpret_cast<const float4*>(p)[0];
    float4 b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void store8(float* p, const float* v) {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void load4(const bf16_t* p, float* v) {
    uint2 u = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
}
__device__ __forceinline__ void store4(bf16_t* p, const float* v) {
    uint2 u; u.x = pack2bf(v[0], v[1]); u.y = pack2bf(v[2], v[3]);
    *reinterpret_cast<uint2*>(p) = u;
}
__device__ __forceinline__ void load4(const float* p, float* v) {
    float4 a = *reinterpret_cast<const float4*>(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}
__device__ __forceinline__ void store4(float* p, const float* v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ float to_f(bf16_t x) { return bf2f(x); }
__device__ __forceinline__ float to_f(float x) { return x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16_t from_f<bf16_t>(float x) { return f2bf(x); }

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64); `red` holds NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += red[i];
    __syncthreads();
    return t;
}

// ---------------------------------------------------------------- math
// GELU / GELU' for the epilogues: the Abramowitz & Stegun 7.1.26 erf (|error| <= 1.5e-7,
// far below bf16 resolution) -- one reciprocal, one exponential and a degree-5 Horner
// chain, branch-free.  With x = z / sqrt(2), t = 1 / (1 + p |x|) and
// erf(x) = sign(x) (1 - t P(t) e^{-x^2}):
//   GELU(z)  = max(z, 0) - w,            w = 0.5 |z| t P(t) e^{-z^2/2}
//   GELU'(z) = 0.5 + copysign(0.5 - 0.5 t P(t) e^{-z^2/2}, z) + z phi(z)
// (no copysign/1+ on the GELU path; the grad shares the one exponential with phi).
// The *2 forms run two elements as packed f32 (v_pk_fma / v_pk_mul: half the issue
// cycles of scalar f32 VALU): the FFN GEMM epilogues evaluate them for 128 values per
// lane per output tile with no MFMA to hide behind, where they were the main cost.
typedef float f32x2_t __attribute__((ext_vector_type(2)));
namespace gelu_c {
constexpr float P1 = 0.3275911f * 0.70710678118654752f;   // p / sqrt(2)
constexpr float A1 = 0.254829592f, A2 = -0.284496736f, A3 = 1.421413741f, A4 = -1.453152027f,
                A5 = 1.061405429f;
constexpr float NH_LOG2E = -0.5f * 1.4426950408889634f;    // e^{-z^2/2} = 2^{z * (z * NH_LOG2E)}
constexpr float INV_SQRT_2PI = 0.3989422804014327f;
}  // namespace gelu_c
__device__ __forceinline__ f32x2_t gelu_erf2(f32x2_t z) {
    using namespace gelu_c;
    const f32x2_t a = {fabsf(z.x), fabsf(z.y)};
    const f32x2_t d = a * P1 + 1.f;
    const f32x2_t t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
    f32x2_t q = t * (0.5f * A5) + (0.5f * A4);
    q = q * t + (0.5f * A3);
    q = q * t + (0.5f * A2);
    q = q * t + (0.5f * A1);
    const f32x2_t s = (z * NH_LOG2E) * z;
    const f32x2_t e = {__builtin_amdgcn_exp2f(s.x), __builtin_amdgcn_exp2f(s.y)};
    const f32x2_t w = (a * t) * (q * e);
    const f32x2_t r = {fmaxf(z.x, 0.f), fmaxf(z.y, 0.f)};
    return r - w;
}
__device__ __forceinline__ f32x2_t gelu_erf_grad2(f32x2_t z) {
    using namespace gelu_c;
    const f32x2_t a = {fabsf(z.x), fabsf(z.y)};
    const f32x2_t d = a * P1 + 1.f;
    const f32x2_t t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
    f32x2_t q = t * (-0.5f * A5) + (-0.5f * A4);
    q = q * t + (-0.5f * A3);
    q = q * t + (-0.5f * A2);
    q = q * t + (-0.5f * A1);
    const f32x2_t s = (z * NH_LOG2E) * z;
    const f32x2_t e = {__builtin_amdgcn_exp2f(s.x), __builtin_amdgcn_exp2f(s.y)};
    const f32x2_t h = (q * t) * e + 0.5f;   // 0.5 - 0.5 t P e, in [0, 0.5]
    const f32x2_t c = {copysignf(h.x, z.x), copysignf(h.y, z.y)};
    return (z * INV_SQRT_2PI) * e + c + 0.5f;
}
__device__ __forceinline__ float gelu_erf(float z) {
    using namespace gelu_c;
    const float a = fabsf(z), t = __builtin_amdgcn_rcpf(a * P1 + 1.f);
    const float q = (((t * (0.5f * A5) + (0.5f * A4)) * t + (0.5f * A3)) * t + (0.5f * A2)) * t + (0.5f * A1);
    return fmaxf(z, 0.f) - (a * t) * (q * __builtin_amdgcn_exp2f((z * NH_LOG2E) * z));
}
__device__ __forceinline__ float gelu_erf_grad(float z) {
    using namespace gelu_c;
    const float t = __builtin_amdgcn_rcpf(fabsf(z) * P1 + 1.f);
    const float q = (((t * (-0.5f * A5) + (-0.5f * A4)) * t + (-0.5f * A3)) * t + (-0.5f * A2)) * t + (-0.5f * A1);
    const float e = __builtin_amdgcn_exp2f((z * NH_LOG2E) * z);
    return (z * INV_SQRT_2PI) * e + copysignf((q * t) * e + 0.5f, z) + 0.5f;
}

// Counter-based dropout RNG: masks are regenerated in backward, never stored.  ONE
// "lowbias32" integer-finaliser round (xor-shift / 32-bit multiply) per PAIR of
// consecutive element indices (idx >> 1), each element thresholded on its 16-bit half
// (the low half for even idx): P(keep) = 1 - thresh16 / 65536.  About 4 VALU ops per
// element -- cheap enough inside bandwidth-bound LayerNorm / attention passes, where a
// two-round hash per element was VALU-bound.
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ uint32_t pair_hash(uint64_t seed, uint64_t pidx) {
    uint32_t x = (uint32_t)pidx ^ (uint32_t)seed;
    x += (uint32_t)(pidx >> 32) * 0x9E3779B9u + (uint32_t)(seed >> 32);
    return lowbias32(x);
}
__host__ __device__ __forceinline__ uint32_t drop_thresh16(float p) {
    const float t = p * 65536.f;
    return t >= 65536.f ? 65536u : (t <= 0.f ? 0u : (uint32_t)t);
}
__device__ __forceinline__ bool keep_half(uint32_t h, uint64_t idx, uint32_t thresh16) {
    return ((h >> ((uint32_t)(idx & 1) * 16)) & 0xffffu) >= thresh16;
}
__device__ __forceinline__ bool keep_elem(uint64_t seed, uint64_t idx, uint32_t thresh16) {
    return keep_half(pair_hash(seed, idx >> 1), idx, thresh16);
}
// keep bits of elements i0 .. i0+3, i0 even (bit j = element i0 + j): two hashes
__device__ __forceinline__ uint32_t keep_bits4(uint64_t seed, uint64_t i0, uint32_t thresh16) {
    const uint32_t h0 = pair_hash(seed, i0 >> 1), h1 = pair_hash(seed, (i0 >> 1) + 1);
    return (uint32_t)((h0 & 0xffffu) >= thresh16) | ((uint32_t)((h0 >> 16) >= thresh16) << 1) |
           ((uint32_t)((h1 & 0xffffu) >= thresh16) << 2) | ((uint32_t)((h1 >> 16) >= thresh16) << 3);
}

// BatchNorm-backward GEMM epilogue (ACT_BNB) side arguments: the BN's ReLU bit mask
// (nullable), saved mean and inverse std.  Set on the launching host thread by
// ddl_gemm_bnb(), consumed by the next GEMM entry call (gemm.hip / gemm_big.hip).
struct BnbArgs {
    const uint8_t* mask;
    const float* mean;
    const float* istd;
};
BnbArgs ddl_take_bnb();

// Sum over the 16 lanes of a DPP row (every lane of the row gets the total):
// xor 1, xor 2 (quad_perm), then half-row and row mirrors -- four DPP adds, no LDS.
template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
    return v + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF,
                                                                     false));
}
__device__ __forceinline__ float row16_sum(float v) {
    v = dpp_add<0xB1>(v);    // quad_perm [1,0,3,2]
    v = dpp_add<0x4E>(v);    // quad_perm [2,3,0,1]
    v = dpp_add<0x141>(v);   // row_half_mirror
    return dpp_add<0x140>(v);   // row_mirror
}
// Whole-wave sum with no LDS traffic: the 16-lane row sums (DPP), then gfx950's
// v_permlane16_swap / v_permlane32_swap exchange rows (0,1), (2,3) and the two halves -- each
// lane adds its own value and its partner's, so every lane ends with the wave's sum.  Six
// dependent VALU steps instead of the six ds_bpermute round trips (and their LDS bank cycles)
// of the __shfl_xor tree.  All 64 lanes must be active.
__device__ __forceinline__ float wave_sum_dpp(float v) {
    v = row16_sum(v);
    const uint32_t u = __float_as_uint(v);
    const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const uint32_t w = __float_as_uint(v);
    const auto b = __builtin_amdgcn_permlane32_swap(w, w, false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Fast unsigned division by a runtime constant (magic multiply), for index math
// in hot loops: q = umulhi(n, mul) >> shift, exact for n < 2^31.
struct FastDiv {
    uint32_t d, mul, shift;
};
__host__ inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f; f.d = d;
    uint32_t s = 0;
    while ((1ull << s) < d) ++s;
    f.shift = s;
    f.mul = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
    if (d == 1) { f.mul = 0; f.shift = 0; }
    return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, FastDiv f) {
    if (f.d == 1) return n;
    uint32_t t = __umulhi(n, f.mul);
    return (t + n) >> f.shift;
}

// Column sum over the rows of a row-major fp32 matrix part[nrows][ld] (per-block
// partials of a two-level reduction).  Block = 1024 threads = 64 columns x 16 row
// groups; each lane keeps 4 independent loads in flight.  `red` holds 1024 floats.
// Result valid in threads 0..63 (column `col` = the caller's column for lane t&63).
__device__ __forceinline__ float colsum64(const float* __restrict__ part, int nrows, long ld, int col, bool ok,
                                          float* red) {
    const int grp = threadIdx.x >> 6;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    if (ok) {
        int r = grp;
        // eight rows in flight per thread (the partial rows were just written: L2 latency,
        // not bandwidth, bounds this loop -- a few hundred rows take 2-4 round trips)
        for (; r + 112 < nrows; r += 128) {
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = part[(long)(r + 16 * i) * ld + col];
            a0 += v[0] + v[4];
            a1 += v[1] + v[5];
            a2 += v[2] + v[6];
            a3 += v[3] + v[7];
        }
        for (; r < nrows; r += 16) a0 += part[(long)r * ld + col];
    }
    red[threadIdx.x] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    float s = 0.f;
    if (threadIdx.x < 64) {
#pragma unroll
        for (int i = 0; i < 16; ++i) s += red[i * 64 + threadIdx.x];
    }
    __syncthreads();
    return s;
}
