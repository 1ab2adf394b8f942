// Fused flat-arena optimizer steps for gfx950 (kernel families K12/K20/K21/K22).
//
// The whole model's parameters / gradients / optimizer state are flat arrays
// with one layout (optim/arena.py), so a step is ONE launch over the arena.  A
// block table int32[nblk][4] = (start, len | decay << 30, tensor_index, param_delta)
// maps each 256-thread block to <= 8192 contiguous elements of a single tensor,
// which gives per-tensor hyper-parameters (weight-decay masks, LAMB trust ratios)
// without per-tensor launches.  Each lane moves 8 elements per access.
//
// `start` indexes the optimizer's own (local) arrays -- gradient, fp32 master,
// moments; the compute-dtype parameter copy is written at start + param_delta.
// Unsharded, local == arena and the delta is 0; a ZeRO-1 rank owns one chunk per
// gradient bucket, stored back to back locally, and each chunk's rows carry the
// offset of that chunk in the arena.
//
// Gradients may be bf16 or fp32; the fp32 master weights are updated in place
// and, when the model computes in bf16, the bf16 copy is written in the same
// pass (no separate cast kernel).  The gradient multiplier (1/world, 1/accum,
// clip factor) is read from device memory so no host sync is needed.
#include "ddl_common.h"

namespace {

constexpr int OPT_NT = 256;

template <typename G>
__device__ __forceinline__ void load_grad8(const G* g, long i, float* v) { load8(g + i, v); }

template <typename G, typename P>
__global__ __launch_bounds__(OPT_NT) void sgd_k(const G* __restrict__ grad, float* __restrict__ master,
                                                 P* __restrict__ param, float* __restrict__ mom,
                                                 const int4* __restrict__ table, const float* __restrict__ scale_p,
                                                 float lr, float mu, float wd, int nesterov, int first) {
    const int4 e = table[blockIdx.x];
    const int len = e.y & 0x3fffffff;
    const bool dec = (e.y >> 30) & 1;
    const float scale = scale_p[0];
    for (int k = threadIdx.x * 8; k < len; k += OPT_NT * 8) {
        const long i = (long)e.x + k;
        float g[8], p[8], b[8];
        load_grad8(grad, i, g);
        load8(master + i, p);
        if (mu != 0.f && !first) load8(mom + i, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float d = g[j] * scale;
            if (dec) d += wd * p[j];
            if (mu != 0.f) {
                b[j] = first ? d : mu * b[j] + d;
                d = nesterov ? d + mu * b[j] : b[j];
            }
            p[j] -= lr * d;
        }
        store8(master + i, p);
        if (mu != 0.f) store8(mom + i, b);
        if (param) store8(param + i + e.w, p);
    }
}

template <typename G, typename P>
__global__ __launch_bounds__(OPT_NT) void adamw_k(const G* __restrict__ grad, float* __restrict__ master,
                                                   P* __restrict__ param, float* __restrict__ m_, float* __restrict__ v_,
                                                   const int4* __restrict__ table, const float* __restrict__ scale_p,
                                                   float lr, float b1, float b2, float eps, float wd, float bc1,
                                                   float bc2) {
    const int4 e = table[blockIdx.x];
    const int len = e.y & 0x3fffffff;
    const float scale = scale_p[0];
    const float step_size = lr / bc1;
    const float inv_sqrt_bc2 = rsqrtf(bc2);
    const float decay = ((e.y >> 30) & 1) ? (1.f - lr * wd) : 1.f;
    for (int k = threadIdx.x * 8; k < len; k += OPT_NT * 8) {
        const long i = (long)e.x + k;
        float g[8], p[8], m[8], v[8];
        load_grad8(grad, i, g);
        load8(master + i, p);
        load8(m_ + i, m);
        load8(v_ + i, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float gg = g[j] * scale;
            m[j] = b1 * m[j] + (1.f - b1) * gg;
            v[j] = b2 * v[j] + (1.f - b2) * gg * gg;
            p[j] = p[j] * decay - step_size * m[j] / (sqrtf(v[j]) * inv_sqrt_bc2 + eps);
        }
        store8(master + i, p);
        store8(m_ + i, m);
        store8(v_ + i, v);
        if (param) store8(param + i + e.w, p);
    }
}

// LAMB phase 1: moments + per-tensor ||p||^2 and ||u||^2 (u = m_hat/(sqrt(v_hat)+eps) + wd p)
template <typename G>
__global__ __launch_bounds__(OPT_NT) void lamb_phase1_k(const G* __restrict__ grad, const float* __restrict__ master,
                                                         float* __restrict__ m_, float* __restrict__ v_,
                                                         const int4* __restrict__ table, const float* __restrict__ scale_p,
                                                         float b1, float b2, float eps, float wd, float bc1, float bc2,
                                                         float* __restrict__ norms) {
    __shared__ float red[4];
    const int4 e = table[blockIdx.x];
    const int len = e.y & 0x3fffffff;
    const bool dec = (e.y >> 30) & 1;
    const float scale = scale_p[0];
    float pn = 0.f, un = 0.f;
    for (int k = threadIdx.x * 8; k < len; k += OPT_NT * 8) {
        const long i = (long)e.x + k;
        float g[8], p[8], m[8], v[8];
        load_grad8(grad, i, g);
        load8(master + i, p);
        load8(m_ + i, m);
        load8(v_ + i, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float gg = g[j] * scale;
            m[j] = b1 * m[j] + (1.f - b1) * gg;
            v[j] = b2 * v[j] + (1.f - b2) * gg * gg;
            float u = (m[j] / bc1) / (sqrtf(v[j] / bc2) + eps);
            if (dec) u += wd * p[j];
            pn += p[j] * p[j];
            un += u * u;
        }
        store8(m_ + i, m);
        store8(v_ + i, v);
    }
    pn = block_sum<OPT_NT>(pn, red);
    un = block_sum<OPT_NT>(un, red);
    if (threadIdx.x == 0) {
        atomicAdd(norms + 2 * e.z, pn);
        atomicAdd(norms + 2 * e.z + 1, un);
    }
}

template <typename P>
__global__ __launch_bounds__(OPT_NT) void lamb_phase2_k(float* __restrict__ master, P* __restrict__ param,
                                                         const float* __restrict__ m_, const float* __restrict__ v_,
                                                         const int4* __restrict__ table, float lr, float eps, float wd,
                                                         float bc1, float bc2, const float* __restrict__ norms) {
    const int4 e = table[blockIdx.x];
    const int len = e.y & 0x3fffffff;
    const bool dec = (e.y >> 30) & 1;
    const float pn = sqrtf(norms[2 * e.z]), un = sqrtf(norms[2 * e.z + 1]);
    const float ratio = (pn > 0.f && un > 0.f) ? pn / un : 1.f;
    const float step = lr * ratio;
    for (int k = threadIdx.x * 8; k < len; k += OPT_NT * 8) {
        const long i = (long)e.x + k;
        float p[8], m[8], v[8];
        load8(master + i, p);
        load8(m_ + i, m);
        load8(v_ + i, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float u = (m[j] / bc1) / (sqrtf(v[j] / bc2) + eps);
            if (dec) u += wd * p[j];
            p[j] -= step * u;
        }
        store8(master + i, p);
        if (param) store8(param + i + e.w, p);
    }
}

template <typename G>
__global__ __launch_bounds__(256) void sumsq_k(const G* __restrict__ x, long n8, float* __restrict__ out) {
    __shared__ float red[4];
    float s = 0.f;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
        float v[8];
        load8(x + i * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[j] * v[j];
    }
    s = block_sum<256>(s, red);
    if (threadIdx.x == 0) atomicAdd(out, s);
}

}  // namespace

// gdtype / pdtype: 0 = fp32, 1 = bf16; param may be null (fp32 model: master IS the param)
DDL_API int ddl_sgd_step(int gdtype, const void* grad, float* master, int pdtype, void* param, float* mom,
                         const int* table, int nblk, const float* scale, float lr, float mu, float wd, int nesterov,
                         int first, hipStream_t st) {
    const int4* t = (const int4*)table;
#define SGD_CALL(G, P) sgd_k<G, P><<<nblk, OPT_NT, 0, st>>>((const G*)grad, master, (P*)param, mom, t, scale, lr, mu, wd, nesterov, first)
    if (gdtype == 1) { if (pdtype == 1) SGD_CALL(bf16_t, bf16_t); else SGD_CALL(bf16_t, float); }
    else { if (pdtype == 1) SGD_CALL(float, bf16_t); else SGD_CALL(float, float); }
#undef SGD_CALL
    DDL_RETURN_LAUNCH();
}

DDL_API int ddl_adamw_step(int gdtype, const void* grad, float* master, int pdtype, void* param, float* m, float* v,
                           const int* table, int nblk, const float* scale, float lr, float b1, float b2, float eps,
                           float wd, float bc1, float bc2, hipStream_t st) {
    const int4* t = (const int4*)table;
#define ADAM_CALL(G, P) adamw_k<G, P><<<nblk, OPT_NT, 0, st>>>((const G*)grad, master, (P*)param, m, v, t, scale, lr, b1, b2, eps, wd, bc1, bc2)
    if (gdtype == 1) { if (pdtype == 1) ADAM_CALL(bf16_t, bf16_t); else ADAM_CALL(bf16_t, float); }
    else { if (pdtype == 1) ADAM_CALL(float, bf16_t); else ADAM_CALL(float, float); }
#undef ADAM_CALL
    DDL_RETURN_LAUNCH();
}

// norms: fp32[2 * ntensors], zeroed by the caller before the call
DDL_API int ddl_lamb_step(int gdtype, const void* grad, float* master, int pdtype, void* param, float* m, float* v,
                          const int* table, int nblk, const float* scale, float lr, float b1, float b2, float eps,
                          float wd, float bc1, float bc2, float* norms, hipStream_t st) {
    const int4* t = (const int4*)table;
    if (gdtype == 1)
        lamb_phase1_k<bf16_t><<<nblk, OPT_NT, 0, st>>>((const bf16_t*)grad, master, m, v, t, scale, b1, b2, eps, wd, bc1,
                                                       bc2, norms);
    else
        lamb_phase1_k<float><<<nblk, OPT_NT, 0, st>>>((const float*)grad, master, m, v, t, scale, b1, b2, eps, wd, bc1,
                                                      bc2, norms);
    if (pdtype == 1)
        lamb_phase2_k<bf16_t><<<nblk, OPT_NT, 0, st>>>(master, (bf16_t*)param, m, v, t, lr, eps, wd, bc1, bc2, norms);
    else
        lamb_phase2_k<float><<<nblk, OPT_NT, 0, st>>>(master, (float*)param, m, v, t, lr, eps, wd, bc1, bc2, norms);
    DDL_RETURN_LAUNCH();
}

// LAMB as two launches, for the sharded optimizer: per-tensor norms of a rank's
// slice are all-reduced between phase 1 (moments + partial norms) and phase 2
DDL_API int ddl_lamb_phase1(int gdtype, const void* grad, float* master, float* m, float* v, const int* table,
                            int nblk, const float* scale, float b1, float b2, float eps, float wd, float bc1, float bc2,
                            float* norms, hipStream_t st) {
    const int4* t = (const int4*)table;
    if (gdtype == 1)
        lamb_phase1_k<bf16_t><<<nblk, OPT_NT, 0, st>>>((const bf16_t*)grad, master, m, v, t, scale, b1, b2, eps, wd, bc1,
                                                       bc2, norms);
    else
        lamb_phase1_k<float><<<nblk, OPT_NT, 0, st>>>((const float*)grad, master, m, v, t, scale, b1, b2, eps, wd, bc1,
                                                      bc2, norms);
    DDL_RETURN_LAUNCH();
}
DDL_API int ddl_lamb_phase2(float* master, int pdtype, void* param, float* m, float* v, const int* table, int nblk,
                            float lr, float eps, float wd, float bc1, float bc2, const float* norms, hipStream_t st) {
    const int4* t = (const int4*)table;
    if (pdtype == 1)
        lamb_phase2_k<bf16_t><<<nblk, OPT_NT, 0, st>>>(master, (bf16_t*)param, m, v, t, lr, eps, wd, bc1, bc2, norms);
    else
        lamb_phase2_k<float><<<nblk, OPT_NT, 0, st>>>(master, (float*)param, m, v, t, lr, eps, wd, bc1, bc2, norms);
    DDL_RETURN_LAUNCH();
}

// out (fp32 scalar, zeroed by caller) += sum(x^2); n % 8 == 0
DDL_API int ddl_sumsq(int dtype, const void* x, long n, float* out, hipStream_t st) {
    if (n % 8) return -1;
    const long n8 = n / 8;
    const int g = (int)std::min<long>(2048, (n8 + 255) / 256);
    if (dtype == 1) sumsq_k<bf16_t><<<g, 256, 0, st>>>((const bf16_t*)x, n8, out);
    else sumsq_k<float><<<g, 256, 0, st>>>((const float*)x, n8, out);
    DDL_RETURN_LAUNCH();
}
