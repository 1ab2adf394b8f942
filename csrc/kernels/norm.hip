// BatchNorm (NHWC, channels innermost) and LayerNorm kernels for gfx950.
//
// BatchNorm training forward = 3 launches:
//   bn_stats_partial  : per-block per-channel (sum, sumsq), 16-byte loads
//   bn_stats_finalize : merge partials in fp64, mean/invstd, running-stat update,
//                       fold gamma/beta into per-channel (scale, shift)
//   bn_apply          : y = x*scale + shift (+ residual) (ReLU), one pass
// BatchNorm backward = bn_bwd_partial (sum dz, sum dz*xhat) -> bn_bwd_finalize
// (dgamma, dbeta) -> bn_bwd_apply (dx, and dresidual = dz when the residual add
// was fused).  The ReLU mask is recomputed from the saved output, never stored.
//
// LayerNorm: one wave per row (H % 256 == 0: BERT-base 768, BERT-large 1024),
// fused residual add, fp32 statistics saved for backward; backward computes dx
// per row and per-block dgamma/dbeta partials reduced by a second kernel.
#include "ddl_common.h"
#include <cstdlib>
#include <mutex>
#include <unordered_map>

namespace {

constexpr int BN_NT = 256;

// ------------------------------------------------------------------ BN stats
template <typename T>
__global__ __launch_bounds__(BN_NT) void bn_stats_partial_k(const T* __restrict__ x, long M, int C,
                                                            int rows_per_blk, float* __restrict__ part) {
    __shared__ float s_red[2 * BN_NT * 8];
    const int tpr = C / 8;            // threads per row (each owns 8 channels)
    const int rpi = BN_NT / tpr;      // rows per iteration
    const int tid = threadIdx.x;
    const int cg = tid % tpr, rr = tid / tpr;
    const long r0 = (long)blockIdx.x * rows_per_blk;
    const long r1 = min(M, r0 + rows_per_blk);
    float s[8], q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { s[j] = 0.f; q[j] = 0.f; }
    long r = r0 + rr;
    for (; r + 3 * rpi < r1; r += 4 * rpi) {   // 4 rows of 16-byte loads in flight
        float v[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) load8(x + (r + u * rpi) * C + cg * 8, v[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int j = 0; j < 8; ++j) { s[j] += v[u][j]; q[j] += v[u][j] * v[u][j]; }
    }
    for (; r < r1; r += rpi) {
        float v[8];
        load8(x + r * C + cg * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) { s[j] += v[j]; q[j] += v[j] * v[j]; }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        s_red[tid * 8 + j] = s[j];
        s_red[BN_NT * 8 + tid * 8 + j] = q[j];
    }
    __syncthreads();
    for (int c = tid; c < C; c += BN_NT) {
        float a = 0.f, b = 0.f;
        for (int i = 0; i < rpi; ++i) {
            a += s_red[i * C + c];
            b += s_red[BN_NT * 8 + i * C + c];
        }
        part[(long)blockIdx.x * 2 * C + c] = a;
        part[(long)blockIdx.x * 2 * C + C + c] = b;
    }
}

// channel c's statistics from its summed [sum | sumsq]: mean / invstd saved, running stats
// updated, gamma / beta folded into (scale, shift)
template <typename TP>
__device__ __forceinline__ void bn_fwd_finish_channel(int c, double s, double q, long M, const TP* __restrict__ gamma,
                                                      const TP* __restrict__ beta, float* __restrict__ running_mean,
                                                      float* __restrict__ running_var, float momentum, float eps,
                                                      float* __restrict__ save_mean, float* __restrict__ save_invstd,
                                                      float* __restrict__ scale, float* __restrict__ shift) {
    const double mean = s / (double)M;
    double var = q / (double)M - mean * mean;
    if (var < 0) var = 0;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    save_mean[c] = (float)mean;
    save_invstd[c] = invstd;
    if (running_mean) {
        const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
        running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unbiased;
    }
    const float g = gamma ? to_f(gamma[c]) : 1.f;
    const float bb = beta ? to_f(beta[c]) : 0.f;
    scale[c] = g * invstd;
    shift[c] = bb - (float)mean * g * invstd;
}

template <typename TP>
__global__ __launch_bounds__(1024) void bn_stats_finalize_k(const float* __restrict__ part, int nblk, int C, long M,
                                    const TP* __restrict__ gamma, const TP* __restrict__ beta,
                                    float* __restrict__ running_mean, float* __restrict__ running_var, float momentum,
                                    float eps, float* __restrict__ save_mean, float* __restrict__ save_invstd,
                                    float* __restrict__ scale, float* __restrict__ shift) {
    __shared__ float red[1024];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const double s = colsum64(part, nblk, 2L * C, c, c < C, red);
    const double q = colsum64(part, nblk, 2L * C, C + c, c < C, red);
    if (threadIdx.x >= 64 || c >= C) return;
    bn_fwd_finish_channel<TP>(c, s, q, M, gamma, beta, running_mean, running_var, momentum, eps, save_mean,
                              save_invstd, scale, shift);
}

// eval mode: scale/shift from running statistics
template <typename TP>
__global__ void bn_eval_coeffs_k(int C, const TP* __restrict__ gamma, const TP* __restrict__ beta,
                                 const float* __restrict__ rm, const float* __restrict__ rv, float eps,
                                 float* __restrict__ scale, float* __restrict__ shift) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float inv = rsqrtf(rv[c] + eps);
    const float g = gamma ? to_f(gamma[c]) : 1.f;
    const float bb = beta ? to_f(beta[c]) : 0.f;
    scale[c] = g * inv;
    shift[c] = bb - rm[c] * g * inv;
}

// RELU + mask: one bit per element (byte i covers elements 8i..8i+7) records
// y > 0, so the backward never re-reads y (16x less traffic than the bf16 output)
template <typename T, bool RES, bool RELU>
__global__ __launch_bounds__(256) void bn_apply_k(const T* __restrict__ x, const T* __restrict__ res,
                                                  const float* __restrict__ scale, const float* __restrict__ shift,
                                                  T* __restrict__ y, uint8_t* __restrict__ mask, long n8, int C) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
        const int c0 = (int)((i * 8) % C);
        float v[8], sc[8], sh[8];
        load8(x + i * 8, v);
        load8(scale + c0, sc);
        load8(shift + c0, sh);
        float r[8];
        if (RES) load8(res + i * 8, r);
        uint32_t bits = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float t = v[j] * sc[j] + sh[j];
            if (RES) t += r[j];
            if (RELU) {
                // the bit must agree with the stored (rounded) output
                t = fmaxf(t, 0.f);
                bits |= (to_f(from_f<T>(t)) > 0.f ? 1u : 0u) << j;
            }
            v[j] = t;
        }
        store8(y + i * 8, v);
        if (RELU && mask) mask[i] = (uint8_t)bits;
    }
}

// Row-major variant of bn_apply for C / 8 dividing 256: a thread owns one
// 8-channel group for the whole launch (coefficients loaded once, no per-element
// channel modulo) and keeps 4 rows of 16-byte loads in flight.
template <typename T, bool RES, bool RELU>
__global__ __launch_bounds__(256) void bn_apply_rows_k(const T* __restrict__ x, const T* __restrict__ res,
                                                       const float* __restrict__ scale, const float* __restrict__ shift,
                                                       T* __restrict__ y, uint8_t* __restrict__ mask, long M, int C) {
    const int tpr = C / 8, rpb = 256 / tpr;
    const int cg = threadIdx.x % tpr, rr = threadIdx.x / tpr;
    float sc[8], sh[8];
    load8(scale + cg * 8, sc);
    load8(shift + cg * 8, sh);
    const long rs = (long)gridDim.x * rpb;
    auto one = [&](const float* v, const float* r, long row) {
        float o[8];
        uint32_t bits = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float t = v[j] * sc[j] + sh[j];
            if (RES) t += r[j];
            if (RELU) {
                // the bit must agree with the stored (rounded) output
                t = fmaxf(t, 0.f);
                bits |= (to_f(from_f<T>(t)) > 0.f ? 1u : 0u) << j;
            }
            o[j] = t;
        }
        store8(y + row * C + cg * 8, o);
        if (RELU && mask) mask[row * tpr + cg] = (uint8_t)bits;
    };
    long r = (long)blockIdx.x * rpb + rr;
    for (; r + 3 * rs < M; r += 4 * rs) {
        float v[4][8], rv[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) {   // non-temporal: read again only by the backward, much later
            load8_nt(x + (r + u * rs) * C + cg * 8, v[u]);
            if (RES) load8_nt(res + (r + u * rs) * C + cg * 8, rv[u]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) one(v[u], rv[u], r + u * rs);
    }
    for (; r < M; r += rs) {
        float v[8], rv[8];
        load8(x + r * C + cg * 8, v);
        if (RES) load8(res + r * C + cg * 8, rv);
        one(v, rv, r);
    }
}

// Two BatchNorms meeting at a residual add (a ResNet downsample block's output):
// y = relu(x * scale + shift + x2 * scale2 + shift2) in one pass -- the downsample BN's
// output is never written and re-read.
template <typename T, bool RELU>
__global__ __launch_bounds__(256) void bn_apply2_rows_k(const T* __restrict__ x, const T* __restrict__ x2,
                                                        const float* __restrict__ scale, const float* __restrict__ shift,
                                                        const float* __restrict__ scale2,
                                                        const float* __restrict__ shift2, T* __restrict__ y,
                                                        uint8_t* __restrict__ mask, long M, int C) {
    const int tpr = C / 8, rpb = 256 / tpr;
    const int cg = threadIdx.x % tpr, rr = threadIdx.x / tpr;
    float sc[8], sh[8], sc2[8];
    load8(scale + cg * 8, sc);
    load8(shift + cg * 8, sh);
    load8(scale2 + cg * 8, sc2);
    {
        float sh2[8];
        load8(shift2 + cg * 8, sh2);
#pragma unroll
        for (int j = 0; j < 8; ++j) sh[j] += sh2[j];
    }
    const long rs = (long)gridDim.x * rpb;
    auto one = [&](const float* v, const float* r, long row) {
        float o[8];
        uint32_t bits = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float t = v[j] * sc[j] + r[j] * sc2[j] + sh[j];
            if (RELU) {
                t = fmaxf(t, 0.f);
                bits |= (to_f(from_f<T>(t)) > 0.f ? 1u : 0u) << j;
            }
            o[j] = t;
        }
        store8(y + row * C + cg * 8, o);
        if (RELU && mask) mask[row * tpr + cg] = (uint8_t)bits;
    };
    long r = (long)blockIdx.x * rpb + rr;
    for (; r + 3 * rs < M; r += 4 * rs) {
        float v[4][8], rv[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) {   // non-temporal: read again only by the backward, much later
            load8_nt(x + (r + u * rs) * C + cg * 8, v[u]);
            load8_nt(x2 + (r + u * rs) * C + cg * 8, rv[u]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) one(v[u], rv[u], r + u * rs);
    }
    for (; r < M; r += rs) {
        float v[8], rv[8];
        load8(x + r * C + cg * 8, v);
        load8(x2 + r * C + cg * 8, rv);
        one(v, rv, r);
    }
}

// blocks for the row-major passes: ONE resident round -- as many blocks of 256 threads as the
// CUs hold at once for THIS kernel (its occupancy), each thread looping over rows.  A fixed 2048
// (8 per CU) left a second round wherever registers allow fewer: at 68 VGPRs (7 waves per SIMD)
// 1792 blocks ran, then 256 more, one per CU, ran alone to finish the pass.
// DDL_BN_ROWS_GRID=0 restores the fixed 2048 (A/B timing).
static int cu_count() {
    static const int n = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
            v = 256;
        return v;
    }();
    return n;
}
static bool rows_grid_fit() {
    static const bool on = [] {
        const char* e = getenv("DDL_BN_ROWS_GRID");
        return !(e && e[0] == '0');
    }();
    return on;
}
static int rows_grid(long M, int C, const void* kernel = nullptr) {
    const long rpb = 256 / (C / 8);
    const long need = (M + rpb - 1) / rpb;
    long cap = 2048;
    if (kernel && rows_grid_fit()) {
        static std::mutex mu;
        static std::unordered_map<const void*, int> per_cu;
        int nb = 0;
        {
            std::lock_guard<std::mutex> lk(mu);
            auto it = per_cu.find(kernel);
            if (it == per_cu.end()) {
                if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, 256, 0) != hipSuccess) nb = 8;
                nb = std::min(8, std::max(1, nb));
                per_cu.emplace(kernel, nb);
            } else {
                nb = it->second;
            }
        }
        cap = (long)nb * cu_count();
    }
    return (int)std::max<long>(1, std::min<long>(cap, need));
}
static bool rows_ok(int C) { return C % 8 == 0 && 256 % (C / 8) == 0; }

// ------------------------------------------------------------------ BN backward
template <typename T, bool RELU>
__global__ __launch_bounds__(BN_NT) void bn_bwd_partial_k(const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                          const T* __restrict__ x, const float* __restrict__ mean,
                                                          const float* __restrict__ invstd, long M, int C,
                                                          int rows_per_blk, float* __restrict__ part) {
    __shared__ float s_red[2 * BN_NT * 8];
    const int tpr = C / 8, rpi = BN_NT / tpr, tid = threadIdx.x;
    const int cg = tid % tpr, rr = tid / tpr;
    const long r0 = (long)blockIdx.x * rows_per_blk;
    const long r1 = min(M, r0 + rows_per_blk);
    float mu[8], is[8], a[8], b[8];
    load8(mean + cg * 8, mu);
    load8(invstd + cg * 8, is);
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = 0.f; b[j] = 0.f; }
#pragma unroll 2
    for (long r = r0 + rr; r < r1; r += rpi) {
        float g[8], xv[8];
        load8_nt(dy + r * C + cg * 8, g);
        load8_nt(x + r * C + cg * 8, xv);
        const uint32_t bits = RELU ? mask[r * tpr + cg] : 0xffu;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float dz = ((bits >> j) & 1u) ? g[j] : 0.f;
            a[j] += dz;
            b[j] += dz * (xv[j] - mu[j]) * is[j];
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        s_red[tid * 8 + j] = a[j];
        s_red[BN_NT * 8 + tid * 8 + j] = b[j];
    }
    __syncthreads();
    for (int c = tid; c < C; c += BN_NT) {
        float s = 0.f, q = 0.f;
        for (int i = 0; i < rpi; ++i) {
            s += s_red[i * C + c];
            q += s_red[BN_NT * 8 + i * C + c];
        }
        part[(long)blockIdx.x * 2 * C + c] = s;
        part[(long)blockIdx.x * 2 * C + C + c] = q;
    }
}

template <typename TP>
__device__ __forceinline__ void bn_bwd_finish_channel(int c, double s, double q, int C, long M,
                                                      const TP* __restrict__ gamma, const float* __restrict__ invstd,
                                                      TP* __restrict__ dgamma, TP* __restrict__ dbeta,
                                                      float* __restrict__ coef, int acc,
                                                      const float* __restrict__ prow) {
    // SyncBatchNorm: the coefficients need the group-summed row, but dgamma / dbeta are
    // this rank's partials (the data-parallel reducer sums them across ranks afterwards)
    const float ps = prow ? prow[c] : (float)s, pq = prow ? prow[C + c] : (float)q;
    if (dgamma) dgamma[c] = from_f<TP>(pq + (acc ? to_f(dgamma[c]) : 0.f));
    if (dbeta) dbeta[c] = from_f<TP>(ps + (acc ? to_f(dbeta[c]) : 0.f));
    const float g = gamma ? to_f(gamma[c]) : 1.f;
    coef[c] = g * invstd[c];                 // k1
    coef[C + c] = (float)(s / (double)M);    // mean(dz)
    coef[2 * C + c] = (float)(q / (double)M);// mean(dz*xhat)
}

template <typename TP>
__global__ __launch_bounds__(1024) void bn_bwd_finalize_k(const float* __restrict__ part, int nblk, int C, long M,
                                  const TP* __restrict__ gamma, const float* __restrict__ invstd,
                                  TP* __restrict__ dgamma, TP* __restrict__ dbeta, float* __restrict__ coef,
                                  int acc, const float* __restrict__ prow = nullptr) {
    __shared__ float red[1024];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const double s = colsum64(part, nblk, 2L * C, c, c < C, red);
    const double q = colsum64(part, nblk, 2L * C, C + c, c < C, red);
    if (threadIdx.x >= 64 || c >= C) return;
    bn_bwd_finish_channel<TP>(c, s, q, C, M, gamma, invstd, dgamma, dbeta, coef, acc, prow);
}

template <typename T, bool RELU, bool DRES>
__global__ __launch_bounds__(256) void bn_bwd_apply_k(const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                      const T* __restrict__ x, const float* __restrict__ mean,
                                                      const float* __restrict__ invstd, const float* __restrict__ coef,
                                                      T* __restrict__ dx, T* __restrict__ dres, long n8, int C) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
        const int c0 = (int)((i * 8) % C);
        float g[8], xv[8], mu[8], is[8], k1[8], mb[8], mg[8];
        load8(dy + i * 8, g);
        load8(x + i * 8, xv);
        const uint32_t bits = RELU ? mask[i] : 0xffu;
        load8(mean + c0, mu);
        load8(invstd + c0, is);
        load8(coef + c0, k1);
        load8(coef + C + c0, mb);
        load8(coef + 2 * C + c0, mg);
        float o[8], dz[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            dz[j] = ((bits >> j) & 1u) ? g[j] : 0.f;
            const float xh = (xv[j] - mu[j]) * is[j];
            o[j] = k1[j] * (dz[j] - mb[j] - xh * mg[j]);
        }
        store8(dx + i * 8, o);
        if (DRES) store8(dres + i * 8, dz);
    }
}

// Row-major backward apply (C / 8 dividing 256): per-thread channel group, the
// five per-channel coefficients folded once into dx = A*dz + B*x + D.
template <typename T, bool RELU, bool DRES>
__global__ __launch_bounds__(256) void bn_bwd_apply_rows_k(const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                           const T* __restrict__ x, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ coef, T* __restrict__ dx,
                                                           T* __restrict__ dres, long M, int C) {
    const int tpr = C / 8, rpb = 256 / tpr;
    const int cg = threadIdx.x % tpr, rr = threadIdx.x / tpr;
    float A[8], B[8], D[8];
    {
        float mu[8], is[8], k1[8], mb[8], mg[8];
        load8(mean + cg * 8, mu);
        load8(invstd + cg * 8, is);
        load8(coef + cg * 8, k1);
        load8(coef + C + cg * 8, mb);
        load8(coef + 2 * C + cg * 8, mg);
        // dx = k1 * (dz - mb - (x - mu) * is * mg)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            A[j] = k1[j];
            B[j] = -k1[j] * is[j] * mg[j];
            D[j] = k1[j] * (mu[j] * is[j] * mg[j] - mb[j]);
        }
    }
    const long rs = (long)gridDim.x * rpb;
    auto one = [&](const float* g, const float* xv, uint32_t bits, long row) {
        float o[8], dz[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            dz[j] = ((bits >> j) & 1u) ? g[j] : 0.f;
            o[j] = A[j] * dz[j] + B[j] * xv[j] + D[j];
        }
        store8(dx + row * C + cg * 8, o);
        if (DRES) store8(dres + row * C + cg * 8, dz);
    };
    long r = (long)blockIdx.x * rpb + rr;
    for (; r + 3 * rs < M; r += 4 * rs) {
        float g[4][8], xv[4][8];
        uint32_t bits[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {   // the last reads of dy and x: non-temporal
            load8_nt(dy + (r + u * rs) * C + cg * 8, g[u]);
            load8_nt(x + (r + u * rs) * C + cg * 8, xv[u]);
            bits[u] = RELU ? mask[(r + u * rs) * tpr + cg] : 0xffu;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) one(g[u], xv[u], bits[u], r + u * rs);
    }
    for (; r < M; r += rs) {
        float g[8], xv[8];
        load8(dy + r * C + cg * 8, g);
        load8(x + r * C + cg * 8, xv);
        one(g, xv, RELU ? mask[r * tpr + cg] : 0xffu, r);
    }
}

// ------------------------------------------------------------------ LayerNorm
// One wave per row; each lane owns VPL = H/256 chunks of 4 contiguous elements
// (lane chunk k covers columns 256*k + 4*lane .. +3): every load is 8 B/lane,
// fully coalesced per wave.
// Dropout fused on the LayerNorm's main input: y = LN(dropout(x) + res).  The keep
// mask is the counter hash of (seed, flat element index), regenerated in the
// backward, which writes the residual gradient g and the x gradient g*mask/(1-p)
// (and the column sums of the latter: the producing Linear's bias gradient).
// raw 4-element loads (bf16: 8 bytes, fp32: 16 bytes) converted later, so a load can stay in
// flight across unrelated work
template <typename T> struct Raw4;
template <> struct Raw4<bf16_t> { typedef uint2 type; };
template <> struct Raw4<float> { typedef float4 type; };
__device__ __forceinline__ uint2 ld_raw4(const bf16_t* p) { return *reinterpret_cast<const uint2*>(p); }
__device__ __forceinline__ float4 ld_raw4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void cvt_raw4(const uint2& u, float* v) {
    v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
}
__device__ __forceinline__ void cvt_raw4(const float4& a, float* v) { v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; }

struct Drop {
    uint64_t seed;
    uint32_t thresh;   // 16-bit threshold (ddl_common.h keep_bits4); 0: no dropout
    float scale;       // 1 / (1 - p)
    void* dres;        // backward: residual gradient (unmasked), only with dropout
};
// idx % 4 == 0 (H % 4 == 0, 4 columns per lane): two pair hashes per 4 elements
__device__ __forceinline__ uint32_t drop_bits4(const Drop& d, long idx) {
    return keep_bits4(d.seed, (uint64_t)idx, d.thresh);
}
__device__ __forceinline__ void apply4(const Drop& d, uint32_t bits, float* v) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = ((bits >> j) & 1u) ? v[j] * d.scale : 0.f;
}
__device__ __forceinline__ void drop4(const Drop& d, long idx, float* v) { apply4(d, drop_bits4(d, idx), v); }

template <typename T, int VPL>
__global__ __launch_bounds__(256) void ln_fwd_k(const T* __restrict__ x, const T* __restrict__ res, long res_rows,
                                                const T* __restrict__ gamma, const T* __restrict__ beta, T* __restrict__ y,
                                                float* __restrict__ save_mean, float* __restrict__ save_rstd, long rows,
                                                int H, float eps, Drop drop) {
    const int lane = threadIdx.x & 63;
    const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    float v[VPL][4];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
        const int col = 256 * k + 4 * lane;
        load4(x + row * H + col, v[k]);
        if (drop.thresh) drop4(drop, row * H + col, v[k]);
        if (res) {
            float r[4];
            load4(res + (row % res_rows) * H + col, r);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[k][j] += r[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) s += v[k][j];
    }
    const float mean = wave_sum_dpp(s) / H;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < VPL; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) { const float d = v[k][j] - mean; q += d * d; }
    const float rstd = rsqrtf(wave_sum_dpp(q) / H + eps);
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
        const int col = 256 * k + 4 * lane;
        float g[4], b[4], o[4];
        load4(gamma + col, g);
        load4(beta + col, b);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (v[k][j] - mean) * rstd * g[j] + b[j];
        store4(y + row * H + col, o);
    }
    if (lane == 0) { save_mean[row] = mean; save_rstd[row] = rstd; }
}

// bf16 LayerNorm forward with 16-byte accesses: half a wave per row (32 lanes x 8 contiguous columns
// per chunk, chunk k covers columns 256 k + 8 lane32 .. +7), two rows per wave.  The wave-per-row
// kernel above moves 8 bytes per lane (H = 768: three 512-B instructions per operand and row); here an
// instruction moves 1 KB (two rows x 512 B).  Half-wave sums: DPP row sums + one permlane16 swap.
__device__ __forceinline__ float half_sum(float v) {
    v = row16_sum(v);
    const uint32_t u = __float_as_uint(v);
    const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    return __uint_as_float(a[0]) + __uint_as_float(a[1]);
}

template <int VPL>
__global__ __launch_bounds__(256) void ln_fwd8_k(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                 long res_rows, const bf16_t* __restrict__ gamma,
                                                 const bf16_t* __restrict__ beta, bf16_t* __restrict__ y,
                                                 float* __restrict__ save_mean, float* __restrict__ save_rstd, long rows,
                                                 int H, float eps, Drop drop) {
    const int lane = threadIdx.x & 63, l32 = lane & 31;
    const long row = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);
    const bool ok = row < rows;             // both halves take part in the DPP sums
    const long rw = ok ? row : rows - 1;
    uint4 xr[VPL], rr[VPL];
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
        const int col = 256 * k + 8 * l32;
        xr[k] = *reinterpret_cast<const uint4*>(x + rw * H + col);
        if (res) rr[k] = *reinterpret_cast<const uint4*>(res + (rw % res_rows) * H + col);
    }
    float v[VPL][8];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
        const int col = 256 * k + 8 * l32;
        const uint32_t wx[4] = {xr[k].x, xr[k].y, xr[k].z, xr[k].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            v[k][2 * e] = __uint_as_float(wx[e] << 16);
            v[k][2 * e + 1] = __uint_as_float(wx[e] & 0xffff0000u);
        }
        if (drop.thresh) {
            drop4(drop, rw * H + col, v[k]);
            drop4(drop, rw * H + col + 4, v[k] + 4);
        }
        if (res) {
            const uint32_t wr[4] = {rr[k].x, rr[k].y, rr[k].z, rr[k].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[k][2 * e] += __uint_as_float(wr[e] << 16);
                v[k][2 * e + 1] += __uint_as_float(wr[e] & 0xffff0000u);
            }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[k][j];
    }
    const float mean = half_sum(s) / H;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < VPL; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float d = v[k][j] - mean; q += d * d; }
    const float rstd = rsqrtf(half_sum(q) / H + eps);
    if (!ok) return;
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
        const int col = 256 * k + 8 * l32;
        float g[8], b[8], o[8];
        load8(gamma + col, g);
        load8(beta + col, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mean) * rstd * g[j] + b[j];
        store8(y + row * H + col, o);
    }
    if (l32 == 0) { save_mean[row] = mean; save_rstd[row] = rstd; }
}

// dx per row + dgamma/dbeta partials per block (ROWS_PER_BLK rows, 4 waves).
// ADD: dadd (the gradient of this LayerNorm's input from its other consumer -- a pre-LN
// block's residual branch) is added to dx in the same pass, before the column sums, so dx is
// the input's WHOLE gradient (no autograd add kernel, and the column sums are the producing
// Linear's complete bias gradient)
// KNOWN (0: run-time checks): 4 | 2 (residual present) | 1 (dropout present) -- the BERT / ViT widths
// are compiled per case, so the row loop carries no uniform branches for absent operands
template <typename T, int VPL, bool ADD = false, int KNOWN = 0>
__global__ __launch_bounds__(256) void ln_bwd_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                const T* __restrict__ res, long res_rows, const T* __restrict__ gamma,
                                                const float* __restrict__ mean, const float* __restrict__ rstd,
                                                T* __restrict__ dx, float* __restrict__ part, long rows, int H,
                                                int rows_per_blk, int dxsum, Drop drop,
                                                const T* __restrict__ dadd = nullptr) {
    // part row per block: [dgamma(H) | dbeta(H) | (dxsum) sum of dx (H)] -- the last is the
    // bias gradient of the Linear that produced this LayerNorm's input
    // (+4 floats per wave row: the column reads below pair a wave row with the next as ds_read2_b32,
    // whose two dwords fell on one bank at a stride of VPL * 256 floats -- 2-way conflicts on every read)
    __shared__ __attribute__((aligned(16))) float s_acc[3][4][VPL * 256 + 4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const bool has_res = KNOWN ? (KNOWN & 2) != 0 : res != nullptr;
    const bool has_drop = KNOWN ? (KNOWN & 1) != 0 : drop.thresh != 0;
    float dg[VPL][4], db[VPL][4], ds[VPL][4], g[VPL][4];
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
        load4(gamma + 256 * k + 4 * lane, g[k]);
#pragma unroll
        for (int j = 0; j < 4; ++j) { dg[k][j] = 0.f; db[k][j] = 0.f; ds[k][j] = 0.f; }
    }
    const long r0 = (long)blockIdx.x * rows_per_blk;
    const long r1 = min(rows, r0 + rows_per_blk);
    // raw (unconverted) loads of one row -- input x, dy and the residual -- so the next row
    // pair's loads stay in flight while the current pair's reductions run; with dropout the
    // row's keep bits (4 per lane and column group) are generated once and reused for dx
    // the row's saved mean / rstd travel with its operands: loaded at finish time they put a
    // dependent scalar-load miss in front of every row's reductions
    struct RowRaw {
        typename Raw4<T>::type x[VPL], d[VPL], r[VPL];
        uint32_t kb[VPL];
        float mu, rs;
    };
    auto load_row = [&](long row, RowRaw& R) {
        R.mu = mean[row];
        R.rs = rstd[row];
#pragma unroll
        for (int k = 0; k < VPL; ++k) {
            const int col = 256 * k + 4 * lane;
            R.x[k] = ld_raw4(x + row * H + col);
            R.d[k] = ld_raw4(dy + row * H + col);
            if (has_res) R.r[k] = ld_raw4(res + (row % res_rows) * H + col);
            R.kb[k] = has_drop ? drop_bits4(drop, row * H + col) : 0xfu;
        }
    };
    // converted input (dropout(x) + residual) and dy of a loaded row
    auto prep_row = [&](const RowRaw& R, float (&xv)[VPL][4], float (&d)[VPL][4]) {
#pragma unroll
        for (int k = 0; k < VPL; ++k) {
            cvt_raw4(R.x[k], xv[k]);
            cvt_raw4(R.d[k], d[k]);
            if (has_drop) apply4(drop, R.kb[k], xv[k]);
            if (has_res) {
                float r[4];
                cvt_raw4(R.r[k], r);
#pragma unroll
                for (int j = 0; j < 4; ++j) xv[k][j] += r[j];
            }
        }
    };
    auto finish_row = [&](long row, const float (&xv)[VPL][4], const float (&d)[VPL][4], const RowRaw& R) {
        const uint32_t (&kb)[VPL] = R.kb;
        // the added gradient is loaded here, ahead of the row reductions, not a row pair ahead
        // with the other operands (4 rows of it in flight cost the second wave per SIMD)
        typename Raw4<T>::type ra[ADD ? VPL : 1];
        if constexpr (ADD) {
#pragma unroll
            for (int k = 0; k < VPL; ++k) ra[k] = ld_raw4(dadd + row * H + 256 * k + 4 * lane);
        }
        const float mu = R.mu, rs = R.rs;
        float xh[VPL][4], gy[VPL][4];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int k = 0; k < VPL; ++k)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                xh[k][j] = (xv[k][j] - mu) * rs;
                gy[k][j] = d[k][j] * g[k][j];
                s1 += gy[k][j];
                s2 += gy[k][j] * xh[k][j];
                dg[k][j] += d[k][j] * xh[k][j];
                db[k][j] += d[k][j];
            }
        const float m1 = wave_sum_dpp(s1) / H, m2 = wave_sum_dpp(s2) / H;
#pragma unroll
        for (int k = 0; k < VPL; ++k) {
            float o[4];
            const long idx = row * H + 256 * k + 4 * lane;
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = rs * (gy[k][j] - m1 - xh[k][j] * m2);
            if (has_drop) {
                store4((T*)drop.dres + idx, o);      // residual gradient: unmasked
                apply4(drop, kb[k], o);              // x gradient: through the dropout mask
            }
            if constexpr (ADD) {
                float a[4];
                cvt_raw4(ra[k], a);
#pragma unroll
                for (int j = 0; j < 4; ++j) o[j] += a[j];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) ds[k][j] += to_f(from_f<T>(o[j]));   // sum of the stored (rounded) dx
            store4(dx + idx, o);
        }
    };
    // two rows per wave per iteration, software-pipelined: the next pair's loads are issued
    // before the current pair's reductions (the kernel was load-latency bound at ~3 TB/s)
    // (H > 768: two pairs in registers would drop occupancy to one wave per SIMD, so one pair)
    constexpr bool PIPE = VPL <= 3;
    RowRaw ra{}, rb{}, rc{}, rd{};
    long row = r0 + w;
    if (PIPE && row < r1) load_row(row, ra);
    if (PIPE && row + 4 < r1) load_row(row + 4, rb);
    for (; row < r1; row += 8) {
        const bool two = row + 4 < r1;   // wave-uniform
        if constexpr (PIPE) {
            if (row + 8 < r1) load_row(row + 8, rc);
            if (row + 12 < r1) load_row(row + 12, rd);
        } else {
            load_row(row, ra);
            if (two) load_row(row + 4, rb);
        }
        {
            float xv[VPL][4], d[VPL][4];
            prep_row(ra, xv, d);
            finish_row(row, xv, d, ra);
        }
        if (two) {
            float xv[VPL][4], d[VPL][4];
            prep_row(rb, xv, d);
            finish_row(row + 4, xv, d, rb);
        }
        if constexpr (PIPE) {
            ra = rc;
            rb = rd;
        }
    }
    // 16-byte stores (one ds_write_b128 per lane and column group): four scalar stores of a
    // 16-byte lane stride put lanes l, l + 8, l + 16, l + 24 on one bank (4-way conflicts)
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
        *reinterpret_cast<float4*>(&s_acc[0][w][256 * k + 4 * lane]) = make_float4(dg[k][0], dg[k][1], dg[k][2], dg[k][3]);
        *reinterpret_cast<float4*>(&s_acc[1][w][256 * k + 4 * lane]) = make_float4(db[k][0], db[k][1], db[k][2], db[k][3]);
        *reinterpret_cast<float4*>(&s_acc[2][w][256 * k + 4 * lane]) = make_float4(ds[k][0], ds[k][1], ds[k][2], ds[k][3]);
    }
    __syncthreads();
    // column sums over the 4 wave rows: 4 consecutive columns per thread, ds_read_b128 (16 lanes x
    // 16 B = one pass over all 64 banks: conflict free) and 16-byte global stores.  The scalar
    // form (one column per thread, the four wave rows paired into ds_read2_b32) was 50 % bank-
    // conflict cycles in the PMC pass (profiles/pmc_bert.md, round 5).
    const int nv = dxsum ? 3 : 2;
    for (int c = 4 * threadIdx.x; c < H; c += 1024) {
        for (int v = 0; v < nv; ++v) {
            const float4 a = *reinterpret_cast<const float4*>(&s_acc[v][0][c]);
            const float4 b = *reinterpret_cast<const float4*>(&s_acc[v][1][c]);
            const float4 e = *reinterpret_cast<const float4*>(&s_acc[v][2][c]);
            const float4 f = *reinterpret_cast<const float4*>(&s_acc[v][3][c]);
            *reinterpret_cast<float4*>(part + (long)blockIdx.x * nv * H + v * H + c) =
                make_float4(a.x + b.x + e.x + f.x, a.y + b.y + e.y + f.y, a.z + b.z + e.z + f.z, a.w + b.w + e.w + f.w);
        }
    }
}

template <typename TP>
__global__ __launch_bounds__(1024) void colsum_partials_k(const float* __restrict__ part, int nblk, int H,
                                                          TP* __restrict__ dg, TP* __restrict__ db, int acc,
                                                          float* __restrict__ dxsum, TP* __restrict__ dxsink) {
    __shared__ float red[1024];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const long stride = (dxsum ? 3L : 2L) * H;
    const float a = colsum64(part, nblk, stride, c, c < H, red);
    const float b = colsum64(part, nblk, stride, H + c, c < H, red);
    float d = 0.f;
    if (dxsum) d = colsum64(part, nblk, stride, 2 * H + c, c < H, red);
    if (threadIdx.x >= 64 || c >= H) return;
    dg[c] = from_f<TP>(a + (acc ? to_f(dg[c]) : 0.f));
    db[c] = from_f<TP>(b + (acc ? to_f(db[c]) : 0.f));
    if (dxsum) dxsum[c] = d;
    // the producing Linear's bias gradient, accumulated straight into its arena slot
    if (dxsink) dxsink[c] = from_f<TP>(d + (acc ? to_f(dxsink[c]) : 0.f));
}

inline int grid_for(long n, int nt = 256, int cap = 4096) {
    long g = (n + nt - 1) / nt;
    return (int)std::max<long>(1, std::min<long>(g, cap));
}

}  // namespace

// =================================================================== C ABI
// dtype codes: 0 = fp32, 1 = bf16

// backward partial pass: two input streams per row, 4 blocks per CU in flight
DDL_API int ddl_bn_bwd_nblk(long M, int C) {
    const int rpi = BN_NT / (C / 8);
    long nblk = std::min<long>(1024, (M + rpi * 8 - 1) / (rpi * 8));
    return (int)std::max<long>(1, nblk);
}

DDL_API int ddl_bn_stats_nblk(long M, int C) {
    const int rpi = BN_NT / (C / 8);
    long nblk = std::min<long>(512, (M + rpi * 8 - 1) / (rpi * 8));
    return (int)std::max<long>(1, nblk);
}

DDL_API int ddl_bn_fwd_train(int dtype, const void* x, long M, int C, const void* gamma, const void* beta,
                             float* running_mean, float* running_var, float momentum, float eps, float* part,
                             float* save_mean, float* save_invstd, float* scale, float* shift, hipStream_t st) {
    if (C % 8 || (BN_NT % (C / 8) != 0)) return -1;
    const int nblk = ddl_bn_stats_nblk(M, C);
    const int rpi = BN_NT / (C / 8);
    long rpb = (M + nblk - 1) / nblk;
    rpb = (rpb + rpi - 1) / rpi * rpi;
    if (dtype == 1) {
        bn_stats_partial_k<bf16_t><<<nblk, BN_NT, 0, st>>>((const bf16_t*)x, M, C, (int)rpb, part);
        bn_stats_finalize_k<bf16_t><<<(C + 63) / 64, 1024, 0, st>>>(part, nblk, C, M, (const bf16_t*)gamma,
            (const bf16_t*)beta, running_mean, running_var, momentum, eps, save_mean, save_invstd, scale, shift);
    } else {
        bn_stats_partial_k<float><<<nblk, BN_NT, 0, st>>>((const float*)x, M, C, (int)rpb, part);
        bn_stats_finalize_k<float><<<(C + 63) / 64, 1024, 0, st>>>(part, nblk, C, M, (const float*)gamma,
            (const float*)beta, running_mean, running_var, momentum, eps, save_mean, save_invstd, scale, shift);
    }
    DDL_RETURN_LAUNCH();
}

// Training-mode BN statistics from partial sums a GEMM epilogue already produced
// (``part`` = [nblk][sum(C) | sumsq(C)], see gemm.hip / gemm_big.hip colstats):
// the statistics read pass over the conv output disappears.
// First level for many partial rows (a GEMM epilogue writes one per 128 output
// rows: 6272 for a 56x56 layer at batch 256): blockIdx.y sums PC_ROWS rows of
// every column (consecutive threads on consecutive columns, all PC_ROWS loads
// in flight as 4 independent chains), so the finalize kernel reads nblk/PC_ROWS
// rows instead of thousands.
constexpr int PC_ROWS = 32;
__global__ __launch_bounds__(256) void bn_partials_collapse_k(const float* __restrict__ part, int nblk, int width,
                                                              float* __restrict__ out) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    if (col >= width) return;
    const int r0 = blockIdx.y * PC_ROWS;
    const float* src = part + (long)r0 * width + col;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (r0 + PC_ROWS <= nblk) {
#pragma unroll
        for (int r = 0; r < PC_ROWS; ++r) acc[r & 3] += src[(long)r * width];
    } else {
        for (int r = 0; r < nblk - r0; ++r) acc[r & 3] += src[(long)r * width];
    }
    out[(long)blockIdx.y * width + col] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
}

// ---------------------------------------------------------------- merged collapse + finalize
// The BatchNorm statistics / backward-coefficient finalize from thousands of partial rows (one
// per 128 rows of a GEMM epilogue) used to be two launches: a 32:1 collapse, then ONE workgroup
// per 64 channels walking every remaining row (latency-bound: each 16-row group of a 1024-thread
// block is a dependent round trip).  Here one launch: grid (C / 64, S) workgroups of 1024
// threads, each summing FIN_RPS rows of its 64 channels with all loads in flight (one round trip),
// writing that slice's sums, then the agent-scope release / arrival-ticket hand-off
// (cdna_hip_programming.md §5 "In-launch split-K reduction"): the workgroup that draws the last
// ticket of its channel group acquires, sums the S slice rows (one more round trip) and finishes
// the channels.  S = 1 (<= FIN_RPS rows) finishes directly.  Deterministic: fixed summation
// order whichever workgroup arrives last.
constexpr int FIN_RPS = 128;        // partial rows per slice (16 row lanes x 8 loads in flight)
constexpr int TICKETS = 8192, TICKET_WIN = 64;

// a window of TICKET_WIN zeroed arrival tickets for one launch (per device; the last arriver of
// each group re-zeroes its ticket, so a window is reusable once its launch has finished --
// TICKETS / TICKET_WIN launches later)
static int* fin_tickets() {
    static std::mutex mu;
    static std::unordered_map<int, int*> pools;
    static unsigned next = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    int*& pool = pools[dev];
    if (!pool) {
        if (hipMalloc(&pool, TICKETS * sizeof(int)) != hipSuccess) { pool = nullptr; return nullptr; }
        if (hipMemset(pool, 0, TICKETS * sizeof(int)) != hipSuccess) return nullptr;
    }
    int* w = pool + (next % (TICKETS / TICKET_WIN)) * TICKET_WIN;
    ++next;
    return w;
}

// this workgroup's sums of rows [r0, r1) for column c and C + c (double, thread < 64 holds them)
__device__ __forceinline__ void fin_slice(const float* __restrict__ part, int r0, int r1, long ld, int C, int c,
                                          bool ok, float* red, double& s, double& q) {
    const int rl = threadIdx.x >> 6;
    float a = 0.f, b = 0.f;
    if (ok) {
        float va[8], vb[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int r = r0 + rl + 16 * i;
            va[i] = r < r1 ? part[(long)r * ld + c] : 0.f;
            vb[i] = r < r1 ? part[(long)r * ld + C + c] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) { a += va[i]; b += vb[i]; }
        for (int r = r0 + rl + 128; r < r1; r += 16) {      // rows beyond one round trip (S capped)
            a += part[(long)r * ld + c];
            b += part[(long)r * ld + C + c];
        }
    }
    red[threadIdx.x] = a;
    red[1024 + threadIdx.x] = b;
    __syncthreads();
    s = 0.0;
    q = 0.0;
    if (threadIdx.x < 64) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            s += (double)red[i * 64 + threadIdx.x];
            q += (double)red[1024 + i * 64 + threadIdx.x];
        }
    }
    __syncthreads();
}

// S > 1: publish this slice's sums, then the last arriver of the channel group returns true with
// (s, q) = the full sums (threads < 64); every other workgroup returns false
__device__ __forceinline__ bool fin_publish(float* __restrict__ ws, int* __restrict__ tickets, int C, int c, bool ok,
                                            float* red, int* flag, double& s, double& q) {
    if (threadIdx.x < 64 && ok) {
        ws[(long)blockIdx.y * 2 * C + c] = (float)s;
        ws[(long)blockIdx.y * 2 * C + C + c] = (float)q;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // keep: the fence's own wait can be dropped
        const int t = __hip_atomic_fetch_add(tickets + blockIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = t == (int)gridDim.y - 1;
        if (last) {
            __hip_atomic_store(tickets + blockIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *flag = last ? 1 : 0;
    }
    __syncthreads();
    if (!*flag) return false;
    fin_slice(ws, 0, gridDim.y, 2L * C, C, c, ok, red, s, q);
    return true;
}

template <typename TP>
__global__ __launch_bounds__(1024) void bn_fwd_finalize_k(const float* __restrict__ part, int nblk, int rps, int C,
                                   long M, float* __restrict__ ws, int* __restrict__ tickets, const TP* __restrict__ gamma,
                                   const TP* __restrict__ beta, float* __restrict__ running_mean,
                                   float* __restrict__ running_var, float momentum, float eps,
                                   float* __restrict__ save_mean, float* __restrict__ save_invstd,
                                   float* __restrict__ scale, float* __restrict__ shift) {
    __shared__ float red[2048];
    __shared__ int flag;
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const bool ok = c < C;
    const int r0 = blockIdx.y * rps;
    double s, q;
    fin_slice(part, r0, min(nblk, r0 + rps), 2L * C, C, c, ok, red, s, q);
    if (gridDim.y > 1 && !fin_publish(ws, tickets, C, c, ok, red, &flag, s, q)) return;
    if (threadIdx.x < 64 && ok)
        bn_fwd_finish_channel<TP>(c, s, q, M, gamma, beta, running_mean, running_var, momentum, eps, save_mean,
                                  save_invstd, scale, shift);
}

template <typename TP>
__global__ __launch_bounds__(1024) void bn_bwd_finalize2_k(const float* __restrict__ part, int nblk, int rps, int C,
                                    long M, float* __restrict__ ws, int* __restrict__ tickets, const TP* __restrict__ gamma,
                                    const float* __restrict__ invstd, TP* __restrict__ dgamma, TP* __restrict__ dbeta,
                                    float* __restrict__ coef, int acc) {
    __shared__ float red[2048];
    __shared__ int flag;
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const bool ok = c < C;
    const int r0 = blockIdx.y * rps;
    double s, q;
    fin_slice(part, r0, min(nblk, r0 + rps), 2L * C, C, c, ok, red, s, q);
    if (gridDim.y > 1 && !fin_publish(ws, tickets, C, c, ok, red, &flag, s, q)) return;
    if (threadIdx.x < 64 && ok)
        bn_bwd_finish_channel<TP>(c, s, q, C, M, gamma, invstd, dgamma, dbeta, coef, acc, nullptr);
}

// The same merged scheme for the LayerNorm backward's column sums: NV = 2 ([dgamma | dbeta]) or 3
// (+ the sum of dx: the producing Linear's bias gradient) columns of width H per partial row, all
// NV loads of a row issued together (the single-workgroup colsum_partials_k walked the three
// columns one after another: 3 x 4 dependent round trips over 512 rows).
template <int NV>
__device__ __forceinline__ void fin_slice_nv(const float* __restrict__ part, int r0, int r1, long ld, int H, int c,
                                             bool ok, float* red, float* out) {
    const int rl = threadIdx.x >> 6;
    float a[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) a[v] = 0.f;
    if (ok) {
        float x[NV][8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int r = r0 + rl + 16 * i;
#pragma unroll
            for (int v = 0; v < NV; ++v) x[v][i] = r < r1 ? part[(long)r * ld + v * H + c] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int v = 0; v < NV; ++v) a[v] += x[v][i];
        for (int r = r0 + rl + 128; r < r1; r += 16)
#pragma unroll
            for (int v = 0; v < NV; ++v) a[v] += part[(long)r * ld + v * H + c];
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) red[v * 1024 + threadIdx.x] = a[v];
    __syncthreads();
    if (threadIdx.x < 64) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            float t = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) t += red[v * 1024 + i * 64 + threadIdx.x];
            out[v] = t;
        }
    }
    __syncthreads();
}

template <typename TP, int NV>
__global__ __launch_bounds__(1024) void ln_colsum_k(const float* __restrict__ part, int nblk, int rps, int H,
                                                    float* __restrict__ ws, int* __restrict__ tickets,
                                                    TP* __restrict__ dg, TP* __restrict__ db, int acc,
                                                    float* __restrict__ dxsum, TP* __restrict__ dxsink) {
    __shared__ float red[NV * 1024];
    __shared__ int flag;
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const bool ok = c < H;
    const int r0 = blockIdx.y * rps;
    float sum[NV];
    fin_slice_nv<NV>(part, r0, min(nblk, r0 + rps), (long)NV * H, H, c, ok, red, sum);
    if (gridDim.y > 1) {
        if (threadIdx.x < 64 && ok) {
#pragma unroll
            for (int v = 0; v < NV; ++v) ws[(long)blockIdx.y * NV * H + v * H + c] = sum[v];
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const int t = __hip_atomic_fetch_add(tickets + blockIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const bool last = t == (int)gridDim.y - 1;
            if (last) {
                __hip_atomic_store(tickets + blockIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            flag = last ? 1 : 0;
        }
        __syncthreads();
        if (!flag) return;
        fin_slice_nv<NV>(ws, 0, gridDim.y, (long)NV * H, H, c, ok, red, sum);
    }
    if (threadIdx.x >= 64 || !ok) return;
    dg[c] = from_f<TP>(sum[0] + (acc ? to_f(dg[c]) : 0.f));
    db[c] = from_f<TP>(sum[1] + (acc ? to_f(db[c]) : 0.f));
    if constexpr (NV == 3) {
        if (dxsum) dxsum[c] = sum[2];
        if (dxsink) dxsink[c] = from_f<TP>(sum[2] + (acc ? to_f(dxsink[c]) : 0.f));
    }
}

// slices for nblk partial rows: S = ceil(nblk / FIN_RPS), capped so the last arriver's pass over
// the slice rows stays one round trip of 16 row lanes x 8 (ws holds S x 2C floats)
// DDL_FIN_RPS (>= 32: the partial-row buffers hold ceil(nblk / 32) slice rows): rows per slice (A/B)
static int fin_rps_target() {
    static const int v = [] { const char* e = getenv("DDL_FIN_RPS"); return e ? std::max(32, atoi(e)) : FIN_RPS; }();
    return v;
}
static int fin_slices(int nblk) {
    const int t = fin_rps_target();
    return std::max(1, std::min(128, (nblk + t - 1) / t));
}
static int fin_rps(int nblk) { return (nblk + fin_slices(nblk) - 1) / fin_slices(nblk); }
// The merged launch took 7.6-8.3 us against 6.7 us for one finalize workgroup on <= 512 rows in
// the round-5 kernel tables, but whole-step A/B prefers it for every row count: ResNet-50 +0.3 %
// same-box, BERT-base neutral (profiles/merged_fin_ab.log) -- the single workgroup's long tail
// delays the dependent apply launch.  DDL_BN_MERGED_FIN=0: never, =1: above 512 rows only, 2:
// always (default).
static int merged_mode() {
    static const int m = [] { const char* e = getenv("DDL_BN_MERGED_FIN"); return e ? atoi(e) : 2; }();
    return m;
}
// (each launch owns one window of TICKET_WIN arrival tickets, one per 64-channel group: wider
// layers than TICKET_WIN * 64 channels take the collapse + single-pass finalize instead, so a
// group index can never reach into the next launch's window or past the pool)
static bool merged_finalize(int nblk, int C) {
    const int m = merged_mode();
    return (C + 63) / 64 <= TICKET_WIN && (m == 2 || (m == 1 && nblk > 512));
}

// Partial rows beyond this are first collapsed 32:1 (a single finalize block per
// 64 columns is too little parallelism for ~1000 rows).  The caller allocates
// `part` with room for the collapsed rows behind the nblk partial rows.
// DDL_BN_COLLAPSE_MIN overrides the threshold (collapse_partials and ddl_bn_partials_ws)
static int collapse_env() {
    static const int v = [] { const char* e = getenv("DDL_BN_COLLAPSE_MIN"); return e ? atoi(e) : 0; }();
    return v;
}
// Up to COLLAPSE_OVER rows the single column-sum kernel reads every row itself (colsum64: 8 rows
// in flight per thread, <= 4 round trips): the collapse launch cost more than it saved there
// (BERT-base: 49 collapse launches of ~5 us per step for 128- and 512-row partials).
constexpr int COLLAPSE_OVER = 512;
static bool needs_collapse(int nblk) { return nblk > (collapse_env() > 0 ? collapse_env() : COLLAPSE_OVER); }
static const float* collapse_partials(const float* part, int& nblk, int width, hipStream_t st,
                                      float* ws = nullptr) {
    if (!needs_collapse(nblk)) return part;
    if (!ws) ws = const_cast<float*>(part) + (long)nblk * width;
    const int chunks = (nblk + PC_ROWS - 1) / PC_ROWS;
    bn_partials_collapse_k<<<dim3((width + 255) / 256, chunks), 256, 0, st>>>(part, nblk, width, ws);
    nblk = chunks;
    return ws;
}

DDL_API long ddl_bn_partials_ws(int nblk, int C) {
    return needs_collapse(nblk) ? (long)((nblk + PC_ROWS - 1) / PC_ROWS) * 2 * C : 0;
}

DDL_API int ddl_bn_fwd_from_partials(int dtype, const float* part, int nblk, long M, int C, const void* gamma,
                                     const void* beta, float* running_mean, float* running_var, float momentum,
                                     float eps, float* save_mean, float* save_invstd, float* scale, float* shift,
                                     float* ws, long ws_elems, hipStream_t st) {
    if (merged_finalize(nblk, C)) {
        const int S = fin_slices(nblk);
        int* tk = S > 1 ? fin_tickets() : nullptr;
        if (S == 1 || (tk && ws && ws_elems >= (long)S * 2 * C)) {
            const dim3 grid((C + 63) / 64, S);
            if (dtype == 1)
                bn_fwd_finalize_k<bf16_t><<<grid, 1024, 0, st>>>(part, nblk, fin_rps(nblk), C, M, ws, tk,
                    (const bf16_t*)gamma, (const bf16_t*)beta, running_mean, running_var, momentum, eps, save_mean,
                    save_invstd, scale, shift);
            else
                bn_fwd_finalize_k<float><<<grid, 1024, 0, st>>>(part, nblk, fin_rps(nblk), C, M, ws, tk,
                    (const float*)gamma, (const float*)beta, running_mean, running_var, momentum, eps, save_mean,
                    save_invstd, scale, shift);
            DDL_RETURN_LAUNCH();
        }
    }
    const long need = ddl_bn_partials_ws(nblk, C);
    if (need > 0) {
        if (!ws || ws_elems < need) return -2;
        const int chunks = (nblk + PC_ROWS - 1) / PC_ROWS;
        bn_partials_collapse_k<<<dim3((2 * C + 255) / 256, chunks), 256, 0, st>>>(part, nblk, 2 * C, ws);
        part = ws;
        nblk = chunks;
    }
    if (dtype == 1)
        bn_stats_finalize_k<bf16_t><<<(C + 63) / 64, 1024, 0, st>>>(part, nblk, C, M, (const bf16_t*)gamma,
            (const bf16_t*)beta, running_mean, running_var, momentum, eps, save_mean, save_invstd, scale, shift);
    else
        bn_stats_finalize_k<float><<<(C + 63) / 64, 1024, 0, st>>>(part, nblk, C, M, (const float*)gamma,
            (const float*)beta, running_mean, running_var, momentum, eps, save_mean, save_invstd, scale, shift);
    DDL_RETURN_LAUNCH();
}

DDL_API int ddl_bn_eval_coeffs(int dtype, int C, const void* gamma, const void* beta, const float* rm,
                               const float* rv, float eps, float* scale, float* shift, hipStream_t st) {
    if (dtype == 1)
        bn_eval_coeffs_k<bf16_t><<<(C + 255) / 256, 256, 0, st>>>(C, (const bf16_t*)gamma, (const bf16_t*)beta, rm, rv,
                                                                  eps, scale, shift);
    else
        bn_eval_coeffs_k<float><<<(C + 255) / 256, 256, 0, st>>>(C, (const float*)gamma, (const float*)beta, rm, rv,
                                                                 eps, scale, shift);
    DDL_RETURN_LAUNCH();
}

template <typename T>
static void bn_apply_dispatch(const T* x, const T* res, const float* sc, const float* sh, T* y, uint8_t* mask, long n,
                              int C, int relu, hipStream_t st) {
    if (rows_ok(C) && n % C == 0) {
        const long M = n / C;
        auto k = res ? (relu ? bn_apply_rows_k<T, true, true> : bn_apply_rows_k<T, true, false>)
                     : (relu ? bn_apply_rows_k<T, false, true> : bn_apply_rows_k<T, false, false>);
        hipLaunchKernelGGL(k, dim3(rows_grid(M, C, (const void*)k)), dim3(256), 0, st, x, res, sc, sh, y, mask, M, C);
        return;
    }
    const long n8 = n / 8;
    const int g = grid_for(n8, 256, 8192);
    if (res) {
        if (relu) bn_apply_k<T, true, true><<<g, 256, 0, st>>>(x, res, sc, sh, y, mask, n8, C);
        else bn_apply_k<T, true, false><<<g, 256, 0, st>>>(x, res, sc, sh, y, mask, n8, C);
    } else {
        if (relu) bn_apply_k<T, false, true><<<g, 256, 0, st>>>(x, res, sc, sh, y, mask, n8, C);
        else bn_apply_k<T, false, false><<<g, 256, 0, st>>>(x, res, sc, sh, y, mask, n8, C);
    }
}

// y = relu?(x * scale + shift + x2 * scale2 + shift2), bit mask as ddl_bn_apply (row-major
// channel counts only: -1 otherwise)
DDL_API int ddl_bn_apply2(int dtype, const void* x, const void* x2, const float* scale, const float* shift,
                          const float* scale2, const float* shift2, void* y, long n, int C, int relu, void* mask,
                          hipStream_t st) {
    if (n % 8 || !rows_ok(C) || n % C) return -1;
    const long M = n / C;
    uint8_t* mk = (uint8_t*)mask;
#define BA2(T) do { auto k = relu ? bn_apply2_rows_k<T, true> : bn_apply2_rows_k<T, false>; \
                    hipLaunchKernelGGL(k, dim3(rows_grid(M, C, (const void*)k)), dim3(256), 0, st, (const T*)x, (const T*)x2, \
                                       scale, shift, scale2, shift2, (T*)y, mk, M, C); } while (0)
    if (dtype == 1) BA2(bf16_t);
    else BA2(float);
#undef BA2
    DDL_RETURN_LAUNCH();
}

DDL_API int ddl_bn_apply(int dtype, const void* x, const void* res, const float* scale, const float* shift, void* y,
                         long n, int C, int relu, void* mask, hipStream_t st) {
    if (n % 8 || C % 8) return -1;
    uint8_t* mk = (uint8_t*)mask;
    if (dtype == 1) bn_apply_dispatch((const bf16_t*)x, (const bf16_t*)res, scale, shift, (bf16_t*)y, mk, n, C, relu, st);
    else bn_apply_dispatch((const float*)x, (const float*)res, scale, shift, (float*)y, mk, n, C, relu, st);
    DDL_RETURN_LAUNCH();
}

// backward coefficients (+ dgamma / dbeta) from nblk partial rows: collapse (if many) + finalize
// ws: null = the room behind the nblk partial rows (ceil(nblk / 32) rows of 2C floats)
template <typename T>
static void bwd_finalize(const float* part, int nblk, float* ws, int C, long M, const T* gamma, const float* invstd,
                         T* dgamma, T* dbeta, float* coef, int acc, hipStream_t st) {
    if (merged_finalize(nblk, C)) {
        const int S = fin_slices(nblk);
        int* tk = S > 1 ? fin_tickets() : nullptr;
        if (S == 1 || tk) {
            if (!ws) ws = const_cast<float*>(part) + (long)nblk * 2 * C;
            bn_bwd_finalize2_k<T><<<dim3((C + 63) / 64, S), 1024, 0, st>>>(part, nblk, fin_rps(nblk), C, M, ws, tk,
                                                                           gamma, invstd, dgamma, dbeta, coef, acc);
            return;
        }
    }
    int nrows = nblk;
    const float* fin = collapse_partials(part, nrows, 2 * C, st, ws);
    bn_bwd_finalize_k<T><<<(C + 63) / 64, 1024, 0, st>>>(fin, nrows, C, M, gamma, invstd, dgamma, dbeta, coef, acc);
}

template <typename T>
static void bn_bwd_dispatch(const T* dy, const uint8_t* yout, const T* x, const float* mean, const float* invstd,
                            const T* gamma, long M, int C, int relu, float* part, T* dgamma, T* dbeta, float* coef,
                            T* dx, T* dres, int acc, hipStream_t st) {
    const int nblk = ddl_bn_bwd_nblk(M, C);
    const int rpi = BN_NT / (C / 8);
    long rpb = (M + nblk - 1) / nblk;
    rpb = (rpb + rpi - 1) / rpi * rpi;
    if (relu) bn_bwd_partial_k<T, true><<<nblk, BN_NT, 0, st>>>(dy, yout, x, mean, invstd, M, C, (int)rpb, part);
    else bn_bwd_partial_k<T, false><<<nblk, BN_NT, 0, st>>>(dy, yout, x, mean, invstd, M, C, (int)rpb, part);
    bwd_finalize<T>(part, nblk, nullptr, C, M, gamma, invstd, dgamma, dbeta, coef, acc, st);
    if (rows_ok(C)) {
        auto k = relu ? (dres ? bn_bwd_apply_rows_k<T, true, true> : bn_bwd_apply_rows_k<T, true, false>)
                      : (dres ? bn_bwd_apply_rows_k<T, false, true> : bn_bwd_apply_rows_k<T, false, false>);
        hipLaunchKernelGGL(k, dim3(rows_grid(M, C, (const void*)k)), dim3(256), 0, st, dy, yout, x, mean, invstd, coef,
                           dx, dres, M, C);
        return;
    }
    const long n8 = M * C / 8;
    const int g = grid_for(n8, 256, 8192);
    if (relu) {
        if (dres) bn_bwd_apply_k<T, true, true><<<g, 256, 0, st>>>(dy, yout, x, mean, invstd, coef, dx, dres, n8, C);
        else bn_bwd_apply_k<T, true, false><<<g, 256, 0, st>>>(dy, yout, x, mean, invstd, coef, dx, dres, n8, C);
    } else {
        if (dres) bn_bwd_apply_k<T, false, true><<<g, 256, 0, st>>>(dy, yout, x, mean, invstd, coef, dx, dres, n8, C);
        else bn_bwd_apply_k<T, false, false><<<g, 256, 0, st>>>(dy, yout, x, mean, invstd, coef, dx, dres, n8, C);
    }
}

// relu: `mask` is the bit mask written by ddl_bn_apply (required when relu != 0);
// part: (nblk + ceil(nblk/32)) * 2C floats, nblk = ddl_bn_bwd_nblk(M, C)
DDL_API int ddl_bn_bwd(int dtype, const void* dy, const void* mask, const void* x, const float* mean,
                       const float* invstd, const void* gamma, long M, int C, int relu, float* part, void* dgamma,
                       void* dbeta, float* coef, void* dx, void* dres, int acc_params, hipStream_t st) {
    if (C % 8 || (BN_NT % (C / 8) != 0) || (relu && !mask)) return -1;
    const uint8_t* yout = (const uint8_t*)mask;
    if (dtype == 1)
        bn_bwd_dispatch((const bf16_t*)dy, yout, (const bf16_t*)x, mean, invstd, (const bf16_t*)gamma, M,
                        C, relu, part, (bf16_t*)dgamma, (bf16_t*)dbeta, coef, (bf16_t*)dx, (bf16_t*)dres, acc_params, st);
    else
        bn_bwd_dispatch((const float*)dy, yout, (const float*)x, mean, invstd, (const float*)gamma, M, C,
                        relu, part, (float*)dgamma, (float*)dbeta, coef, (float*)dx, (float*)dres, acc_params, st);
    DDL_RETURN_LAUNCH();
}

// ---------------------------------------------------------------- stem backward
// BatchNorm + ReLU backward of the ResNet stem straight from the max-pool's output gradient:
// the max-pool 3x3/2/pad1 backward (a gather over the <= 4 windows covering a pixel, matched
// against the stored window argmax) is evaluated in both BatchNorm passes instead of
// writing the full-resolution activation gradient and reading it twice.
namespace {
template <typename T>
__device__ __forceinline__ void pool_grad8(const T* __restrict__ dy, const uint8_t* __restrict__ idx, long n, int h,
                                           int w, int cg, int C, int P, int Q, float* acc) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    const int p_lo = h >> 1, p_hi = min(P - 1, (h + 1) >> 1);
    const int q_lo = w >> 1, q_hi = min(Q - 1, (w + 1) >> 1);
    for (int p = p_lo; p <= p_hi; ++p) {
        const int r = h - 2 * p + 1;
        for (int q = q_lo; q <= q_hi; ++q) {
            const int s_ = w - 2 * q + 1;
            const long o = ((n * P + p) * Q + q) * C + cg * 8;
            float g[8];
            load8(dy + o, g);
            const uint2 packed = *reinterpret_cast<const uint2*>(idx + o);
            const uint32_t want = (uint32_t)(r * 3 + s_);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t word = j < 4 ? packed.x : packed.y;
                acc[j] += ((word >> (8 * (j & 3))) & 0xffu) == want ? g[j] : 0.f;
            }
        }
    }
}

// per block: [sum dz | sum dz * xhat] (dz = relu_mask * maxpool_bwd(dy)); a thread keeps one
// channel group for the whole launch (256 % (C / 8) == 0)
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_pool_partial_k(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                             const uint8_t* __restrict__ mask, const T* __restrict__ x,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ invstd, int N, int H, int W,
                                                             int C, int P, int Q, float* __restrict__ part) {
    __shared__ float s_red[256 * 16];
    const int c8 = C / 8, tid = threadIdx.x, cg = tid % c8;
    float mu[8], is[8], a[8], b[8];
    load8(mean + cg * 8, mu);
    load8(invstd + cg * 8, is);
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = 0.f; b[j] = 0.f; }
    const long total = (long)N * H * W * c8;
    for (long i = (long)blockIdx.x * 256 + tid; i < total; i += (long)gridDim.x * 256) {
        const long pix = i / c8;
        const int w = (int)(pix % W);
        const long t = pix / W;
        const int h = (int)(t % H);
        const long n = t / H;
        float da[8], xv[8];
        pool_grad8(dy, idx, n, h, w, cg, C, P, Q, da);
        load8(x + i * 8, xv);
        const uint32_t bits = mask[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float dz = ((bits >> j) & 1u) ? da[j] : 0.f;
            a[j] += dz;
            b[j] += dz * (xv[j] - mu[j]) * is[j];
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        s_red[tid * 16 + j] = a[j];
        s_red[tid * 16 + 8 + j] = b[j];
    }
    __syncthreads();
    for (int c = tid; c < 2 * C; c += 256) {
        const int ch = c % C, g = ch / 8, j = ch % 8, off = c < C ? 0 : 8;
        float s = 0.f;
        for (int u = g; u < 256; u += c8) s += s_red[u * 16 + off + j];
        part[(long)blockIdx.x * 2 * C + c] = s;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_pool_apply_k(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                           const uint8_t* __restrict__ mask, const T* __restrict__ x,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ coef, T* __restrict__ dx, int N,
                                                           int H, int W, int C, int P, int Q) {
    const int c8 = C / 8, cg = threadIdx.x % c8;
    float A[8], B[8], D[8];
    {
        float mu[8], is[8], k1[8], mb[8], mg[8];
        load8(mean + cg * 8, mu);
        load8(invstd + cg * 8, is);
        load8(coef + cg * 8, k1);
        load8(coef + C + cg * 8, mb);
        load8(coef + 2 * C + cg * 8, mg);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            A[j] = k1[j];
            B[j] = -k1[j] * is[j] * mg[j];
            D[j] = k1[j] * (mu[j] * is[j] * mg[j] - mb[j]);
        }
    }
    const long total = (long)N * H * W * c8;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const long pix = i / c8;
        const int w = (int)(pix % W);
        const long t = pix / W;
        const int h = (int)(t % H);
        const long n = t / H;
        float da[8], xv[8], o[8];
        pool_grad8(dy, idx, n, h, w, cg, C, P, Q, da);
        load8(x + i * 8, xv);
        const uint32_t bits = mask[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = A[j] * (((bits >> j) & 1u) ? da[j] : 0.f) + B[j] * xv[j] + D[j];
        store8(dx + i * 8, o);
    }
}
}  // namespace

DDL_API int ddl_bn_bwd_pool_nblk() { return 1024; }

// dx = BatchNorm + ReLU backward of the stem given the max-pool 3x3/2/pad1 output gradient dy
// [N, P, Q, C] and window argmax idx (ddl_bn_relu_maxpool); part: (nblk + ceil(nblk / 32)) * 2C
DDL_API int ddl_bn_bwd_pool(int dtype, const void* dy, const uint8_t* idx, const uint8_t* mask, const void* x,
                            const float* mean, const float* invstd, const void* gamma, int N, int H, int W, int C,
                            int P, int Q, float* part, void* dgamma, void* dbeta, float* coef, void* dx,
                            int acc_params, hipStream_t st) {
    if (C % 8 || 256 % (C / 8) || H != 2 * P || W != 2 * Q || !mask) return -1;
    const int nblk = ddl_bn_bwd_pool_nblk();
    const long M = (long)N * H * W;
    int nrows = nblk;
#define BBP(T) do {                                                                                                     \
        bn_bwd_pool_partial_k<T><<<nblk, 256, 0, st>>>((const T*)dy, idx, mask, (const T*)x, mean, invstd, N, H, W, C,  \
                                                       P, Q, part);                                                     \
        bwd_finalize<T>(part, nrows, nullptr, C, M, (const T*)gamma, invstd, (T*)dgamma, (T*)dbeta, coef, acc_params,   \
                        st);                                                                                            \
        bn_bwd_pool_apply_k<T><<<grid_for(M * (C / 8), 256, 8192), 256, 0, st>>>((const T*)dy, idx, mask, (const T*)x,   \
                                                                                mean, invstd, coef, (T*)dx, N, H, W, C, \
                                                                                P, Q);                                   \
    } while (0)
    if (dtype == 1) BBP(bf16_t);
    else BBP(float);
#undef BBP
    DDL_RETURN_LAUNCH();
}

// ---------------------------------------------------------------- LayerNorm
// DDL_LN_FWD8=0: the wave-per-row bf16 forward (A/B timing)
static bool ln_fwd8_enabled() {
    static const bool on = [] { const char* e = getenv("DDL_LN_FWD8"); return !(e && e[0] == '0'); }();
    return on;
}

template <typename T>
static int ln_fwd_dispatch(const T* x, const T* res, long res_rows, const T* g, const T* b, T* y, float* mean,
                           float* rstd, long rows, int H, float eps, Drop drop, hipStream_t st) {
    if constexpr (sizeof(T) == 2) {
        if (ln_fwd8_enabled() && (H / 256 == 3 || H / 256 == 4)) {
            const int grid8 = (int)((rows + 7) / 8);
            if (H / 256 == 3) ln_fwd8_k<3><<<grid8, 256, 0, st>>>(x, res, res_rows, g, b, y, mean, rstd, rows, H, eps, drop);
            else ln_fwd8_k<4><<<grid8, 256, 0, st>>>(x, res, res_rows, g, b, y, mean, rstd, rows, H, eps, drop);
            return 0;
        }
    }
    const int grid = (int)((rows + 3) / 4);
    switch (H / 256) {
        case 1: ln_fwd_k<T, 1><<<grid, 256, 0, st>>>(x, res, res_rows, g, b, y, mean, rstd, rows, H, eps, drop); break;
        case 2: ln_fwd_k<T, 2><<<grid, 256, 0, st>>>(x, res, res_rows, g, b, y, mean, rstd, rows, H, eps, drop); break;
        case 3: ln_fwd_k<T, 3><<<grid, 256, 0, st>>>(x, res, res_rows, g, b, y, mean, rstd, rows, H, eps, drop); break;
        case 4: ln_fwd_k<T, 4><<<grid, 256, 0, st>>>(x, res, res_rows, g, b, y, mean, rstd, rows, H, eps, drop); break;
        case 5: ln_fwd_k<T, 5><<<grid, 256, 0, st>>>(x, res, res_rows, g, b, y, mean, rstd, rows, H, eps, drop); break;
        case 6: ln_fwd_k<T, 6><<<grid, 256, 0, st>>>(x, res, res_rows, g, b, y, mean, rstd, rows, H, eps, drop); break;
        case 8: ln_fwd_k<T, 8><<<grid, 256, 0, st>>>(x, res, res_rows, g, b, y, mean, rstd, rows, H, eps, drop); break;
        default: return -1;
    }
    return 0;
}

DDL_API int ddl_ln_supported(int H) {
    const int v = H / 256;
    return (H % 256 == 0) && (v >= 1 && v <= 8 && v != 7);
}

static Drop make_drop(unsigned long long seed, float p, void* dres) {
    Drop d{};
    if (p > 0.f) {
        d.seed = seed;
        d.thresh = drop_thresh16(p);
        d.scale = 1.f / (1.f - p);
        d.dres = dres;
    }
    return d;
}

// drop_p > 0: y = LN(dropout(x) + res) with the hash mask of drop_seed
DDL_API int ddl_ln_fwd(int dtype, const void* x, const void* res, long res_rows, const void* g, const void* b, void* y,
                       float* mean, float* rstd, long rows, int H, float eps, unsigned long long drop_seed,
                       float drop_p, hipStream_t st) {
    if (!ddl_ln_supported(H)) return -1;
    if (res_rows <= 0) res_rows = rows;
    const Drop drop = make_drop(drop_seed, drop_p, nullptr);
    int rc = dtype == 1 ? ln_fwd_dispatch((const bf16_t*)x, (const bf16_t*)res, res_rows, (const bf16_t*)g,
                                          (const bf16_t*)b, (bf16_t*)y, mean, rstd, rows, H, eps, drop, st)
                        : ln_fwd_dispatch((const float*)x, (const float*)res, res_rows, (const float*)g,
                                          (const float*)b, (float*)y, mean, rstd, rows, H, eps, drop, st);
    if (rc) return rc;
    DDL_RETURN_LAUNCH();
}

// rows per block (DDL_LN_BWD_ROWS, default 32: +0.6% BERT-base over 16, 64 -2%) and block cap (DDL_LN_BWD_MAXBLK, default 1024)
static int ln_env(const char* name, int dflt) {
    const char* v = getenv(name);
    return v && atoi(v) > 0 ? atoi(v) : dflt;
}
// Blocks of ~32 rows, rounded UP to whole rounds of the blocks the CUs hold at once (2 per CU at the
// 230-240 VGPRs of the H = 768 / 1024 kernels): ViT's 25216 rows made 788 blocks -- one full round
// of 512 and a 276-block second one; now 1024 equal blocks of 24-25 rows (rpb = ceil(rows / nblk))
// run two full rounds.  DDL_LN_BWD_ROUNDS=0: the plain count (A/B timing).
DDL_API int ddl_ln_bwd_nblk(long rows) {
    static const int rpb = ln_env("DDL_LN_BWD_ROWS", 32), cap = ln_env("DDL_LN_BWD_MAXBLK", 1024);
    static const bool rounds = [] { const char* e = getenv("DDL_LN_BWD_ROUNDS"); return !(e && e[0] == '0'); }();
    long nblk = std::max<long>(1, std::min<long>(cap, (rows + rpb - 1) / rpb));
    const long slots = 2L * cu_count();
    if (rounds && nblk > slots && nblk % slots) nblk = std::min<long>(std::max<long>(cap, slots), (nblk + slots - 1) / slots * slots);
    return (int)std::min<long>(nblk, rows);
}

template <typename T>
static int ln_bwd_dispatch(const T* dy, const T* x, const T* res, long res_rows, const T* g, const float* mean,
                           const float* rstd, T* dx, float* part, T* dg, T* db, long rows, int H, int acc,
                           float* dxsum, T* dxsink, Drop drop, const T* dadd, hipStream_t st) {
    const int nblk = ddl_ln_bwd_nblk(rows);
    const int rpb = (int)((rows + nblk - 1) / nblk);
#define LNB(V, A, KN) ln_bwd_k<T, V, A, KN><<<nblk, 256, 0, st>>>(dy, x, res, res_rows, g, mean, rstd, dx, part, rows, H, rpb, dxsum != nullptr, drop, dadd)
    // H = 768 / 1024 (BERT, ViT): compiled per (residual, dropout) case; other widths check at run time
    const int known = 4 | (res ? 2 : 0) | (drop.thresh ? 1 : 0);
#define LNB_KNOWN(V, A) do { switch (known) { case 4: LNB(V, A, 4); break; case 5: LNB(V, A, 5); break; \
                                             case 6: LNB(V, A, 6); break; default: LNB(V, A, 7); break; } } while (0)
    if (dadd) {
        switch (H / 256) {
            case 1: LNB(1, true, 0); break;
            case 2: LNB(2, true, 0); break;
            case 3: LNB_KNOWN(3, true); break;
            case 4: LNB_KNOWN(4, true); break;
            default: return -4;
        }
    } else switch (H / 256) {
        case 1: ln_bwd_k<T, 1><<<nblk, 256, 0, st>>>(dy, x, res, res_rows, g, mean, rstd, dx, part, rows, H, rpb, dxsum != nullptr, drop); break;
        case 2: ln_bwd_k<T, 2><<<nblk, 256, 0, st>>>(dy, x, res, res_rows, g, mean, rstd, dx, part, rows, H, rpb, dxsum != nullptr, drop); break;
        case 3: LNB_KNOWN(3, false); break;
        case 4: LNB_KNOWN(4, false); break;
        case 5: ln_bwd_k<T, 5><<<nblk, 256, 0, st>>>(dy, x, res, res_rows, g, mean, rstd, dx, part, rows, H, rpb, dxsum != nullptr, drop); break;
        case 6: ln_bwd_k<T, 6><<<nblk, 256, 0, st>>>(dy, x, res, res_rows, g, mean, rstd, dx, part, rows, H, rpb, dxsum != nullptr, drop); break;
        case 8: ln_bwd_k<T, 8><<<nblk, 256, 0, st>>>(dy, x, res, res_rows, g, mean, rstd, dx, part, rows, H, rpb, dxsum != nullptr, drop); break;
        default: return -1;
    }
#undef LNB_KNOWN
#undef LNB
    if (merged_finalize(nblk, H)) {
        // one launch: 128-row slices + last-arriver combine (ws: the room behind the partial rows)
        const int S = fin_slices(nblk);
        int* tk = S > 1 ? fin_tickets() : nullptr;
        if (S == 1 || tk) {
            const int nv = dxsum ? 3 : 2;
            float* ws = part + (long)nblk * nv * H;
            const dim3 grid((H + 63) / 64, S);
            if (dxsum) ln_colsum_k<T, 3><<<grid, 1024, 0, st>>>(part, nblk, fin_rps(nblk), H, ws, tk, dg, db, acc, dxsum,
                                                               dxsink);
            else ln_colsum_k<T, 2><<<grid, 1024, 0, st>>>(part, nblk, fin_rps(nblk), H, ws, tk, dg, db, acc, nullptr,
                                                         nullptr);
            return 0;
        }
    }
    int nrows = nblk;
    const float* fin = collapse_partials(part, nrows, (dxsum ? 3 : 2) * H, st);
    colsum_partials_k<T><<<(H + 63) / 64, 1024, 0, st>>>(fin, nrows, H, dg, db, acc, dxsum, dxsink);
    return 0;
}

// part: (nblk + ceil(nblk/32)) * (dxsum ? 3 : 2) * H floats (partial rows + their
// collapse); dxsum (nullable, fp32 [H]) receives the
// column sums of dx -- the bias gradient of the Linear feeding this LayerNorm
// drop_p > 0: dx = gradient of x through the dropout mask, dres (required) = the
// unmasked gradient of (dropout(x) + res); dxsum then sums the masked dx.
// dxsink (nullable, dtype of dg): the same column sums also added to (acc_params) or
// stored in that Linear's bias gradient -- needs dxsum
DDL_API int ddl_ln_bwd(int dtype, const void* dy, const void* x, const void* res, long res_rows, const void* g,
                       const float* mean, const float* rstd, void* dx, float* part, void* dg, void* db, long rows, int H,
                       int acc_params, float* dxsum, unsigned long long drop_seed, float drop_p, void* dres,
                       void* dxsink, const void* dadd, hipStream_t st) {
    if (!ddl_ln_supported(H)) return -1;
    if (res_rows <= 0) res_rows = rows;
    if (drop_p > 0.f && (!dres || res_rows != rows)) return -2;
    if (dxsink && !dxsum) return -3;
    const Drop drop = make_drop(drop_seed, drop_p, dres);
    int rc = dtype == 1
                 ? ln_bwd_dispatch((const bf16_t*)dy, (const bf16_t*)x, (const bf16_t*)res, res_rows, (const bf16_t*)g,
                                   mean, rstd, (bf16_t*)dx, part, (bf16_t*)dg, (bf16_t*)db, rows, H, acc_params, dxsum,
                                   (bf16_t*)dxsink, drop, (const bf16_t*)dadd, st)
                 : ln_bwd_dispatch((const float*)dy, (const float*)x, (const float*)res, res_rows, (const float*)g, mean,
                                   rstd, (float*)dx, part, (float*)dg, (float*)db, rows, H, acc_params, dxsum,
                                   (float*)dxsink, drop, (const float*)dadd, st);
    if (rc) return rc;
    DDL_RETURN_LAUNCH();
}

// ---------------------------------------------------------------- SyncBatchNorm pieces
// Cross-rank BatchNorm needs the per-channel sums as ONE row before the finalize (the
// all-reduce runs between): partial passes, rows -> one row, finalize / apply with
// the global row count.
namespace {
__global__ __launch_bounds__(1024) void rows_sum_k(const float* __restrict__ part, int nrows, int width,
                                                   float* __restrict__ out) {
    __shared__ float red[1024];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const float s = colsum64(part, nrows, width, c, c < width, red);
    if (threadIdx.x < 64 && c < width) out[c] = s;
}
// sink[c] (+)= sum_r part[r][c] for c < n (row stride `width`): a column sum straight into a
// parameter's gradient slot (bf16 / fp32), no fp32 row + accumulate launch
template <typename TP>
__global__ __launch_bounds__(1024) void rows_sum_sink_k(const float* __restrict__ part, int nrows, int width, int n,
                                                        TP* __restrict__ sink, int acc) {
    __shared__ float red[1024];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const float s = colsum64(part, nrows, width, c, c < n, red);
    if (threadIdx.x < 64 && c < n) sink[c] = from_f<TP>(s + (acc ? to_f(sink[c]) : 0.f));
}
}  // namespace

DDL_API int ddl_rows_sum_sink(int dtype, const float* part, int nblk, int width, int n, void* sink, int acc,
                              float* ws, hipStream_t st) {
    if (n > width) return -1;
    int nrows = nblk;
    const float* src = collapse_partials(part, nrows, width, st, ws);
    if (dtype == 1) rows_sum_sink_k<bf16_t><<<(n + 63) / 64, 1024, 0, st>>>(src, nrows, width, n, (bf16_t*)sink, acc);
    else rows_sum_sink_k<float><<<(n + 63) / 64, 1024, 0, st>>>(src, nrows, width, n, (float*)sink, acc);
    DDL_RETURN_LAUNCH();
}

// out[c] = sum_r part[r][c]; ws (ceil(nblk/32) * width floats) may be null when part
// itself holds (nblk + ceil(nblk/32)) * width floats
DDL_API int ddl_bn_rows_sum(const float* part, int nblk, int width, float* out, float* ws, hipStream_t st) {
    int nrows = nblk;
    const float* src = collapse_partials(part, nrows, width, st, ws);
    rows_sum_k<<<(width + 63) / 64, 1024, 0, st>>>(src, nrows, width, out);
    DDL_RETURN_LAUNCH();
}

// forward statistics partials only: nblk = ddl_bn_stats_nblk(M, C) rows of [sum | sumsq]
DDL_API int ddl_bn_stats_partials(int dtype, const void* x, long M, int C, float* part, hipStream_t st) {
    if (C % 8 || (BN_NT % (C / 8) != 0)) return -1;
    const int nblk = ddl_bn_stats_nblk(M, C);
    const int rpi = BN_NT / (C / 8);
    long rpb = (M + nblk - 1) / nblk;
    rpb = (rpb + rpi - 1) / rpi * rpi;
    if (dtype == 1) bn_stats_partial_k<bf16_t><<<nblk, BN_NT, 0, st>>>((const bf16_t*)x, M, C, (int)rpb, part);
    else bn_stats_partial_k<float><<<nblk, BN_NT, 0, st>>>((const float*)x, M, C, (int)rpb, part);
    DDL_RETURN_LAUNCH();
}

// backward partials only: nblk = ddl_bn_bwd_nblk(M, C) rows of [sum dz | sum dz*xhat]
DDL_API int ddl_bn_bwd_partials(int dtype, const void* dy, const void* mask, const void* x, const float* mean,
                                const float* invstd, long M, int C, int relu, float* part, hipStream_t st) {
    if (C % 8 || (BN_NT % (C / 8) != 0) || (relu && !mask)) return -1;
    const int nblk = ddl_bn_bwd_nblk(M, C);
    const int rpi = BN_NT / (C / 8);
    long rpb = (M + nblk - 1) / nblk;
    rpb = (rpb + rpi - 1) / rpi * rpi;
    const uint8_t* mk = (const uint8_t*)mask;
#define BWP(T) do { if (relu) bn_bwd_partial_k<T, true><<<nblk, BN_NT, 0, st>>>((const T*)dy, mk, (const T*)x, mean, invstd, M, C, (int)rpb, part); \
                    else bn_bwd_partial_k<T, false><<<nblk, BN_NT, 0, st>>>((const T*)dy, mk, (const T*)x, mean, invstd, M, C, (int)rpb, part); } while (0)
    if (dtype == 1) BWP(bf16_t);
    else BWP(float);
#undef BWP
    DDL_RETURN_LAUNCH();
}

// backward finish from ONE (all-reduced) row [sum dz | sum dz*xhat]: the coefficients use it
// and the global row count M_total, the apply walks the local M rows; dgamma / dbeta come from
// local_row (this rank's own [sum dz | sum dz*xhat], taken before the all-reduce) when given
template <typename T>
static void bn_bwd_apply_only(const T* dy, const uint8_t* mk, const T* x, const float* mean, const float* invstd,
                              long M, int C, int relu, const float* coef, T* dx, T* dres, hipStream_t st) {
    if (!rows_ok(C)) return;
    auto k = relu ? (dres ? bn_bwd_apply_rows_k<T, true, true> : bn_bwd_apply_rows_k<T, true, false>)
                  : (dres ? bn_bwd_apply_rows_k<T, false, true> : bn_bwd_apply_rows_k<T, false, false>);
    hipLaunchKernelGGL(k, dim3(rows_grid(M, C, (const void*)k)), dim3(256), 0, st, dy, mk, x, mean, invstd, coef, dx,
                       dres, M, C);
}

template <typename T>
static void bn_bwd_finish_t(const T* dy, const uint8_t* mk, const T* x, const float* mean, const float* invstd,
                            const T* gamma, long M, long M_total, int C, int relu, const float* row, int nrows,
                            T* dgamma, T* dbeta, float* coef, T* dx, T* dres, int acc, hipStream_t st,
                            const float* prow = nullptr) {
    bn_bwd_finalize_k<T><<<(C + 63) / 64, 1024, 0, st>>>(row, nrows, C, M_total, gamma, invstd, dgamma, dbeta, coef,
                                                         acc, prow);
    bn_bwd_apply_only(dy, mk, x, mean, invstd, M, C, relu, coef, dx, dres, st);
}

DDL_API int ddl_bn_bwd_finish(int dtype, const void* dy, const void* mask, const void* x, const float* mean,
                              const float* invstd, const void* gamma, long M, long M_total, int C, int relu,
                              const float* row, const float* local_row, void* dgamma, void* dbeta, float* coef,
                              void* dx, void* dres, int acc_params, hipStream_t st) {
    if (!rows_ok(C) || (relu && !mask)) return -1;
    const uint8_t* mk = (const uint8_t*)mask;
    if (dtype == 1)
        bn_bwd_finish_t((const bf16_t*)dy, mk, (const bf16_t*)x, mean, invstd, (const bf16_t*)gamma, M, M_total, C,
                        relu, row, 1, (bf16_t*)dgamma, (bf16_t*)dbeta, coef, (bf16_t*)dx, (bf16_t*)dres, acc_params, st,
                        local_row);
    else
        bn_bwd_finish_t((const float*)dy, mk, (const float*)x, mean, invstd, (const float*)gamma, M, M_total, C,
                        relu, row, 1, (float*)dgamma, (float*)dbeta, coef, (float*)dx, (float*)dres, acc_params, st,
                        local_row);
    DDL_RETURN_LAUNCH();
}

// backward from [sum dz | sum dz*xhat] partial rows written by the dgrad GEMM that
// produced dz (ACT_BNB epilogue: dz already carries the ReLU mask); ws: ceil(nrows/32) * 2C
// floats for the 32:1 collapse (may be null when nrows <= 256)
DDL_API int ddl_bn_bwd_from_partials(int dtype, const float* part, int nrows, float* ws, long ws_elems,
                                     const void* dz, const void* x, const float* mean, const float* invstd,
                                     const void* gamma, long M, int C, void* dgamma, void* dbeta, float* coef, void* dx,
                                     void* dres, int acc_params, hipStream_t st) {
    if (!rows_ok(C) || dtype != 1) return -1;
    if (merged_finalize(nrows, C) && (fin_slices(nrows) == 1 || (ws && ws_elems >= (long)fin_slices(nrows) * 2 * C))) {
        bwd_finalize<bf16_t>(part, nrows, fin_slices(nrows) == 1 ? nullptr : ws, C, M, (const bf16_t*)gamma, invstd,
                             (bf16_t*)dgamma, (bf16_t*)dbeta, coef, acc_params, st);
        bn_bwd_apply_only((const bf16_t*)dz, nullptr, (const bf16_t*)x, mean, invstd, M, C, 0, coef, (bf16_t*)dx,
                          (bf16_t*)dres, st);
        DDL_RETURN_LAUNCH();
    }
    const long need = ddl_bn_partials_ws(nrows, C);
    if (need > 0 && (!ws || ws_elems < need)) return -2;
    if (need > 0) {
        bwd_finalize<bf16_t>(part, nrows, ws, C, M, (const bf16_t*)gamma, invstd, (bf16_t*)dgamma, (bf16_t*)dbeta, coef,
                             acc_params, st);
        bn_bwd_apply_only((const bf16_t*)dz, nullptr, (const bf16_t*)x, mean, invstd, M, C, 0, coef, (bf16_t*)dx,
                          (bf16_t*)dres, st);
        DDL_RETURN_LAUNCH();
    }
    bn_bwd_finish_t((const bf16_t*)dz, nullptr, (const bf16_t*)x, mean, invstd, (const bf16_t*)gamma, M, M, C, 0, part,
                    nrows, (bf16_t*)dgamma, (bf16_t*)dbeta, coef, (bf16_t*)dx, (bf16_t*)dres, acc_params, st);
    DDL_RETURN_LAUNCH();
}
