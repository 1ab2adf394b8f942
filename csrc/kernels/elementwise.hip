// Memory-bound elementwise / reduction kernels for gfx950: GELU, dropout,
// bias-gradient column sums, softmax cross-entropy, NHWC pooling, embedding.
// Every kernel moves 8 elements (16 B of bf16) per lane per access.
#include "ddl_common.h"

namespace {

inline int grid_for(long n, int nt = 256, int cap = 8192) {
    long g = (n + nt - 1) / nt;
    return (int)std::max<long>(1, std::min<long>(g, cap));
}

// ------------------------------------------------------------------ GELU
template <typename T>
__global__ __launch_bounds__(256) void gelu_fwd_k(const T* __restrict__ x, T* __restrict__ y, long n8) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
        float v[8];
        load8(x + i * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = gelu_erf(v[j]);
        store8(y + i * 8, v);
    }
}
template <typename T>
__global__ __launch_bounds__(256) void gelu_bwd_k(const T* __restrict__ dy, const T* __restrict__ x, T* __restrict__ dx,
                                                  long n8) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
        float g[8], v[8];
        load8(dy + i * 8, g);
        load8(x + i * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = g[j] * gelu_erf_grad(v[j]);
        store8(dx + i * 8, v);
    }
}

// ------------------------------------------------------------------ dropout
// keep bits from the pair hash of ddl_common.h (16-bit threshold); regenerated in backward.
template <typename T>
__global__ __launch_bounds__(256) void dropout_k(const T* __restrict__ x, T* __restrict__ y, long n8, uint64_t seed,
                                                 uint32_t thresh, float scale) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
        float v[8];
        load8(x + i * 8, v);
        const uint32_t kb = keep_bits4(seed, (uint64_t)i * 8, thresh) | (keep_bits4(seed, (uint64_t)i * 8 + 4, thresh) << 4);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = ((kb >> j) & 1u) ? v[j] * scale : 0.f;
        store8(y + i * 8, v);
    }
}

// ------------------------------------------------------------------ column sums
// out[c] = sum_r x[r, c] (bias gradient).  Partial per block then finalize.
template <typename T>
__global__ __launch_bounds__(256) void colsum_partial_k(const T* __restrict__ x, long rows, int C, int rows_per_blk,
                                                        float* __restrict__ part) {
    // each thread owns 8 columns; the block covers 256*8 columns x rows_per_blk rows
    const int c0 = (blockIdx.y * 256 + threadIdx.x) * 8;
    if (c0 >= C) return;
    const long r0 = (long)blockIdx.x * rows_per_blk;
    const long r1 = std::min<long>(rows, r0 + rows_per_blk);
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll 4
    for (long r = r0; r < r1; ++r) {
        float v[8];
        load8(x + r * C + c0, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += v[j];
    }
    store8(part + (long)blockIdx.x * C + c0, s);
}
// dz = dy * gelu'(z) written once, with its column partial sums (the Linear's bias
// gradient) accumulated in the same pass
template <typename T>
__global__ __launch_bounds__(256) void gelu_bwd_colsum_k(const T* __restrict__ dy, const T* __restrict__ z,
                                                         T* __restrict__ dz, long rows, int C, int rows_per_blk,
                                                         float* __restrict__ part) {
    const int c0 = (blockIdx.y * 256 + threadIdx.x) * 8;
    if (c0 >= C) return;
    const long r0 = (long)blockIdx.x * rows_per_blk;
    const long r1 = std::min<long>(rows, r0 + rows_per_blk);
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll 2
    for (long r = r0; r < r1; ++r) {
        float g[8], v[8];
        load8(dy + r * C + c0, g);
        load8(z + r * C + c0, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            g[j] *= gelu_erf_grad(v[j]);
            s[j] += to_f(from_f<T>(g[j]));
        }
        store8(dz + r * C + c0, g);
    }
    store8(part + (long)blockIdx.x * C + c0, s);
}

template <typename TO>
__global__ __launch_bounds__(1024) void colsum_final_k(const float* __restrict__ part, int nblk, int C,
                                                       TO* __restrict__ out, int accumulate) {
    __shared__ float red[1024];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    float s = colsum64(part, nblk, C, c, c < C, red);
    if (threadIdx.x >= 64 || c >= C) return;
    if (accumulate) s += to_f(out[c]);
    out[c] = from_f<TO>(s);
}

// ------------------------------------------------------------------ softmax CE
// One block (256 threads) per row.  Writes per-row loss and d(loss)/d(logits)
// for mean reduction (softmax - onehot) / B, in one pass over the logits.
template <typename T>
__global__ __launch_bounds__(256) void softmax_ce_k(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                    int C, float inv_b, float* __restrict__ row_loss,
                                                    T* __restrict__ dlogits) {
    __shared__ float red[4];
    const long row = blockIdx.x;
    const T* x = logits + row * C;
    float m = -INFINITY;
    for (int c = threadIdx.x; c < C; c += 256) m = fmaxf(m, to_f(x[c]));
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    __syncthreads();
    float s = 0.f;
    for (int c = threadIdx.x; c < C; c += 256) s += __expf(to_f(x[c]) - m);
    s = block_sum<256>(s, red);
    const float lse = m + __logf(s);
    const long lab = labels[row];
    if (threadIdx.x == 0) row_loss[row] = lse - to_f(x[lab]);
    if (dlogits) {
        const float inv_s = 1.f / s;
        for (int c = threadIdx.x; c < C; c += 256) {
            const float p = __expf(to_f(x[c]) - m) * inv_s;
            dlogits[row * C + c] = from_f<T>((p - (c == lab ? 1.f : 0.f)) * inv_b);
        }
    }
}
// Inference post-processing (K11): softmax over a row and its k largest
// probabilities, one 256-thread block per row (the reference's batch-1 top-5 over
// 1000 ImageNet classes).  Probabilities are staged in LDS (C <= 4096); the top-k
// is k rounds of a block-wide (value, index) argmax that masks the winner --
// ties resolve to the lower index, like torch.topk on distinct values.
template <typename T>
__global__ __launch_bounds__(256) void softmax_topk_k(const T* __restrict__ logits, int C, int k,
                                                      float* __restrict__ probs, float* __restrict__ top_v,
                                                      int64_t* __restrict__ top_i) {
    __shared__ float pr[4096];
    __shared__ float red[4];
    __shared__ float bv[4];
    __shared__ int bi[4];
    const long row = blockIdx.x;
    const T* x = logits + row * C;
    float m = -INFINITY;
    for (int c = threadIdx.x; c < C; c += 256) m = fmaxf(m, to_f(x[c]));
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    __syncthreads();
    float s = 0.f;
    for (int c = threadIdx.x; c < C; c += 256) {
        const float e = __expf(to_f(x[c]) - m);
        pr[c] = e;
        s += e;
    }
    s = block_sum<256>(s, red);
    const float inv_s = 1.f / s;
    for (int c = threadIdx.x; c < C; c += 256) {
        pr[c] *= inv_s;
        if (probs) probs[row * C + c] = pr[c];
    }
    __syncthreads();
    for (int r = 0; r < k; ++r) {
        float v = -1.f;
        int vi = C;
        for (int c = threadIdx.x; c < C; c += 256)
            if (pr[c] > v) { v = pr[c]; vi = c; }
        // wave argmax (higher value, then lower index)
        for (int o = 32; o > 0; o >>= 1) {
            const float ov = __shfl_xor(v, o);
            const int oi = __shfl_xor(vi, o);
            if (ov > v || (ov == v && oi < vi)) { v = ov; vi = oi; }
        }
        if ((threadIdx.x & 63) == 0) { bv[threadIdx.x >> 6] = v; bi[threadIdx.x >> 6] = vi; }
        __syncthreads();
        if (threadIdx.x == 0) {
            float best = bv[0];
            int besti = bi[0];
            for (int w = 1; w < 4; ++w)
                if (bv[w] > best || (bv[w] == best && bi[w] < besti)) { best = bv[w]; besti = bi[w]; }
            top_v[row * k + r] = best;
            top_i[row * k + r] = besti;
            pr[besti] = -2.f;     // remove the winner for the next round
        }
        __syncthreads();
    }
}

__global__ void mean_k(const float* __restrict__ v, long n, float* __restrict__ out) {
    __shared__ float red[4];
    float s = 0.f;
    for (long i = threadIdx.x; i < n; i += 256) s += v[i];
    s = block_sum<256>(s, red);
    if (threadIdx.x == 0) out[0] = s / (float)n;
}
template <typename T>
__global__ __launch_bounds__(256) void scale_k(const T* __restrict__ x, const float* __restrict__ s, T* __restrict__ y,
                                               long n) {
    const float a = s[0];
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        y[i] = from_f<T>(to_f(x[i]) * a);
}

// ------------------------------------------------------------------ NHWC max-pool 3x3/2
// Forward also records the window argmax (0..8) so backward is a gather.
template <typename T>
__global__ __launch_bounds__(256) void maxpool_fwd_k(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ idx,
                                                     int N, int H, int W, int C, int P, int Q, int K, int S, int pad) {
    const int c8 = C / 8;
    const long total = (long)N * P * Q * c8;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int cg = (int)(i % c8);
        long t = i / c8;
        const int q = (int)(t % Q); t /= Q;
        const int p = (int)(t % P);
        const int n = (int)(t / P);
        float best[8];
        uint8_t arg[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; arg[j] = 0; }
        for (int r = 0; r < K; ++r) {
            const int h = p * S - pad + r;
            if (h < 0 || h >= H) continue;
            for (int s = 0; s < K; ++s) {
                const int w = q * S - pad + s;
                if (w < 0 || w >= W) continue;
                float v[8];
                load8(x + (((long)n * H + h) * W + w) * C + cg * 8, v);
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (v[j] > best[j] || (v[j] != v[j])) { best[j] = v[j]; arg[j] = (uint8_t)(r * K + s); }
            }
        }
        store8(y + i * 8, best);
        uint2 packed;
        packed.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | ((uint32_t)arg[3] << 24);
        packed.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | ((uint32_t)arg[7] << 24);
        *reinterpret_cast<uint2*>(idx + i * 8) = packed;
    }
}
// ResNet stem: training BatchNorm apply + ReLU + max-pool 3x3/2 (pad 1) in one pass over the
// conv output (the full-resolution activation is never written).  Needs H == 2P, W == 2Q:
// output pixel (p, q) owns input pixels (2p..2p+1, 2q..2q+1) and writes their ReLU-mask
// bits (bn_apply's layout: bit j of byte e/8 for flat NHWC element e).  Pools the
// bf16-rounded activations with maxpool_fwd_k's tie / NaN rules, so y and idx equal the
// unfused BN apply -> max-pool.
template <typename T>
__global__ __launch_bounds__(256) void bn_relu_maxpool_k(const T* __restrict__ x, const float* __restrict__ scale,
                                                         const float* __restrict__ shift, T* __restrict__ y,
                                                         uint8_t* __restrict__ idx, uint8_t* __restrict__ mask, int N,
                                                         int H, int W, int C, int P, int Q) {
    const int c8 = C / 8;
    const long total = (long)N * P * Q * c8;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int cg = (int)(i % c8);
        long t = i / c8;
        const int q = (int)(t % Q); t /= Q;
        const int p = (int)(t % P);
        const int n = (int)(t / P);
        float sc[8], sh[8], best[8];
        uint8_t arg[8];
        load8(scale + cg * 8, sc);
        load8(shift + cg * 8, sh);
#pragma unroll
        for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; arg[j] = 0; }
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const int h = 2 * p - 1 + r;
            if (h < 0) continue;
#pragma unroll
            for (int s_ = 0; s_ < 3; ++s_) {
                const int w = 2 * q - 1 + s_;
                if (w < 0) continue;
                const long e = (((long)n * H + h) * W + w) * C + cg * 8;
                float v[8];
                load8(x + e, v);
                uint32_t bits = 0;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float a = to_f(from_f<T>(fmaxf(v[j] * sc[j] + sh[j], 0.f)));
                    bits |= (a > 0.f ? 1u : 0u) << j;
                    if (a > best[j] || (a != a)) { best[j] = a; arg[j] = (uint8_t)(r * 3 + s_); }
                }
                if (r >= 1 && s_ >= 1) mask[e >> 3] = (uint8_t)bits;   // an owned pixel
            }
        }
        store8(y + i * 8, best);
        uint2 packed;
        packed.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | ((uint32_t)arg[3] << 24);
        packed.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | ((uint32_t)arg[7] << 24);
        *reinterpret_cast<uint2*>(idx + i * 8) = packed;
    }
}

// Row forms of the two kernels above and below for the ResNet stem: one block per output (input) row,
// 32-bit index math.  The flat forms decompose a 64-bit element index per thread with 64-bit div /
// mod (software sequences) and ran at ~2.3-2.5 TB/s on the 411 MB stem activation.
// Workgroups are dispatched round-robin over the 8 XCDs (block b on XCD b & 7), each with its own L2.
// This bijection of [0, n) gives XCD x a CONTIGUOUS range of logical block ids, so neighbouring blocks
// that share input rows (pooling windows) share them in one L2 instead of fetching them twice.
__device__ __forceinline__ int xcd_contiguous(int bid, int n) {
    const int xcd = bid & 7, qn = n >> 3, rn = n & 7;
    return (xcd < rn ? xcd * (qn + 1) : rn * (qn + 1) + (xcd - rn) * qn) + (bid >> 3);
}

// Rows in XCD-contiguous order (xcd_contiguous): output rows p and p + 1 share input row 2p + 1, and
// round-robin placement put them on different XCDs, i.e. two L2s fetching it (stem shape, batch 256:
// forward 234 -> 225 us, backward 206 -> 193 us; blocks sized to one pass per row, 448 / 896 threads,
// were slower: 237 / 265 us -- profiles/pool_ab_r06.log).
template <typename T>
__global__ __launch_bounds__(256) void bn_relu_maxpool_rows_k(const T* __restrict__ x, const float* __restrict__ scale,
                                                              const float* __restrict__ shift, T* __restrict__ y,
                                                              uint8_t* __restrict__ idx, uint8_t* __restrict__ mask,
                                                              int H, int W, int C, int P, int Q) {
    const int row = xcd_contiguous(blockIdx.x, gridDim.x);
    const int c8 = C / 8, n = row / P, p = row - n * P;
    const long img = (long)n * H * W * C;
    for (int t = threadIdx.x; t < Q * c8; t += 256) {
        const int q = t / c8, cg = t - q * c8;
        float sc[8], sh[8], best[8];
        uint8_t arg[8];
        load8(scale + cg * 8, sc);
        load8(shift + cg * 8, sh);
#pragma unroll
        for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; arg[j] = 0; }
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const int h = 2 * p - 1 + r;
            if (h < 0) continue;
#pragma unroll
            for (int s_ = 0; s_ < 3; ++s_) {
                const int w = 2 * q - 1 + s_;
                if (w < 0) continue;
                const long e = img + ((long)h * W + w) * C + cg * 8;
                float v[8];
                load8(x + e, v);
                uint32_t bits = 0;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float a = to_f(from_f<T>(fmaxf(v[j] * sc[j] + sh[j], 0.f)));
                    bits |= (a > 0.f ? 1u : 0u) << j;
                    if (a > best[j] || (a != a)) { best[j] = a; arg[j] = (uint8_t)(r * 3 + s_); }
                }
                if (r >= 1 && s_ >= 1) mask[e >> 3] = (uint8_t)bits;   // an owned pixel
            }
        }
        const long o = (((long)n * P + p) * Q + q) * C + cg * 8;
        store8(y + o, best);
        uint2 packed;
        packed.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | ((uint32_t)arg[3] << 24);
        packed.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | ((uint32_t)arg[7] << 24);
        *reinterpret_cast<uint2*>(idx + o) = packed;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void maxpool_bwd_rows_k(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                          T* __restrict__ dx, int H, int W, int C, int P, int Q, int K,
                                                          int S, int pad) {
    const int row = xcd_contiguous(blockIdx.x, gridDim.x);   // input rows 2p, 2p + 1 read pooled row p
    const int c8 = C / 8, n = row / H, h = row - n * H;
    const int p_lo = max(0, (h + pad - K + S) / S), p_hi = min(P - 1, (h + pad) / S);
    for (int t = threadIdx.x; t < W * c8; t += 256) {
        const int w = t / c8, cg = t - w * c8;
        float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const int q_lo = max(0, (w + pad - K + S) / S), q_hi = min(Q - 1, (w + pad) / S);
        for (int p = p_lo; p <= p_hi; ++p) {
            const int r = h - (p * S - pad);
            if (r < 0 || r >= K) continue;
            for (int q = q_lo; q <= q_hi; ++q) {
                const int s = w - (q * S - pad);
                if (s < 0 || s >= K) continue;
                const long o = (((long)n * P + p) * Q + q) * C + cg * 8;
                float g[8];
                load8(dy + o, g);
                const uint2 packed = *reinterpret_cast<const uint2*>(idx + o);
                const uint8_t want = (uint8_t)(r * K + s);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t word = j < 4 ? packed.x : packed.y;
                    const uint8_t a = (uint8_t)(word >> (8 * (j & 3)));
                    if (a == want) acc[j] += g[j];
                }
            }
        }
        store8(dx + (((long)n * H + h) * W + w) * C + cg * 8, acc);
    }
}

template <typename T>
__global__ __launch_bounds__(256) void maxpool_bwd_k(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                     T* __restrict__ dx, int N, int H, int W, int C, int P, int Q, int K,
                                                     int S, int pad) {
    const int c8 = C / 8;
    const long total = (long)N * H * W * c8;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int cg = (int)(i % c8);
        long t = i / c8;
        const int w = (int)(t % W); t /= W;
        const int h = (int)(t % H);
        const int n = (int)(t / H);
        float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        // outputs whose window covers (h, w): p*S - pad <= h <= p*S - pad + K - 1
        const int p_lo = std::max(0, (h + pad - K + S) / S), p_hi = std::min(P - 1, (h + pad) / S);
        const int q_lo = std::max(0, (w + pad - K + S) / S), q_hi = std::min(Q - 1, (w + pad) / S);
        for (int p = p_lo; p <= p_hi; ++p) {
            const int r = h - (p * S - pad);
            if (r < 0 || r >= K) continue;
            for (int q = q_lo; q <= q_hi; ++q) {
                const int s = w - (q * S - pad);
                if (s < 0 || s >= K) continue;
                const long o = (((long)n * P + p) * Q + q) * C + cg * 8;
                float g[8];
                load8(dy + o, g);
                const uint2 packed = *reinterpret_cast<const uint2*>(idx + o);
                const uint8_t want = (uint8_t)(r * K + s);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t word = j < 4 ? packed.x : packed.y;
                    const uint8_t a = (uint8_t)(word >> (8 * (j & 3)));
                    if (a == want) acc[j] += g[j];
                }
            }
        }
        store8(dx + i * 8, acc);
    }
}

// ------------------------------------------------------------------ global avg-pool
template <typename T>
__global__ __launch_bounds__(256) void avgpool_fwd_k(const T* __restrict__ x, T* __restrict__ y, int N, int HW, int C) {
    const int c8 = C / 8;
    const long total = (long)N * c8;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int cg = (int)(i % c8);
        const long n = i / c8;
        float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int k = 0; k < HW; ++k) {
            float v[8];
            load8(x + (n * HW + k) * C + cg * 8, v);
#pragma unroll
            for (int j = 0; j < 8; ++j) s[j] += v[j];
        }
        const float inv = 1.f / HW;
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] *= inv;
        store8(y + n * C + cg * 8, s);
    }
}
template <typename T>
__global__ __launch_bounds__(256) void avgpool_bwd_k(const T* __restrict__ dy, T* __restrict__ dx, int N, int HW, int C) {
    const int c8 = C / 8;
    const long total = (long)N * HW * c8;
    const float inv = 1.f / HW;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int cg = (int)(i % c8);
        const long n = i / ((long)HW * c8);
        float g[8];
        load8(dy + n * C + cg * 8, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] *= inv;
        store8(dx + i * 8, g);
    }
}

// ------------------------------------------------------------------ embedding
template <typename T>
__global__ __launch_bounds__(256) void embed_fwd_k(const int64_t* __restrict__ ids, const T* __restrict__ w,
                                                   T* __restrict__ y, long n_tok, int D) {
    const int d8 = D / 8;
    const long total = n_tok * d8;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const long t = i / d8;
        const int dg = (int)(i % d8);
        const long id = ids[t];
        *reinterpret_cast<uint4*>(y + t * D + dg * 8) = *reinterpret_cast<const uint4*>(w + id * D + dg * 8);
        if (sizeof(T) == 4)
            *reinterpret_cast<uint4*>(y + t * D + dg * 8 + 4) = *reinterpret_cast<const uint4*>(w + id * D + dg * 8 + 4);
    }
}
// scatter-add into an fp32 accumulator (one 256-B row segment per wave instruction)
template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_k(const int64_t* __restrict__ ids, const T* __restrict__ dy,
                                                   float* __restrict__ acc, long n_tok, int D) {
    const long total = n_tok * D;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const long t = i / D;
        const int d = (int)(i % D);
        atomicAdd(acc + ids[t] * D + d, to_f(dy[i]));
    }
}
// Deterministic embedding backward over the ids sorted stably on the host side (s = sorted ids,
// pi = their token positions).  One wave per chunk of EMB_CH sorted positions sums every run of equal
// ids inside the chunk in token order (fp32, 8 columns per lane, column slabs of 512).  A run that
// starts and ends inside the chunk is written straight into dw; a piece of a run that crosses a chunk
// edge goes to part[chunk][0] (the chunk's head piece: the run began earlier) or part[chunk][1] (its
// tail piece: the run begins here and continues), and embed_bwd_join_k adds the pieces in chunk order.
// No atomics (the same bits every run) and no V x D fp32 buffer to fill and cast.
constexpr int EMB_CH = 16;

template <typename T>
__device__ __forceinline__ void emb_row_out(T* __restrict__ dst, const float* a, int accumulate) {
    float o[8];
    if (accumulate) {
        load8(dst, o);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += a[j];
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = a[j];
    }
    store8(dst, o);
}

template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_seg_k(const int* __restrict__ s, const int64_t* __restrict__ pi,
                                                       const T* __restrict__ dy, T* __restrict__ dw,
                                                       float* __restrict__ part, long n, int D, int accumulate) {
    const long chunk = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long c0 = chunk * EMB_CH;
    if (c0 >= n) return;                                      // wave-uniform
    const int cnt = (int)min((long)EMB_CH, n - c0);
    const int G = D / 8;
    const bool cont_in = c0 > 0 && s[c0 - 1] == s[c0];        // the chunk's first run began earlier
    const bool cont_out = c0 + cnt < n && s[c0 + cnt] == s[c0 + cnt - 1];
    // the chunk's ids and token positions: one vector load (lane j holds position j), then read back
    // as wave-uniform values per unrolled position -- no scalar-load round trip per position
    const int sv = lane < cnt ? s[c0 + lane] : -1;
    const long pv = lane < cnt ? pi[c0 + lane] : 0;
    const int pv_lo = (int)(uint32_t)pv, pv_hi = (int)(pv >> 32);
    for (int g0 = 0; g0 < G; g0 += 64) {
        const int g = g0 + lane;
        const bool on = g < G;
        float v[EMB_CH][8];                                   // every row's load in flight at once
#pragma unroll
        for (int j = 0; j < EMB_CH; ++j) {
            // unconditional (a load under a branch waits at the branch's end): positions past the chunk
            // read token 0's row, idle lanes the last column group -- both valid, both ignored
            const long row = ((long)__builtin_amdgcn_readlane(pv_hi, j) << 32) |
                             (uint32_t)__builtin_amdgcn_readlane(pv_lo, j);
            load8(dy + row * D + (on ? g : G - 1) * 8, v[j]);
        }
        // pass 1: run sums; a run complete inside the chunk keeps its sum in v[j] (j = its last position)
        float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        int start = 0;
        uint32_t done = 0;                                    // wave-uniform: bit j = complete run ends at j
#pragma unroll
        for (int j = 0; j < EMB_CH; ++j) {
            if (j < cnt) {
#pragma unroll
                for (int e = 0; e < 8; ++e) a[e] += v[j][e];
                const int sj = __builtin_amdgcn_readlane(sv, j);
                const bool last = j == cnt - 1 || __builtin_amdgcn_readlane(sv, j < EMB_CH - 1 ? j + 1 : j) != sj;
                if (last) {
                    const bool starts = start > 0 || !cont_in;
                    const bool ends = j < cnt - 1 || !cont_out;
                    if (starts && ends) {
                        done |= 1u << j;
#pragma unroll
                        for (int e = 0; e < 8; ++e) v[j][e] = a[e];
                    } else if (on) {
                        store8(part + (chunk * 2 + (starts ? 1 : 0)) * D + g * 8, a);
                    }
#pragma unroll
                    for (int e = 0; e < 8; ++e) a[e] = 0.f;
                    start = j + 1;
                }
            }
        }
        // pass 2: the complete runs' rows, every accumulate read in flight before the first store
        if (on) {
            float w[EMB_CH][8];
            if (accumulate) {                                 // unconditional loads (see above): row of
#pragma unroll                                                    // position 0 where no run ends
                for (int j = 0; j < EMB_CH; ++j)
                    load8(dw + (long)__builtin_amdgcn_readlane(sv, ((done >> j) & 1u) ? j : 0) * D + g * 8, w[j]);
            }
#pragma unroll
            for (int j = 0; j < EMB_CH; ++j) {
                if ((done >> j) & 1u) {
                    if (accumulate) {
#pragma unroll
                        for (int e = 0; e < 8; ++e) v[j][e] += w[j][e];
                    }
                    store8(dw + (long)__builtin_amdgcn_readlane(sv, j) * D + g * 8, v[j]);
                }
            }
        }
    }
}

// One workgroup per chunk whose tail piece starts a run that continues past the chunk: that piece
// plus the head pieces of the following chunks, in a fixed order, until the run ends.  Real batches
// have LONG runs (padding id 0; token-type ids, V = 2, half the batch each: hundreds of chunks), so
// the run's last chunk is found by a binary search over the sorted ids (log2 n dependent loads, not
// one per chunk), and the 256 threads split the chunks: thread (r, g) sums column group g of the
// chunks r, r + R, ... (R = 256 / groups, each thread's loads independent, four in flight), then
// the R partial sums are added in r order through LDS -- the same bits every run.
template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_join_k(const int* __restrict__ s, T* __restrict__ dw,
                                                        const float* __restrict__ part, long n, int D, int accumulate) {
    __shared__ float red[256 * 8];
    __shared__ long s_last;
    const long chunk = blockIdx.x;
    const long c0 = chunk * EMB_CH;
    if (c0 >= n) return;
    const long c1 = min(c0 + EMB_CH, n);
    const int v = s[c1 - 1];
    if (c1 >= n || s[c1] != v) return;                        // the last run ends in this chunk
    if (s[c0] == v && c0 > 0 && s[c0 - 1] == v) return;       // ... or began before it
    if (threadIdx.x == 0) {
        long lo = c1, hi = n;                                 // first position past the run
        while (lo < hi) {
            const long mid = (lo + hi) >> 1;
            if (s[mid] == v) lo = mid + 1;
            else hi = mid;
        }
        s_last = lo - 1;
    }
    __syncthreads();
    const long cend = s_last / EMB_CH;                        // chunk holding the run's last position
    const long k = cend - chunk;                              // head pieces: chunks chunk+1 .. cend
    const int G = D / 8;
    for (int g0 = 0; g0 < G; g0 += 256) {
        const int gs = min(256, G - g0);                      // column groups of this slab
        const int R = 256 / gs;                               // chunk lanes
        const int r = threadIdx.x / gs, g = g0 + threadIdx.x % gs;
        float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (r < R) {
            if (r == 0) load8(part + (chunk * 2 + 1) * D + g * 8, a);
            long i = 1 + r;
            for (; i + 3L * R <= k; i += 4L * R) {
                float b[4][8];
#pragma unroll
                for (int u = 0; u < 4; ++u) load8(part + (chunk + i + (long)u * R) * 2 * D + g * 8, b[u]);
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int e = 0; e < 8; ++e) a[e] += b[u][e];
            }
            for (; i <= k; i += R) {
                float b[8];
                load8(part + (chunk + i) * 2 * D + g * 8, b);
#pragma unroll
                for (int e = 0; e < 8; ++e) a[e] += b[e];
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) red[threadIdx.x * 8 + e] = a[e];
        }
        __syncthreads();
        if (r == 0) {
            for (int rr = 1; rr < R; ++rr)
#pragma unroll
                for (int e = 0; e < 8; ++e) a[e] += red[(rr * gs + threadIdx.x) * 8 + e];
            emb_row_out(dw + (long)v * D + g * 8, a, accumulate);
        }
        __syncthreads();
    }
}

template <typename TO>
__global__ __launch_bounds__(256) void cast_f32_k(const float* __restrict__ x, TO* __restrict__ y, long n, int acc) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        y[i] = from_f<TO>(x[i] + (acc ? to_f(y[i]) : 0.f));
}

}  // namespace

// =================================================================== C ABI
// dst (bf16 / fp32) += src (fp32): folds an fp32 side-channel result (e.g. the bias
// gradient a LayerNorm backward summed) into a parameter-gradient slot in one launch
template <typename T>
__global__ __launch_bounds__(256) void acc_f32_k(T* __restrict__ dst, const float* __restrict__ src, long n) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        dst[i] = from_f<T>(to_f(dst[i]) + src[i]);
}

// Gradient-accumulation drain (micro-step of grad_accum): acc (fp32) += g; g = 0 -- one pass
// over the arena instead of an ATen add plus a zero fill; 8 elements per thread per
// iteration (16-byte gradient loads / stores, two float4 on the accumulator).
// Gradient accumulation into the fp32 accumulator, one pass: acc = g (FIRST: the accumulator's
// previous contents are dead, so it is neither zero-filled per step nor read) or acc += g, and g = 0
// when ZERO (a micro-step's drain; the last micro-step's gradients are summed in place and left).
template <typename T, bool FIRST, bool ZERO>
__global__ __launch_bounds__(256) void acc_grad_k(float* __restrict__ acc, T* __restrict__ g, long n8) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
        float v[8], a[8];
        load8(g + i * 8, v);
        if (!FIRST) {
            load8(acc + i * 8, a);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += a[e];
        }
        store8(acc + i * 8, v);
        if (ZERO) {
            const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            store8(g + i * 8, z);
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void drain_acc_k(float* __restrict__ acc, T* __restrict__ g, long n8) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
        float v[8], a[8];
        load8(g + i * 8, v);
        load8(acc + i * 8, a);
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] += v[e];
        store8(acc + i * 8, a);
        const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        store8(g + i * 8, z);
    }
}

#define DISPATCH_T(dtype, KERNEL_CALL_BF16, KERNEL_CALL_F32) \
    do { if ((dtype) == 1) { KERNEL_CALL_BF16; } else { KERNEL_CALL_F32; } } while (0)

DDL_API int ddl_gelu_fwd(int dtype, const void* x, void* y, long n, hipStream_t st) {
    if (n % 8) return -1;
    const long n8 = n / 8;
    DISPATCH_T(dtype, (gelu_fwd_k<bf16_t><<<grid_for(n8), 256, 0, st>>>((const bf16_t*)x, (bf16_t*)y, n8)),
               (gelu_fwd_k<float><<<grid_for(n8), 256, 0, st>>>((const float*)x, (float*)y, n8)));
    DDL_RETURN_LAUNCH();
}
DDL_API int ddl_gelu_bwd(int dtype, const void* dy, const void* x, void* dx, long n, hipStream_t st) {
    if (n % 8) return -1;
    const long n8 = n / 8;
    DISPATCH_T(dtype,
               (gelu_bwd_k<bf16_t><<<grid_for(n8), 256, 0, st>>>((const bf16_t*)dy, (const bf16_t*)x, (bf16_t*)dx, n8)),
               (gelu_bwd_k<float><<<grid_for(n8), 256, 0, st>>>((const float*)dy, (const float*)x, (float*)dx, n8)));
    DDL_RETURN_LAUNCH();
}
DDL_API int ddl_dropout(int dtype, const void* x, void* y, long n, uint64_t seed, float p, hipStream_t st) {
    if (n % 8) return -1;
    const long n8 = n / 8;
    const uint32_t thresh = drop_thresh16(p);
    const float scale = 1.f / (1.f - p);
    DISPATCH_T(dtype,
               (dropout_k<bf16_t><<<grid_for(n8), 256, 0, st>>>((const bf16_t*)x, (bf16_t*)y, n8, seed, thresh, scale)),
               (dropout_k<float><<<grid_for(n8), 256, 0, st>>>((const float*)x, (float*)y, n8, seed, thresh, scale)));
    DDL_RETURN_LAUNCH();
}

DDL_API int ddl_colsum_nblk(long rows) { return (int)std::max<long>(1, std::min<long>(1024, (rows + 15) / 16)); }

// out[c] (+)= sum_r x[r, c]; `part` needs ddl_colsum_nblk(rows) * C floats.
DDL_API int ddl_colsum(int dtype, const void* x, long rows, int C, float* part, void* out, int out_dtype,
                       int accumulate, hipStream_t st) {
    if (C % 8) return -1;
    const int nblk = ddl_colsum_nblk(rows);
    const int rpb = (int)((rows + nblk - 1) / nblk);
    dim3 g(nblk, (C / 8 + 255) / 256);
    DISPATCH_T(dtype, (colsum_partial_k<bf16_t><<<g, 256, 0, st>>>((const bf16_t*)x, rows, C, rpb, part)),
               (colsum_partial_k<float><<<g, 256, 0, st>>>((const float*)x, rows, C, rpb, part)));
    if (out_dtype == 1) colsum_final_k<bf16_t><<<(C + 63) / 64, 1024, 0, st>>>(part, nblk, C, (bf16_t*)out, accumulate);
    else colsum_final_k<float><<<(C + 63) / 64, 1024, 0, st>>>(part, nblk, C, (float*)out, accumulate);
    DDL_RETURN_LAUNCH();
}

// dz = dy * gelu'(z) and out[c] (+)= sum_r dz[r, c] in one pass over dy / z
DDL_API int ddl_gelu_bwd_colsum(int dtype, const void* dy, const void* z, void* dz, long rows, int C, float* part,
                                void* out, int out_dtype, int accumulate, hipStream_t st) {
    if (C % 8) return -1;
    const int nblk = ddl_colsum_nblk(rows);
    const int rpb = (int)((rows + nblk - 1) / nblk);
    dim3 g(nblk, (C / 8 + 255) / 256);
    DISPATCH_T(dtype,
               (gelu_bwd_colsum_k<bf16_t><<<g, 256, 0, st>>>((const bf16_t*)dy, (const bf16_t*)z, (bf16_t*)dz, rows,
                                                              C, rpb, part)),
               (gelu_bwd_colsum_k<float><<<g, 256, 0, st>>>((const float*)dy, (const float*)z, (float*)dz, rows, C,
                                                             rpb, part)));
    if (out_dtype == 1) colsum_final_k<bf16_t><<<(C + 63) / 64, 1024, 0, st>>>(part, nblk, C, (bf16_t*)out, accumulate);
    else colsum_final_k<float><<<(C + 63) / 64, 1024, 0, st>>>(part, nblk, C, (float*)out, accumulate);
    DDL_RETURN_LAUNCH();
}

DDL_API int ddl_softmax_ce(int dtype, const void* logits, const int64_t* labels, long B, int C, float* row_loss,
                           float* loss, void* dlogits, hipStream_t st) {
    const float inv_b = 1.f / (float)B;
    DISPATCH_T(dtype,
               (softmax_ce_k<bf16_t><<<B, 256, 0, st>>>((const bf16_t*)logits, labels, C, inv_b, row_loss,
                                                        (bf16_t*)dlogits)),
               (softmax_ce_k<float><<<B, 256, 0, st>>>((const float*)logits, labels, C, inv_b, row_loss,
                                                       (float*)dlogits)));
    mean_k<<<1, 256, 0, st>>>(row_loss, B, loss);
    DDL_RETURN_LAUNCH();
}
DDL_API int ddl_scale_by(int dtype, const void* x, const float* s, void* y, long n, hipStream_t st) {
    DISPATCH_T(dtype, (scale_k<bf16_t><<<grid_for(n), 256, 0, st>>>((const bf16_t*)x, s, (bf16_t*)y, n)),
               (scale_k<float><<<grid_for(n), 256, 0, st>>>((const float*)x, s, (float*)y, n)));
    DDL_RETURN_LAUNCH();
}

DDL_API int ddl_maxpool_fwd(int dtype, const void* x, void* y, uint8_t* idx, int N, int H, int W, int C, int P, int Q,
                            int K, int S, int pad, hipStream_t st) {
    if (C % 8) return -1;
    const long tot = (long)N * P * Q * (C / 8);
    DISPATCH_T(dtype,
               (maxpool_fwd_k<bf16_t><<<grid_for(tot), 256, 0, st>>>((const bf16_t*)x, (bf16_t*)y, idx, N, H, W, C, P,
                                                                      Q, K, S, pad)),
               (maxpool_fwd_k<float><<<grid_for(tot), 256, 0, st>>>((const float*)x, (float*)y, idx, N, H, W, C, P, Q,
                                                                     K, S, pad)));
    DDL_RETURN_LAUNCH();
}
// DDL_POOL_ROWS=0: the flat-index stem pooling kernels (A/B timing)
static bool rows_form_enabled() {
    static const bool on = [] { const char* e = getenv("DDL_POOL_ROWS"); return !(e && e[0] == '0'); }();
    return on;
}
DDL_API int ddl_bn_relu_maxpool(int dtype, const void* x, const float* scale, const float* shift, void* y,
                                uint8_t* idx, uint8_t* mask, int N, int H, int W, int C, int P, int Q, hipStream_t st) {
    if (C % 8 || H != 2 * P || W != 2 * Q) return -1;
    const long tot = (long)N * P * Q * (C / 8);
    if ((long)N * P < (1L << 31) && rows_form_enabled()) {
        DISPATCH_T(dtype,
                   (bn_relu_maxpool_rows_k<bf16_t><<<N * P, 256, 0, st>>>(
                       (const bf16_t*)x, scale, shift, (bf16_t*)y, idx, mask, H, W, C, P, Q)),
                   (bn_relu_maxpool_rows_k<float><<<N * P, 256, 0, st>>>(
                       (const float*)x, scale, shift, (float*)y, idx, mask, H, W, C, P, Q)));
        DDL_RETURN_LAUNCH();
    }
    DISPATCH_T(dtype,
               (bn_relu_maxpool_k<bf16_t><<<grid_for(tot), 256, 0, st>>>((const bf16_t*)x, scale, shift, (bf16_t*)y,
                                                                          idx, mask, N, H, W, C, P, Q)),
               (bn_relu_maxpool_k<float><<<grid_for(tot), 256, 0, st>>>((const float*)x, scale, shift, (float*)y, idx,
                                                                         mask, N, H, W, C, P, Q)));
    DDL_RETURN_LAUNCH();
}
DDL_API int ddl_maxpool_bwd(int dtype, const void* dy, const uint8_t* idx, void* dx, int N, int H, int W, int C, int P,
                            int Q, int K, int S, int pad, hipStream_t st) {
    if (C % 8) return -1;
    const long tot = (long)N * H * W * (C / 8);
    if ((long)N * H < (1L << 31) && rows_form_enabled()) {
        DISPATCH_T(dtype,
                   (maxpool_bwd_rows_k<bf16_t><<<N * H, 256, 0, st>>>(
                       (const bf16_t*)dy, idx, (bf16_t*)dx, H, W, C, P, Q, K, S, pad)),
                   (maxpool_bwd_rows_k<float><<<N * H, 256, 0, st>>>(
                       (const float*)dy, idx, (float*)dx, H, W, C, P, Q, K, S, pad)));
        DDL_RETURN_LAUNCH();
    }
    DISPATCH_T(dtype,
               (maxpool_bwd_k<bf16_t><<<grid_for(tot), 256, 0, st>>>((const bf16_t*)dy, idx, (bf16_t*)dx, N, H, W, C,
                                                                      P, Q, K, S, pad)),
               (maxpool_bwd_k<float><<<grid_for(tot), 256, 0, st>>>((const float*)dy, idx, (float*)dx, N, H, W, C, P, Q,
                                                                     K, S, pad)));
    DDL_RETURN_LAUNCH();
}
DDL_API int ddl_avgpool_fwd(int dtype, const void* x, void* y, int N, int HW, int C, hipStream_t st) {
    if (C % 8) return -1;
    const long tot = (long)N * (C / 8);
    DISPATCH_T(dtype, (avgpool_fwd_k<bf16_t><<<grid_for(tot), 256, 0, st>>>((const bf16_t*)x, (bf16_t*)y, N, HW, C)),
               (avgpool_fwd_k<float><<<grid_for(tot), 256, 0, st>>>((const float*)x, (float*)y, N, HW, C)));
    DDL_RETURN_LAUNCH();
}
DDL_API int ddl_avgpool_bwd(int dtype, const void* dy, void* dx, int N, int HW, int C, hipStream_t st) {
    if (C % 8) return -1;
    const long tot = (long)N * HW * (C / 8);
    DISPATCH_T(dtype, (avgpool_bwd_k<bf16_t><<<grid_for(tot), 256, 0, st>>>((const bf16_t*)dy, (bf16_t*)dx, N, HW, C)),
               (avgpool_bwd_k<float><<<grid_for(tot), 256, 0, st>>>((const float*)dy, (float*)dx, N, HW, C)));
    DDL_RETURN_LAUNCH();
}
DDL_API int ddl_embedding_fwd(int dtype, const int64_t* ids, const void* w, void* y, long n_tok, int D, hipStream_t st) {
    if (D % 8) return -1;
    const long tot = n_tok * (D / 8);
    DISPATCH_T(dtype, (embed_fwd_k<bf16_t><<<grid_for(tot), 256, 0, st>>>(ids, (const bf16_t*)w, (bf16_t*)y, n_tok, D)),
               (embed_fwd_k<float><<<grid_for(tot), 256, 0, st>>>(ids, (const float*)w, (float*)y, n_tok, D)));
    DDL_RETURN_LAUNCH();
}
// acc must be zeroed (fp32 [V, D]); then cast into dw (dtype) of V*D elements.
DDL_API int ddl_embedding_bwd(int dtype, const int64_t* ids, const void* dy, float* acc, void* dw, long n_tok, long V,
                              int D, int accumulate, hipStream_t st) {
    const long tot = n_tok * D;
    DISPATCH_T(dtype, (embed_bwd_k<bf16_t><<<grid_for(tot), 256, 0, st>>>(ids, (const bf16_t*)dy, acc, n_tok, D)),
               (embed_bwd_k<float><<<grid_for(tot), 256, 0, st>>>(ids, (const float*)dy, acc, n_tok, D)));
    const long n = V * D;
    DISPATCH_T(dtype, (cast_f32_k<bf16_t><<<grid_for(n), 256, 0, st>>>(acc, (bf16_t*)dw, n, accumulate)),
               (cast_f32_k<float><<<grid_for(n), 256, 0, st>>>(acc, (float*)dw, n, accumulate)));
    DDL_RETURN_LAUNCH();
}
// Deterministic form: s / pi = the ids (int32: a radix sort of half the passes) sorted stably and their
// token positions (int64), n_tok each;
// part = fp32 workspace of 2 * ceil(n_tok / 16) * D elements (no initialisation needed).  Writes
// (accumulate: adds to) only the rows of dw whose id occurs; the caller zeroes dw otherwise.
DDL_API int ddl_embedding_bwd_sorted(int dtype, const int* s, const int64_t* pi, const void* dy, void* dw,
                                     float* part, long n_tok, int D, int accumulate, hipStream_t st) {
    if (D % 8 || n_tok <= 0) return -1;
    const long nch = (n_tok + EMB_CH - 1) / EMB_CH;
    const long blocks = (nch + 3) / 4;
    if (nch >= (1L << 31)) return -1;
    DISPATCH_T(dtype,
               (embed_bwd_seg_k<bf16_t><<<(int)blocks, 256, 0, st>>>(s, pi, (const bf16_t*)dy, (bf16_t*)dw, part,
                                                                      n_tok, D, accumulate)),
               (embed_bwd_seg_k<float><<<(int)blocks, 256, 0, st>>>(s, pi, (const float*)dy, (float*)dw, part,
                                                                     n_tok, D, accumulate)));
    DISPATCH_T(dtype,
               (embed_bwd_join_k<bf16_t><<<(int)nch, 256, 0, st>>>(s, (bf16_t*)dw, part, n_tok, D, accumulate)),
               (embed_bwd_join_k<float><<<(int)nch, 256, 0, st>>>(s, (float*)dw, part, n_tok, D, accumulate)));
    DDL_RETURN_LAUNCH();
}

// ------------------------------------------------------------------ conv dgrad weight layout
// out[c][r'][s'][k] = w[k][rmap[r']][smap[s']][c]  (bf16): the transposed (and for
// stride-1 dgrad: spatially flipped; for a stride-s parity class: tap-subset)
// weight the implicit-GEMM dgrad reads as its KC operand.  One launch replaces
// the index / flip / permute / contiguous chain (4-6 small ATen kernels per conv).
struct TapMap {
    int r[8], s[8];
};
// 32x32 (k, c) tiles per tap through LDS: reads coalesce along c (w's contiguous
// dimension), writes along k (out's); 32-bit index math (weights < 2^31 elements)
__global__ __launch_bounds__(256) void conv_w_dgrad_k(const bf16_t* __restrict__ w, bf16_t* __restrict__ out, int K,
                                                      int R, int S, int C, int Rp, int Sp, TapMap tm) {
    __shared__ bf16_t tile[32][33];
    const int k0 = blockIdx.x * 32, c0 = blockIdx.y * 32, tap = blockIdx.z;
    const int rp = tap / Sp, sp = tap - rp * Sp;
    const int r = tm.r[rp], s_ = tm.s[sp];
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = k0 + ty + 8 * i, c = c0 + tx;
        if (k < K && c < C) tile[ty + 8 * i][tx] = w[((k * R + r) * S + s_) * C + c];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = c0 + ty + 8 * i, k = k0 + tx;
        if (k < K && c < C) out[((c * Rp + rp) * Sp + sp) * K + k] = tile[tx][ty + 8 * i];
    }
}

DDL_API int ddl_conv_w_dgrad(const void* w, void* out, int K, int R, int S, int C, int Rp, int Sp, const int* rmap,
                             const int* smap, hipStream_t st) {
    if (Rp > 8 || Sp > 8 || Rp < 1 || Sp < 1) return -1;
    TapMap tm{};
    for (int i = 0; i < Rp; ++i) tm.r[i] = rmap[i];
    for (int i = 0; i < Sp; ++i) tm.s[i] = smap[i];
    if ((long)K * R * S * C >= (1L << 31)) return -2;
    const dim3 grid((K + 31) / 32, (C + 31) / 32, Rp * Sp);
    conv_w_dgrad_k<<<grid, 256, 0, st>>>((const bf16_t*)w, (bf16_t*)out, K, R, S, C, Rp, Sp, tm);
    DDL_RETURN_LAUNCH();
}

// Every conv's dgrad weight layout of one optimizer step in ONE launch (ResNet-50: 61
// re-layouts of 2-600 KB each were 61 launch-latency-bound kernels, ~0.3 ms per step).
// Job table in device memory, WJ_FIELDS int64 per job:
//   [w, out, K, R, S, C, Rp, Sp, gk, gc, block0, r[8], s[8]]
// gk / gc: 32-wide k / c tiles; block0: first flat block of the job (ascending).
constexpr int WJ_FIELDS = 27;
__global__ __launch_bounds__(256) void conv_w_dgrad_batch_k(const int64_t* __restrict__ tab, int njobs) {
    __shared__ bf16_t tile[32][33];
    const long b = blockIdx.x;
    int lo = 0, hi = njobs - 1;          // last job with block0 <= b
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (tab[mid * WJ_FIELDS + 10] <= b) lo = mid; else hi = mid - 1;
    }
    const int64_t* j = tab + lo * WJ_FIELDS;
    const bf16_t* w = (const bf16_t*)j[0];
    bf16_t* out = (bf16_t*)j[1];
    const int K = (int)j[2], R = (int)j[3], S = (int)j[4], C = (int)j[5], Sp = (int)j[7];
    const int Rp = (int)j[6], gk = (int)j[8], gc = (int)j[9];
    const int loc = (int)(b - j[10]);
    const int tap = loc / (gk * gc), rem = loc - tap * gk * gc;
    const int k0 = (rem % gk) * 32, c0 = (rem / gk) * 32;
    const int rp = tap / Sp, sp = tap - rp * Sp;
    const int r = (int)j[11 + rp], s_ = (int)j[19 + sp];
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = k0 + ty + 8 * i, c = c0 + tx;
        if (k < K && c < C) tile[ty + 8 * i][tx] = w[((k * R + r) * S + s_) * C + c];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = c0 + ty + 8 * i, k = k0 + tx;
        if (k < K && c < C) out[((c * Rp + rp) * Sp + sp) * K + k] = tile[tx][ty + 8 * i];
    }
}

// tab: device copy of the job table; host_tab: the same table on the host (validated here)
DDL_API int ddl_conv_w_dgrad_batch(const int64_t* tab, const int64_t* host_tab, int njobs, hipStream_t st) {
    if (njobs <= 0) return 0;
    long total = 0;
    for (int i = 0; i < njobs; ++i) {
        const int64_t* j = host_tab + (long)i * WJ_FIELDS;
        const long K = j[2], R = j[3], S = j[4], C = j[5], Rp = j[6], Sp = j[7];
        if (Rp > 8 || Sp > 8 || Rp < 1 || Sp < 1 || K * R * S * C >= (1L << 31)) return -1;
        if (j[8] != (K + 31) / 32 || j[9] != (C + 31) / 32 || j[10] != total) return -2;
        for (int t = 0; t < Rp; ++t) if (j[11 + t] < 0 || j[11 + t] >= R) return -3;
        for (int t = 0; t < Sp; ++t) if (j[19 + t] < 0 || j[19 + t] >= S) return -3;
        total += j[8] * j[9] * Rp * Sp;
    }
    if (total >= (1L << 31)) return -4;
    conv_w_dgrad_batch_k<<<(unsigned)total, 256, 0, st>>>(tab, njobs);
    DDL_RETURN_LAUNCH();
}

DDL_API int ddl_acc_f32(int dtype, void* dst, const float* src, long n, hipStream_t st) {
    const int g = (int)std::min<long>(1024, (n + 255) / 256);
    DISPATCH_T(dtype, (acc_f32_k<bf16_t><<<g, 256, 0, st>>>((bf16_t*)dst, src, n)),
               (acc_f32_k<float><<<g, 256, 0, st>>>((float*)dst, src, n)));
    DDL_RETURN_LAUNCH();
}

// acc (fp32) = / += g (bf16 / fp32), then g = 0 if zero_g (see acc_grad_k).  n % 8 == 0, 16-byte aligned.
DDL_API int ddl_acc_grad(int dtype, float* acc, void* g, long n, int first, int zero_g, hipStream_t st) {
    if (n % 8) return -1;
    const long n8 = n / 8;
    const int grid = (int)std::min<long>(4096, (n8 + 255) / 256);
#define AGK(T, F, Z) acc_grad_k<T, F, Z><<<grid, 256, 0, st>>>(acc, (T*)g, n8)
#define AGT(T) do { if (first) { if (zero_g) AGK(T, true, true); else AGK(T, true, false); } \
                    else { if (zero_g) AGK(T, false, true); else AGK(T, false, false); } } while (0)
    if (dtype == 1) AGT(bf16_t);
    else AGT(float);
#undef AGT
#undef AGK
    DDL_RETURN_LAUNCH();
}

// acc (fp32) += g (bf16 / fp32); g = 0.  n % 8 == 0, 16-byte aligned buffers.
DDL_API int ddl_drain_acc(int dtype, float* acc, void* g, long n, hipStream_t st) {
    if (n % 8) return -1;
    const long n8 = n / 8;
    const int grid = (int)std::min<long>(4096, (n8 + 255) / 256);
    DISPATCH_T(dtype, (drain_acc_k<bf16_t><<<grid, 256, 0, st>>>(acc, (bf16_t*)g, n8)),
               (drain_acc_k<float><<<grid, 256, 0, st>>>(acc, (float*)g, n8)));
    DDL_RETURN_LAUNCH();
}

// probs (nullable) [B, C], top_v [B, k], top_i (int64) [B, k]; C <= 4096, k <= C
DDL_API int ddl_softmax_topk(int dtype, const void* logits, long B, int C, int k, float* probs, float* top_v,
                             int64_t* top_i, hipStream_t st) {
    if (C > 4096 || k < 1 || k > C) return -1;
    DISPATCH_T(dtype,
               (softmax_topk_k<bf16_t><<<B, 256, 0, st>>>((const bf16_t*)logits, C, k, probs, top_v, top_i)),
               (softmax_topk_k<float><<<B, 256, 0, st>>>((const float*)logits, C, k, probs, top_v, top_i)));
    DDL_RETURN_LAUNCH();
}

// ======================================================================= step glue
// Small kernels that replace the ATen launches still left in a training step: the pooler's tanh
// backward, zero-padded / strided 2-D copies (classifier-head padding, first-token gather and its
// backward), in-place adds into gradient slots, the gradient-arena zero fill, and the embedding
// backward's stable id sort.  Each is one launch where ATen took two to six.
namespace {

// dz = dy * (1 - y^2) (tanh from its output), 8 elements per thread
template <typename T>
__global__ __launch_bounds__(256) void tanh_bwd_k(const T* __restrict__ dy, const T* __restrict__ y, T* __restrict__ dz,
                                                  long n8) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
        float g[8], v[8];
        load8(dy + i * 8, g);
        load8(y + i * 8, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] *= 1.f - v[e] * v[e];
        store8(dz + i * 8, g);
    }
}
template <typename T>
__global__ __launch_bounds__(256) void tanh_bwd_tail_k(const T* __restrict__ dy, const T* __restrict__ y,
                                                       T* __restrict__ dz, long n0, long n) {
    const long i = n0 + (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const float v = to_f(y[i]);
        dz[i] = from_f<T>(to_f(dy[i]) * (1.f - v * v));
    }
}

// dst[r][c] = (r < srows && c < scols) ? src[r][c] : 0 for r < drows, c < dcols (element strides ldd / lds):
// zero padding, slicing and strided gathers in one pass; V = 8 when every row start is 16-byte aligned
template <typename T, int V>
__global__ __launch_bounds__(256) void copy2d_k(T* __restrict__ dst, long ldd, long drows, long dcols,
                                                const T* __restrict__ src, long lds, long srows, long scols) {
    const long cv = dcols / V, total = drows * cv;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const long r = i / cv, c = (i - r * cv) * V;
        if constexpr (V == 8) {
            float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if (r < srows && c + 8 <= scols) load8(src + r * lds + c, v);
            else if (r < srows && c < scols)
                for (int e = 0; e < 8; ++e) v[e] = c + e < scols ? to_f(src[r * lds + c + e]) : 0.f;
            store8(dst + r * ldd + c, v);
        } else {
            dst[r * ldd + c] = (r < srows && c < scols) ? src[r * lds + c] : from_f<T>(0.f);
        }
    }
}

// dst (+)= src, same dtype (a returned gradient folded into its arena slot)
template <typename T>
__global__ __launch_bounds__(256) void add_into_k(T* __restrict__ dst, const T* __restrict__ src, long n) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        dst[i] = from_f<T>(to_f(dst[i]) + to_f(src[i]));
}

// dst[r][c] = a[r][c] + v[c] (the embedding residual: position rows + the token-type row)
template <typename T>
__global__ __launch_bounds__(256) void rows_add_row_k(T* __restrict__ dst, const T* __restrict__ a, const T* __restrict__ v,
                                                      long rows, long cols) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < rows * cols; i += (long)gridDim.x * blockDim.x)
        dst[i] = from_f<T>(to_f(a[i]) + to_f(v[i % cols]));
}

// ViT token assembly: out[b][s] = (s == 0 ? head : src[b][s - 1]) + table[s] for s < S, i.e. the
// class token prepended to the patch tokens plus the position table, in one pass (it was an ATen
// cat + broadcast add).  V = 8: 16-byte bf16 vectors (H % 8 == 0), V = 1: scalar.
template <typename T, int V>
__global__ __launch_bounds__(256) void seq_prepend_add_k(T* __restrict__ out, const T* __restrict__ src,
                                                         const T* __restrict__ head, const T* __restrict__ table,
                                                         long B, long S, long H) {
    const long hv = H / V, n = B * S * hv;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const long row = i / hv, c = (i - row * hv) * V;
        const long b = row / S, s = row - b * S;
        const T* a = s == 0 ? head + c : src + (b * (S - 1) + s - 1) * H + c;
        const T* t = table + s * H + c;
        if constexpr (V == 8) {
            float x[8], y[8];
            load8(a, x);
            load8(t, y);
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] += y[e];
            store8(out + row * H + c, x);
        } else {
            out[row * H + c] = from_f<T>(to_f(*a) + to_f(*t));
        }
    }
}

__global__ __launch_bounds__(256) void zero16_k(uint4* __restrict__ p, long n16) {
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (long)gridDim.x * blockDim.x) p[i] = z;
}
__global__ void zero_bytes_k(unsigned char* __restrict__ p, long n) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = 0;
}

// Stable sort of n <= 32768 token ids: key = id * n + position (unique, ordered by (id, position): any
// sort of these keys is the stable sort of the ids), then s = key / n, pi = key % n.  Replaces rocPRIM's
// block sort + merge passes + ATen's index fill and int32 cast.
//   1. sort_chunk_k: one workgroup per 2048-key chunk (one chunk: the whole job, results written
//      directly), a bitonic network with thread t holding keys t R .. t R + R - 1 in registers, so a
//      compare-exchange at distance j runs
//        j < R:        inside the thread (register pairs);
//        R <= j < 64R: against lane t ^ (j / R) of the same wave (__shfl_xor, no barrier);
//        j >= 64R:     through LDS (store, barrier, partner read, barrier), the image XOR-swizzled by
//                      32-key block so R-strided stores and partner reads hit 32 distinct banks;
//   2. sort_merge_k: one workgroup merges the sorted chunks in LDS (log2(chunks) merge-path levels:
//      each thread binary-searches its diagonal, then merges E = N / 1024 keys into registers).
// A bitonic network is VALU-bound on ONE CU (~9,400 instructions per wave at N = 16384 in registers;
// 81 us), and the first version -- every one of its 105 stages through LDS with a barrier -- took
// 125 us per BERT-base step (profiles/kernels_bert.md); chunks spread the network over 8-16 CUs and
// the merge levels cost ~log2(N) + E steps per thread.
constexpr int SORT_CHUNK = 2048;
__device__ __forceinline__ int sort_swz(int e) { return e ^ ((e >> 5) & 31); }

template <int R, int J>
__device__ __forceinline__ void sort_reg_stage(uint32_t (&v)[R], int tid, int k) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (r & J) continue;
        const bool asc = ((tid * R + r) & k) == 0;
        const uint32_t a = v[r], b = v[r | J];
        v[r] = asc ? min(a, b) : max(a, b);
        v[r | J] = asc ? max(a, b) : min(a, b);
    }
}

// tmp == null: the one chunk is the whole job (s / pi written); else the sorted keys of chunk
// blockIdx.x go to tmp[blockIdx.x * 1024 R ..]
template <int R>
__global__ __launch_bounds__(1024) void sort_chunk_k(const int64_t* __restrict__ ids, int n, int* __restrict__ s,
                                                     int64_t* __restrict__ pi, uint32_t* __restrict__ tmp) {
    extern __shared__ uint32_t keys[];
    constexpr int N = 1024 * R;
    const int tid = threadIdx.x, base = blockIdx.x * N;
    // keys in and results out through the LDS image, so the global loads and stores are coalesced
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int e = base + q * 1024 + tid;
        keys[sort_swz(q * 1024 + tid)] = e < n ? (uint32_t)ids[e] * (uint32_t)n + (uint32_t)e : ~0u;
    }
    __syncthreads();
    uint32_t v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = keys[sort_swz(tid * R + r)];
    __syncthreads();
    for (int k = 2; k <= N; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= 64 * R) {
#pragma unroll
                for (int r = 0; r < R; ++r) keys[sort_swz(tid * R + r)] = v[r];
                __syncthreads();
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int e = tid * R + r;
                    const uint32_t b = keys[sort_swz(e ^ j)];
                    const bool asc = (e & k) == 0, lower = (e & j) == 0;
                    v[r] = lower == asc ? min(v[r], b) : max(v[r], b);
                }
                __syncthreads();
            } else if (j >= R) {
                const int tj = j / R;
                const bool lower = (tid & tj) == 0;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t b = (uint32_t)__shfl_xor((int)v[r], tj, 64);
                    const bool asc = ((tid * R + r) & k) == 0;
                    v[r] = lower == asc ? min(v[r], b) : max(v[r], b);
                }
            } else {
                if constexpr (R > 1) { if (j == 1) sort_reg_stage<R, 1>(v, tid, k); }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) keys[sort_swz(tid * R + r)] = v[r];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int e = q * 1024 + tid;
        const uint32_t kk = keys[sort_swz(e)];
        if (tmp) {
            tmp[base + e] = kk;
        } else if (e < n) {
            s[e] = (int)(kk / (uint32_t)n);
            pi[e] = (int64_t)(kk % (uint32_t)n);
        }
    }
}

// merge nc sorted chunks of SORT_CHUNK keys (tmp) into the sorted whole: N = 1024 E keys in LDS
// (chunks past nc read as ~0u), merge-path levels of run length L = SORT_CHUNK .. N / 2.  tmp may
// alias pi: every key is read into LDS before the first output is written.
template <int E>
__global__ __launch_bounds__(1024) void sort_merge_k(const uint32_t* __restrict__ tmp, int nc, int n,
                                                     int* __restrict__ s, int64_t* __restrict__ pi) {
    extern __shared__ uint32_t keys[];
    constexpr int N = 1024 * E;
    const int tid = threadIdx.x;
    const int nk = nc * SORT_CHUNK;
#pragma unroll
    for (int q = 0; q < E; ++q) {
        const int e = q * 1024 + tid;
        keys[sort_swz(e)] = e < nk ? tmp[e] : ~0u;
    }
    __syncthreads();
    const int o0 = tid * E;
    for (int L = SORT_CHUNK; L < N; L <<= 1) {
        const int blk = o0 & ~(2 * L - 1), d = o0 - blk;
        const int A = blk, B = blk + L;
        // diagonal d: i keys of run A and d - i of run B come first
        int lo = max(0, d - L), hi = min(d, L);
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (keys[sort_swz(A + mid)] < keys[sort_swz(B + d - 1 - mid)]) lo = mid + 1;
            else hi = mid;
        }
        int i = lo, j = d - lo;
        uint32_t out[E];
        uint32_t a = i < L ? keys[sort_swz(A + i)] : ~0u, b = j < L ? keys[sort_swz(B + j)] : ~0u;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const bool takeA = j >= L || (i < L && a <= b);
            out[e] = takeA ? a : b;
            if (takeA) { ++i; a = i < L ? keys[sort_swz(A + i)] : ~0u; }
            else { ++j; b = j < L ? keys[sort_swz(B + j)] : ~0u; }
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < E; ++e) keys[sort_swz(o0 + e)] = out[e];
        __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < E; ++q) {
        const int e = q * 1024 + tid;
        if (e < n) {
            const uint32_t kk = keys[sort_swz(e)];
            s[e] = (int)(kk / (uint32_t)n);
            pi[e] = (int64_t)(kk % (uint32_t)n);
        }
    }
}

}  // namespace

DDL_API int ddl_tanh_bwd(int dtype, const void* dy, const void* y, void* dz, long n, hipStream_t st) {
    const long n8 = n / 8, tail = n - n8 * 8;
    if (n8 > 0)
        DISPATCH_T(dtype,
                   (tanh_bwd_k<bf16_t><<<grid_for(n8), 256, 0, st>>>((const bf16_t*)dy, (const bf16_t*)y, (bf16_t*)dz, n8)),
                   (tanh_bwd_k<float><<<grid_for(n8), 256, 0, st>>>((const float*)dy, (const float*)y, (float*)dz, n8)));
    if (tail > 0)
        DISPATCH_T(dtype,
                   (tanh_bwd_tail_k<bf16_t><<<1, 256, 0, st>>>((const bf16_t*)dy, (const bf16_t*)y, (bf16_t*)dz, n8 * 8, n)),
                   (tanh_bwd_tail_k<float><<<1, 256, 0, st>>>((const float*)dy, (const float*)y, (float*)dz, n8 * 8, n)));
    DDL_RETURN_LAUNCH();
}

// zero-padded / strided 2-D copy (element strides); dst and src must not overlap
DDL_API int ddl_copy2d(int dtype, void* dst, long ldd, long drows, long dcols, const void* src, long lds, long srows,
                       long scols, hipStream_t st) {
    if (drows <= 0 || dcols <= 0) return 0;
    const int esz = dtype == 1 ? 2 : 4;
    const bool v8 = dtype == 1 && dcols % 8 == 0 && ldd % 8 == 0 && lds % 8 == 0 &&
                    ((uintptr_t)dst % 16) == 0 && (scols == 0 || ((uintptr_t)src % 16) == 0);
    (void)esz;
    const long work = v8 ? drows * (dcols / 8) : drows * dcols;
    if (v8)
        copy2d_k<bf16_t, 8><<<grid_for(work), 256, 0, st>>>((bf16_t*)dst, ldd, drows, dcols, (const bf16_t*)src, lds,
                                                            srows, scols);
    else
        DISPATCH_T(dtype,
                   (copy2d_k<bf16_t, 1><<<grid_for(work), 256, 0, st>>>((bf16_t*)dst, ldd, drows, dcols,
                                                                      (const bf16_t*)src, lds, srows, scols)),
                   (copy2d_k<float, 1><<<grid_for(work), 256, 0, st>>>((float*)dst, ldd, drows, dcols,
                                                                     (const float*)src, lds, srows, scols)));
    DDL_RETURN_LAUNCH();
}

DDL_API int ddl_add_into(int dtype, void* dst, const void* src, long n, hipStream_t st) {
    if (n <= 0) return 0;
    DISPATCH_T(dtype, (add_into_k<bf16_t><<<grid_for(n), 256, 0, st>>>((bf16_t*)dst, (const bf16_t*)src, n)),
               (add_into_k<float><<<grid_for(n), 256, 0, st>>>((float*)dst, (const float*)src, n)));
    DDL_RETURN_LAUNCH();
}

DDL_API int ddl_rows_add_row(int dtype, void* dst, const void* a, const void* v, long rows, long cols, hipStream_t st) {
    if (rows * cols <= 0) return 0;
    DISPATCH_T(dtype,
               (rows_add_row_k<bf16_t><<<grid_for(rows * cols), 256, 0, st>>>((bf16_t*)dst, (const bf16_t*)a,
                                                                            (const bf16_t*)v, rows, cols)),
               (rows_add_row_k<float><<<grid_for(rows * cols), 256, 0, st>>>((float*)dst, (const float*)a,
                                                                           (const float*)v, rows, cols)));
    DDL_RETURN_LAUNCH();
}

// out [B][S][H] = [head | src[b] (S - 1 rows)] + table [S][H] (see seq_prepend_add_k)
DDL_API int ddl_seq_prepend_add(int dtype, void* out, const void* src, const void* head, const void* table, long B,
                                long S, long H, hipStream_t st) {
    if (B <= 0 || S <= 0 || H <= 0) return 0;
    const bool v8 = dtype == 1 && H % 8 == 0 && ((uintptr_t)out % 16) == 0 && ((uintptr_t)src % 16) == 0 &&
                    ((uintptr_t)head % 16) == 0 && ((uintptr_t)table % 16) == 0;
    if (v8)
        seq_prepend_add_k<bf16_t, 8><<<grid_for(B * S * (H / 8)), 256, 0, st>>>(
            (bf16_t*)out, (const bf16_t*)src, (const bf16_t*)head, (const bf16_t*)table, B, S, H);
    else
        DISPATCH_T(dtype,
                   (seq_prepend_add_k<bf16_t, 1><<<grid_for(B * S * H), 256, 0, st>>>(
                       (bf16_t*)out, (const bf16_t*)src, (const bf16_t*)head, (const bf16_t*)table, B, S, H)),
                   (seq_prepend_add_k<float, 1><<<grid_for(B * S * H), 256, 0, st>>>(
                       (float*)out, (const float*)src, (const float*)head, (const float*)table, B, S, H)));
    DDL_RETURN_LAUNCH();
}

DDL_API int ddl_zero(void* p, long nbytes, hipStream_t st) {
    if (nbytes <= 0) return 0;
    unsigned char* b = (unsigned char*)p;
    long head = (long)((16 - ((uintptr_t)b & 15)) & 15);
    if (head > nbytes) head = nbytes;
    if (head) zero_bytes_k<<<1, 64, 0, st>>>(b, head);
    const long n16 = (nbytes - head) / 16;
    if (n16 > 0) zero16_k<<<grid_for(n16), 256, 0, st>>>((uint4*)(b + head), n16);
    const long tail = nbytes - head - n16 * 16;
    if (tail > 0) zero_bytes_k<<<1, 64, 0, st>>>(b + head + n16 * 16, tail);
    DDL_RETURN_LAUNCH();
}

// 1 when ddl_sort_ids can sort n ids below vocab (else the caller sorts another way)
DDL_API int ddl_sort_ids_ok(long n, long vocab) {
    return n > 0 && n <= 32768 && (unsigned long long)vocab * (unsigned long long)n < (1ull << 32) ? 1 : 0;
}

static bool sort_lds_ok(const void* k, int bytes) {
    return bytes <= 65536 || hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess;
}

template <int E>
static int sort_merge_launch(const int64_t* ids, long n, int* s, int64_t* pi, hipStream_t st) {
    static const bool ok = sort_lds_ok((const void*)sort_merge_k<E>, 1024 * E * 4);
    if (!ok) return -1;
    const int nc = (int)((n + SORT_CHUNK - 1) / SORT_CHUNK);
    // the sorted chunks (nc x 2048 keys, <= 8 n bytes for nc >= 2) live in pi's storage until merged
    uint32_t* tmp = reinterpret_cast<uint32_t*>(pi);
    sort_chunk_k<SORT_CHUNK / 1024><<<nc, 1024, SORT_CHUNK * 4, st>>>(ids, (int)n, s, pi, tmp);
    sort_merge_k<E><<<1, 1024, (size_t)1024 * E * 4, st>>>(tmp, nc, (int)n, s, pi);
    DDL_RETURN_LAUNCH();
}

DDL_API int ddl_sort_ids(const int64_t* ids, long n, int* s, int64_t* pi, hipStream_t st) {
    if (n <= 0 || n > 32768) return -1;
    if (n <= 1024) {
        sort_chunk_k<1><<<1, 1024, 1024 * 4, st>>>(ids, (int)n, s, pi, nullptr);
        DDL_RETURN_LAUNCH();
    }
    if (n <= 2048) {
        sort_chunk_k<2><<<1, 1024, 2048 * 4, st>>>(ids, (int)n, s, pi, nullptr);
        DDL_RETURN_LAUNCH();
    }
    if (n <= 4096) return sort_merge_launch<4>(ids, n, s, pi, st);
    if (n <= 8192) return sort_merge_launch<8>(ids, n, s, pi, st);
    if (n <= 16384) return sort_merge_launch<16>(ids, n, s, pi, st);
    return sort_merge_launch<32>(ids, n, s, pi, st);
}
