// Fused multi-head attention (flash-style) for gfx950, head dim 64 (BERT-base/large,
// ViT-B/16).  Kernel families K14 (forward) and K15 (backward).
//
// Layout: packed QKV straight from the fused QKV GEMM, row (b, s) holds
// [q(H*D) | k(H*D) | v(H*D)]; the output is [B, S, H*D] ready for the output
// projection; gradients are written into a packed dQKV of the same layout.
//
// Forward (one workgroup = 4 wave64 = 64 query rows of one (b, h)):
//   S^T = K Q^T with v_mfma_f32_16x16x32_bf16 so each lane holds one query row's
//   scores in registers (query on the lane, keys in the accumulator registers);
//   online softmax on exp2 with per-lane partial row sums (no shuffles per tile);
//   O^T += V^T P^T with P fed from the accumulator registers as the B operand
//   (the MFMA's k order is permuted consistently for both operands, so P never
//   goes through LDS) and V^T fragments read by ds_read_b64_tr_b16.
//   K/V tiles of 64 keys are register-staged into double-buffered, XOR-swizzled
//   LDS; the next tile's global loads are in flight under the current MFMAs.
// Backward: dKV kernel (one workgroup per 64 keys, loops over queries) and dQ
// kernel (one workgroup per 64 queries, loops over keys): every sum stays on
// chip, no atomics; P is recomputed from the saved log-sum-exp.
// Dropout on the attention probabilities uses the counter hash of ddl_common.h
// keyed by ((b*H+h)*S + q)*S + k, regenerated in backward.
#include "ddl_common.h"

namespace {

constexpr int D = 64;          // head dim
constexpr int TQ = 64;         // queries per workgroup
constexpr int TK = 64;         // keys per tile
constexpr int ROWB = 128;      // bytes per LDS row (64 bf16)
constexpr float LOG2E = 1.4426950408889634f;

typedef __attribute__((address_space(3))) s16x4 lds_v4;

// Row image swizzle (128-B rows; ds_read_b128 fragment reads conflict free).
__device__ __forceinline__ int swz_row(int r, int c) { return c ^ ((r >> 1) & 7); }
// V / transposed-read image: 8 consecutive rows x 2 chunks conflict free for tr reads.
__device__ __forceinline__ int swz_tr(int r, int c) { return c ^ (2 * ((r >> 1) & 3)); }

template <bool TR>
__device__ __forceinline__ int lds_off(int r, int c) {
    return r * ROWB + ((TR ? swz_tr(r, c) : swz_row(r, c)) << 4);
}

// fragment: rows rbase..+15 (lane&15), k = 32kk + 8(lane>>4) + 0..7, from a row image
template <bool TR>
__device__ __forceinline__ bf16x8 frag_rows(const char* lds, int rbase, int kk) {
    const int l = threadIdx.x & 63;
    const int r = rbase + (l & 15);
    return *reinterpret_cast<const bf16x8*>(lds + lds_off<TR>(r, kk * 4 + (l >> 4)));
}

// transposed fragment with the permuted k order used for accumulator operands:
// lane l gets column cbase + (l&15) of rows  kb + 16h + 4g + {0..3}, h = 0,1
// (kb = 32 s), i.e. element j <-> row kb + 16 (j>>2) + 4 g + (j&3).
template <bool TR>
__device__ __forceinline__ bf16x8 frag_tr(const char* lds, int kb, int cbase) {
    const int l = threadIdx.x & 63;
    const int g = l >> 4, q = (l >> 2) & 3, p = l & 3;
    const int col = cbase + 4 * p;
    const int ra = kb + 4 * g + q, rb = ra + 16;
    const char* pa = lds + lds_off<TR>(ra, col >> 3) + (p & 1) * 8;
    const char* pb = lds + lds_off<TR>(rb, col >> 3) + (p & 1) * 8;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)pa);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)pb);
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
}

// pack 8 fp32 (two accumulator 4-vectors, blocks 2s and 2s+1) into an operand
__device__ __forceinline__ bf16x8 pack_acc(const f32x4& a, const f32x4& b) {
    bf16x8 r;
    r[0] = (__bf16)a[0]; r[1] = (__bf16)a[1]; r[2] = (__bf16)a[2]; r[3] = (__bf16)a[3];
    r[4] = (__bf16)b[0]; r[5] = (__bf16)b[1]; r[6] = (__bf16)b[2]; r[7] = (__bf16)b[3];
    return r;
}

// stage a [64 rows][64] bf16 tile (rows >= nrows -> 0) with 256 threads: 2 chunks each
struct Stager {
    uint4 v[2];
    __device__ __forceinline__ void load(const bf16_t* base, long row_stride, int row0, int nrows) {
        const int t = threadIdx.x;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int r = (t >> 3) + 32 * i, c = t & 7;
            const bool ok = row0 + r < nrows;
            const uint4 x = *reinterpret_cast<const uint4*>(base + (long)(ok ? row0 + r : 0) * row_stride + c * 8);
            v[i] = ok ? x : make_uint4(0, 0, 0, 0);
        }
    }
    template <bool TR>
    __device__ __forceinline__ void store(char* lds) {
        const int t = threadIdx.x;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int r = (t >> 3) + 32 * i, c = t & 7;
            *reinterpret_cast<uint4*>(lds + lds_off<TR>(r, c)) = v[i];
        }
    }
};

__device__ __forceinline__ uint32_t drop_thresh(float p) {
    const double t = (double)p * 4294967296.0;
    return t >= 4294967295.0 ? 4294967295u : (uint32_t)t;
}

__device__ __forceinline__ bf16x8 load_frag_global(const bf16_t* rowp, int kk) {
    const int l = threadIdx.x & 63;
    return *reinterpret_cast<const bf16x8*>(rowp + kk * 32 + 8 * (l >> 4));
}

// ============================================================ forward
__global__ __launch_bounds__(256) void attn_fwd_k(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                                                  bf16_t* __restrict__ out, float* __restrict__ lse, int B, int S, int H,
                                                  float scale, float p_drop, uint64_t seed) {
    __shared__ __attribute__((aligned(16))) char smem[4 * TK * ROWB];   // K0 V0 K1 V1
    const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4;
    const long rs = 3L * H * D;                              // qkv row stride
    const bf16_t* qb = qkv + (long)b * S * rs + h * D;
    const bf16_t* kb = qb + H * D;
    const bf16_t* vb = qb + 2 * H * D;
    const int q0 = blockIdx.x * TQ + w * 16;
    const int myq = q0 + (lane & 15);
    const bool qok = myq < S;
    // Q fragments (B operand of S^T = K Q^T): lane holds Q[myq][32kk + 8g + 0..7]
    bf16x8 qf[2];
    {
        const bf16_t* qr = qb + (long)(qok ? myq : 0) * rs;
        qf[0] = load_frag_global(qr, 0);
        qf[1] = load_frag_global(qr, 1);
    }
    const float c2 = scale * LOG2E;
    float m = -INFINITY, lsum = 0.f;
    f32x4 o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const uint32_t thresh = drop_thresh(p_drop);
    const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;

    const int nt = (S + TK - 1) / TK;
    Stager sk, sv;
    sk.load(kb, rs, 0, S);
    sv.load(vb, rs, 0, S);
    sk.store<false>(smem);
    sv.store<true>(smem + TK * ROWB);
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
        char* sK = smem + (t & 1) * 2 * TK * ROWB;
        char* sV = sK + TK * ROWB;
        const bool more = t + 1 < nt;
        if (more) {
            sk.load(kb, rs, (t + 1) * TK, S);
            sv.load(vb, rs, (t + 1) * TK, S);
        }
        // ---- S^T block: lane holds s[blk][r] = score(q = myq, k = t*64 + 16 blk + 4 g + r)
        f32x4 s[4];
#pragma unroll
        for (int blk = 0; blk < 4; ++blk) {
            s[blk] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
                s[blk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<false>(sK, 16 * blk, kk), qf[kk], s[blk],
                                                                  0, 0, 0);
        }
        // ---- scale, mask, online softmax (log2 domain)
        float tmax = -INFINITY;
#pragma unroll
        for (int blk = 0; blk < 4; ++blk)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int key = t * TK + 16 * blk + 4 * g + r;
                float v = s[blk][r] * c2;
                if (mask) v += (key < S ? mask[(long)b * S + key] : 0.f) * LOG2E;
                if (key >= S) v = -INFINITY;
                s[blk][r] = v;
                tmax = fmaxf(tmax, v);
            }
        tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        const float mnew = fmaxf(m, tmax);
        const float alpha = (m == -INFINITY) ? 0.f : exp2f(m - mnew);
        const float msub = mnew == -INFINITY ? 0.f : mnew;
        m = mnew;
        float psum = 0.f;
#pragma unroll
        for (int blk = 0; blk < 4; ++blk)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float pv = exp2f(s[blk][r] - msub);
                psum += pv;
                if (p_drop > 0.f) {
                    const int key = t * TK + 16 * blk + 4 * g + r;
                    const uint64_t idx = ((uint64_t)bh * S + myq) * S + key;
                    pv = keep_elem(seed, idx, thresh) ? pv * inv_keep : 0.f;
                }
                s[blk][r] = pv;
            }
        lsum = lsum * alpha + psum;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] *= alpha;
        // ---- O^T[d][q] += V^T[d][k] P^T[k][q]
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            const bf16x8 pf = pack_acc(s[2 * st], s[2 * st + 1]);
#pragma unroll
            for (int db = 0; db < 4; ++db)
                o[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<true>(sV, 32 * st, 16 * db), pf, o[db], 0, 0, 0);
        }
        if (more) {
            char* nK = smem + ((t + 1) & 1) * 2 * TK * ROWB;
            sk.store<false>(nK);
            sv.store<true>(nK + TK * ROWB);
        }
        __syncthreads();
    }
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    if (!qok) return;
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    bf16_t* orow = out + ((long)b * S + myq) * H * D + h * D;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
        float v[4] = {o[db][0] * inv, o[db][1] * inv, o[db][2] * inv, o[db][3] * inv};
        store4(orow + 16 * db + 4 * g, v);
    }
    if (g == 0) lse[(long)bh * S + myq] = (m + log2f(lsum)) / LOG2E;   // natural-log LSE of scaled scores
}

// delta[b,h,q] = sum_d dO[q][d] * O[q][d]
// delta[b,h,q] = sum_d dO * O.  8 lanes per (b, s, h) row, 16-B loads, a 3-step
// xor-shuffle reduction: a pure streaming pass over dO and O.
__global__ __launch_bounds__(256) void attn_delta_k(const bf16_t* __restrict__ dout, const bf16_t* __restrict__ out,
                                                    float* __restrict__ delta, int B, int S, int H) {
    const long row = ((long)blockIdx.x * 256 + threadIdx.x) >> 3;   // (b*S + s)*H + h
    const int part = threadIdx.x & 7;
    const bool ok = row < (long)B * S * H;
    float a = 0.f;
    if (ok) {
        float x[8], y[8];
        load8(dout + row * D + part * 8, x);
        load8(out + row * D + part * 8, y);
#pragma unroll
        for (int j = 0; j < 8; ++j) a += x[j] * y[j];
    }
    a += __shfl_xor(a, 1);
    a += __shfl_xor(a, 2);
    a += __shfl_xor(a, 4);
    if (ok && part == 0) {
        const long bs = row / H;
        const int h = (int)(row - bs * H);
        const long b = bs / S, q = bs - b * S;
        delta[(b * H + h) * S + q] = a;
    }
}

// ============================================================ backward dK, dV
// workgroup = 64 keys of one (b, h); wave w owns keys k0 + 16 w .. +15 (key on the lane).
__global__ __launch_bounds__(256) void attn_bwd_dkv_k(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout,
                                                      const float* __restrict__ lse, const float* __restrict__ delta,
                                                      const float* __restrict__ mask, bf16_t* __restrict__ dqkv, int B,
                                                      int S, int H, float scale, float p_drop, uint64_t seed) {
    __shared__ __attribute__((aligned(16))) char smem[2 * TQ * ROWB];   // Q, dO tiles
    __shared__ float s_lse[TQ], s_delta[TQ];
    const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4;
    const long rs = 3L * H * D;
    const bf16_t* qb = qkv + (long)b * S * rs + h * D;
    const bf16_t* kb = qb + H * D;
    const bf16_t* vb = qb + 2 * H * D;
    const bf16_t* dob = dout + (long)b * S * H * D + h * D;
    const int k0 = blockIdx.x * TK + w * 16;
    const int myk = k0 + (lane & 15);
    const bool kok = myk < S;
    // K and V rows of my key as B operands (lane: row myk, d = 32kk + 8g + ..)
    bf16x8 kf[2], vf[2];
    {
        const bf16_t* kr = kb + (long)(kok ? myk : 0) * rs;
        const bf16_t* vr = vb + (long)(kok ? myk : 0) * rs;
        kf[0] = load_frag_global(kr, 0); kf[1] = load_frag_global(kr, 1);
        vf[0] = load_frag_global(vr, 0); vf[1] = load_frag_global(vr, 1);
    }
    const float mbias = (mask && kok) ? mask[(long)b * S + myk] : 0.f;
    const float c2 = scale * LOG2E;
    const uint32_t thresh = drop_thresh(p_drop);
    const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    f32x4 dv[4], dk[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { dv[i] = (f32x4){0, 0, 0, 0}; dk[i] = (f32x4){0, 0, 0, 0}; }
    char* sQ = smem;
    char* sO = smem + TQ * ROWB;
    const int nt = (S + TQ - 1) / TQ;
    for (int t = 0; t < nt; ++t) {
        Stager a, c;
        a.load(qb, rs, t * TQ, S);
        c.load(dob, (long)H * D, t * TQ, S);
        __syncthreads();             // previous tile fully consumed
        a.store<false>(sQ);
        c.store<false>(sO);
        if (threadIdx.x < TQ) {
            const int q = t * TQ + threadIdx.x;
            s_lse[threadIdx.x] = q < S ? lse[(long)bh * S + q] : 0.f;
            s_delta[threadIdx.x] = q < S ? delta[(long)bh * S + q] : 0.f;
        }
        __syncthreads();
        // S[q][k] and dP[q][k]: lane holds q = t*64 + 16 qb + 4 g + r, k = myk
        f32x4 sc[4], dp[4];
#pragma unroll
        for (int qbk = 0; qbk < 4; ++qbk) {
            sc[qbk] = (f32x4){0, 0, 0, 0};
            dp[qbk] = (f32x4){0, 0, 0, 0};
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                sc[qbk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<false>(sQ, 16 * qbk, kk), kf[kk], sc[qbk], 0, 0, 0);
                dp[qbk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<false>(sO, 16 * qbk, kk), vf[kk], dp[qbk], 0, 0, 0);
            }
        }
        f32x4 pd[4], ds[4];
#pragma unroll
        for (int qbk = 0; qbk < 4; ++qbk)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ql = 16 * qbk + 4 * g + r;
                const int q = t * TQ + ql;
                float pv = (q < S && kok) ? exp2f(sc[qbk][r] * c2 + mbias * LOG2E - s_lse[ql] * LOG2E) : 0.f;
                float dpv = dp[qbk][r];
                float pdrop = pv;
                if (p_drop > 0.f) {
                    const uint64_t idx = ((uint64_t)bh * S + q) * S + myk;
                    const bool keep = keep_elem(seed, idx, thresh);
                    pdrop = keep ? pv * inv_keep : 0.f;
                    dpv = keep ? dpv * inv_keep : 0.f;
                }
                pd[qbk][r] = pdrop;
                ds[qbk][r] = pv * (dpv - s_delta[ql]);
            }
        // dV^T[d][k] += dO^T[d][q] Pd[q][k];  dK^T[d][k] += Q^T[d][q] dS[q][k]
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            const bf16x8 pf = pack_acc(pd[2 * st], pd[2 * st + 1]);
            const bf16x8 sf = pack_acc(ds[2 * st], ds[2 * st + 1]);
#pragma unroll
            for (int db = 0; db < 4; ++db) {
                dv[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<false>(sO, 32 * st, 16 * db), pf, dv[db], 0, 0, 0);
                dk[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<false>(sQ, 32 * st, 16 * db), sf, dk[db], 0, 0, 0);
            }
        }
    }
    if (!kok) return;
    bf16_t* dkr = dqkv + ((long)b * S + myk) * rs + H * D + h * D;
    bf16_t* dvr = dkr + H * D;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
        float a4[4] = {dk[db][0] * scale, dk[db][1] * scale, dk[db][2] * scale, dk[db][3] * scale};
        float b4[4] = {dv[db][0], dv[db][1], dv[db][2], dv[db][3]};
        store4(dkr + 16 * db + 4 * g, a4);
        store4(dvr + 16 * db + 4 * g, b4);
    }
}

// ============================================================ backward dQ
// workgroup = 64 queries; wave owns 16 queries (query on the lane), loops over key tiles.
__global__ __launch_bounds__(256) void attn_bwd_dq_k(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout,
                                                     const float* __restrict__ lse, const float* __restrict__ delta,
                                                     const float* __restrict__ mask, bf16_t* __restrict__ dqkv, int B,
                                                     int S, int H, float scale, float p_drop, uint64_t seed) {
    __shared__ __attribute__((aligned(16))) char smem[2 * TK * ROWB];   // K, V tiles
    const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4;
    const long rs = 3L * H * D;
    const bf16_t* qb = qkv + (long)b * S * rs + h * D;
    const bf16_t* kb = qb + H * D;
    const bf16_t* vb = qb + 2 * H * D;
    const bf16_t* dob = dout + (long)b * S * H * D + h * D;
    const int myq = blockIdx.x * TQ + w * 16 + (lane & 15);
    const bool qok = myq < S;
    bf16x8 qf[2], of[2];
    {
        const bf16_t* qr = qb + (long)(qok ? myq : 0) * rs;
        const bf16_t* orr = dob + (long)(qok ? myq : 0) * H * D;
        qf[0] = load_frag_global(qr, 0); qf[1] = load_frag_global(qr, 1);
        of[0] = load_frag_global(orr, 0); of[1] = load_frag_global(orr, 1);
    }
    const float my_lse = qok ? lse[(long)bh * S + myq] : 0.f;
    const float my_delta = qok ? delta[(long)bh * S + myq] : 0.f;
    const float c2 = scale * LOG2E;
    const uint32_t thresh = drop_thresh(p_drop);
    const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    f32x4 dq[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) dq[i] = (f32x4){0, 0, 0, 0};
    char* sK = smem;
    char* sV = smem + TK * ROWB;
    const int nt = (S + TK - 1) / TK;
    for (int t = 0; t < nt; ++t) {
        Stager a, c;
        a.load(kb, rs, t * TK, S);
        c.load(vb, rs, t * TK, S);
        __syncthreads();
        a.store<false>(sK);
        c.store<false>(sV);
        __syncthreads();
        // S^T[k][q], dP^T[k][q]: lane holds k = t*64 + 16 blk + 4 g + r, q = myq
        f32x4 sc[4], dp[4];
#pragma unroll
        for (int blk = 0; blk < 4; ++blk) {
            sc[blk] = (f32x4){0, 0, 0, 0};
            dp[blk] = (f32x4){0, 0, 0, 0};
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                sc[blk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<false>(sK, 16 * blk, kk), qf[kk], sc[blk], 0, 0, 0);
                dp[blk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<false>(sV, 16 * blk, kk), of[kk], dp[blk], 0, 0, 0);
            }
        }
        f32x4 ds[4];
#pragma unroll
        for (int blk = 0; blk < 4; ++blk)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int key = t * TK + 16 * blk + 4 * g + r;
                const bool ok = qok && key < S;
                const float mb = (mask && key < S) ? mask[(long)b * S + key] : 0.f;
                const float pv = ok ? exp2f(sc[blk][r] * c2 + mb * LOG2E - my_lse * LOG2E) : 0.f;
                float dpv = dp[blk][r];
                if (p_drop > 0.f) {
                    const uint64_t idx = ((uint64_t)bh * S + myq) * S + key;
                    dpv = keep_elem(seed, idx, thresh) ? dpv * inv_keep : 0.f;
                }
                ds[blk][r] = pv * (dpv - my_delta);
            }
        // dQ^T[d][q] += K^T[d][k] dS^T[k][q]
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            const bf16x8 sf = pack_acc(ds[2 * st], ds[2 * st + 1]);
#pragma unroll
            for (int db = 0; db < 4; ++db)
                dq[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<false>(sK, 32 * st, 16 * db), sf, dq[db], 0, 0, 0);
        }
    }
    if (!qok) return;
    bf16_t* dqr = dqkv + ((long)b * S + myq) * rs + h * D;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
        float a4[4] = {dq[db][0] * scale, dq[db][1] * scale, dq[db][2] * scale, dq[db][3] * scale};
        store4(dqr + 16 * db + 4 * g, a4);
    }
}

}  // namespace

// qkv [B, S, 3*H*64] bf16; mask: additive key bias [B, S] fp32 or null; out [B, S, H*64]; lse [B, H, S] fp32
DDL_API int ddl_attn_fwd(const void* qkv, const float* mask, void* out, float* lse, int B, int S, int H, float scale,
                         float p_drop, uint64_t seed, hipStream_t st) {
    dim3 grid((S + TQ - 1) / TQ, B * H);
    attn_fwd_k<<<grid, 256, 0, st>>>((const bf16_t*)qkv, mask, (bf16_t*)out, lse, B, S, H, scale, p_drop, seed);
    DDL_RETURN_LAUNCH();
}

// dqkv [B, S, 3*H*64] bf16 (fully written); delta scratch [B, H, S] fp32
DDL_API int ddl_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse, const float* mask,
                         float* delta, void* dqkv, int B, int S, int H, float scale, float p_drop, uint64_t seed,
                         hipStream_t st) {
    const long rows = (long)B * S * H;
    attn_delta_k<<<(int)((rows * 8 + 255) / 256), 256, 0, st>>>((const bf16_t*)dout, (const bf16_t*)out, delta, B, S, H);
    dim3 grid((S + TK - 1) / TK, B * H);
    attn_bwd_dkv_k<<<grid, 256, 0, st>>>((const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, mask, (bf16_t*)dqkv, B,
                                         S, H, scale, p_drop, seed);
    attn_bwd_dq_k<<<grid, 256, 0, st>>>((const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, mask, (bf16_t*)dqkv, B, S,
                                        H, scale, p_drop, seed);
    DDL_RETURN_LAUNCH();
}
