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
// Dropout on the attention probabilities: one lowbias32 hash per pair of score
// indices ((b*H+h)*S + q)*S + k (attn_hash below), drawn in the forward, which also
// stores the keep decisions as a bit mask (1 bit per score, dmask_word below); the
// backward kernels read the bits instead of re-hashing every score (lane = key in
// the dK/dV passes: one hash per score there cost ~2.4x the pass's MFMA time).
#include "ddl_common.h"

#include <algorithm>
#include <cstdlib>

namespace {

constexpr int D = 64;          // head dim
constexpr int TQ = 64;         // query rows per staged tile
constexpr int TK = 64;         // keys per tile
// waves per workgroup of the tiled (S > 256) kernels, 16 rows each; a staged tile is shared by all
// of them.  Forward: 8 (each K / V tile staged once per 128 queries: fwd 63 -> 57 us at BERT-large's
// shape); backward: 4 (at 8 the dK/dV and dQ kernels' 130-160 VGPRs leave one 8-wave workgroup
// per CU instead of three 4-wave ones, and fwd+bwd went 178 -> 200 us)
constexpr int TWF = 8, TWB = 4;
constexpr int TROWS_F = 16 * TWF, TROWS_B = 16 * TWB;
constexpr int ROWB = 128;      // bytes per LDS row (64 bf16)
constexpr int FS = 128;        // longest sequence of the one-workgroup-per-(b, h) kernels
constexpr float LOG2E = 1.4426950408889634f;

typedef __attribute__((address_space(3))) s16x4 lds_v4;

// 2^x as the bare v_exp_f32: exp2f adds a denormal-range fix-up (ldexp, compare, select)
// per call; softmax arguments are <= 0 and a result below 2^-126 may as well be 0
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Row image swizzle (128-B rows; ds_read_b128 fragment reads conflict free).
__device__ __forceinline__ int swz_row(int r, int c) { return c ^ ((r >> 1) & 7); }
// V / transposed-read image: 8 consecutive rows x 2 chunks conflict free for tr reads.  It is
// conflict free for frag_rows' ds_read_b128 groups too (16-row fragments: the 8 even and the 8
// odd rows of a lane group land on 8 distinct 16-B slots), so images read BOTH ways (Q, dO, K
// and the dS^T images of the fused backward kernels) use it; the row swizzle above put pairs of
// rows on the same slots for the tr reads (2-way conflicts: ~32 % extra LDS cycles).
__device__ __forceinline__ int swz_tr(int r, int c) { return c ^ (2 * ((r >> 1) & 3)); }

// dS^T images of the fused backward kernels: written as 8-byte pieces, one key row per lane (16 rows
// x one chunk per half-wave pass) and read transposed (8 rows x 2 chunks per pass).  swz_tr repeats
// its pattern every 8 rows, so rows r and r + 8 of a write pass collided (2-way: the 16.7 % LDS
// bank conflicts of attn_bwd_fused_k); bit 3 of the row in the chunk's low bit separates them and
// keeps the transposed reads conflict free.  A ds_write_b64 lane group is 16 lanes banked over 128 B
// (one row), so rows r and r ^ 1 -- same chunk -- still shared 8-byte slots: odd rows also swap the
// two 8-byte halves of every chunk (ds_half; frag_tr<., true> reads them back), which makes the 16
// pieces of a write pass 16 distinct slots and leaves every transposed read pass's slot set as it was.
__device__ __forceinline__ int swz_ds(int r, int c) { return c ^ ((2 * ((r >> 1) & 3)) | ((r >> 3) & 1)); }

// byte offset of the 8-byte half `h` (0 / 1) of a chunk in row r of a dS^T image
__device__ __forceinline__ int ds_half(int r, int h) { return ((h ^ r) & 1) * 8; }

template <bool TR, bool DS = false>
__device__ __forceinline__ int lds_off(int r, int c) {
    return r * ROWB + ((TR ? (DS ? swz_ds(r, c) : swz_tr(r, c)) : swz_row(r, c)) << 4);
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
template <bool TR, bool DS = false>
__device__ __forceinline__ bf16x8 frag_tr(const char* lds, int kb, int cbase) {
    const int l = threadIdx.x & 63;
    const int g = l >> 4, q = (l >> 2) & 3, p = l & 3;
    const int col = cbase + 4 * p;
    const int ra = kb + 4 * g + q, rb = ra + 16;
    // dS^T images also swap the 8-byte halves of odd rows (swz_ds below); rb = ra + 16 has ra's parity
    const int half = DS ? ((p ^ ra) & 1) : (p & 1);
    const char* pa = lds + lds_off<TR, DS>(ra, col >> 3) + half * 8;
    const char* pb = lds + lds_off<TR, DS>(rb, col >> 3) + half * 8;
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

// ok ? v : 0 per component: a select of whole vectors made hipcc park both in scratch and
// select a scratch POINTER (a scratch store + load on every staged chunk)
__device__ __forceinline__ uint4 zero_unless(bool ok, uint4 v) {
    return make_uint4(ok ? v.x : 0u, ok ? v.y : 0u, ok ? v.z : 0u, ok ? v.w : 0u);
}

// stage a [64 rows][64] bf16 tile (rows >= nrows -> 0) with NT threads: 512 / NT chunks each.
// load() keeps the RAW loaded chunks and only records which rows are past the end; the zero
// select happens in store(): a select right after the load made the compiler wait for the
// load there (s_waitcnt vmcnt(0) straight behind the prefetch), so a tile "prefetched" under
// the previous tile's compute was in fact waited for before that compute started
template <int NT = 256>
struct Stager {
    static constexpr int PER = 512 / NT;
    uint4 v[PER];
    bool ok[PER];
    __device__ __forceinline__ void load(const bf16_t* base, long row_stride, int row0, int nrows) {
        const int t = threadIdx.x;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int r = (t >> 3) + (NT / 8) * i, c = t & 7;
            ok[i] = row0 + r < nrows;
            v[i] = *reinterpret_cast<const uint4*>(base + (long)(ok[i] ? row0 + r : 0) * row_stride + c * 8);
        }
    }
    template <bool TR>
    __device__ __forceinline__ void store(char* lds) {
        const int t = threadIdx.x;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int r = (t >> 3) + (NT / 8) * i, c = t & 7;
            *reinterpret_cast<uint4*>(lds + lds_off<TR>(r, c)) = zero_unless(ok[i], v[i]);
        }
    }
};

// Probability dropout: the pair hash of ddl_common.h over the score index
// idx = ((b*H + h)*S + q)*S + k, the same decision in the forward and in both
// backward kernels.
__device__ __forceinline__ uint32_t attn_hash(uint64_t seed, uint64_t pidx) { return pair_hash(seed, pidx); }
__device__ __forceinline__ bool attn_keep_half(uint32_t h, uint64_t idx, uint32_t thresh16) {
    return keep_half(h, idx, thresh16);
}
// the 4 consecutive score indices i0 .. i0+3 (one lane's keys 4g..4g+3 of a 16-key block)
__device__ __forceinline__ void attn_keep4(uint64_t seed, uint64_t i0, uint32_t thresh16, bool odd_rows,
                                          bool (&keep)[4]) {
    const uint64_t p0 = i0 >> 1;
    const uint32_t h0 = attn_hash(seed, p0), h1 = attn_hash(seed, p0 + 1);
    const uint32_t h2 = odd_rows ? attn_hash(seed, p0 + 2) : 0u;   // i0 odd only when S is odd
    const int o = (int)(i0 & 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int e = o + r;
        const uint32_t h = (e >> 1) == 0 ? h0 : ((e >> 1) == 1 ? h1 : h2);
        keep[r] = ((h >> ((e & 1) * 16)) & 0xffffu) >= thresh16;
    }
}

// additive key mask of keys k0 + {0..3} (k0 = a lane's first key of a 16-key block),
// one 16-byte load when the whole group is in range and aligned
__device__ __forceinline__ void mask4(const float* mrow, int k0, int S, float (&m)[4]) {
    if (k0 + 3 < S && ((S | k0) & 3) == 0) {
        const float4 v = *reinterpret_cast<const float4*>(mrow + k0);
        m[0] = v.x; m[1] = v.y; m[2] = v.z; m[3] = v.w;
    } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) m[r] = k0 + r < S ? mrow[k0 + r] : 0.f;
    }
}

// Dropout keep-bit layout: word ((bh * NKW + kw) * 4 + g) * S + q, NKW = ceil(S / 128), bit
// 4 * blk + r  <->  key kw * 128 + 16 * blk + 4 * g + r (blk 0..7): the bits one forward lane
// holds (query on the lane, keys 16 blk + 4 g + r in its accumulators) are one word.
__host__ __device__ __forceinline__ int dmask_nkw(int S) { return (S + 127) >> 7; }
__device__ __forceinline__ long dmask_word(int bh, int S, int kw, int g, int q) {
    return ((long)(bh * dmask_nkw(S) + kw) * 4 + g) * S + q;
}
// keep bits of queries q0 .. q0+3 for one key (lane = key): the 4 words of (kw, g) of that key
__device__ __forceinline__ uint4 dmask_words4(const uint32_t* __restrict__ dm, long w0, int q0, int S) {
    if (((S | q0) & 3) == 0 && q0 + 3 < S) return *reinterpret_cast<const uint4*>(dm + w0);
    return make_uint4(q0 < S ? dm[w0] : 0u, q0 + 1 < S ? dm[w0 + 1] : 0u, q0 + 2 < S ? dm[w0 + 2] : 0u,
                      q0 + 3 < S ? dm[w0 + 3] : 0u);
}

// bit `bit` of each of the 4 words, packed into bits 0..3 (one register per 4 queries)
__device__ __forceinline__ uint32_t dmask_pick4(uint4 w, int bit) {
    return ((w.x >> bit) & 1u) | (((w.y >> bit) & 1u) << 1) | (((w.z >> bit) & 1u) << 2) | (((w.w >> bit) & 1u) << 3);
}

__device__ __forceinline__ bf16x8 load_frag_global(const bf16_t* rowp, int kk) {
    const int l = threadIdx.x & 63;
    return *reinterpret_cast<const bf16x8*>(rowp + kk * 32 + 8 * (l >> 4));
}

// ============================================================ forward
// 8 waves (128 queries) per workgroup: each K / V tile is staged once for 128 queries (it was
// once per 64 with 4 waves: half the staging per query); (512, 1) leaves the compiler its
// register budget, LDS allows two workgroups per CU
// MASK / DROP: key-padding mask / probability dropout present (uniform per launch; as run-time
// checks they put ~50 branches into the tile loop: VALU:MFMA 36 in pmc_bert_large.md)
template <bool MASK, bool DROP>
__global__ __launch_bounds__(64 * TWF, 1) void attn_fwd_k(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                                                  bf16_t* __restrict__ out, float* __restrict__ lse, int B, int S, int H,
                                                  float scale, float p_drop, uint64_t seed, uint32_t* __restrict__ dmask) {
    __shared__ __attribute__((aligned(16))) char smem[4 * TK * ROWB];   // K0 V0 K1 V1
    // the tiles' additive key mask (scaled to log2), staged with K / V: an in-loop global load of
    // it made the compiler wait out the K / V prefetch (vmcnt counts every load in order)
    __shared__ __attribute__((aligned(16))) float s_mk[2][TK];
    const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4;
    const long rs = 3L * H * D;                              // qkv row stride
    const bf16_t* qb = qkv + (long)b * S * rs + h * D;
    const bf16_t* kb = qb + H * D;
    const bf16_t* vb = qb + 2 * H * D;
    const int q0 = blockIdx.x * TROWS_F + w * 16;
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
    const uint32_t thresh = drop_thresh16(p_drop);
    const float inv_keep = DROP ? 1.f / (1.f - p_drop) : 1.f;
    const uint64_t rowidx = ((uint64_t)bh * S + myq) * S;     // score index of (myq, key 0)
    const float* mrow = MASK ? mask + (long)b * S : nullptr;

    const int nt = (S + TK - 1) / TK;
    uint32_t kbits = 0;                                      // dropout keep bits of a 128-key word
    Stager<64 * TWF> sk, sv;
    float nmk = 0.f;                                         // raw load; scaled / bounded at the store
    bool mk_ok = false;
    auto load_mk = [&](int t) __attribute__((always_inline)) {
        const int k = t * TK + (int)threadIdx.x;
        mk_ok = k < S;
        if (MASK && threadIdx.x < TK) nmk = mrow[min(k, S - 1)];
    };
    sk.load(kb, rs, 0, S);
    sv.load(vb, rs, 0, S);
    load_mk(0);
    sk.store<false>(smem);
    sv.store<true>(smem + TK * ROWB);
    if (MASK && threadIdx.x < TK) s_mk[0][threadIdx.x] = mk_ok ? nmk * LOG2E : 0.f;
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
        char* sK = smem + (t & 1) * 2 * TK * ROWB;
        char* sV = sK + TK * ROWB;
        const float* sM = s_mk[t & 1];
        const bool more = t + 1 < nt;
        if (more) {
            sk.load(kb, rs, (t + 1) * TK, S);
            sv.load(vb, rs, (t + 1) * TK, S);
            load_mk(t + 1);
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
        const bool tail = (t + 1) * TK > S;          // uniform: keys past S in this tile
#pragma unroll
        for (int blk = 0; blk < 4; ++blk) {
            const int k0 = t * TK + 16 * blk + 4 * g;
            float4 mk4 = make_float4(0.f, 0.f, 0.f, 0.f);
            if (MASK) mk4 = *reinterpret_cast<const float4*>(sM + 16 * blk + 4 * g);
            const float mk[4] = {mk4.x, mk4.y, mk4.z, mk4.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float v = s[blk][r] * c2;
                if (MASK) v += mk[r];
                if (tail && k0 + r >= S) v = -INFINITY;
                s[blk][r] = v;
                tmax = fmaxf(tmax, v);
            }
        }
        tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        const float mnew = fmaxf(m, tmax);
        const float alpha = (m == -INFINITY) ? 0.f : fast_exp2(m - mnew);
        const float msub = mnew == -INFINITY ? 0.f : mnew;
        m = mnew;
        float psum = 0.f;
#pragma unroll
        for (int blk = 0; blk < 4; ++blk) {
            bool keep[4] = {true, true, true, true};
            if (DROP) attn_keep4(seed, rowidx + t * TK + 16 * blk + 4 * g, thresh, S & 1, keep);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float pv = fast_exp2(s[blk][r] - msub);
                psum += pv;
                if (DROP) {
                    pv = keep[r] ? pv * inv_keep : 0.f;
                    kbits |= (uint32_t)keep[r] << ((t & 1) * 16 + 4 * blk + r);
                }
                s[blk][r] = pv;
            }
        }
        if (DROP && ((t & 1) || t == nt - 1)) {      // a 128-key word is complete
            if (qok) dmask[dmask_word(bh, S, t >> 1, g, myq)] = kbits;
            kbits = 0;
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
            if (MASK && threadIdx.x < TK) s_mk[(t + 1) & 1][threadIdx.x] = mk_ok ? nmk * LOG2E : 0.f;
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
// workgroup = 16 TWB keys of one (b, h); wave w owns keys k0 + 16 w .. +15 (key on the lane).
// (256, 3): three waves per SIMD -- the compiler then allocates ~160 VGPRs instead of 176 (two
// waves per SIMD) without spilling; the tiled kernels wait on memory ~45-50 % of wave time,
// which more resident waves hide (same for the dQ kernel below)
template <bool DROP>
__global__ __launch_bounds__(64 * TWB, 3) void attn_bwd_dkv_k(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout,
                                                      const float* __restrict__ lse, const float* __restrict__ delta,
                                                      const float* __restrict__ mask, bf16_t* __restrict__ dqkv, int B,
                                                      int S, int H, float scale, float p_drop,
                                                      const uint32_t* __restrict__ dmask,
                                                      float* __restrict__ colsum) {
    // Q, dO tiles as ONE image each on the transposed-read swizzle, read both as rows (S, dP
    // fragments) and transposed (dK, dV fragments) without bank conflicts (the row swizzle had
    // 23 % conflicted tr reads; a second, transposed copy of each tile doubled the staging)
    __shared__ __attribute__((aligned(16))) char smem[2 * TQ * ROWB];
    __shared__ float s_lse[TQ], s_delta[TQ];
    // this tile's keep words [g][q], rows TQ + 8 words apart (at TQ words = 256 B, the 4 rows a lane
    // group's 16-byte reads hit at one q shared banks: 2-way)
    constexpr int DMT = TQ + 8;
    __shared__ __attribute__((aligned(16))) uint32_t s_dm[4 * DMT];
    const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4;
    const long rs = 3L * H * D;
    const bf16_t* qb = qkv + (long)b * S * rs + h * D;
    const bf16_t* kb = qb + H * D;
    const bf16_t* vb = qb + 2 * H * D;
    const bf16_t* dob = dout + (long)b * S * H * D + h * D;
    const int k0 = blockIdx.x * TROWS_B + w * 16;
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
    const float inv_keep = DROP ? 1.f / (1.f - p_drop) : 1.f;
    // my key's keep bits: word (kw, gk) of each query (staged per tile in s_dm), bit kbit; the
    // workgroup's keys share kw
    static_assert(TROWS_B <= 128 && 128 % TROWS_B == 0, "a workgroup's keys in one 128-key keep word");
    const int kq = kok ? myk : 0;
    const int kw_blk = (blockIdx.x * TROWS_B) >> 7;
    const uint32_t* dmw = s_dm + ((kq >> 2) & 3) * DMT;
    const int kbit = ((kq >> 4) & 7) * 4 + (kq & 3);
    f32x4 dv[4], dk[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { dv[i] = (f32x4){0, 0, 0, 0}; dk[i] = (f32x4){0, 0, 0, 0}; }
    char* sQ = smem;
    char* sO = smem + TQ * ROWB;
    const int nt = (S + TQ - 1) / TQ;
    // tile t+1's Q / dO rows, keep words, LSE and delta are loaded into registers while tile t
    // computes (the single-buffered loop waited out every tile's loads)
    Stager<64 * TWB> a, c;
    uint32_t wd = 0;
    float nlse = 0.f, ndel = 0.f;
    auto fetch = [&](int t) __attribute__((always_inline)) {
        a.load(qb, rs, t * TQ, S);
        c.load(dob, (long)H * D, t * TQ, S);
        const int q = t * TQ + (threadIdx.x & (TQ - 1));
        if (DROP && threadIdx.x < 4 * TQ)   // keep word (g, q) of the tile, one per thread
            wd = q < S ? dmask[dmask_word(bh, S, kw_blk, threadIdx.x >> 6, q)] : 0u;
        if (threadIdx.x < TQ) {
            nlse = q < S ? lse[(long)bh * S + q] : 0.f;
            ndel = q < S ? delta[(long)bh * S + q] : 0.f;
        }
    };
    fetch(0);
    for (int t = 0; t < nt; ++t) {
        __syncthreads();             // previous tile fully consumed
        a.store<true>(sQ);
        c.store<true>(sO);
        if (DROP && threadIdx.x < 4 * TQ) s_dm[(threadIdx.x >> 6) * DMT + (threadIdx.x & (TQ - 1))] = wd;
        if (threadIdx.x < TQ) {
            s_lse[threadIdx.x] = nlse;
            s_delta[threadIdx.x] = ndel;
        }
        __syncthreads();
        if (t + 1 < nt) fetch(t + 1);
        // S[q][k] and dP[q][k]: lane holds q = t*64 + 16 qb + 4 g + r, k = myk
        f32x4 sc[4], dp[4];
#pragma unroll
        for (int qbk = 0; qbk < 4; ++qbk) {
            sc[qbk] = (f32x4){0, 0, 0, 0};
            dp[qbk] = (f32x4){0, 0, 0, 0};
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                sc[qbk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<true>(sQ, 16 * qbk, kk), kf[kk], sc[qbk], 0, 0, 0);
                dp[qbk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<true>(sO, 16 * qbk, kk), vf[kk], dp[qbk], 0, 0, 0);
            }
        }
        f32x4 pd[4], ds[4];
#pragma unroll
        for (int qbk = 0; qbk < 4; ++qbk) {
            const int qa = t * TQ + 16 * qbk + 4 * g;
            const uint32_t kb4 = DROP ? dmask_pick4(*reinterpret_cast<const uint4*>(dmw + (qa - t * TQ)), kbit)
                                              : 0xfu;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ql = 16 * qbk + 4 * g + r;
                const int q = t * TQ + ql;
                float pv = (q < S && kok) ? fast_exp2(sc[qbk][r] * c2 + mbias * LOG2E - s_lse[ql] * LOG2E) : 0.f;
                float dpv = dp[qbk][r];
                float pdrop = pv;
                if (DROP) {
                    const bool keep = (kb4 >> r) & 1u;
                    pdrop = keep ? pv * inv_keep : 0.f;
                    dpv = keep ? dpv * inv_keep : 0.f;
                }
                pd[qbk][r] = pdrop;
                ds[qbk][r] = pv * (dpv - s_delta[ql]);
            }
        }
        // dV^T[d][k] += dO^T[d][q] Pd[q][k];  dK^T[d][k] += Q^T[d][q] dS[q][k]
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            const bf16x8 pf = pack_acc(pd[2 * st], pd[2 * st + 1]);
            const bf16x8 sf = pack_acc(ds[2 * st], ds[2 * st + 1]);
#pragma unroll
            for (int db = 0; db < 4; ++db) {
                dv[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<true>(sO, 32 * st, 16 * db), pf, dv[db], 0, 0, 0);
                dk[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<true>(sQ, 32 * st, 16 * db), sf, dk[db], 0, 0, 0);
            }
        }
    }
    if (colsum) {
        // the QKV bias gradient's share of this wave's 16 keys: column sums of their dK, dV
        // rows, row (b * tiles + tile) * 4 + wave of colsum [B * tiles * 4][3 H D] (keys past S
        // contribute zero).  Per wave, no barrier: a workgroup-wide reduction held every wave
        // until the slowest finished (+10 us per launch at ViT's 6144 workgroups)
        float* crow = colsum + (((long)b * gridDim.x + blockIdx.x) * TWB + w) * rs + h * D + 4 * g;
#pragma unroll
        for (int db = 0; db < 4; ++db) {
            float sk[4], sv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                sk[r] = row16_sum(kok ? dk[db][r] * scale : 0.f);     // over the DPP row = 16 keys
                sv[r] = row16_sum(kok ? dv[db][r] : 0.f);
            }
            if ((lane & 15) == 0) {
                *reinterpret_cast<float4*>(crow + H * D + 16 * db) = make_float4(sk[0], sk[1], sk[2], sk[3]);
                *reinterpret_cast<float4*>(crow + 2 * H * D + 16 * db) = make_float4(sv[0], sv[1], sv[2], sv[3]);
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
// workgroup = 16 TWB queries; wave owns 16 queries (query on the lane), loops over key tiles.
template <bool MASK, bool DROP>
__global__ __launch_bounds__(64 * TWB, 3) void attn_bwd_dq_k(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout,
                                                     const float* __restrict__ lse, const float* __restrict__ delta,
                                                     const float* __restrict__ mask, bf16_t* __restrict__ dqkv, int B,
                                                     int S, int H, float scale, float p_drop,
                                                     const uint32_t* __restrict__ dmask,
                                                     float* __restrict__ colsum) {
    __shared__ __attribute__((aligned(16))) char smem[2 * TK * ROWB];   // K (tr swizzle: read both ways), V tiles
    __shared__ __attribute__((aligned(16))) float s_mk[TK];            // the tile's additive key mask (log2)
    const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4;
    const long rs = 3L * H * D;
    const bf16_t* qb = qkv + (long)b * S * rs + h * D;
    const bf16_t* kb = qb + H * D;
    const bf16_t* vb = qb + 2 * H * D;
    const bf16_t* dob = dout + (long)b * S * H * D + h * D;
    const int myq = blockIdx.x * TROWS_B + w * 16 + (lane & 15);
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
    const float inv_keep = DROP ? 1.f / (1.f - p_drop) : 1.f;
    const float* mrow = MASK ? mask + (long)b * S : nullptr;
    // this query's keep words, one per 128 keys, loaded up front (S <= 512 here: 4 words)
    constexpr int MAXKW = 4;
    uint32_t kwds[MAXKW] = {~0u, ~0u, ~0u, ~0u};
    if (DROP && qok) {
#pragma unroll
        for (int i = 0; i < MAXKW; ++i)
            if (i < dmask_nkw(S)) kwds[i] = dmask[dmask_word(bh, S, i, g, myq)];
    }
    f32x4 dq[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) dq[i] = (f32x4){0, 0, 0, 0};
    char* sK = smem;
    char* sV = smem + TK * ROWB;
    const int nt = (S + TK - 1) / TK;
    // tile t+1's K / V rows (and key mask) are loaded into registers while tile t computes
    Stager<64 * TWB> a, c;
    float nmk = 0.f;                                         // raw load; scaled / bounded at the store
    bool mk_ok = false;
    auto load_mk = [&](int t) __attribute__((always_inline)) {
        const int k = t * TK + (int)threadIdx.x;
        mk_ok = k < S;
        if (MASK && threadIdx.x < TK) nmk = mrow[min(k, S - 1)];
    };
    a.load(kb, rs, 0, S);
    c.load(vb, rs, 0, S);
    load_mk(0);
    for (int t = 0; t < nt; ++t) {
        __syncthreads();
        a.store<true>(sK);
        c.store<false>(sV);
        if (MASK && threadIdx.x < TK) s_mk[threadIdx.x] = mk_ok ? nmk * LOG2E : 0.f;
        __syncthreads();
        if (t + 1 < nt) {
            a.load(kb, rs, (t + 1) * TK, S);
            c.load(vb, rs, (t + 1) * TK, S);
            load_mk(t + 1);
        }
        // S^T[k][q], dP^T[k][q]: lane holds k = t*64 + 16 blk + 4 g + r, q = myq
        f32x4 sc[4], dp[4];
#pragma unroll
        for (int blk = 0; blk < 4; ++blk) {
            sc[blk] = (f32x4){0, 0, 0, 0};
            dp[blk] = (f32x4){0, 0, 0, 0};
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                sc[blk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<true>(sK, 16 * blk, kk), qf[kk], sc[blk], 0, 0, 0);
                dp[blk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<false>(sV, 16 * blk, kk), of[kk], dp[blk], 0, 0, 0);
            }
        }
        f32x4 ds[4];
        const float lse2 = my_lse * LOG2E;
        // the forward's keep bits of my query for this tile's keys (one word per 128 keys)
        uint32_t kbits = ~0u;
        if (DROP && qok) {
            const int kwi = t >> 1;
            const uint32_t wv = kwi < MAXKW ? (kwi == 0 ? kwds[0] : kwi == 1 ? kwds[1] : kwi == 2 ? kwds[2] : kwds[3])
                                            : dmask[dmask_word(bh, S, kwi, g, myq)];
            kbits = wv >> ((t & 1) * 16);
        }
#pragma unroll
        for (int blk = 0; blk < 4; ++blk) {
            const int k0 = t * TK + 16 * blk + 4 * g;
            float4 mk4 = make_float4(0.f, 0.f, 0.f, 0.f);
            if (MASK) mk4 = *reinterpret_cast<const float4*>(s_mk + 16 * blk + 4 * g);
            const float mk[4] = {mk4.x, mk4.y, mk4.z, mk4.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const bool ok = qok && k0 + r < S;
                const float pv = ok ? fast_exp2(sc[blk][r] * c2 + mk[r] - lse2) : 0.f;
                float dpv = dp[blk][r];
                if (DROP) dpv = ((kbits >> (4 * blk + r)) & 1u) ? dpv * inv_keep : 0.f;
                ds[blk][r] = pv * (dpv - my_delta);
            }
        }
        // dQ^T[d][q] += K^T[d][k] dS^T[k][q]
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            const bf16x8 sf = pack_acc(ds[2 * st], ds[2 * st + 1]);
#pragma unroll
            for (int db = 0; db < 4; ++db)
                dq[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<true>(sK, 32 * st, 16 * db), sf, dq[db], 0, 0, 0);
        }
    }
    if (colsum) {
        // column sums of this wave's 16 dQ rows (the same colsum row as the dKV kernel's wave
        // over these positions' keys)
        float* crow = colsum + (((long)b * gridDim.x + blockIdx.x) * TWB + w) * rs + h * D + 4 * g;
#pragma unroll
        for (int db = 0; db < 4; ++db) {
            float sq[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) sq[r] = row16_sum(qok ? dq[db][r] * scale : 0.f);
            if ((lane & 15) == 0)
                *reinterpret_cast<float4*>(crow + 16 * db) = make_float4(sq[0], sq[1], sq[2], sq[3]);
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


// ============================================================ forward, S <= 128
// One workgroup (8 waves) per (b, h): K and V of the whole sequence staged into LDS once
// (the tiled forward stages them once per 64-query workgroup), wave w owns queries
// 16w..16w+15 with every key's score in registers, so the softmax needs no online
// rescaling: one max, one exponential per score, one sum.
// FULL: S == 128 (every score block valid: no per-block branches, so the compiler can
// interleave one block's fragment reads with the previous block's MFMAs); MASK / DROP:
// key-padding mask / probability dropout present (uniform per launch)
template <bool FULL, bool MASK, bool DROP>
__global__ __launch_bounds__(512, 2) void attn_fwd_short_k(const bf16_t* __restrict__ qkv,
                                                            const float* __restrict__ mask, bf16_t* __restrict__ out,
                                                            float* __restrict__ lse, int S, int H, float scale,
                                                            float p_drop, uint64_t seed, int BH,
                                                            uint32_t* __restrict__ dmask) {
    // persistent: a workgroup walks (b, h) = blockIdx.x, + gridDim.x, ...; the next pair's K / V rows,
    // mask entry and Q fragments are loaded into registers while the current pair computes, and
    // staged into the other half of the double-buffered LDS images (the single-pair version
    // waited out every pair's loads: ~40 % of its wave time)
    // per buffer: K (row image), V (transposed-read image), the key-padding mask row (fp32)
    constexpr int BUF = 2 * FS * ROWB + FS * 4;
    __shared__ __attribute__((aligned(16))) char smem_all[2 * BUF];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
    const long rs = 3L * H * D;
    const int myq = 16 * w + (lane & 15);
    const bool qok = myq < S;
    // next pair, in registers (plain arrays: a struct copy went through scratch)
    uint4 nk4[2], nv4[2];
    float nm = 0.f;
    bf16x8 nq[2], qf[2];
    auto fetch = [&](int bhp) __attribute__((always_inline)) {
        const int bp = bhp / H, hp = bhp - bp * H;
        const bf16_t* qb = qkv + (long)bp * S * rs + hp * D;
        const bf16_t* kb = qb + H * D;
        const bf16_t* vb = qb + 2 * H * D;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int r = (tid >> 3) + 64 * i, c = tid & 7;
            const int rr = r < S ? r : 0;
            nk4[i] = *reinterpret_cast<const uint4*>(kb + (long)rr * rs + c * 8);
            nv4[i] = *reinterpret_cast<const uint4*>(vb + (long)rr * rs + c * 8);
        }
        if (MASK) nm = tid < FS ? mask[(long)bp * S + (tid < S ? tid : 0)] : 0.f;
        const bf16_t* qr = qb + (long)(qok ? myq : 0) * rs;
        nq[0] = load_frag_global(qr, 0);
        nq[1] = load_frag_global(qr, 1);
    };
    auto stage = [&](char* smem) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int r = (tid >> 3) + 64 * i, c = tid & 7;
            const bool ok = r < S;
            *reinterpret_cast<uint4*>(smem + lds_off<false>(r, c)) = zero_unless(ok, nk4[i]);
            *reinterpret_cast<uint4*>(smem + FS * ROWB + lds_off<true>(r, c)) = zero_unless(ok, nv4[i]);
        }
        if (MASK && tid < FS) reinterpret_cast<float*>(smem + 2 * FS * ROWB)[tid] = tid < S ? nm : 0.f;
        qf[0] = nq[0];
        qf[1] = nq[1];
    };
    int bh = blockIdx.x;
    if (bh >= BH) return;
    fetch(bh);
    stage(smem_all);
    __syncthreads();
    for (int it = 0; bh < BH; ++it, bh += gridDim.x) {
    const int nbh = bh + gridDim.x;
    if (nbh < BH) fetch(nbh);
    char* smem = smem_all + (it & 1) * BUF;
    const int b = bh / H, h = bh - b * H;
    char* sK = smem;
    char* sV = smem + FS * ROWB;
    const float c2 = scale * LOG2E;
    float* sM = reinterpret_cast<float*>(smem + 2 * FS * ROWB);
    const int nblk = FULL ? 8 : (S + 15) / 16;
    // S^T blocks: lane holds s[blk][r] = score(q = myq, k = 16 blk + 4 g + r)
    f32x4 s[8];
    float mx = -INFINITY;
    // all QK^T MFMAs first (fragment reads only), then the scale / mask / max pass: the
    // softmax math no longer waits on each block's MFMA result in turn
#pragma unroll
    for (int blk = 0; blk < 8; ++blk) {
        s[blk] = (f32x4){0.f, 0.f, 0.f, 0.f};
        if (blk < nblk) {
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
                s[blk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<false>(sK, 16 * blk, kk), qf[kk], s[blk], 0, 0, 0);
        }
    }
#pragma unroll
    for (int blk = 0; blk < 8; ++blk) {
        const int k0 = 16 * blk + 4 * g;
        float4 mk = make_float4(0.f, 0.f, 0.f, 0.f);
        if (MASK) mk = *reinterpret_cast<const float4*>(sM + k0);
        const float mka[4] = {mk.x, mk.y, mk.z, mk.w};
        const bool edge = !FULL && 16 * blk + 16 > S;   // uniform: this block reaches past S
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v = MASK ? s[blk][r] * c2 + mka[r] * LOG2E : s[blk][r] * c2;
            if (edge && k0 + r >= S) v = -INFINITY;
            s[blk][r] = v;
            mx = fmaxf(mx, v);
        }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float msub = mx == -INFINITY ? 0.f : mx;
    const uint32_t thresh = drop_thresh16(p_drop);
    const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    const uint64_t rowidx = ((uint64_t)bh * S + myq) * S;
    float lsum = 0.f;
    uint32_t kbits = 0;
#pragma unroll
    for (int blk = 0; blk < 8; ++blk) {
        bool keep[4] = {true, true, true, true};
        if (DROP && blk < nblk) attn_keep4(seed, rowidx + 16 * blk + 4 * g, thresh, !FULL && (S & 1), keep);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float pv = fast_exp2(s[blk][r] - msub);
            lsum += pv;
            if (DROP) {
                pv = keep[r] ? pv * inv_keep : 0.f;
                kbits |= (uint32_t)keep[r] << (4 * blk + r);
            }
            s[blk][r] = pv;
        }
    }
    if (DROP && qok) dmask[dmask_word(bh, S, 0, g, myq)] = kbits;   // for the backward
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    // O^T[d][q] = V^T[d][k] P^T[k][q]
    f32x4 o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < 4; ++st) {
        if (2 * st >= nblk) break;
        const bf16x8 pf = pack_acc(s[2 * st], s[2 * st + 1]);
#pragma unroll
        for (int db = 0; db < 4; ++db)
            o[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<true>(sV, 32 * st, 16 * db), pf, o[db], 0, 0, 0);
    }
    if (qok) {
        const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
        bf16_t* orow = out + ((long)b * S + myq) * H * D + h * D;
#pragma unroll
        for (int db = 0; db < 4; ++db) {
            float v[4] = {o[db][0] * inv, o[db][1] * inv, o[db][2] * inv, o[db][3] * inv};
            store4(orow + 16 * db + 4 * g, v);
        }
        if (g == 0) lse[(long)bh * S + myq] = (mx + log2f(lsum)) / LOG2E;
    }
    // the next pair into the other buffer (last read by the previous pair, before the barrier
    // that ended it); the barrier below publishes it
    if (nbh < BH) stage(smem_all + ((it + 1) & 1) * BUF);
    __syncthreads();
    }
}

// ============================================================ fused backward, S <= 128
// One workgroup (8 waves) per (b, h) holds the whole sequence: Q, K and dO are staged
// into LDS once, delta = rowsum(dO * O) is computed in the prologue, and
//   phase 1 (lane = key, wave w owns keys 16w..16w+15): S, dP over all 128 queries in
//           chunks of 32, P (saved LSE), dropout, dS -> dV, dK complete in registers; the
//           lane's dS column stays in registers (bf16) until every wave is done with Q and
//           dO, then goes to LDS as two [128 keys][64 queries] dS^T row images over them
//           (48 KB of LDS: two workgroups per CU);
//   phase 2 (lane = query, wave w owns queries 16w..16w+15): dQ = dS K from the dS^T
//           images and K, both read transposed.
// Every input byte is read once and nothing is recomputed (the two-kernel path re-derives
// P and dP in both its dK/dV and its dQ kernel and reads Q/K/V/dO once per tile pair).
// FULL: S == 128 (the query / key chunk loops unroll, no bounds checks); DROP: dropout on
template <bool FULL, bool DROP>
__global__ __launch_bounds__(512, 4) void attn_bwd_fused_k(const bf16_t* __restrict__ qkv,
                                                            const bf16_t* __restrict__ out,
                                                            const bf16_t* __restrict__ dout,
                                                            const float* __restrict__ lse,
                                                            const float* __restrict__ mask, bf16_t* __restrict__ dqkv,
                                                            int S, int H, float scale, float p_drop,
                                                            const uint32_t* __restrict__ dmask,
                                                            float* __restrict__ colsum) {
    __shared__ __attribute__((aligned(16))) char smem[3 * FS * ROWB];   // Q, K, dO; then dS^T halves over Q, dO
    // colsum (nullable, [B][3 H D] fp32): this (b, h)'s column sums of dQ / dK / dV over the sequence --
    // the QKV Linear's bias gradient without another pass over dQKV: per-wave sums, then over waves
    __shared__ float s_cs[8][3][D];
    __shared__ __attribute__((aligned(16))) float s_lse[FS];
    __shared__ __attribute__((aligned(16))) float s_delta[FS];
    __shared__ float s_mask[FS];
    // keep-bit words [g][q], rows DMS words apart: a lane group's 16-byte reads hit 4 rows at one q,
    // and at FS words (2 x 256 B) apart those rows shared banks (2-way)
    constexpr int DMS = FS + 8;
    __shared__ __attribute__((aligned(16))) uint32_t s_dm[DROP ? 4 * DMS : 4];
    const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
    const long rs = 3L * H * D;
    const long ors = (long)H * D;
    const bf16_t* qb = qkv + (long)b * S * rs + h * D;
    const bf16_t* kb = qb + H * D;
    const bf16_t* vb = qb + 2 * H * D;
    const bf16_t* dob = dout + (long)b * S * ors + h * D;
    const bf16_t* ob = out + (long)b * S * ors + h * D;
    char* sQ = smem;
    char* sK = sQ + FS * ROWB;
    char* sO = sK + FS * ROWB;
    char* sT0 = sQ;                 // dS^T[:, 0:64]   (after phase 1)
    char* sT1 = sO;                 // dS^T[:, 64:128] (after phase 1)
    uint2 dsk[8];                   // this lane's dS column, bf16, blocks of 4 queries (qc, j)

    // ---- prologue: Q, K, dO row images (rows >= S are zeros), delta, scaled LSE, mask
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = (tid >> 3) + 64 * i, c = tid & 7;
        const bool ok = r < S;
        const int rr = ok ? r : 0;
        const uint4 q4 = *reinterpret_cast<const uint4*>(qb + (long)rr * rs + c * 8);
        const uint4 k4 = *reinterpret_cast<const uint4*>(kb + (long)rr * rs + c * 8);
        const uint4 o4 = *reinterpret_cast<const uint4*>(dob + (long)rr * ors + c * 8);
        *reinterpret_cast<uint4*>(sQ + lds_off<true>(r, c)) = zero_unless(ok, q4);
        *reinterpret_cast<uint4*>(sK + lds_off<true>(r, c)) = zero_unless(ok, k4);
        *reinterpret_cast<uint4*>(sO + lds_off<true>(r, c)) = zero_unless(ok, o4);
    }
    {
        // delta[q] = sum_d dO[q][d] O[q][d]: 4 threads per query, 16 d each
        const int q = tid >> 2, part = tid & 3;
        float a = 0.f;
        if (q < S) {
            float x[8], y[8];
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                load8(dob + (long)q * ors + part * 16 + hh * 8, x);
                load8(ob + (long)q * ors + part * 16 + hh * 8, y);
#pragma unroll
                for (int j = 0; j < 8; ++j) a += x[j] * y[j];
            }
        }
        a += __shfl_xor(a, 1);
        a += __shfl_xor(a, 2);
        if (part == 0) s_delta[q] = a;
    }
    if (tid < FS) {
        s_lse[tid] = tid < S ? lse[(long)bh * S + tid] * LOG2E : 0.f;
        s_mask[tid] = (mask && tid < S) ? mask[(long)b * S + tid] * LOG2E : 0.f;
    }
    if (DROP) {   // the forward's dropout keep bits of this (b, h): word (g, q), one per thread
        const int gq = tid >> 7, q = tid & (FS - 1);
        s_dm[gq * DMS + q] = q < S ? dmask[dmask_word(bh, S, 0, gq, q)] : 0u;
    }
    __syncthreads();

    const float c2 = scale * LOG2E;
    const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;

    // ---- phase 1: lane = key
    {
        const int myk = 16 * w + (lane & 15);
        const bool kok = myk < S;
        bf16x8 kf[2], vf[2];
        const bf16_t* vr = vb + (long)(kok ? myk : 0) * rs;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            kf[kk] = frag_rows<true>(sK, 16 * w, kk);   // B operand: my key's row, d = 32kk + 8g ..
            vf[kk] = load_frag_global(vr, kk);
        }
        const float mb2 = s_mask[kok ? myk : 0];
        // my key's dropout keep bits: LDS words (gk, q), bit kbit
        const int kq = kok ? myk : 0;
        const uint32_t* dmw = s_dm + (DROP ? ((kq >> 2) & 3) * DMS : 0);
        const int kbit = (kq >> 4) * 4 + (kq & 3);
        f32x4 dv[4], dk[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) { dv[i] = (f32x4){0, 0, 0, 0}; dk[i] = (f32x4){0, 0, 0, 0}; }
        const int nqc = FULL ? 4 : (S + 31) / 32;
#pragma unroll
        for (int qc = 0; qc < 4; ++qc) {
            if (!FULL && qc >= nqc) break;
            f32x4 sc[2], dp[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                sc[j] = (f32x4){0, 0, 0, 0};
                dp[j] = (f32x4){0, 0, 0, 0};
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) {
                    sc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<true>(sQ, 32 * qc + 16 * j, kk), kf[kk],
                                                                    sc[j], 0, 0, 0);
                    dp[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<true>(sO, 32 * qc + 16 * j, kk), vf[kk],
                                                                    dp[j], 0, 0, 0);
                }
            }
            f32x4 pd[2], ds[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int q0 = 32 * qc + 16 * j + 4 * g;
                const f32x4 lse4 = *reinterpret_cast<const f32x4*>(s_lse + q0);     // one LDS read per 4 queries
                const f32x4 del4 = *reinterpret_cast<const f32x4*>(s_delta + q0);
                // queries q0 .. q0+3: their keep bits for my key, packed into bits 0..3
                const uint32_t kb4 = DROP ? dmask_pick4(*reinterpret_cast<const uint4*>(dmw + q0), kbit) : 0xfu;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int ql = q0 + r;
                    const float pv = (FULL || (ql < S && kok)) ? fast_exp2(sc[j][r] * c2 + (mb2 - lse4[r])) : 0.f;
                    float dpv = dp[j][r];
                    float pdrop = pv;
                    if (DROP) {
                        const bool keep = (kb4 >> r) & 1u;
                        pdrop = keep ? pv * inv_keep : 0.f;
                        dpv = keep ? dpv * inv_keep : 0.f;
                    }
                    pd[j][r] = pdrop;
                    ds[j][r] = pv * (dpv - del4[r]);
                }
                // dS^T row myk, query columns 32qc + 16j + 4g .. +3 (written after phase 1)
                dsk[2 * qc + j] = make_uint2(pack2bf(ds[j][0], ds[j][1]), pack2bf(ds[j][2], ds[j][3]));
            }
            // dV^T[d][k] += dO^T[d][q] Pd[q][k];  dK^T[d][k] += Q^T[d][q] dS[q][k]
            const bf16x8 pf = pack_acc(pd[0], pd[1]);
            const bf16x8 sf = pack_acc(ds[0], ds[1]);
#pragma unroll
            for (int db = 0; db < 4; ++db) {
                dv[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<true>(sO, 32 * qc, 16 * db), pf, dv[db], 0, 0, 0);
                dk[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<true>(sQ, 32 * qc, 16 * db), sf, dk[db], 0, 0, 0);
            }
        }
        // query chunks past S: their dS^T columns read as zeros in phase 2
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (c >= nqc) dsk[2 * c] = dsk[2 * c + 1] = make_uint2(0u, 0u);
        if (kok) {
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
        if (colsum) {   // keys past S hold zero gradients
#pragma unroll
            for (int db = 0; db < 4; ++db)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float sk = row16_sum(dk[db][e] * scale), sv = row16_sum(dv[db][e]);
                    if ((lane & 15) == 0) {
                        s_cs[w][1][16 * db + 4 * g + e] = sk;
                        s_cs[w][2][16 * db + 4 * g + e] = sv;
                    }
                }
        }
    }
    __syncthreads();               // every wave is done with the Q and dO images
    {
        const int myk = 16 * w + (lane & 15);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int q0 = 16 * c + 4 * g;             // block c = (qc, j) = (c / 2, c % 2)
            char* img = q0 < 64 ? sT0 : sT1;
            const int qq = q0 & 63;
            *reinterpret_cast<uint2*>(img + lds_off<true, true>(myk, qq >> 3) + ds_half(myk, (qq >> 2) & 1)) = dsk[c];
        }
    }
    __syncthreads();

    // ---- phase 2: lane = query; dQ^T[d][q] = K^T[d][k] dS^T[k][q] over all keys
    {
        const int myq = 16 * w + (lane & 15);
        const char* img = w < 4 ? sT0 : sT1;
        const int cb = (16 * w) & 63;
        f32x4 dq[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) dq[i] = (f32x4){0, 0, 0, 0};
        const int nkc = FULL ? 4 : (S + 31) / 32;
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            if (!FULL && st >= nkc) break;
            const bf16x8 sf = frag_tr<true, true>(img, 32 * st, cb);
#pragma unroll
            for (int db = 0; db < 4; ++db)
                dq[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<true>(sK, 32 * st, 16 * db), sf, dq[db], 0, 0, 0);
        }
        if (myq < S) {
            bf16_t* dqr = dqkv + ((long)b * S + myq) * rs + h * D;
#pragma unroll
            for (int db = 0; db < 4; ++db) {
                float a4[4] = {dq[db][0] * scale, dq[db][1] * scale, dq[db][2] * scale, dq[db][3] * scale};
                store4(dqr + 16 * db + 4 * g, a4);
            }
        }
        if (colsum) {   // queries past S hold zero gradients
#pragma unroll
            for (int db = 0; db < 4; ++db)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float sq = row16_sum(dq[db][e] * scale);
                    if ((lane & 15) == 0) s_cs[w][0][16 * db + 4 * g + e] = sq;
                }
        }
    }
    if (colsum) {
        __syncthreads();
        if (tid < 3 * D) {
            const int part = tid / D, d = tid - part * D;
            float acc = 0.f;
#pragma unroll
            for (int ww = 0; ww < 8; ++ww) acc += s_cs[ww][part][d];
            colsum[(long)b * 3 * H * D + part * H * D + h * D + d] = acc;
        }
    }
}

// ============================================================ forward, 128 < S <= 256
// ViT-B/16 (S = 197) and BERT at seq 256: one workgroup (8 waves) per (b, h) with K and V of
// the whole sequence in LDS (64 KB: two workgroups per CU, so one stages while the other
// computes); wave w owns query blocks w and w + 8, each with all 16 key blocks' scores in
// registers (64 accumulator VGPRs), so the softmax is exact in one pass as in the S <= 128
// kernel.  The tiled forward re-staged K / V once per 64 queries and rescaled its running
// output per 64-key tile.  Both query blocks' Q fragments are loaded in the prologue, under
// the K / V staging.
constexpr int FM = 256;        // longest sequence of the medium kernels

template <bool MASK, bool DROP>
__global__ __launch_bounds__(512, 2) void attn_fwd_med_k(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                                                          bf16_t* __restrict__ out, float* __restrict__ lse, int S, int H,
                                                          float scale, float p_drop, uint64_t seed,
                                                          uint32_t* __restrict__ dmask) {
    __shared__ __attribute__((aligned(16))) char smem[2 * FM * ROWB + FM * 4];   // K rows, V^T image, mask
    const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
    const long rs = 3L * H * D;
    const bf16_t* qb = qkv + (long)b * S * rs + h * D;
    const bf16_t* kb = qb + H * D;
    const bf16_t* vb = qb + 2 * H * D;
    char* sK = smem;
    char* sV = smem + FM * ROWB;
    float* sM = reinterpret_cast<float*>(smem + 2 * FM * ROWB);
    const int nblk = (S + 15) >> 4;          // key blocks = query blocks (> 8: S > 128)
    uint4 k4[4], v4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = (tid >> 3) + 64 * i, c = tid & 7;
        const int rr = r < S ? r : 0;
        k4[i] = *reinterpret_cast<const uint4*>(kb + (long)rr * rs + c * 8);
        v4[i] = *reinterpret_cast<const uint4*>(vb + (long)rr * rs + c * 8);
    }
    float nm = 0.f;
    if (MASK && tid < FM) nm = tid < S ? mask[(long)b * S + tid] : 0.f;
    bf16x8 qf[2][2];
#pragma unroll
    for (int qi = 0; qi < 2; ++qi) {
        const int q = 16 * (w + 8 * qi) + (lane & 15);
        const bf16_t* qr = qb + (long)(q < S ? q : 0) * rs;
        qf[qi][0] = load_frag_global(qr, 0);
        qf[qi][1] = load_frag_global(qr, 1);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = (tid >> 3) + 64 * i, c = tid & 7;
        const bool ok = r < S;
        *reinterpret_cast<uint4*>(sK + lds_off<false>(r, c)) = zero_unless(ok, k4[i]);
        *reinterpret_cast<uint4*>(sV + lds_off<true>(r, c)) = zero_unless(ok, v4[i]);
    }
    if (MASK && tid < FM) sM[tid] = nm * LOG2E;
    __syncthreads();
    const float c2 = scale * LOG2E;
    const uint32_t thresh = drop_thresh16(p_drop);
    const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
#pragma unroll
    for (int qi = 0; qi < 2; ++qi) {
        const int qblk = w + 8 * qi;
        if (qblk < nblk) {                       // uniform per wave
        const int myq = 16 * qblk + (lane & 15);
        const bool qok = myq < S;
        // S^T blocks: lane holds s[blk][r] = score(q = myq, k = 16 blk + 4 g + r); blocks past
        // the last key block stay 0 and are never exponentiated (P = 0 there)
        f32x4 s[16];
#pragma unroll
        for (int blk = 0; blk < 16; ++blk) {
            s[blk] = (f32x4){0.f, 0.f, 0.f, 0.f};
            if (blk < nblk) {
#pragma unroll
                for (int kk = 0; kk < 2; ++kk)
                    s[blk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<false>(sK, 16 * blk, kk), qf[qi][kk],
                                                                      s[blk], 0, 0, 0);
            }
        }
        float mx = -INFINITY;
#pragma unroll
        for (int blk = 0; blk < 16; ++blk) {
            if (blk >= nblk) continue;
            const int k0 = 16 * blk + 4 * g;
            float4 mk = make_float4(0.f, 0.f, 0.f, 0.f);
            if (MASK) mk = *reinterpret_cast<const float4*>(sM + k0);
            const float mka[4] = {mk.x, mk.y, mk.z, mk.w};
            const bool edge = 16 * blk + 16 > S;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float v = MASK ? s[blk][r] * c2 + mka[r] : s[blk][r] * c2;
                if (edge && k0 + r >= S) v = -INFINITY;
                s[blk][r] = v;
                mx = fmaxf(mx, v);
            }
        }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float msub = mx == -INFINITY ? 0.f : mx;
        const uint64_t rowidx = ((uint64_t)bh * S + myq) * S;
        float lsum = 0.f;
        uint32_t kbits[2] = {0u, 0u};            // keep bits of keys 0..127 / 128..255
#pragma unroll
        for (int blk = 0; blk < 16; ++blk) {
            if (blk >= nblk) continue;
            bool keep[4] = {true, true, true, true};
            if (DROP) attn_keep4(seed, rowidx + 16 * blk + 4 * g, thresh, S & 1, keep);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float pv = fast_exp2(s[blk][r] - msub);
                lsum += pv;
                if (DROP) {
                    pv = keep[r] ? pv * inv_keep : 0.f;
                    kbits[blk >> 3] |= (uint32_t)keep[r] << (4 * (blk & 7) + r);
                }
                s[blk][r] = pv;
            }
        }
        if (DROP && qok) {
            dmask[dmask_word(bh, S, 0, g, myq)] = kbits[0];
            dmask[dmask_word(bh, S, 1, g, myq)] = kbits[1];
        }
        lsum += __shfl_xor(lsum, 16, 64);
        lsum += __shfl_xor(lsum, 32, 64);
        // O^T[d][q] = V^T[d][k] P^T[k][q], 32 keys per step
        f32x4 o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int st = 0; st < 8; ++st) {
            if (2 * st >= nblk) continue;
            const bf16x8 pf = pack_acc(s[2 * st], s[2 * st + 1]);
#pragma unroll
            for (int db = 0; db < 4; ++db)
                o[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<true>(sV, 32 * st, 16 * db), pf, o[db], 0, 0, 0);
        }
        if (qok) {
            const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
            bf16_t* orow = out + ((long)b * S + myq) * H * D + h * D;
#pragma unroll
            for (int db = 0; db < 4; ++db) {
                float v[4] = {o[db][0] * inv, o[db][1] * inv, o[db][2] * inv, o[db][3] * inv};
                store4(orow + 16 * db + 4 * g, v);
            }
            if (g == 0) lse[(long)bh * S + myq] = (mx + log2f(lsum)) / LOG2E;
        }
        }
    }
}

// ============================================================ fused backward, 128 < S <= 256
// The S <= 128 fused backward scaled to 256 rows, with 16 waves (1024 threads: four per SIMD
// to cover the LDS and MFMA latencies of the one workgroup a CU holds): Q, K, dO row images
// (96 KB), delta / LSE / mask / dropout words in LDS, then
//   phase 1 (lane = key): wave w owns key block w -- S, dP over all queries in 32-query
//           chunks, P, dS -> dK, dV complete in registers and stored; the lane's dS column
//           stays in registers as bf16 (32 VGPRs);
//   phase 2 (lane = query), in two halves of 128 queries: the half's dS^T columns go to LDS as
//           two [256 keys][64 queries] row images over the Q and dO images (64 KB), then
//           dQ = dS K, wave w computing query block (w & 7) of the half, head dims
//           32 (w >> 3) .. +31.
// Replaces the delta pass + dK/dV kernel + dQ kernel of the tiled path, which re-derived P and
// dP in both kernels and re-read Q / K / V / dO once per 64 x 64 tile pair.
constexpr int MW = 16;         // waves per workgroup of the medium backward

template <bool DROP>
__global__ __launch_bounds__(64 * MW, 1) void attn_bwd_med_k(const bf16_t* __restrict__ qkv,
                                                              const bf16_t* __restrict__ out,
                                                              const bf16_t* __restrict__ dout,
                                                              const float* __restrict__ lse,
                                                              const float* __restrict__ mask, bf16_t* __restrict__ dqkv,
                                                              int S, int H, float scale, float p_drop,
                                                              const uint32_t* __restrict__ dmask,
                                                              float* __restrict__ colsum) {
    // one LDS object, carved by hand: Q, K, dO images | col sums [MW][3][D] | LSE | delta | mask | keep words
    constexpr int NT = 64 * MW;
    constexpr int IMG = FM * ROWB;
    constexpr int OFF_CS = 3 * IMG;
    constexpr int OFF_LSE = OFF_CS + MW * 3 * D * 4;
    constexpr int OFF_DEL = OFF_LSE + FM * 4;
    constexpr int OFF_MSK = OFF_DEL + FM * 4;
    constexpr int OFF_DM = OFF_MSK + FM * 4;
    constexpr int DMM = FM + 8;     // keep-word row stride (see attn_bwd_fused_k's DMS)
    __shared__ __attribute__((aligned(16))) char smem[OFF_DM + (DROP ? 2 * 4 * DMM * 4 : 16)];
    float* s_cs = reinterpret_cast<float*>(smem + OFF_CS);     // [w][part][d]
    float* s_lse = reinterpret_cast<float*>(smem + OFF_LSE);
    float* s_delta = reinterpret_cast<float*>(smem + OFF_DEL);
    float* s_mask = reinterpret_cast<float*>(smem + OFF_MSK);
    uint32_t* s_dm = reinterpret_cast<uint32_t*>(smem + OFF_DM);   // keep-bit words [kw][g][q]
    const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
    const long rs = 3L * H * D;
    const long ors = (long)H * D;
    const bf16_t* qb = qkv + (long)b * S * rs + h * D;
    const bf16_t* kb = qb + H * D;
    const bf16_t* vb = qb + 2 * H * D;
    const bf16_t* dob = dout + (long)b * S * ors + h * D;
    const bf16_t* ob = out + (long)b * S * ors + h * D;
    char* sQ = smem;
    char* sK = sQ + IMG;
    char* sO = sK + IMG;
    char* sT0 = sQ;                 // dS^T[:, half + 0:64]   (phase 2)
    char* sT1 = sO;                 // dS^T[:, half + 64:128] (phase 2)
    const int nblk = (S + 15) >> 4;
    const int nch = (S + 31) >> 5;  // 32-row chunks
    const int myk = 16 * w + (lane & 15);
    const bool kok = myk < S;

    // ---- prologue: my key block's V fragments (B operand of dP^T), then the row images
    bf16x8 vf[2];
    {
        const bf16_t* vr = vb + (long)(kok ? myk : 0) * rs;
        vf[0] = load_frag_global(vr, 0);
        vf[1] = load_frag_global(vr, 1);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = (tid >> 3) + (NT / 8) * i, c = tid & 7;
        const bool ok = r < S;
        const int rr = ok ? r : 0;
        const uint4 q4 = *reinterpret_cast<const uint4*>(qb + (long)rr * rs + c * 8);
        const uint4 k4 = *reinterpret_cast<const uint4*>(kb + (long)rr * rs + c * 8);
        const uint4 o4 = *reinterpret_cast<const uint4*>(dob + (long)rr * ors + c * 8);
        *reinterpret_cast<uint4*>(sQ + lds_off<true>(r, c)) = zero_unless(ok, q4);
        *reinterpret_cast<uint4*>(sK + lds_off<true>(r, c)) = zero_unless(ok, k4);
        *reinterpret_cast<uint4*>(sO + lds_off<true>(r, c)) = zero_unless(ok, o4);
    }
    {
        // delta[q] = sum_d dO[q][d] O[q][d]: 4 threads per query, 16 d each
        const int q = tid >> 2, part = tid & 3;
        float a = 0.f;
        if (q < S) {
            float x[8], y[8];
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                load8(dob + (long)q * ors + part * 16 + hh * 8, x);
                load8(ob + (long)q * ors + part * 16 + hh * 8, y);
#pragma unroll
                for (int e = 0; e < 8; ++e) a += x[e] * y[e];
            }
        }
        a += __shfl_xor(a, 1);
        a += __shfl_xor(a, 2);
        if (part == 0) s_delta[q] = a;
    }
    if (tid < FM) {
        s_lse[tid] = tid < S ? lse[(long)bh * S + tid] * LOG2E : 0.f;
        s_mask[tid] = (mask && tid < S) ? mask[(long)b * S + tid] * LOG2E : 0.f;
    }
    if (DROP) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int idx = tid + NT * i, kw = idx >> 10, gq = (idx >> 8) & 3, q = idx & (FM - 1);
            s_dm[(kw * 4 + gq) * DMM + q] = q < S ? dmask[dmask_word(bh, S, kw, gq, q)] : 0u;
        }
    }
    __syncthreads();

    const float c2 = scale * LOG2E;
    const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    uint2 dsk[16];                  // my key's dS column, bf16, blocks of 4 queries per query block
#pragma unroll
    for (int c = 0; c < 16; ++c) dsk[c] = make_uint2(0u, 0u);

    // ---- phase 1: lane = key
    if (w < nblk) {                 // uniform per wave
        bf16x8 kf[2];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) kf[kk] = frag_rows<true>(sK, 16 * w, kk);
        const float mb2 = s_mask[kok ? myk : 0];
        const int kq = kok ? myk : 0;
        const uint32_t* dmw = s_dm + (DROP ? ((kq >> 7) * 4 + ((kq >> 2) & 3)) * DMM : 0);
        const int kbit = ((kq >> 4) & 7) * 4 + (kq & 3);
        f32x4 dv[4], dk[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) { dv[i] = (f32x4){0, 0, 0, 0}; dk[i] = (f32x4){0, 0, 0, 0}; }
#pragma unroll
        for (int qc = 0; qc < 8; ++qc) {
            if (qc < nch) {
                f32x4 sc[2], dp[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    sc[j] = (f32x4){0, 0, 0, 0};
                    dp[j] = (f32x4){0, 0, 0, 0};
#pragma unroll
                    for (int kk = 0; kk < 2; ++kk) {
                        sc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<true>(sQ, 32 * qc + 16 * j, kk),
                                                                        kf[kk], sc[j], 0, 0, 0);
                        dp[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<true>(sO, 32 * qc + 16 * j, kk),
                                                                        vf[kk], dp[j], 0, 0, 0);
                    }
                }
                f32x4 pd[2], ds[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int q0 = 32 * qc + 16 * j + 4 * g;
                    const f32x4 lse4 = *reinterpret_cast<const f32x4*>(s_lse + q0);
                    const f32x4 del4 = *reinterpret_cast<const f32x4*>(s_delta + q0);
                    const uint32_t kb4 = DROP ? dmask_pick4(*reinterpret_cast<const uint4*>(dmw + q0), kbit) : 0xfu;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int ql = q0 + r;
                        const float pv = (ql < S && kok) ? fast_exp2(sc[j][r] * c2 + (mb2 - lse4[r])) : 0.f;
                        float dpv = dp[j][r];
                        float pdrop = pv;
                        if (DROP) {
                            const bool keep = (kb4 >> r) & 1u;
                            pdrop = keep ? pv * inv_keep : 0.f;
                            dpv = keep ? dpv * inv_keep : 0.f;
                        }
                        pd[j][r] = pdrop;
                        ds[j][r] = pv * (dpv - del4[r]);
                    }
                    dsk[2 * qc + j] = make_uint2(pack2bf(ds[j][0], ds[j][1]), pack2bf(ds[j][2], ds[j][3]));
                }
                const bf16x8 pf = pack_acc(pd[0], pd[1]);
                const bf16x8 sf = pack_acc(ds[0], ds[1]);
#pragma unroll
                for (int db = 0; db < 4; ++db) {
                    dv[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<true>(sO, 32 * qc, 16 * db), pf, dv[db],
                                                                     0, 0, 0);
                    dk[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<true>(sQ, 32 * qc, 16 * db), sf, dk[db],
                                                                     0, 0, 0);
                }
            }
        }
        if (kok) {
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
        if (colsum) {   // keys past S hold zero gradients
#pragma unroll
            for (int db = 0; db < 4; ++db)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float sk = row16_sum(dk[db][e] * scale), sv = row16_sum(dv[db][e]);
                    if ((lane & 15) == 0) {
                        s_cs[(w * 3 + 1) * D + 16 * db + 4 * g + e] = sk;
                        s_cs[(w * 3 + 2) * D + 16 * db + 4 * g + e] = sv;
                    }
                }
        }
    } else if (colsum && lane < D) {   // no key block: zero dK / dV column sums
        s_cs[(w * 3 + 1) * D + lane] = 0.f;
        s_cs[(w * 3 + 2) * D + lane] = 0.f;
    }

    // ---- phase 2, two halves of 128 queries: dQ^T[d][q] = K^T[d][k] dS^T[k][q] over all keys
    const int qsub = w & 7, dh = w >> 3;        // query block within the half, head-dim half
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        __syncthreads();            // phase 1 / the previous half is done with the images it overwrites
#pragma unroll
        for (int c = 0; c < 8; ++c) {   // rows of absent key blocks / keys past S get zeros
            const int q0 = 16 * c + 4 * g;
            char* img = q0 < 64 ? sT0 : sT1;
            const int qq = q0 & 63;
            *reinterpret_cast<uint2*>(img + lds_off<true, true>(myk, qq >> 3) + ds_half(myk, (qq >> 2) & 1)) =
                dsk[8 * half + c];
        }
        __syncthreads();
        const int qblk = 8 * half + qsub;
        if (qblk < nblk) {
            const int myq = 16 * qblk + (lane & 15);
            const char* img = qsub < 4 ? sT0 : sT1;
            const int cb = (16 * qsub) & 63;
            f32x4 dq[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) dq[i] = (f32x4){0, 0, 0, 0};
#pragma unroll
            for (int st = 0; st < 8; ++st) {
                if (st < nch) {
                    const bf16x8 sf = frag_tr<true, true>(img, 32 * st, cb);
#pragma unroll
                    for (int i = 0; i < 2; ++i)
                        dq[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<true>(sK, 32 * st, 32 * dh + 16 * i),
                                                                        sf, dq[i], 0, 0, 0);
                }
            }
            if (myq < S) {
                bf16_t* dqr = dqkv + ((long)b * S + myq) * rs + h * D + 32 * dh;
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    float a4[4] = {dq[i][0] * scale, dq[i][1] * scale, dq[i][2] * scale, dq[i][3] * scale};
                    store4(dqr + 16 * i + 4 * g, a4);
                }
            }
            if (colsum) {   // queries past S hold zero gradients; wave w sums head dims 32 dh .. +31
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float sq = row16_sum(dq[i][e] * scale);
                        if ((lane & 15) == 0) {
                            float* c0 = s_cs + (w * 3 + 0) * D + 32 * dh + 16 * i + 4 * g + e;
                            *c0 = half ? *c0 + sq : sq;
                        }
                    }
            }
        }
    }
    if (colsum) {
        __syncthreads();
        if (tid < 3 * D) {
            const int part = tid / D, d = tid - part * D;
            float acc = 0.f;
            if (part == 0) {        // dQ: waves 8 (d >> 5) .. +7 hold head dim d
#pragma unroll
                for (int ww = 0; ww < 8; ++ww) acc += s_cs[((8 * (d >> 5) + ww) * 3) * D + d];
            } else {
#pragma unroll
                for (int ww = 0; ww < MW; ++ww) acc += s_cs[(ww * 3 + part) * D + d];
            }
            colsum[(long)b * 3 * H * D + part * H * D + h * D + d] = acc;
        }
    }
}
}  // namespace

namespace {
int num_cus() {
    static const int n = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
            v = 256;
        return v;
    }();
    return n;
}
// DDL_ATTN_FUSED_BWD=0: the tiled forward and two-kernel backward for every S (A/B timing, tests)
bool fused_bwd_enabled() {
    static const bool on = [] {
        const char* e = getenv("DDL_ATTN_FUSED_BWD");
        return !(e && e[0] == '0');
    }();
    return on;
}
// DDL_ATTN_MED=0: 128 < S <= 256 takes the tiled forward and two-kernel backward (A/B timing)
bool med_enabled() {
    static const bool on = [] {
        const char* e = getenv("DDL_ATTN_MED");
        return fused_bwd_enabled() && !(e && e[0] == '0');
    }();
    return on;
}
}  // namespace

// dropout keep-bit words the forward writes and the backward reads (p_drop > 0)
DDL_API long ddl_attn_dmask_words(int B, int S, int H) { return (long)B * H * dmask_nkw(S) * 4 * S; }

// qkv [B, S, 3*H*64] bf16; mask: additive key bias [B, S] fp32 or null; out [B, S, H*64]; lse [B, H, S] fp32
// dmask: ddl_attn_dmask_words uint32 (required when p_drop > 0): the dropout keep bits
DDL_API int ddl_attn_fwd(const void* qkv, const float* mask, void* out, float* lse, int B, int S, int H, float scale,
                         float p_drop, uint64_t seed, uint32_t* dmask, hipStream_t st) {
    if (p_drop > 0.f && !dmask) return -5;
    if (S <= FS && fused_bwd_enabled()) {
        const bool full = S == FS, msk = mask != nullptr, drp = p_drop > 0.f;
        const int grid = std::min(B * H, 2 * num_cus());   // persistent: two workgroups per CU
#define FWD_SHORT(F, M, D) attn_fwd_short_k<F, M, D><<<grid, 512, 0, st>>>((const bf16_t*)qkv, mask, (bf16_t*)out, lse, S, H, scale, p_drop, seed, B * H, dmask)
        if (full) {
            if (msk) { if (drp) FWD_SHORT(true, true, true); else FWD_SHORT(true, true, false); }
            else { if (drp) FWD_SHORT(true, false, true); else FWD_SHORT(true, false, false); }
        } else {
            if (msk) { if (drp) FWD_SHORT(false, true, true); else FWD_SHORT(false, true, false); }
            else { if (drp) FWD_SHORT(false, false, true); else FWD_SHORT(false, false, false); }
        }
#undef FWD_SHORT
        DDL_RETURN_LAUNCH();
    }
    if (S <= FM && med_enabled()) {
#define FWD_MED(M, D) attn_fwd_med_k<M, D><<<B * H, 512, 0, st>>>((const bf16_t*)qkv, mask, (bf16_t*)out, lse, S, H, scale, p_drop, seed, dmask)
        if (mask) { if (p_drop > 0.f) FWD_MED(true, true); else FWD_MED(true, false); }
        else { if (p_drop > 0.f) FWD_MED(false, true); else FWD_MED(false, false); }
#undef FWD_MED
        DDL_RETURN_LAUNCH();
    }
    dim3 grid((S + TROWS_F - 1) / TROWS_F, B * H);
#define FWD_TILED(M, D) attn_fwd_k<M, D><<<grid, 64 * TWF, 0, st>>>((const bf16_t*)qkv, mask, (bf16_t*)out, lse, B, S, H, scale, p_drop, seed, dmask)
    if (mask) { if (p_drop > 0.f) FWD_TILED(true, true); else FWD_TILED(true, false); }
    else { if (p_drop > 0.f) FWD_TILED(false, true); else FWD_TILED(false, false); }
#undef FWD_TILED
    DDL_RETURN_LAUNCH();
}

// dqkv [B, S, 3*H*64] bf16 (fully written); delta scratch [B, H, S] fp32
// colsum (nullable, [B * 4 ceil(S / 64)][3 H 64] fp32): column sums of dqkv per batch (single-
// workgroup paths: rows 0..B-1, returns 0) or per batch and 16-row group (tiled path: every row,
// returns 2) -- the QKV bias gradient is the column sum of the written rows
DDL_API int ddl_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse, const float* mask,
                         float* delta, void* dqkv, int B, int S, int H, float scale, float p_drop,
                         const uint32_t* dmask, float* colsum, hipStream_t st) {
    if (p_drop > 0.f && !dmask) return -5;
    if (S <= FS && fused_bwd_enabled()) {   // the whole sequence fits one workgroup's LDS
#define BWD_FUSED(F, DR) attn_bwd_fused_k<F, DR><<<B * H, 512, 0, st>>>((const bf16_t*)qkv, (const bf16_t*)out, \
        (const bf16_t*)dout, lse, mask, (bf16_t*)dqkv, S, H, scale, p_drop, dmask, colsum)
        if (S == FS) { if (p_drop > 0.f) BWD_FUSED(true, true); else BWD_FUSED(true, false); }
        else { if (p_drop > 0.f) BWD_FUSED(false, true); else BWD_FUSED(false, false); }
#undef BWD_FUSED
        DDL_RETURN_LAUNCH();
    }
    if (S <= FM && med_enabled()) {   // 96 KB of row images: one workgroup per CU
#define BWD_MED(DR) attn_bwd_med_k<DR><<<B * H, 64 * MW, 0, st>>>((const bf16_t*)qkv, (const bf16_t*)out, \
        (const bf16_t*)dout, lse, mask, (bf16_t*)dqkv, S, H, scale, p_drop, dmask, colsum)
        if (p_drop > 0.f) BWD_MED(true); else BWD_MED(false);
#undef BWD_MED
        DDL_RETURN_LAUNCH();
    }
    const long rows = (long)B * S * H;
    attn_delta_k<<<(int)((rows * 8 + 255) / 256), 256, 0, st>>>((const bf16_t*)dout, (const bf16_t*)out, delta, B, S, H);
    dim3 grid((S + TROWS_B - 1) / TROWS_B, B * H);    // the dKV and dQ workgroups share the colsum rows
    const bool drp = p_drop > 0.f;
#define BWD_DKV(DR) attn_bwd_dkv_k<DR><<<grid, 64 * TWB, 0, st>>>((const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, \
        mask, (bf16_t*)dqkv, B, S, H, scale, p_drop, dmask, colsum)
#define BWD_DQ(M, DR) attn_bwd_dq_k<M, DR><<<grid, 64 * TWB, 0, st>>>((const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, \
        mask, (bf16_t*)dqkv, B, S, H, scale, p_drop, dmask, colsum)
    if (drp) BWD_DKV(true); else BWD_DKV(false);
    if (mask) { if (drp) BWD_DQ(true, true); else BWD_DQ(true, false); }
    else { if (drp) BWD_DQ(false, true); else BWD_DQ(false, false); }
#undef BWD_DKV
#undef BWD_DQ
    const int rc = (int)hipGetLastError();
    return rc ? rc : (colsum ? 2 : 0);
}
