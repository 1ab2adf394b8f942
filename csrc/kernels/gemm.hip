// bf16 MFMA GEMM + implicit-GEMM convolution for gfx950 (kernel families K1/K2/K3/K9/K13).
//
//   C[m][n] = sum_k A(m,k) * B(n,k)  (+ bias[n]) (activation)     fp32 accumulate
//
// Operand loaders (template parameters) cover every GEMM the models issue
// without any transpose copies:
//   KC  : X(r,k) = X[r*ld + k]          (row-major, reduction contiguous)
//   KO  : X(r,k) = X[k*ld + r]          (reduction outer: dgrad weights, wgrad activations)
//   CONV: A(m,k) = implicit im2col of an NHWC tensor (conv fwd / dgrad)
//   CONVW: B(n,k) = im2col with the reduction over output pixels (conv wgrad)
//
// Tiling (CDNA4): 128x128x64 block tile, 256 threads = 4 wave64 in a 2x2 grid,
// each wave 64x64 = 4x4 v_mfma_f32_16x16x32_bf16 tiles.  Operands are staged
// global -> registers -> LDS (double-buffered, one barrier per K-step; the next
// tile's global loads are in flight under the current tile's MFMAs).  LDS
// images are XOR-swizzled so both fragment reads are bank-conflict free:
//   KC image  [128 rows][64 k], 128-B rows, chunk' = chunk ^ ((row>>1)&7),
//             fragments by ds_read_b128;
//   KO image  [64 k][128 cols], 256-B rows, chunk' = chunk ^ 2*((r&3)|((r>>3)&1)<<2),
//             fragments by ds_read_b64_tr_b16 (hardware transpose).
// The MFMA is issued as (B-fragment, A-fragment) so each lane's accumulator
// holds 4 consecutive output COLUMNS of one row: the epilogue stores 8/16 B per
// lane and applies bias / GELU / ReLU / tanh from fp32 before rounding once.
// Split-K writes fp32 partial slabs reduced (with the epilogue) by gemm_reduce.
// Block ids are remapped so the blocks that share an XCD's L2 (ids congruent
// mod 8) walk neighbouring tiles (bijective remap, §5.5 T1).
#include "ddl_common.h"

#include <cstdlib>

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_BYTES = 128 * 64 * 2;   // 16 KB per operand tile

enum Layout { KC = 0, KO = 1, CONV = 2, CONVW = 3 };
// LDS bytes of one pipeline stage (A image + B image).  A narrow tile's 64-row B image
// is 8 KB (KC: the first half of the 128-row layout; k-major: packed 128-byte rows), so
// its stage packs to 24 KB: 48 KB a block, three blocks (12 waves) a CU.
template <int LB, int BNT>
constexpr int stage_bytes() { return TILE_BYTES + (BNT == 64 ? TILE_BYTES / 2 : TILE_BYTES); }
template <int LB, int BNT>
constexpr int waves_per_eu() { return BNT == 64 ? 3 : 2; }
enum Act { ACT_NONE = 0, ACT_GELU = 1, ACT_RELU = 2, ACT_TANH = 3, ACT_DGELU = 4, ACT_BNB = 5 };

struct ConvDesc {
    int N, H, W, C;                 // input NHWC
    int P, Q;                       // GEMM output-pixel grid
    int stride, h_off, w_off, h_step, w_step;
    int R, S;                       // taps (after sub-setting for dgrad classes)
    FastDiv fd_PQ, fd_Q, fd_C, fd_S;
    int OH, OW, ostep, oa, ob;      // output pixel (n, p*ostep+oa, q*ostep+ob) in [OH, OW]
    int bk_dq, bk_dp;               // BK output pixels = bk_dp grid rows + bk_dq columns
};

struct Params {
    const bf16_t* A;
    const bf16_t* B;
    long lda, ldb;
    void* C;
    long ldc;
    int M, N, K;
    const void* bias;
    int bias_bf16;
    int act;
    void* aux;        // ACT_GELU: pre-activation output (bf16, ldc); ACT_DGELU: pre-activation input
    int out_f32;
    int splits, kt_per_split;
    long split_stride;
    int row_remap;    // conv output rows -> strided output pixels
    int trans_out;    // store C^T: element (m, n) at C[n * ldc + m] (narrow-Cout weight gradients)
    float* colstats;  // BN statistics of the (bf16-rounded) output: per 128-row tile,
                      // [tile_m][0..N) column sums and [tile_m][N..2N) sums of squares
    long ldw;         // split-K slab row stride
    const bf16_t* res;  // optional residual added before the activation (same layout as C)
    int accumulate;     // C += result (gradient accumulation straight into the parameter-grad arena)
    // ACT_BNB (BatchNorm backward fused into the dgrad that produces the BN output's
    // gradient): C = (acc + res) * relu_mask, colstats = [sum C | sum C * xhat] with
    // xhat = (aux - bn_mean) * bn_istd -- the BN backward's reduction pass
    const uint8_t* bn_mask;
    const float* bn_mean;
    const float* bn_istd;
    ConvDesc cd;
    int tiles_m, tiles_n;
    int stage_out;      // wide plain-bf16 tiles leave through LDS as whole rows (DDL_GEMM_STAGE_OUT)
};

// Loads are unconditional from a clamped (always valid) address and the VALUE is
// selected, so hipcc never materialises a zero vector in scratch for a
// select-of-pointers.
__device__ __forceinline__ uint4 ldg16(const bf16_t* ptr) { return *reinterpret_cast<const uint4*>(ptr); }
__device__ __forceinline__ uint4 sel(bool ok, uint4 a, uint4 z) {
    return make_uint4(ok ? a.x : z.x, ok ? a.y : z.y, ok ? a.z : z.z, ok ? a.w : z.w);
}

__device__ __forceinline__ int swz_ko(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }
// 64-column k-major image (narrow B operand), 128-byte rows: a fragment read touches rows
// 8g + q (g, q < 4), two chunks each; rows of one parity share a bank half, so the chunk
// pair is XORed with (q >> 1) | (g & 1) << 1 -- the same 2-way (g, g + 2) overlap as the
// 256-byte layout
__device__ __forceinline__ int swz_kon(int r) { return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }

// ------------------------------------------------------------------ loaders
// Each thread stages 4 chunks (16 B) of each operand per K-step.
template <int L, bool IS_A, int ROWS = 128>
struct Loader {
    // ROWS = 64 (narrow B tile): KC rows (t>>3) + 32 i for i < 2 (the first half of the
    // 128-row image, fragment reads unchanged); KO/CONVW chunk c = t&7 and k-rows
    // (t>>3) + 32 i into packed 128-byte rows (read_frag<L, true>).
    static constexpr int NCH = ROWS / 32;   // 16-B chunks per thread
    // KC / CONV: thread -> chunk c = t&7, rows (t>>3) + 32 i
    // KO / CONVW: thread -> chunk c = t&15, k-rows (t>>4) + 16 i
    const bf16_t* base;
    long ld;
    int rows_total;   // M or N extent of this operand
    int K;
    int r0;           // tile origin (m0 or n0)
    // conv state
    int hb[4], wb[4];
    const bf16_t* img[4];
    bool rowok[4];
    int ctap_r, ctap_s, cci;   // CONVW: column tap decomposition (fixed per thread)
    bool colok;
    // CONVW: output-pixel state of this thread's rows, advanced by BK per K-step
    // instead of two divisions per 16-byte chunk (the loader was VALU-bound)
    int wn_[4], wp_[4], wq_[4];
    int knext;

    __device__ __forceinline__ void init(const Params& p, int origin) {
        const int t = threadIdx.x;
        base = IS_A ? p.A : p.B;
        ld = IS_A ? p.lda : p.ldb;
        rows_total = IS_A ? p.M : p.N;
        K = p.K;
        r0 = origin;
        if (L == CONV) {
            const ConvDesc& cd = p.cd;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int m = r0 + (t >> 3) + 32 * i;
                rowok[i] = m < rows_total;
                const int mm = rowok[i] ? m : 0;
                const int n = (int)fdiv((uint32_t)mm, cd.fd_PQ);
                const int rem = mm - n * cd.P * cd.Q;
                const int pp = (int)fdiv((uint32_t)rem, cd.fd_Q);
                const int qq = rem - pp * cd.Q;
                hb[i] = pp * cd.stride + cd.h_off;
                wb[i] = qq * cd.stride + cd.w_off;
                img[i] = base + (long)n * cd.H * cd.W * cd.C;
            }
        }
        if (L == CONVW) {
            const ConvDesc& cd = p.cd;
            const int col = r0 + 8 * (ROWS == 128 ? (t & 15) : (t & 7));
            colok = col < rows_total;
            const int cc = colok ? col : 0;
            const int tap = (int)fdiv((uint32_t)cc, cd.fd_C);
            cci = cc - tap * cd.C;
            ctap_r = (int)fdiv((uint32_t)tap, cd.fd_S);
            ctap_s = tap - ctap_r * cd.S;
            knext = -1;
        }
    }

    __device__ __forceinline__ void load(const Params& p, int k0, uint4 (&v)[4]) {
        const int t = threadIdx.x;
        const uint4 z = make_uint4(0, 0, 0, 0);
        if (L == KC) {
            const int c = t & 7;
            const int k = k0 + 8 * c;
#pragma unroll
            for (int i = 0; i < NCH; ++i) {
                const int r = r0 + (t >> 3) + 32 * i;
                const bool ok = r < rows_total && k < K;
                v[i] = sel(ok, ldg16(ok ? base + (long)r * ld + k : base), z);
            }
        } else if (L == KO) {
            const int col = r0 + 8 * (ROWS == 128 ? (t & 15) : (t & 7));
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int k = k0 + (ROWS == 128 ? (t >> 4) + 16 * i : (t >> 3) + 32 * (i & 1));
                if (ROWS != 128 && i >= 2) break;
                const bool ok = k < K && col < rows_total;
                v[i] = sel(ok, ldg16(ok ? base + (long)k * ld + col : base), z);
            }
        } else if (L == CONV) {
            const ConvDesc& cd = p.cd;
            const int k = k0 + 8 * (t & 7);
            const int kk = k < K ? k : 0;
            const int tap = (int)fdiv((uint32_t)kk, cd.fd_C);
            const int ci = kk - tap * cd.C;
            const int rr = (int)fdiv((uint32_t)tap, cd.fd_S);
            const int ss = tap - rr * cd.S;
            const int dh = rr * cd.h_step, dw = ss * cd.w_step;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int h = hb[i] + dh, w = wb[i] + dw;
                const bool ok = rowok[i] && k < K && (unsigned)h < (unsigned)cd.H && (unsigned)w < (unsigned)cd.W;
                v[i] = sel(ok, ldg16(ok ? img[i] + ((long)h * cd.W + w) * cd.C + ci : base), z);
            }
        } else {  // CONVW: reduction rows are output pixels m
            const ConvDesc& cd = p.cd;
            if (k0 != knext) {   // first K-step of this block: full decomposition of each row
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int m = k0 + (ROWS == 128 ? (t >> 4) + 16 * i : (t >> 3) + 32 * i);
                    const int mm = m < K ? m : 0;
                    wn_[i] = (int)fdiv((uint32_t)mm, cd.fd_PQ);
                    const int rem = mm - wn_[i] * cd.P * cd.Q;
                    wp_[i] = (int)fdiv((uint32_t)rem, cd.fd_Q);
                    wq_[i] = rem - wp_[i] * cd.Q;
                }
            }
            const int hof = cd.h_off + ctap_r * cd.h_step, wof = cd.w_off + ctap_s * cd.w_step;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (ROWS != 128 && i >= 2) break;
                const int m = k0 + (ROWS == 128 ? (t >> 4) + 16 * i : (t >> 3) + 32 * i);
                const int h = wp_[i] * cd.stride + hof;
                const int w = wq_[i] * cd.stride + wof;
                const bool ok = colok && m < K && (unsigned)h < (unsigned)cd.H && (unsigned)w < (unsigned)cd.W;
                // 32-bit element offset: activations stay < 2^31 elements (host-checked)
                const uint32_t off = ((uint32_t)(wn_[i] * cd.H + h) * (uint32_t)cd.W + (uint32_t)w) * (uint32_t)cd.C +
                                     (uint32_t)cci;
                v[i] = sel(ok, ldg16(ok ? base + off : base), z);
                // advance this row by BK output pixels: q += BK % Q (carry into p), p += BK / Q,
                // then wrap p into the next image(s)
                int q = wq_[i] + cd.bk_dq, pq = wp_[i] + cd.bk_dp;
                if (q >= cd.Q) { q -= cd.Q; ++pq; }
                int nn = wn_[i];
                while (pq >= cd.P) { pq -= cd.P; ++nn; }
                wq_[i] = q;
                wp_[i] = pq;
                wn_[i] = nn;
            }
            knext = k0 + BK;
        }
    }

    __device__ __forceinline__ void store(char* lds, const uint4 (&v)[4]) {
        const int t = threadIdx.x;
        if (L == KC || L == CONV) {
            const int c = t & 7;
#pragma unroll
            for (int i = 0; i < NCH; ++i) {
                const int r = (t >> 3) + 32 * i;
                *reinterpret_cast<uint4*>(lds + r * 128 + ((c ^ ((r >> 1) & 7)) << 4)) = v[i];
            }
        } else if (ROWS == 128) {
            const int c = t & 15;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = (t >> 4) + 16 * i;
                *reinterpret_cast<uint4*>(lds + r * 256 + ((c ^ swz_ko(r)) << 4)) = v[i];
            }
        } else {   // 64-column k-major image, packed 128-byte rows (read_frag<L, true>)
            const int c = t & 7;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int r = (t >> 3) + 32 * i;
                *reinterpret_cast<uint4*>(lds + r * 128 + ((c ^ swz_kon(r)) << 4)) = v[i];
            }
        }
    }
};

// Fragment for rows [rbase, rbase+16) of the tile, k-subtile kk (0/1):
// lane l gets row rbase + (l&15), k = 32 kk + 8 (l>>4) + 0..7.
template <int L, bool NARROW = false>
__device__ __forceinline__ bf16x8 read_frag(const char* lds, int rbase, int kk) {
    const int l = threadIdx.x & 63;
    if (L == KC || L == CONV) {
        const int r = rbase + (l & 15);
        const int c = kk * 4 + (l >> 4);
        return *reinterpret_cast<const bf16x8*>(lds + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
    } else {
        const int g = l >> 4, q = (l >> 2) & 3, pq = l & 3;
        const int col = rbase + 4 * pq;
        const int chunk = col >> 3;
        const int r_a = kk * 32 + 8 * g + q;
        const int r_b = r_a + 4;
        typedef __attribute__((address_space(3))) s16x4 lds_v4;
        const char* pa = NARROW ? lds + r_a * 128 + ((chunk ^ swz_kon(r_a)) << 4) + (pq & 1) * 8
                                : lds + r_a * 256 + ((chunk ^ swz_ko(r_a)) << 4) + (pq & 1) * 8;
        const char* pb = NARROW ? lds + r_b * 128 + ((chunk ^ swz_kon(r_b)) << 4) + (pq & 1) * 8
                                : lds + r_b * 256 + ((chunk ^ swz_ko(r_b)) << 4) + (pq & 1) * 8;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)pa);
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)pb);
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, r);
    }
}

__device__ __forceinline__ float apply_act(float v, int act) {
    switch (act) {
        case ACT_GELU: return gelu_erf(v);
        case ACT_RELU: return fmaxf(v, 0.f);
        case ACT_TANH: return tanhf(v);
        default: return v;
    }
}

__device__ __forceinline__ long out_row(const Params& p, int m) {
    if (!p.row_remap) return m;
    const ConvDesc& cd = p.cd;
    const int n = (int)fdiv((uint32_t)m, cd.fd_PQ);
    const int rem = m - n * cd.P * cd.Q;
    const int pp = (int)fdiv((uint32_t)rem, cd.fd_Q);
    const int qq = rem - pp * cd.Q;
    return ((long)n * cd.OH + pp * cd.ostep + cd.oa) * cd.OW + qq * cd.ostep + cd.ob;
}

// BNB: the BatchNorm-backward epilogue variant (own instantiation: its registers
// never weigh on the other epilogues)
template <int LA, int LB, int BNT, bool BNB = false>
__device__ __forceinline__ void gemm_body(const Params& p, char* smem) {
    constexpr int WN = BNT / 2;        // wave tile N extent (64 or 32)
    constexpr int NJ = WN / 16;        // MFMA column tiles per wave
    // ---- XCD-aware bijective tile remap
    const int nwg = p.tiles_m * p.tiles_n;
    const int bid = blockIdx.x;
    const int xcd = bid & 7, qn = nwg >> 3, rn = nwg & 7;
    const int wg = (xcd < rn ? xcd * (qn + 1) : rn * (qn + 1) + (xcd - rn) * qn) + (bid >> 3);
    const int tm = wg / p.tiles_n, tn = wg - tm * p.tiles_n;
    const int m0 = tm * BM, n0 = tn * BNT;
    const int split = blockIdx.y;

    const int nk_total = (p.K + BK - 1) / BK;
    const int kt0 = split * p.kt_per_split;
    const int kt1 = min(nk_total, kt0 + p.kt_per_split);

    Loader<LA, true> la;
    Loader<LB, false, BNT> lb;
    la.init(p, m0);
    lb.init(p, n0);

    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm = w & 1, wn = w >> 1;
    const int g = lane >> 4;

    f32x4 acc[4][NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    // wide plain-bf16 tiles with a residual: the residual tile is loaded up front, in flight
    // under the operand loads and MFMAs (short-K GEMMs are epilogue-bound: loading it in the
    // epilogue serialised a second memory latency behind the operand loads every tile)
    const bool wide_early = m0 + BM <= p.M && n0 + BNT <= p.N && (p.N & 7) == 0 && (p.ldc & 7) == 0;
    const bool wide_plain = !BNB && wide_early && !(p.out_f32) && !p.trans_out && !p.row_remap && !p.bias &&
                            p.act == ACT_NONE && !p.accumulate;
    uint2 rb_pre[NJ][4];
    // BNB: the epilogue's BN input / residual / ReLU-mask sites, likewise loaded up front
    // (unconditional loads from clamped addresses; absent operands read aux and are
    // replaced afterwards -- a load under a branch gets waited at the join)
    // (not for the implicit-GEMM conv variants: their loaders leave no registers for it)
    constexpr bool EARLY_BNB = BNB && LA == KC;
    uint2 xr[4][NJ], rr[4][NJ];
    uint32_t mb[4][NJ];
    // Interior tiles with 64-aligned rows (bnb_vec) load 16 bytes per lane -- 8 columns of
    // row block i (g even) or i + 1 (g odd), the pair-store layout -- and un-pair them with
    // v_permlane16_swap in the epilogue; the ReLU mask as one 32 / 64-bit word per row.
    // (per-site 8-byte and 1-byte loads left the epilogue issue-stalled on the VMEM queue)
    const bool bnb_vec = wide_early && (p.ldc & 63) == 0;
    auto bnb_load = [&]() {
        const bf16_t* auxp = (const bf16_t*)p.aux;
        const bf16_t* resp = p.res ? p.res : auxp;
        const uint8_t* mp = p.bn_mask ? p.bn_mask : (const uint8_t*)auxp;
        if (bnb_vec) {
#pragma unroll
            for (int ip = 0; ip < 2; ++ip) {
                const long mrow = m0 + wm * 64 + (2 * ip + (g & 1)) * 16 + (lane & 15);
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const long o = mrow * p.ldc + n0 + wn * WN + j * 16 + (g >> 1) * 8;
                    const uint4 vx = *reinterpret_cast<const uint4*>(auxp + o);
                    const uint4 vr = *reinterpret_cast<const uint4*>(resp + o);
                    xr[2 * ip][j] = make_uint2(vx.x, vx.y);
                    xr[2 * ip + 1][j] = make_uint2(vx.z, vx.w);
                    rr[2 * ip][j] = make_uint2(vr.x, vr.y);
                    rr[2 * ip + 1][j] = make_uint2(vr.z, vr.w);
                }
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const long mw = ((long)(m0 + wm * 64 + i * 16 + (lane & 15)) * p.ldc + n0 + wn * WN) >> 3;
                if constexpr (NJ == 4) {
                    const uint2 w2 = *reinterpret_cast<const uint2*>(mp + mw);
                    mb[i][0] = w2.x;
                    mb[i][1] = w2.y;
                } else {
                    mb[i][0] = *reinterpret_cast<const uint32_t*>(mp + mw);
                }
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const long mc = min(m0 + wm * 64 + i * 16 + (lane & 15), p.M - 1);
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int nc = min(n0 + wn * WN + j * 16 + 4 * g, p.N - 4);
                const long o = mc * p.ldc + nc;
                xr[i][j] = *reinterpret_cast<const uint2*>(auxp + o);
                rr[i][j] = *reinterpret_cast<const uint2*>(resp + o);
                mb[i][j] = (uint32_t)mp[o >> 3] >> (nc & 4);
            }
        }
    };
    if (kt0 < kt1) {
        // two K-steps of global loads in flight (register sets 0 / 1 alternate): the
        // 128-row tiles do little MFMA work per K-step, so one step of prefetch left
        // them latency-bound on the operand loads (im2col gathers above all)
        uint4 ra0[4], rb0[4], ra1[4], rb1[4];
        la.load(p, kt0 * BK, ra0);
        lb.load(p, kt0 * BK, rb0);
        if (kt0 + 1 < kt1) {
            la.load(p, (kt0 + 1) * BK, ra1);
            lb.load(p, (kt0 + 1) * BK, rb1);
        }
        // (issued after the first operand loads: vmcnt retires in order, so the operand
        // wait does not also wait for the residual)
        if constexpr (EARLY_BNB) bnb_load();
        if (wide_plain && p.res) {
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    rb_pre[j][i] = *reinterpret_cast<const uint2*>(
                        p.res + (long)(m0 + (threadIdx.x >> 6 & 1) * 64 + i * 16 + (threadIdx.x & 15)) * p.ldc + n0 +
                        (threadIdx.x >> 7) * WN + j * 16 + 4 * ((threadIdx.x & 63) >> 4));
        }
        la.store(smem, ra0);
        lb.store(smem + TILE_BYTES, rb0);
        __syncthreads();
        // one K-step: (ran, rbn) hold K-step kt+1, (raf, rbf) are free and receive kt+2
        auto step = [&](int kt, uint4 (&ran)[4], uint4 (&rbn)[4], uint4 (&raf)[4], uint4 (&rbf)[4]) {
            const int cur = (kt - kt0) & 1;
            char* sa = smem + cur * stage_bytes<LB, BNT>();
            char* sb = sa + TILE_BYTES;
            if (kt + 2 < kt1) {
                la.load(p, (kt + 2) * BK, raf);
                lb.load(p, (kt + 2) * BK, rbf);
            }
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                bf16x8 af[4], bfr[NJ];
#pragma unroll
                for (int i = 0; i < 4; ++i) af[i] = read_frag<LA>(sa, wm * 64 + i * 16, kk);
#pragma unroll
                for (int j = 0; j < NJ; ++j) bfr[j] = read_frag<LB, BNT == 64>(sb, wn * WN + j * 16, kk);
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < NJ; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
            }
            if (kt + 1 < kt1) {
                char* na = smem + (cur ^ 1) * stage_bytes<LB, BNT>();
                la.store(na, ran);
                lb.store(na + TILE_BYTES, rbn);
            }
            __syncthreads();
        };
        for (int kt = kt0; kt < kt1; kt += 2) {
            step(kt, ra1, rb1, ra0, rb0);
            if (kt + 1 < kt1) step(kt + 1, ra0, rb0, ra1, rb1);
        }
    }

    // ---- epilogue: lane holds C[m][n..n+3]
    // Interior tiles with 8-element-aligned rows store two row blocks (i, i + 1) of a
    // column group per lane as ONE 16-byte store: v_permlane16_swap gives the odd lane
    // rows (g = 1, 3) block i + 1's quads of the even rows in exchange for theirs of
    // block i, so every lane holds 8 consecutive columns of one row (8-byte stores left
    // these output-heavy tiles store-issue bound).  Needs every lane active.
    const bool wide = m0 + BM <= p.M && n0 + BNT <= p.N && (p.N & 7) == 0 && (p.ldc & 7) == 0;
    auto store_pair = [&](bf16_t* base, uint32_t lo0, uint32_t hi0, uint32_t lo1, uint32_t hi1, int mA, int nb) {
        const auto x = __builtin_amdgcn_permlane16_swap(lo0, lo1, false, false);
        const auto y = __builtin_amdgcn_permlane16_swap(hi0, hi1, false, false);
        const int mrow = (lane & 16) ? mA + 16 : mA;       // g odd: row block i + 1
        *reinterpret_cast<uint4*>(base + (long)mrow * p.ldc + nb + (lane >> 5) * 8) = make_uint4(x[0], y[0], x[1], y[1]);
    };
    float st_s[NJ][4], st_q[NJ][4];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) st_s[j][r] = st_q[j][r] = 0.f;
    if constexpr (BNB) {
        // BatchNorm backward (N % 8 == 0: a site is whole or outside): dz = (acc + res) *
        // relu_mask stored, column sums of dz and dz * xhat.  Pass 1 puts every site's
        // loads in flight at once (clamped addresses; out-of-range sites are dropped in
        // pass 2) -- one site at a time the epilogue is load-latency bound.
        // (the loads were issued with the first operand loads where that fits: bnb_load)
        if constexpr (!EARLY_BNB) bnb_load();
        if (bnb_vec) {
#pragma unroll
            for (int ip = 0; ip < 2; ++ip)
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const auto a = __builtin_amdgcn_permlane16_swap(xr[2 * ip][j].x, xr[2 * ip + 1][j].x, false, false);
                    const auto b = __builtin_amdgcn_permlane16_swap(xr[2 * ip][j].y, xr[2 * ip + 1][j].y, false, false);
                    xr[2 * ip][j] = make_uint2(a[0], b[0]);
                    xr[2 * ip + 1][j] = make_uint2(a[1], b[1]);
                    const auto c = __builtin_amdgcn_permlane16_swap(rr[2 * ip][j].x, rr[2 * ip + 1][j].x, false, false);
                    const auto d = __builtin_amdgcn_permlane16_swap(rr[2 * ip][j].y, rr[2 * ip + 1][j].y, false, false);
                    rr[2 * ip][j] = make_uint2(c[0], d[0]);
                    rr[2 * ip + 1][j] = make_uint2(c[1], d[1]);
                }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint32_t bits[NJ];
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    bits[j] = NJ == 4 ? mb[i][j >> 1] >> ((j & 1) * 16 + 4 * g) : mb[i][0] >> (j * 16 + 4 * g);
#pragma unroll
                for (int j = 0; j < NJ; ++j) mb[i][j] = bits[j];
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                if (!p.res) rr[i][j] = make_uint2(0u, 0u);
                mb[i][j] = p.bn_mask ? mb[i][j] & 0xfu : 0xfu;
            }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int n = n0 + wn * WN + j * 16 + 4 * g;
            float mu[4], is[4];
            load4(p.bn_mean + min(n, p.N - 4), mu);
            load4(p.bn_istd + min(n, p.N - 4), is);
            if (wide) {
                uint32_t plo = 0, phi = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float xv[4] = {__uint_as_float(xr[i][j].x << 16), __uint_as_float(xr[i][j].x & 0xffff0000u),
                                         __uint_as_float(xr[i][j].y << 16), __uint_as_float(xr[i][j].y & 0xffff0000u)};
                    const float rv[4] = {__uint_as_float(rr[i][j].x << 16), __uint_as_float(rr[i][j].x & 0xffff0000u),
                                         __uint_as_float(rr[i][j].y << 16), __uint_as_float(rr[i][j].y & 0xffff0000u)};
                    float v[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = ((mb[i][j] >> r) & 1u) ? acc[i][j][r] + rv[r] : 0.f;
                    const uint32_t lo = pack2bf(v[0], v[1]), hi = pack2bf(v[2], v[3]);
                    if ((i & 1) == 0) { plo = lo; phi = hi; }
                    else store_pair((bf16_t*)p.C, plo, phi, lo, hi, m0 + wm * 64 + (i - 1) * 16 + (lane & 15),
                                    n0 + wn * WN + j * 16);
                    const float t[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                                        __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        st_s[j][r] += t[r];
                        st_q[j][r] += t[r] * (xv[r] - mu[r]) * is[r];
                    }
                }
                continue;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int m = m0 + wm * 64 + i * 16 + (lane & 15);
                if (m >= p.M || n >= p.N) continue;
                const float xv[4] = {__uint_as_float(xr[i][j].x << 16), __uint_as_float(xr[i][j].x & 0xffff0000u),
                                     __uint_as_float(xr[i][j].y << 16), __uint_as_float(xr[i][j].y & 0xffff0000u)};
                const float rv[4] = {__uint_as_float(rr[i][j].x << 16), __uint_as_float(rr[i][j].x & 0xffff0000u),
                                     __uint_as_float(rr[i][j].y << 16), __uint_as_float(rr[i][j].y & 0xffff0000u)};
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = ((mb[i][j] >> r) & 1u) ? acc[i][j][r] + rv[r] : 0.f;
                store4((bf16_t*)p.C + (long)m * p.ldc + n, v);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float q = bf2f(f2bf(v[r]));     // what the BN backward reads
                    st_s[j][r] += q;
                    st_q[j][r] += q * (xv[r] - mu[r]) * is[r];
                }
            }
        }
    }
    if (wide_plain) {
        // bf16 (+ residual, loaded up front) (+ BatchNorm statistics of the stored values).
        // stage_out: the tile goes through LDS (the operand stages are free after the last
        // K-step's barrier) and out as whole rows -- a pair store writes 32 rows x 32 B per
        // instruction, a row store 1 KB of 4 (or 8) contiguous rows
        constexpr int RB = BNT * 2, CH16 = RB / 16;            // staging row bytes, 16-B chunks per row
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int nb = n0 + wn * WN + j * 16;
            const uint2* rb = rb_pre[j];
            uint32_t plo = 0, phi = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                if (p.res) {
                    v[0] += __uint_as_float(rb[i].x << 16);
                    v[1] += __uint_as_float(rb[i].x & 0xffff0000u);
                    v[2] += __uint_as_float(rb[i].y << 16);
                    v[3] += __uint_as_float(rb[i].y & 0xffff0000u);
                }
                const uint32_t lo = pack2bf(v[0], v[1]), hi = pack2bf(v[2], v[3]);
                if (p.stage_out) {
                    const int row = wm * 64 + i * 16 + (lane & 15), c = (wn * WN + j * 16) / 8 + (g >> 1);
                    *reinterpret_cast<uint2*>(smem + row * RB + ((c ^ (row & (CH16 - 1))) << 4) + (g & 1) * 8) =
                        make_uint2(lo, hi);
                } else if ((i & 1) == 0) {
                    plo = lo;
                    phi = hi;
                } else {
                    store_pair((bf16_t*)p.C, plo, phi, lo, hi, m0 + wm * 64 + (i - 1) * 16 + (lane & 15), nb);
                }
                if (p.colstats) {
                    const float t[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                                        __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        st_s[j][r] += t[r];
                        st_q[j][r] += t[r] * t[r];
                    }
                }
            }
        }
        if (p.stage_out) {
            __syncthreads();
            constexpr int RPI = 1024 / RB;                     // rows per store instruction
#pragma unroll
            for (int q = 0; q < BM * RB / 1024 / 4; ++q) {
                const int row = (q * 4 + w) * RPI + lane / CH16, c = lane % CH16;
                const uint4 d = *reinterpret_cast<const uint4*>(smem + row * RB + ((c ^ (row & (CH16 - 1))) << 4));
                *reinterpret_cast<uint4*>((bf16_t*)p.C + (long)(m0 + row) * p.ldc + n0 + c * 8) = d;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if constexpr (BNB) break;
        if (wide_plain) break;
        const int m = m0 + wm * 64 + i * 16 + (lane & 15);
        if (m >= p.M) continue;
        const long orow = out_row(p, m);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int n = n0 + wn * WN + j * 16 + 4 * g;
            if (n >= p.N) continue;
            float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
            const bool full = n + 3 < p.N;
            if (p.out_f32 && p.splits > 1) {
                float* c = (float*)p.C + split * p.split_stride + orow * p.ldw + n;
                if (full) store4(c, v);
                else {
#pragma unroll
                    for (int r = 0; r < 4; ++r) if (n + r < p.N) c[r] = v[r];
                }
                continue;
            }
            if (p.trans_out) {   // plain (or accumulating) transposed store; no other epilogue ops
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (n + r >= p.N) continue;
                    const long o = (long)(n + r) * p.ldc + m;
                    float t = v[r];
                    if (p.out_f32) {
                        if (p.accumulate) t += ((float*)p.C)[o];
                        ((float*)p.C)[o] = t;
                    } else {
                        if (p.accumulate) t += bf2f(((bf16_t*)p.C)[o]);
                        ((bf16_t*)p.C)[o] = f2bf(t);
                    }
                }
                continue;
            }
            if (p.bias) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (n + r < p.N)
                        v[r] += p.bias_bf16 ? bf2f(((const bf16_t*)p.bias)[n + r]) : ((const float*)p.bias)[n + r];
            }
            if (p.res) {
                float rr[4];
                const bf16_t* rp = p.res + orow * p.ldc + n;
                if (full) load4(rp, rr);
                else {
#pragma unroll
                    for (int r = 0; r < 4; ++r) rr[r] = n + r < p.N ? bf2f(rp[r]) : 0.f;
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] += rr[r];
            }
            if (p.act == ACT_DGELU) {
                float z[4];
                const bf16_t* ap = (const bf16_t*)p.aux + orow * p.ldc + n;
                if (full) load4(ap, z);
                else {
#pragma unroll
                    for (int r = 0; r < 4; ++r) z[r] = n + r < p.N ? bf2f(ap[r]) : 0.f;
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] *= gelu_erf_grad(z[r]);
            } else if (p.act != ACT_NONE) {
                if (p.aux) {  // keep the pre-activation for backward
                    bf16_t* ap = (bf16_t*)p.aux + orow * p.ldc + n;
                    if (full) store4(ap, v);
                    else {
#pragma unroll
                        for (int r = 0; r < 4; ++r) if (n + r < p.N) ap[r] = f2bf(v[r]);
                    }
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
            }
            if (p.accumulate) {
                float o[4] = {0.f, 0.f, 0.f, 0.f};
                if (p.out_f32) {
                    const float* c = (const float*)p.C + orow * p.ldc + n;
                    if (full) load4(c, o);
                    else {
#pragma unroll
                        for (int r = 0; r < 4; ++r) if (n + r < p.N) o[r] = c[r];
                    }
                } else {
                    const bf16_t* c = (const bf16_t*)p.C + orow * p.ldc + n;
                    if (full) load4(c, o);
                    else {
#pragma unroll
                        for (int r = 0; r < 4; ++r) if (n + r < p.N) o[r] = bf2f(c[r]);
                    }
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] += o[r];
            }
            if (p.out_f32) {
                float* c = (float*)p.C + orow * p.ldc + n;
                if (full) store4(c, v);
                else {
#pragma unroll
                    for (int r = 0; r < 4; ++r) if (n + r < p.N) c[r] = v[r];
                }
            } else {
                bf16_t* c = (bf16_t*)p.C + orow * p.ldc + n;
                if (full) store4(c, v);
                else {
#pragma unroll
                    for (int r = 0; r < 4; ++r) if (n + r < p.N) c[r] = f2bf(v[r]);
                }
                if (p.colstats) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float q = n + r < p.N ? bf2f(f2bf(v[r])) : 0.f;   // what BN will read
                        st_s[j][r] += q;
                        st_q[j][r] += q * q;
                    }
                }
            }
        }
    }
    if (p.colstats) {
        // rows of this wave: reduce over the 16 lanes that share a column group,
        // then over the two M-waves through LDS (the tile buffers are free here)
        float* red = reinterpret_cast<float*>(smem);     // [2][BNT] sums, squares
        __syncthreads();
        for (int t = threadIdx.x; t < 2 * BNT; t += NT) red[t] = 0.f;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                // the 16 lanes holding these columns are one DPP row
                const float a = row16_sum(st_s[j][r]), b = row16_sum(st_q[j][r]);
                if ((lane & 15) == 0) {
                    const int col = wn * WN + j * 16 + 4 * g + r;
                    atomicAdd(&red[col], a);
                    atomicAdd(&red[BNT + col], b);
                }
            }
        __syncthreads();
        for (int t = threadIdx.x; t < BNT; t += NT) {
            const int n = n0 + t;
            if (n < p.N) {
                p.colstats[(long)tm * 2 * p.N + n] = red[t];
                p.colstats[(long)tm * 2 * p.N + p.N + n] = red[BNT + t];
            }
        }
    }
}

template <int LA, int LB, int BNT, bool BNB = false>
__global__ __launch_bounds__(NT, (waves_per_eu<LB, BNT>())) void gemm_k(Params p) {
    __shared__ __attribute__((aligned(16))) char smem[2 * stage_bytes<LB, BNT>()];
    gemm_body<LA, LB, BNT, BNB>(p, smem);
}

// Several independent GEMMs of one shape class in one launch (blockIdx.z picks the
// problem): the stride-s conv dgrad's s*s output-parity classes run concurrently
// instead of as s*s short serial launches.
constexpr int MAX_MC = 4;
struct ParamsMC {
    Params c[MAX_MC];
};

template <int LA, int LB, int BNT>
__global__ __launch_bounds__(NT, (waves_per_eu<LB, BNT>())) void gemm_mc_k(ParamsMC pm) {
    __shared__ __attribute__((aligned(16))) char smem[2 * stage_bytes<LB, BNT>()];
    const Params& p = pm.c[blockIdx.z];
    if ((int)blockIdx.x >= p.tiles_m * p.tiles_n) return;   // this class has fewer tiles
    gemm_body<LA, LB, BNT>(p, smem);
}

// Sum split-K fp32 partials, apply the epilogue, write bf16/fp32.
__global__ __launch_bounds__(256) void gemm_reduce_k(const float* __restrict__ part, int splits, long split_stride,
                                                     long ldw, int M, int N, long ldc, void* out, int out_f32,
                                                     const void* bias, int bias_bf16, int act, void* aux,
                                                     const bf16_t* __restrict__ res, int accumulate, int trans) {
    const long total = (long)M * N;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        // transposed output: walk the output contiguously (n major) so the stores coalesce
        const int m = trans ? (int)(i % M) : (int)(i / N);
        const int n = trans ? (int)(i / M) : (int)(i - (long)m * N);
        float v = 0.f;
        for (int s = 0; s < splits; ++s) v += part[s * split_stride + (long)m * ldw + n];
        if (trans) {
            const long o = (long)n * ldc + m;
            if (accumulate) v += out_f32 ? ((float*)out)[o] : bf2f(((bf16_t*)out)[o]);
            if (out_f32) ((float*)out)[o] = v;
            else ((bf16_t*)out)[o] = f2bf(v);
            continue;
        }
        if (bias) v += bias_bf16 ? bf2f(((const bf16_t*)bias)[n]) : ((const float*)bias)[n];
        if (res) v += bf2f(res[(long)m * ldc + n]);
        if (act == ACT_DGELU) v *= gelu_erf_grad(bf2f(((const bf16_t*)aux)[(long)m * ldc + n]));
        else if (act != ACT_NONE) {
            if (aux) ((bf16_t*)aux)[(long)m * ldc + n] = f2bf(v);
            v = apply_act(v, act);
        }
        if (accumulate) v += out_f32 ? ((float*)out)[(long)m * ldc + n] : bf2f(((bf16_t*)out)[(long)m * ldc + n]);
        if (out_f32) ((float*)out)[(long)m * ldc + n] = v;
        else ((bf16_t*)out)[(long)m * ldc + n] = f2bf(v);
    }
}

// Vectorised split-K reduce: a thread owns 4 consecutive output elements along the
// output's contiguous dimension (n, or m for the transposed store), 16-byte slab
// loads when the slab dimension is contiguous, no 64-bit division per element.
// SG threads share one output quad (splits g, g+SG, ..., summed through LDS): weight
// gradients have small outputs (64x256) and up to 256 slabs, so one thread per quad
// left a few dozen blocks each walking hundreds of dependent load latencies.
template <int SG>
__global__ __launch_bounds__(256) void gemm_reduce4_k(const float* __restrict__ part, int splits, long split_stride,
                                                      long ldw, int M, int N, long ldc, void* out, int out_f32,
                                                      const void* bias, int bias_bf16, int act, void* aux,
                                                      const bf16_t* __restrict__ res, int accumulate, int trans,
                                                      FastDiv fd_w, int w4, int total4) {
    constexpr int QPB = 256 / SG;   // output quads per block
    __shared__ float4 s_part[SG > 1 ? SG - 1 : 1][QPB];
    const int ql = threadIdx.x % QPB, g = threadIdx.x / QPB;
    // plain: i = m * (N/4) + n/4;   transposed: i = (m/4) * N + n
    // (block-uniform trip count: the LDS combine below has barriers)
    for (int base = blockIdx.x * QPB; base < total4; base += gridDim.x * QPB) {
        const bool live = base + ql < total4;
        const int i = live ? base + ql : total4 - 1;   // dead lanes re-read a valid quad
        const int row = (int)fdiv((uint32_t)i, fd_w);
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        if (!trans) {
            // row = m, columns c4..c4+3 (consecutive threads: consecutive column groups)
            const int c4 = (i - row * w4) * 4;
            const float* src = part + (long)row * ldw + c4;
            float u[4] = {0.f, 0.f, 0.f, 0.f};
            int s = g;
            for (; s + SG < splits; s += 2 * SG) {   // two independent chains
                const float4 t0 = *reinterpret_cast<const float4*>(src + (long)s * split_stride);
                const float4 t1 = *reinterpret_cast<const float4*>(src + (long)(s + SG) * split_stride);
                v[0] += t0.x; v[1] += t0.y; v[2] += t0.z; v[3] += t0.w;
                u[0] += t1.x; u[1] += t1.y; u[2] += t1.z; u[3] += t1.w;
            }
            if (s < splits) {
                const float4 t = *reinterpret_cast<const float4*>(src + (long)s * split_stride);
                v[0] += t.x; v[1] += t.y; v[2] += t.z; v[3] += t.w;
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += u[r];
            if (SG > 1) {
                if (g > 0) s_part[g - 1][ql] = make_float4(v[0], v[1], v[2], v[3]);
                __syncthreads();
                if (g == 0) {
#pragma unroll
                    for (int k = 0; k < SG - 1; ++k) {
                        const float4 t = s_part[k][ql];
                        v[0] += t.x; v[1] += t.y; v[2] += t.z; v[3] += t.w;
                    }
                }
                __syncthreads();
            }
            if (g != 0 || !live) continue;
            const long o = (long)row * ldc + c4;
            if (bias) {
                float bv[4];
                if (bias_bf16) load4((const bf16_t*)bias + c4, bv);
                else load4((const float*)bias + c4, bv);
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] += bv[r];
            }
            if (res) {
                float rv[4];
                load4(res + o, rv);
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] += rv[r];
            }
            if (act == ACT_DGELU) {
                float z[4];
                load4((const bf16_t*)aux + o, z);
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] *= gelu_erf_grad(z[r]);
            } else if (act != ACT_NONE) {
                if (aux) store4((bf16_t*)aux + o, v);
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], act);
            }
            if (out_f32) {
                if (accumulate) {
                    float t[4];
                    load4((const float*)out + o, t);
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] += t[r];
                }
                store4((float*)out + o, v);
            } else {
                if (accumulate) {
                    float t[4];
                    load4((const bf16_t*)out + o, t);
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] += t[r];
                }
                store4((bf16_t*)out + o, v);
            }
        } else {
            // rows m = 4*row .. +3 of slab column n (consecutive threads: consecutive n, so
            // the slab reads coalesce); stored as 4 consecutive elements of C^T row n
            const int n = i - row * w4, m4 = row * 4;
            const float* src = part + (long)m4 * ldw + n;
            for (int s = g; s < splits; s += SG)
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] += src[(long)s * split_stride + r * ldw];
            if (SG > 1) {
                if (g > 0) s_part[g - 1][ql] = make_float4(v[0], v[1], v[2], v[3]);
                __syncthreads();
                if (g == 0) {
#pragma unroll
                    for (int k = 0; k < SG - 1; ++k) {
                        const float4 t = s_part[k][ql];
                        v[0] += t.x; v[1] += t.y; v[2] += t.z; v[3] += t.w;
                    }
                }
                __syncthreads();
            }
            if (g != 0 || !live) continue;
            const long o = (long)n * ldc + m4;
            if (out_f32) {
                if (accumulate) {
                    float t[4];
                    load4((const float*)out + o, t);
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] += t[r];
                }
                store4((float*)out + o, v);
            } else {
                if (accumulate) {
                    float t[4];
                    load4((const bf16_t*)out + o, t);
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] += t[r];
                }
                store4((bf16_t*)out + o, v);
            }
        }
    }
}

template <int LA, int LB, int BNT = 128>
int launch(Params& p, float* workspace, long ws_elems, int splits, hipStream_t st) {
    p.tiles_m = (p.M + BM - 1) / BM;
    p.tiles_n = (p.N + BNT - 1) / BNT;
    const int nk = (p.K + BK - 1) / BK;
    if (splits < 1) splits = 1;
    if (splits > nk) splits = nk > 0 ? nk : 1;
    p.kt_per_split = (nk + splits - 1) / splits;
    splits = nk > 0 ? (nk + p.kt_per_split - 1) / p.kt_per_split : 1;
    p.splits = splits;
    void* final_out = p.C;
    const int final_f32 = p.out_f32;
    int acc_final = 0;
    p.ldw = p.trans_out ? p.N : p.ldc;
    if (splits > 1) {
        p.split_stride = (long)p.M * p.ldw;
        if (!workspace || ws_elems < p.split_stride * splits) return -2;
        if (p.row_remap) return -3;
        p.C = workspace;
        p.out_f32 = 1;
        acc_final = p.accumulate;
        p.accumulate = 0;
    }
    dim3 grid(p.tiles_m * p.tiles_n, splits);
    if (p.act == ACT_BNB) {
        if constexpr (LB == KC && (LA == KC || LA == CONV)) {   // dgrad operand layouts
            hipLaunchKernelGGL((gemm_k<LA, LB, BNT, true>), grid, dim3(NT), 0, st, p);
            return (int)hipGetLastError();
        }
        return -8;
    }
    hipLaunchKernelGGL((gemm_k<LA, LB, BNT>), grid, dim3(NT), 0, st, p);
    if (splits > 1) {
        const long total = (long)p.M * p.N;
        // 4 outputs per thread along the output's contiguous dimension (n; m for C^T)
        const bool vec = (p.trans_out ? p.M % 4 == 0 : (p.N % 4 == 0 && p.ldw % 4 == 0 && p.split_stride % 4 == 0)) &&
                         p.ldc % 4 == 0 && total < (1L << 31);
        if (vec) {
            const int w4 = p.trans_out ? p.N : p.N / 4;     // index divisor: i = row * w4 + col
            const int total4 = (int)(total / 4);
            // threads per output quad: enough to put ~1024 blocks on the chip, >= 4 slabs each
            int sg = 1;
            while (sg < 16 && sg * 4 <= splits && (long)total4 * sg < 256L * 1024) sg *= 2;
            const int g = std::min(8192, (total4 + 256 / sg - 1) / (256 / sg));
            const FastDiv fd = make_fastdiv((uint32_t)w4);
#define DDL_REDUCE4(SG_)                                                                                        \
    gemm_reduce4_k<SG_><<<g, 256, 0, st>>>(workspace, splits, p.split_stride, p.ldw, p.M, p.N, p.ldc, final_out, \
                                           final_f32, p.bias, p.bias_bf16, p.act, p.aux, p.res, acc_final,       \
                                           p.trans_out, fd, w4, total4)
            switch (sg) {
                case 1: DDL_REDUCE4(1); break;
                case 2: DDL_REDUCE4(2); break;
                case 4: DDL_REDUCE4(4); break;
                case 8: DDL_REDUCE4(8); break;
                default: DDL_REDUCE4(16); break;
            }
#undef DDL_REDUCE4
        } else {
            const int g = (int)std::min<long>(8192, (total + 255) / 256);
            gemm_reduce_k<<<g, 256, 0, st>>>(workspace, splits, p.split_stride, p.ldw, p.M, p.N, p.ldc, final_out,
                                              final_f32, p.bias, p.bias_bf16, p.act, p.aux, p.res, acc_final,
                                              p.trans_out);
        }
    }
    return (int)hipGetLastError();
}

void fill_conv(ConvDesc& cd, const int* d) {
    // d: N H W C P Q stride h_off w_off h_step w_step R S OH OW ostep oa ob
    cd.N = d[0]; cd.H = d[1]; cd.W = d[2]; cd.C = d[3]; cd.P = d[4]; cd.Q = d[5];
    cd.stride = d[6]; cd.h_off = d[7]; cd.w_off = d[8]; cd.h_step = d[9]; cd.w_step = d[10];
    cd.R = d[11]; cd.S = d[12]; cd.OH = d[13]; cd.OW = d[14]; cd.ostep = d[15]; cd.oa = d[16]; cd.ob = d[17];
    cd.fd_PQ = make_fastdiv((uint32_t)(cd.P * cd.Q));
    cd.fd_Q = make_fastdiv((uint32_t)cd.Q);
    cd.fd_C = make_fastdiv((uint32_t)cd.C);
    cd.fd_S = make_fastdiv((uint32_t)std::max(1, cd.S));
    cd.bk_dq = BK % std::max(1, cd.Q);
    cd.bk_dp = BK / std::max(1, cd.Q);
}

}  // namespace

// =================================================================== C ABI
// mode: 0 = A KC, B KC   (y = x W^T, Linear fwd)
//       1 = A KC, B KO   (dx = dy W,  Linear dgrad)
//       2 = A KO, B KO   (dW = dy^T x, Linear wgrad)
//       3 = A CONV, B KC (conv fwd / dgrad by implicit GEMM; conv desc required)
//       4 = A KO, B CONVW (conv wgrad; conv desc required)
//       5 = A CONVW, B KO (conv wgrad computed as dW^T: the im2col side on M, so a
//           64-channel output is the N side and fits the 128x64 tile)
//       | 16 = store C^T (element (m, n) at C[n * ldc + m]); no bias/act/residual
// act: 0 none, 1 gelu (aux <- pre-activation if aux), 2 relu, 3 tanh, 4 dgelu (v *= gelu'(aux))
static int gemm_entry(int narrow, int mode, const void* A, long lda, const void* B, long ldb, void* C, long ldc,
                      int M, int N, int K, const void* bias, int bias_bf16, int act, void* aux, int out_f32,
                      int splits, float* workspace, long ws_elems, const int* conv, int row_remap, const void* res,
                      int accumulate, float* colstats, hipStream_t st) {
    Params p{};
    p.A = (const bf16_t*)A; p.B = (const bf16_t*)B; p.lda = lda; p.ldb = ldb;
    p.C = C; p.ldc = ldc; p.M = M; p.N = N; p.K = K;
    p.bias = bias; p.bias_bf16 = bias_bf16; p.act = act; p.aux = aux; p.out_f32 = out_f32;
    p.row_remap = row_remap;
    p.trans_out = (mode & 16) ? 1 : 0;
    mode &= 15;
    if (p.trans_out && (bias || act || res || row_remap)) return -5;
    p.colstats = colstats;
    static const int stage_out = getenv("DDL_GEMM_STAGE_OUT") ? atoi(getenv("DDL_GEMM_STAGE_OUT")) : 1;
    p.stage_out = stage_out;
    if (act == ACT_BNB) {
        const BnbArgs bn = ddl_take_bnb();
        // whole-K tiles writing a dense bf16 [M, C] gradient: the mask is indexed by element
        if (!colstats || !aux || !bn.mean || !bn.istd || ldc != N || N % 8 || p.trans_out || out_f32 || accumulate ||
            splits > 1 || bias || row_remap)
            return -8;
        p.bn_mask = bn.mask; p.bn_mean = bn.mean; p.bn_istd = bn.istd;
    } else if (colstats && (p.trans_out || out_f32 || accumulate || (splits > 1) || bias || act || res)) {
        return -6;
    }
    p.res = (const bf16_t*)res;
    p.accumulate = accumulate;
    if (conv) fill_conv(p.cd, conv);
    if (M <= 0 || N <= 0) return 0;
    // the wgrad im2col loader addresses the activation with 32-bit element offsets
    if ((mode == 4 || mode == 5) && conv && (long)p.cd.N * p.cd.H * p.cd.W * p.cd.C >= (1L << 31)) return -7;
    if (narrow) {   // 128 x 64 tiles: outputs with 64 (or 64 + k*128) columns waste no MFMA work
        switch (mode) {
            case 0: return launch<KC, KC, 64>(p, workspace, ws_elems, splits, st);
            case 1: return launch<KC, KO, 64>(p, workspace, ws_elems, splits, st);
            case 2: return launch<KO, KO, 64>(p, workspace, ws_elems, splits, st);
            case 3: return launch<CONV, KC, 64>(p, workspace, ws_elems, splits, st);
            case 4: return launch<KO, CONVW, 64>(p, workspace, ws_elems, splits, st);
            case 5: return launch<CONVW, KO, 64>(p, workspace, ws_elems, splits, st);
            default: return -1;
        }
    }
    switch (mode) {
        case 0: return launch<KC, KC>(p, workspace, ws_elems, splits, st);
        case 1: return launch<KC, KO>(p, workspace, ws_elems, splits, st);
        case 2: return launch<KO, KO>(p, workspace, ws_elems, splits, st);
        case 3: return launch<CONV, KC>(p, workspace, ws_elems, splits, st);
        case 4: return launch<KO, CONVW>(p, workspace, ws_elems, splits, st);
        case 5: return launch<CONVW, KO>(p, workspace, ws_elems, splits, st);
        default: return -1;
    }
}



static thread_local BnbArgs t_bnb{};

BnbArgs ddl_take_bnb() {
    const BnbArgs a = t_bnb;
    t_bnb = BnbArgs{};
    return a;
}

// ACT_BNB side arguments for the next GEMM call on this thread (see BnbArgs)
DDL_API int ddl_gemm_bnb(const void* mask, const float* mean, const float* istd) {
    t_bnb = BnbArgs{(const uint8_t*)mask, mean, istd};
    return 0;
}

// colstats (nullable): BN statistics partials of the output, one row pair per 128-row tile
DDL_API int ddl_gemm(int mode, const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N,
                     int K, const void* bias, int bias_bf16, int act, void* aux, int out_f32, int splits,
                     float* workspace, long ws_elems, const int* conv, int row_remap, const void* res,
                     int accumulate, float* colstats, hipStream_t st) {
    return gemm_entry(0, mode, A, lda, B, ldb, C, ldc, M, N, K, bias, bias_bf16, act, aux, out_f32, splits, workspace,
                      ws_elems, conv, row_remap, res, accumulate, colstats, st);
}

DDL_API int ddl_gemm_n64(int mode, const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N,
                         int K, const void* bias, int bias_bf16, int act, void* aux, int out_f32, int splits,
                         float* workspace, long ws_elems, const int* conv, int row_remap, const void* res,
                         int accumulate, float* colstats, hipStream_t st) {
    return gemm_entry(1, mode, A, lda, B, ldb, C, ldc, M, N, K, bias, bias_bf16, act, aux, out_f32, splits, workspace,
                      ws_elems, conv, row_remap, res, accumulate, colstats, st);
}

// Multi-problem launch: n (<= 4) CONV-mode GEMMs sharing A, N and the output tensor,
// each with its own B, K and conv descriptor (18 ints per problem, as ddl_gemm) and
// output-row remap -- the parity classes of a strided convolution's dgrad.
// No split-K, no epilogue ops.
DDL_API int ddl_gemm_conv_multi(int narrow, int n, const void* A, const void* const* Bs, const int* Ms, const int* Ks,
                                void* C, long ldc, int N, const int* convs, hipStream_t st) {
    if (n < 1 || n > MAX_MC) return -1;
    ParamsMC pm{};
    int max_tiles = 0;
    const int bnt = narrow ? 64 : 128;
    for (int i = 0; i < n; ++i) {
        Params& p = pm.c[i];
        p.A = (const bf16_t*)A;
        p.B = (const bf16_t*)Bs[i];
        p.lda = 0;
        p.ldb = Ks[i];
        p.C = C;
        p.ldc = ldc;
        p.M = Ms[i];
        p.N = N;
        p.K = Ks[i];
        p.row_remap = 1;
        p.splits = 1;
        p.kt_per_split = (Ks[i] + BK - 1) / BK;
        p.ldw = ldc;
        fill_conv(p.cd, convs + 18 * i);
        p.tiles_m = (p.M + BM - 1) / BM;
        p.tiles_n = (p.N + bnt - 1) / bnt;
        if (p.M <= 0) p.tiles_m = 0;
        max_tiles = std::max(max_tiles, p.tiles_m * p.tiles_n);
    }
    if (max_tiles == 0) return 0;
    dim3 grid(max_tiles, 1, n);
    if (narrow) hipLaunchKernelGGL((gemm_mc_k<CONV, KC, 64>), grid, dim3(NT), 0, st, pm);
    else hipLaunchKernelGGL((gemm_mc_k<CONV, KC, 128>), grid, dim3(NT), 0, st, pm);
    return (int)hipGetLastError();
}
