// Large-tile bf16 GEMM / implicit-GEMM convolution for gfx950 (kernel families K1/K2/K3/K9/K13).
//
//   C[m][n] (+)= sum_k A(m,k) * B(n,k)  (+bias[n]) (+residual) (activation)
//
// Same operand-loader vocabulary as gemm.hip (KC: reduction-contiguous, KO:
// reduction-outer, CONV / CONVW: implicit im2col of an NHWC tensor), so every
// Linear / conv GEMM of fwd, dgrad and wgrad runs here without transposes.
//
// Structure (the CDNA4 256x256 8-phase schedule):
//   * block tile 256x256, BK = 64, 8 wave64 (512 threads) as 2 (M) x 4 (N);
//     each wave owns a 128x64 output tile held as four 64x32 quadrants
//     (8 v_mfma_f32_16x16x32_bf16 accumulators each = 128 accumulator VGPRs);
//   * operands reach LDS by global_load_lds (LDS-DMA, 16 B per lane, per-lane
//     source address -> gathers for free; out-of-range lanes read a 16-byte zero
//     page, which is how padding pixels, K tails and M/N tails become zeros);
//     a K-tile is four 16 KB half-tiles (A rows 0-127 / 128-255, B rows 0-127 /
//     128-255), two LDS buffers = 128 KB;
//   * every K-tile is computed in 4 phases, one quadrant each:
//       {ds_read the new fragments, issue one half-tile prefetch,
//        s_barrier, lgkmcnt(0), 16 MFMA (setprio 1), s_barrier};
//     the prefetch stays in flight across barriers (counted vmcnt(6) twice per
//     2 K-tiles, never vmcnt(0) in steady state), 3 half-tiles ahead;
//   * wave quadrants are interleaved (rows wm*64 and 128+wm*64, cols wn*32 and
//     128+wn*32) so each phase reads exactly one A half and/or one B half, which
//     is what lets a half-tile be restaged one phase after its last read;
//   * LDS images: reduction-contiguous operands as 16x32 subtiles of 1 KB with
//     the st_16x32 swizzle (byte bit 5 ^= bit 9), read by ds_read_b128;
//     reduction-outer operands as [64 k][128] rows of 256 B with an XOR chunk
//     swizzle, read by ds_read_b64_tr_b16 (hardware transpose).  Both swizzles
//     are applied on the DMA SOURCE address and on the read, so the DMA image
//     stays lane-linear and every fragment read is conflict-free;
//   * split-K over blockIdx.y with fp32 partial slabs reduced (with the
//     epilogue) by a second kernel; XCD-aware bijective block remap.
#include "ddl_common.h"

#include <cstdlib>
#include <mutex>

namespace {

#ifndef DDL_STAGGER
#define DDL_STAGGER 1
#endif
#ifndef DDL_GROUP_M
#define DDL_GROUP_M 8      // tile rows per L2 group (tile order inside an XCD's share)
#endif
// Retire depth of the operand DMA (A/B variants, csrc/bench/gemm_stamps.cpp, profiles/gemm_stamps_dr*.log):
//   0: the whole E / O tile is waited for at phases 4 / 8 (three half-tiles in flight);
//   1: each half-tile is waited for in the phase right before its first read (five in flight,
//      runtime-counted waits) -- measured 1.5-2.2x SLOWER (the counted-wait branches), kept for A/B;
//   2 (default): phases 4 / 8 retire three halves, the fourth (staged last) two phases later --
//      constant waits; neutral on 256-wide tiles, 10-15 % faster on 256 x 192 ones.
#ifndef DDL_DEEP_RETIRE
#define DDL_DEEP_RETIRE 2
#endif
// Phases 1 / 5 issue the B fragments of phases 2 / 6 (quadrant (0,1)) right after their own reads
// complete, so they land under that phase's MFMAs: the halves they read (E-B1 / O-B1) were retired
// two phases earlier and are restaged only at phases 4 / 8; fb1 is free from phase 7 / 3 on.
// Phases 2 / 6 then issue no fragment reads.  (DR 0 / 2 main loops, B k-contiguous only: PF_B1 in
// gemm_big_k; 0 = read in phases 2 / 6)
#ifndef DDL_PREFETCH_B1
#define DDL_PREFETCH_B1 1
#endif
#ifndef DDL_GEMM_EPI_LDS_CODE
#define DDL_GEMM_EPI_LDS_CODE 0   // whole-row LDS epilogue experiment (epi_lds_bf16): not compiled in
#endif
constexpr int EP_LD = 132;   // epilogue LDS row stride (floats)
constexpr int TB = 256, BK = 64, NTH = 512;
constexpr int HALF = 128 * 64 * 2;   // 16 KB half-tile

enum Layout { KC = 0, KO = 1, CONV = 2, CONVW = 3 };
enum Act { ACT_NONE = 0, ACT_GELU = 1, ACT_RELU = 2, ACT_TANH = 3, ACT_DGELU = 4, ACT_BNB = 5 };

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_v4;

struct ConvDesc {
    int N, H, W, C;
    int P, Q;
    int stride, h_off, w_off, h_step, w_step;
    int R, S;
    FastDiv fd_PQ, fd_Q, fd_C, fd_S;
    int OH, OW, ostep, oa, ob;
};

struct BigParams {
    const bf16_t* A;
    const bf16_t* B;
    long lda, ldb;
    void* C;
    long ldc;
    int M, N, K;
    const void* bias;
    int bias_bf16;
    int act;
    bf16_t* aux;
    const bf16_t* res;
    int accumulate;
    int out_f32;
    int splits, kt_per_split;
    long split_stride;
    int row_remap;
    const bf16_t* zero;       // >= 16 zero bytes
    float* colstats;          // BN statistics partials of the bf16 output: [tile_m][2][N]
    ConvDesc cd;
    int tiles_m, tiles_n;
    int ek;                   // register-epilogue variant (EK_*), set by the launcher
    int behind_mask;          // store-behind beyond plain bf16 tiles: BEHIND_* bits (DDL_GEMM_BEHIND)
    int epi_lds;              // DDL_GEMM_EPI_LDS=1: plain bf16 tiles stored as whole rows through LDS
    const uint8_t* bn_mask;   // ACT_BNB: BatchNorm backward reduction fused into the dgrad (gemm.hip Params)
    const float* bn_mean;
    const float* bn_istd;
    int* sched;               // persistent grid: per-XCD tile tickets (null: static tile striding)
    int xsplit;               // split-K on a 1-D grid whose XCDs run contiguous (split, tile) runs
    int part_bf16;            // split-K partial slabs stored as bf16 (DDL_GEMM_PART_BF16, default on)
    int zero_b1;              // 256 x 192 NT tiles: unused B rows from the zero page (DDL_GEMM_ZB1, default on)
    int wg_tbl;               // gemm_wg_k CONVW: output-pixel row table in LDS (the split's rows fit; host)
};
// tile-ticket slot layout: 8 per-XCD counters + one exit counter, 128 B apart
constexpr int SCHED_STRIDE = 32;
enum BehindBits { BEHIND_BIAS = 1, BEHIND_GELU = 2, BEHIND_RES = 4 };
enum EpiKind { EK_GEN = 0, EK_BF16 = 1, EK_F32 = 2, EK_GELU = 3, EK_DGELU = 4, EK_BNB = 5, EK_BNBC = 6 };

__device__ __forceinline__ int half_off(int buf, int x, int h) { return ((buf * 2 + x) * 2 + h) * HALF; }
__device__ __forceinline__ int swz_kc(int b) { return b ^ (((b >> 9) & 1) << 5); }
__device__ __forceinline__ int swz_ko(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }

__device__ __forceinline__ void glds(const bf16_t* g, char* dst) {
    __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)dst, 16, 0, 0);
}

// pixel decomposition of a GEMM row m (conv): image pointer + top-left input coords
struct Pix {
    const bf16_t* img;
    int hb, wb;
    bool ok;
};
__device__ __forceinline__ Pix decompose(const ConvDesc& cd, const bf16_t* base, int m, int mlimit) {
    Pix px;
    px.ok = m < mlimit;
    const int mm = px.ok ? m : 0;
    const int n = (int)fdiv((uint32_t)mm, cd.fd_PQ);
    const int rem = mm - n * cd.P * cd.Q;
    const int pp = (int)fdiv((uint32_t)rem, cd.fd_Q);
    const int qq = rem - pp * cd.Q;
    px.hb = pp * cd.stride + cd.h_off;
    px.wb = qq * cd.stride + cd.w_off;
    px.img = base + (long)n * cd.H * cd.W * cd.C;
    return px;
}
__device__ __forceinline__ void tap_of(const ConvDesc& cd, int k, int& dh, int& dw, int& ci) {
    const int tap = (int)fdiv((uint32_t)k, cd.fd_C);
    ci = k - tap * cd.C;
    const int rr = (int)fdiv((uint32_t)tap, cd.fd_S);
    const int ss = tap - rr * cd.S;
    dh = rr * cd.h_step;
    dw = ss * cd.w_step;
}

// ------------------------------------------------------------------ operand staging
// Per-lane source pointers are computed once (init) so a stage costs a 64-bit
// add and a select per DMA: the non-MFMA segment between barriers is on the
// critical path of the 8-phase schedule.  Out-of-range lanes point at the zero
// page with a zero stride.
template <int L, bool IS_A, bool KTAIL>
struct Stager {
    const bf16_t* base;
    long ld;
    int rows;        // extent of this operand's M (A) / N (B) side
    int K;
    int r0;          // tile origin on the M / N side
    const bf16_t* lp[2];   // KC / KO: lane pointer for half 0 / 1 at K-tile 0, sub j = 0
    bool lok[2];
    Pix px[2];       // CONV: this lane's row in half 0 / half 1
    int kcol;        // KC/CONV: lane's k offset inside a subtile (8 c); KO/CONVW: unused
    bool zero_h1;    // KC B of a 256 x 192 tile: this wave's rows of half 1 lie past the tile (zero page)

    // n192: a 192-wide B tile (N192).  Its second 128-row half holds 64 useful rows, those of waves
    // 0-3; waves 4-7 stage theirs from the zero page (every lane one 16-byte address: one cache
    // line per instruction instead of 1 KB of operand rows) -- the same DMA count per wave, so the
    // counted vmcnt waits are unchanged, and 1/8 fewer operand bytes per k-tile through L2.
    __device__ __forceinline__ void init(const BigParams& p, int origin, bool n192 = false) {
        base = IS_A ? p.A : p.B;
        ld = IS_A ? p.lda : p.ldb;
        rows = IS_A ? p.M : p.N;
        K = p.K;
        r0 = origin;
        const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
        zero_h1 = L == KC && !IS_A && n192 && w >= 4;
        if (L == KC || L == CONV) {
            const int lb = swz_kc(l * 16);
            const int r = lb >> 6;
            kcol = ((lb >> 4) & 3) * 8;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int row = r0 + h * 128 + w * 16 + r;
                if (L == KC) {
                    // rows past the edge re-read the last row: their results are never stored
                    lok[h] = row < rows;
                    lp[h] = base + (long)(lok[h] ? row : rows - 1) * ld + kcol;
                } else {
                    px[h] = decompose(p.cd, base, row, rows);
                    // padding / out-of-range rows: coordinates that fail every bounds check
                    if (!px[h].ok) px[h].hb = -(1 << 20);
                    lp[h] = px[h].img + ((long)px[h].hb * p.cd.W + px[h].wb) * p.cd.C + kcol;
                }
            }
        } else if (L == KO) {
            const int krow = (w * 2) * 4 + (l >> 4);      // sub j = 0; j = 1 adds 4 rows
            const int c = (l & 15) ^ swz_ko(krow);         // same swizzle for krow + 4 (bits 0,1,3 unchanged)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int col = r0 + h * 128 + 8 * c;
                lok[h] = col < rows;
                lp[h] = base + (long)krow * ld + (lok[h] ? col : ((rows - 1) & ~7));
            }
        }
    }

    // half-tile h of K-tile kt (kt < kt_end: the caller never stages padding
    // tiles).  Without KTAIL the KC / KO paths are a 64-bit add of a uniform
    // offset per DMA; the K-tail variant swaps lanes past K onto the zero page.
    __device__ __forceinline__ void stage(const BigParams& p, char* smem, int buf, int h, int kt) {
        // (scalar wave index: the LDS-DMA destinations are SGPR values for M0, no v_readfirstlane per DMA)
        const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
        char* hbase = smem + half_off(buf, IS_A ? 0 : 1, h);
        const bool ktail = KTAIL && (kt + 1) * BK > K;       // uniform: partial last tile
        if (L == KC) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int off = kt * BK + j * 32;
                const bf16_t* g = lp[h] + off;
                if (ktail) g = (off + kcol < K) ? g : p.zero;
                if (!IS_A && h == 1 && zero_h1) g = p.zero;
                glds(g, hbase + (w * 2 + j) * 1024);
            }
        } else if (L == KO) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const bf16_t* g = lp[h] + (long)(kt * BK + j * 4) * ld;
                if (ktail) g = (kt * BK + j * 4 + (w * 2) * 4 + (l >> 4) < K) ? g : p.zero;
                glds(g, hbase + (w * 2 + j) * 1024);
            }
        } else if (L == CONV) {
            const Pix& x = px[h];
            if (!KTAIL) {
                // C % 64 == 0: the whole K-tile lies in one (r, s) tap -> uniform offset
                int dh, dw, ci;
                tap_of(p.cd, kt * BK, dh, dw, ci);
                const long toff = ((long)dh * p.cd.W + dw) * p.cd.C + ci;
                const bool ok = (unsigned)(x.hb + dh) < (unsigned)p.cd.H && (unsigned)(x.wb + dw) < (unsigned)p.cd.W;
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    glds(ok ? lp[h] + toff + j * 32 : p.zero, hbase + (w * 2 + j) * 1024);
            } else {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int k = kt * BK + j * 32 + kcol;
                    int dh, dw, ci;
                    tap_of(p.cd, k < K ? k : 0, dh, dw, ci);
                    const int hh = x.hb + dh, ww = x.wb + dw;
                    const bool ok = k < K && (unsigned)hh < (unsigned)p.cd.H && (unsigned)ww < (unsigned)p.cd.W;
                    glds(ok ? x.img + ((long)hh * p.cd.W + ww) * p.cd.C + ci : p.zero, hbase + (w * 2 + j) * 1024);
                }
            }
        } else {   // CONVW: reduction rows are output pixels, columns are (tap, channel)
            const int pc = l & 15;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int krow = (w * 2 + j) * 4 + (l >> 4);
                const int c = pc ^ swz_ko(krow);
                const int col = r0 + h * 128 + 8 * c;
                const int k = kt * BK + krow;
                const bf16_t* g = p.zero;
                if (k < K && col < rows) {
                    int dh, dw, ci;
                    tap_of(p.cd, col, dh, dw, ci);
                    const Pix x = decompose(p.cd, base, k, K);
                    const int hh = x.hb + dh, ww = x.wb + dw;
                    if ((unsigned)hh < (unsigned)p.cd.H && (unsigned)ww < (unsigned)p.cd.W)
                        g = x.img + ((long)hh * p.cd.W + ww) * p.cd.C + ci;
                }
                glds(g, hbase + (w * 2 + j) * 1024);
            }
        }
    }
};

// Transposed LDS read through a restrict-qualified parameter: inlined, the read
// carries alias-scope metadata, which is what keeps the compiler's LDS-DMA tracking
// from putting an `s_waitcnt vmcnt(0)` in front of every ds_read_b64_tr_b16 (a bare
// builtin read has no alias info, so it waited out ALL in-flight operand DMA -- the
// whole 3-half-tile prefetch of the reduction-outer (NN / TN) kernels, every phase).
// The schedule's own counted vmcnt waits + barriers order DMA and reads.
__device__ __forceinline__ s16x4 ds_read_tr(lds_v4* __restrict__ p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(p);
}

// fragment: operand rows rbase..rbase+15 of half h, k = 32 kk + 8 (lane>>4) + 0..7
template <int L>
__device__ __forceinline__ bf16x8 frag(const char* hbase, int rbase, int kk) {
    const int l = threadIdx.x & 63;
    if (L == KC || L == CONV) {
        const int pb = swz_kc((l & 15) * 64 + (l >> 4) * 16);
        return *reinterpret_cast<const bf16x8*>(hbase + ((rbase >> 4) * 2 + kk) * 1024 + pb);
    } else {
        const int g = l >> 4, q = (l >> 2) & 3, pq = l & 3;
        const int col = rbase + 4 * pq;
        const int chunk = col >> 3;
        const int ra = kk * 32 + 8 * g + q, rb = ra + 4;
        const char* pa = hbase + ra * 256 + ((chunk ^ swz_ko(ra)) << 4) + (pq & 1) * 8;
        const char* pb = hbase + rb * 256 + ((chunk ^ swz_ko(rb)) << 4) + (pq & 1) * 8;
        s16x4 lo = ds_read_tr((lds_v4*)pa);
        s16x4 hi = ds_read_tr((lds_v4*)pb);
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, r);
    }
}

#define BARRIER() __builtin_amdgcn_s_barrier()
// End of a read phase.  With the staggered wave groups a half-tile may be
// restaged by the other group in the very next phase, so this wave's fragment
// reads must have completed BEFORE it arrives at the barrier (WAR); the wait
// costs nothing visible because the other group is in its MFMA cluster.
#if DDL_STAGGER
#define READS_DONE_BARRIER() do { LGKM0(); BARRIER(); } while (0)
#else
#define READS_DONE_BARRIER() do { BARRIER(); LGKM0(); } while (0)
#endif
#define LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
#define VM6() asm volatile("s_waitcnt vmcnt(6)" ::: "memory")
#define VMN(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
#define VM0() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")

// Diagnostic build only (-DDDL_GEMM_STAMPS, csrc/bench/gemm_stamps.cpp): waves 0 and 4 record
// s_memrealtime / s_memtime at four points of every tile (start, main loop start / end,
// epilogue issued) into a buffer of their own; never compiled into the library.
#ifdef DDL_GEMM_STAMPS
__device__ unsigned long long* g_stamps;
constexpr int STAMP_TILES = 16;
#define STAMP(ev)                                                                                           \
    do {                                                                                                    \
        if ((threadIdx.x & 255) == 0 && stamp_ti < STAMP_TILES) {                                            \
            const unsigned long long rt = __builtin_amdgcn_s_memrealtime(), ct = __builtin_amdgcn_s_memtime(); \
            unsigned long long* d = g_stamps + ((((long)blockIdx.y * gridDim.x + blockIdx.x) * STAMP_TILES + stamp_ti) * 2 + \
                                                (threadIdx.x >> 8)) * 8 + (ev) * 2;                           \
            d[0] = rt;                                                                                      \
            d[1] = ct;                                                                                      \
        }                                                                                                   \
    } while (0)
__device__ unsigned long long* g_kstamps;   // [block][k-tile pair < 32]: first tile only, wave 0
// (a store in wave 0's vector-memory stream shifts its counted vmcnt waits: off unless asked for)
#ifdef DDL_GEMM_KSTAMPS
#define KSTAMP(it)                                                                                          \
    do {                                                                                                    \
        if (threadIdx.x == 0 && stamp_ti == 0 && (it) < 32)                                                 \
            g_kstamps[((long)blockIdx.y * gridDim.x + blockIdx.x) * 32 + (it)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define KSTAMP(it) do {} while (0)
#endif
#else
#define STAMP(ev) do {} while (0)
#define KSTAMP(it) do {} while (0)
#endif

__device__ __forceinline__ float act_fn(float v, int act) {
    switch (act) {
        case ACT_GELU: return gelu_erf(v);
        case ACT_RELU: return fmaxf(v, 0.f);
        case ACT_TANH: return tanhf(v);
        default: return v;
    }
}

__device__ __forceinline__ long out_row(const BigParams& p, int m) {
    if (!p.row_remap) return m;
    const ConvDesc& cd = p.cd;
    const int n = (int)fdiv((uint32_t)m, cd.fd_PQ);
    const int rem = m - n * cd.P * cd.Q;
    const int pp = (int)fdiv((uint32_t)rem, cd.fd_Q);
    const int qq = rem - pp * cd.Q;
    return ((long)n * cd.OH + pp * cd.ostep + cd.oa) * cd.OW + qq * cd.ostep + cd.ob;
}

template <typename T>
__device__ __forceinline__ void load4g(const T* ptr, bool full, int nvalid, float* o) {
    if (full) load4(ptr, o);
    else {
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = r < nvalid ? to_f(ptr[r]) : 0.f;
    }
}
template <typename T>
__device__ __forceinline__ void store4g(T* ptr, bool full, int nvalid, const float* v) {
    if (full) store4(ptr, v);
    else {
#pragma unroll
        for (int r = 0; r < 4; ++r) if (r < nvalid) ptr[r] = from_f<T>(v[r]);
    }
}

// bias / residual / activation / accumulate and the final store of 4 columns
__device__ __forceinline__ void epilogue4(const BigParams& p, long orow, int n, float* v) {
    const bool full = n + 3 < p.N;
    const int nv = p.N - n;
    if (p.bias) {
        float bv[4];
        if (p.bias_bf16) load4g((const bf16_t*)p.bias + n, full, nv, bv);
        else load4g((const float*)p.bias + n, full, nv, bv);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bv[r];
    }
    if (p.res) {
        float rv[4];
        load4g(p.res + orow * p.ldc + n, full, nv, rv);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += rv[r];
    }
    if (p.act == ACT_DGELU) {
        float z[4];
        load4g(p.aux + orow * p.ldc + n, full, nv, z);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] *= gelu_erf_grad(z[r]);
    } else if (p.act != ACT_NONE) {
        if (p.aux) store4g(p.aux + orow * p.ldc + n, full, nv, v);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = act_fn(v[r], p.act);
    }
    if (p.out_f32) {
        float* cp = (float*)p.C + orow * p.ldc + n;
        if (p.accumulate) {
            float o[4];
            load4g(cp, full, nv, o);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += o[r];
        }
        store4g(cp, full, nv, v);
    } else {
        bf16_t* cp = (bf16_t*)p.C + orow * p.ldc + n;
        if (p.accumulate) {
            float o[4];
            load4g(cp, full, nv, o);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += o[r];
        }
        store4g(cp, full, nv, v);
    }
}


// Direct epilogue site: the MFMA output layout gives a lane 4 consecutive
// columns of one row, so a site is finished in registers and written with one
// 8-byte (bf16) or 16-byte (fp32) store -- no LDS round trip, which is what lets
// a persistent block restage the next tile's operands while this tile drains.
// Covers bias / residual / ReLU / GELU (+pre-activation) / accumulate / fp32 /
// split-K partial outputs; tanh, dGELU and row remap take the LDS-staged epilogue.
// `fin` receives the four values as stored (for column statistics of the output)
template <bool PB = false>
__device__ __forceinline__ void direct4(const BigParams& p, int m, int n, const f32x4& a, int split, float* fin) {
    if (m >= p.M || n >= p.N) return;
    const bool full = n + 3 < p.N;
    const int nv = p.N - n;
    float v[4] = {a[0], a[1], a[2], a[3]};
    if (p.splits > 1) {
        if constexpr (PB) store4g((bf16_t*)p.C + split * p.split_stride + (long)m * p.ldc + n, full, nv, v);
        else store4g((float*)p.C + split * p.split_stride + (long)m * p.ldc + n, full, nv, v);
        return;
    }
    if (p.bias) {
        float bv[4];
        if (p.bias_bf16) load4g((const bf16_t*)p.bias + n, full, nv, bv);
        else load4g((const float*)p.bias + n, full, nv, bv);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bv[r];
    }
    if (p.res) {
        float rv[4];
        load4g(p.res + (long)m * p.ldc + n, full, nv, rv);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += rv[r];
    }
    if (p.act == ACT_RELU) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
    } else if (p.act == ACT_GELU) {
        if (p.aux) store4g(p.aux + (long)m * p.ldc + n, full, nv, v);   // pre-activation for the backward
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = gelu_erf(v[r]);
    } else if (p.act == ACT_DGELU) {
        float z[4];
        load4g(p.aux + (long)m * p.ldc + n, full, nv, z);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] *= gelu_erf_grad(z[r]);
    }
    if (p.out_f32) {
        float* cp = (float*)p.C + (long)m * p.ldc + n;
        if (p.accumulate) {
            float o[4];
            load4g(cp, full, nv, o);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += o[r];
        }
        store4g(cp, full, nv, v);
    } else {
        bf16_t* cp = (bf16_t*)p.C + (long)m * p.ldc + n;
        if (p.accumulate) {
            float o[4];
            load4g(cp, full, nv, o);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += o[r];
        }
        store4g(cp, full, nv, v);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) fin[r] = v[r];
}

// Register epilogue of one 256x256 tile.  Lane layout: acc[qm][qn][i][j] holds
// row m0 + qm*128 + wm*64 + i*16 + (lane & 15), columns n0 + qn*128 + wn*32 +
// j*16 + 4*(lane >> 4) .. +3.
//   EK_BF16: interior tile, bf16 out, optional bf16 bias / residual -- one 16-byte store per
//            two sites (N, ldc % 8 == 0)
//   EK_GELU: interior tile, bf16 out = GELU(acc + bf16 bias), pre-activation to aux (likewise)
//   EK_DGELU: interior tile, bf16 out = acc * GELU'(aux) (+ column sums for the bias gradient), pair
//             stores like EK_BF16 (N, ldc % 8 == 0)
//   EK_F32 : interior tile, fp32 split-K partial or fp32 out (+accumulate) -- one 16-byte store
//   EK_GEN : anything direct4 covers, with bounds checks (edge tiles)
// With colstats (EK_BF16 / EK_GEN) the BatchNorm statistics of the bf16 output --
// what BN will read -- are summed per lane over its 8 rows, then over the 16
// lanes holding the same columns; one partial row per (tile, wave row).
// Column of an accumulator block: quadrant qn, 16-column block j of wave column wn.  A 192-wide
// N tile (N192) keeps quadrant 0 as is (128 columns, 32 per wave) and gives each wave ONE 16-column
// block of quadrant 1 (64 columns): acc[.][1][.][1] is not used.
template <bool N192>
__device__ __forceinline__ int col_base(int n0, int qn, int wn, int j) {
    return n0 + qn * 128 + ((N192 && qn) ? wn * 16 : wn * 32 + j * 16);
}

// HOIST: the residual / pre-activation loads of all column groups up front (off in the weight-gradient
// kernels, whose only bf16 tiles are rare unsplit ones: the extra registers spilled their main loop)
// PB: the split-K partials are bf16 (the weight-gradient instantiations, compile-time: a run-time
// choice between two store paths spilled 128 scratch ops into their MFMA main loops, and so did
// a bf16 path in the other kernels' epilogues -- scripts/check_spills.py)
template <int EK, bool N192 = false, bool HOIST = true, bool PB = false>
__device__ __forceinline__ void epi_direct(const BigParams& p, f32x4 (&acc)[2][2][4][2], int m0, int n0, int tm,
                                           int wm, int wn, int lane, int split) {
    const int g4 = (lane >> 4) * 4, r16 = lane & 15;
    const bool stats = (EK == EK_BF16 || EK == EK_GEN || EK == EK_DGELU || EK == EK_BNB || EK == EK_BNBC) &&
                       p.colstats;
    // interior bf16 / GELU tiles: the bias of all four column groups up front, so no
    // load sits between this tile's stores (a load's wait also waits out every store
    // issued before it: vmcnt counts both)
    uint2 bpre[2][2];
    if ((EK == EK_BF16 || EK == EK_GELU) && p.bias) {
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                bpre[qn][j] = (N192 && qn && j) ? make_uint2(0u, 0u)
                                                : *reinterpret_cast<const uint2*>((const bf16_t*)p.bias +
                                                                                  col_base<N192>(n0, qn, wn, j) + g4);
    }
    // residual (bf16 tiles) / saved pre-activation (dGELU): ALL column groups' loads go out before
    // the first store -- per group they cost one exposed load latency each (p.C may alias them, so
    // no load can move above an earlier group's stores); 16 / 32 extra VGPRs, free after the loop
    const bf16_t* pre = EK == EK_BF16 ? p.res : (EK == EK_DGELU ? (const bf16_t*)p.aux : nullptr);
    uint2 rball[2][2][2][4];
    auto load_pre = [&](int qn, int j) {
        const int n = col_base<N192>(n0, qn, wn, j) + g4;
#pragma unroll
        for (int qm = 0; qm < 2; ++qm)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                rball[qn][j][qm][i] = *reinterpret_cast<const uint2*>(
                    pre + (long)(m0 + qm * 128 + wm * 64 + i * 16 + r16) * p.ldc + n);
    };
    if (HOIST && (EK == EK_BF16 || EK == EK_DGELU) && pre) {
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (N192 && qn && j) continue;
                load_pre(qn, j);
            }
    }
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (N192 && qn && j) continue;
            const int n = col_base<N192>(n0, qn, wn, j) + g4;
            float bv[4] = {0.f, 0.f, 0.f, 0.f}, rs[4] = {0.f, 0.f, 0.f, 0.f};
            if ((EK == EK_BF16 || EK == EK_GELU) && p.bias) {
                const uint2 b2 = bpre[qn][j];
                bv[0] = __uint_as_float(b2.x << 16);
                bv[1] = __uint_as_float(b2.x & 0xffff0000u);
                bv[2] = __uint_as_float(b2.y << 16);
                bv[3] = __uint_as_float(b2.y & 0xffff0000u);
            }
            if (EK == EK_BNB || EK == EK_BNBC) {   // BN mean / inverse std of these 4 channels
                load4(p.bn_mean + min(n, p.N - 4), bv);
                load4(p.bn_istd + min(n, p.N - 4), rs);
            }
            float cs[4] = {0.f, 0.f, 0.f, 0.f}, cq[4] = {0.f, 0.f, 0.f, 0.f};
            if (EK == EK_BNB || EK == EK_BNBC) {
                // BatchNorm backward (N % 8 == 0: a site is whole or outside): dz = (acc + res) *
                // relu_mask stored, column sums of dz and dz * xhat.  The column group's 8
                // sites issue their loads together (clamped addresses, out-of-range sites
                // dropped afterwards): one site at a time the epilogue is load-latency bound.
                const int nc = min(n, p.N - 4);
                uint2 xr[2][4], rr[2][4];
                uint32_t mb[2][4];
#pragma unroll
                for (int qm = 0; qm < 2; ++qm)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const long mc = min(m0 + qm * 128 + wm * 64 + i * 16 + r16, p.M - 1);
                        const long o = mc * p.ldc + nc;
                        xr[qm][i] = *reinterpret_cast<const uint2*>(p.aux + o);
                        rr[qm][i] = p.res ? *reinterpret_cast<const uint2*>(p.res + o) : make_uint2(0u, 0u);
                        mb[qm][i] = p.bn_mask ? (uint32_t)p.bn_mask[o >> 3] >> (nc & 4) : 0xfu;
                    }
#pragma unroll
                for (int qm = 0; qm < 2; ++qm)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int m = m0 + qm * 128 + wm * 64 + i * 16 + r16;
                        if (EK == EK_BNBC && (m >= p.M || n >= p.N)) continue;
                        const f32x4& a = acc[qm][qn][i][j];
                        const uint2 x2 = xr[qm][i], r2 = rr[qm][i];
                        const float xv[4] = {__uint_as_float(x2.x << 16), __uint_as_float(x2.x & 0xffff0000u),
                                             __uint_as_float(x2.y << 16), __uint_as_float(x2.y & 0xffff0000u)};
                        const float rv[4] = {__uint_as_float(r2.x << 16), __uint_as_float(r2.x & 0xffff0000u),
                                             __uint_as_float(r2.y << 16), __uint_as_float(r2.y & 0xffff0000u)};
                        float v[4];
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = ((mb[qm][i] >> e) & 1u) ? a[e] + rv[e] : 0.f;
                        const uint32_t lo = pack2bf(v[0], v[1]), hi = pack2bf(v[2], v[3]);
                        *reinterpret_cast<uint2*>((bf16_t*)p.C + (long)m * p.ldc + n) = make_uint2(lo, hi);
                        const float t[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                                            __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            cs[e] += t[e];
                            cq[e] += t[e] * (xv[e] - bv[e]) * rs[e];
                        }
                    }
            } else {
            // (the residual / pre-activation sites of this group were loaded above, rball; without
            // HOIST the group's 8 sites load together here, before any of its stores)
            if (!HOIST && (EK == EK_BF16 || EK == EK_DGELU) && pre) load_pre(qn, j);
            uint2 (&rb)[2][4] = rball[qn][j];
            // EK_BF16 / EK_GELU store two sites (row blocks i, i + 1) per lane as ONE 16-byte
            // store: v_permlane16_swap hands the odd lane rows (g = 1, 3) the even rows' quads
            // of row block i + 1 in exchange for theirs of row block i, so each lane holds 8
            // consecutive columns of one row (half the store instructions; 8-byte stores kept
            // the epilogue store-issue bound).  Row-block i values wait in (plo, phi) / (zlo, zhi).
            uint32_t plo = 0, phi = 0, zlo = 0, zhi = 0;
            const int wcol = col_base<N192>(n0, qn, wn, j) + (lane >> 5) * 8;   // (g >> 1) * 8
            auto store_pair = [&](void* base, uint32_t lo0, uint32_t hi0, uint32_t lo1, uint32_t hi1, int m1) {
                const auto x = __builtin_amdgcn_permlane16_swap(lo0, lo1, false, false);
                const auto y = __builtin_amdgcn_permlane16_swap(hi0, hi1, false, false);
                const int mrow = (lane & 16) ? m1 : m1 - 16;      // g odd: row block i + 1
                *reinterpret_cast<uint4*>((bf16_t*)base + (long)mrow * p.ldc + wcol) = make_uint4(x[0], y[0], x[1], y[1]);
            };
#pragma unroll
            for (int qm = 0; qm < 2; ++qm)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int m = m0 + qm * 128 + wm * 64 + i * 16 + r16;
                    const f32x4& a = acc[qm][qn][i][j];
                    if (EK == EK_BF16) {
                        float rv[4] = {0.f, 0.f, 0.f, 0.f};
                        if (p.res) {
                            const uint2 r2 = rb[qm][i];
                            rv[0] = __uint_as_float(r2.x << 16);
                            rv[1] = __uint_as_float(r2.x & 0xffff0000u);
                            rv[2] = __uint_as_float(r2.y << 16);
                            rv[3] = __uint_as_float(r2.y & 0xffff0000u);
                        }
                        const uint32_t lo = pack2bf(a[0] + bv[0] + rv[0], a[1] + bv[1] + rv[1]);
                        const uint32_t hi = pack2bf(a[2] + bv[2] + rv[2], a[3] + bv[3] + rv[3]);
                        if ((i & 1) == 0) { plo = lo; phi = hi; }
                        else store_pair(p.C, plo, phi, lo, hi, m);
                        if (stats) {
                            const float t[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                                                __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                cs[e] += t[e];
                                cq[e] += t[e] * t[e];
                            }
                        }
                    } else if (EK == EK_GELU) {
                        // z = acc + bias kept for the backward (aux), y = GELU(z)
                        float z[4] = {a[0] + bv[0], a[1] + bv[1], a[2] + bv[2], a[3] + bv[3]};
                        const uint32_t zl = pack2bf(z[0], z[1]), zh = pack2bf(z[2], z[3]);
                        const f32x2_t y0 = gelu_erf2(f32x2_t{z[0], z[1]}), y1 = gelu_erf2(f32x2_t{z[2], z[3]});
                        const uint32_t yl = pack2bf(y0.x, y0.y), yh = pack2bf(y1.x, y1.y);
                        if ((i & 1) == 0) { zlo = zl; zhi = zh; plo = yl; phi = yh; }
                        else {
                            if (p.aux) store_pair(p.aux, zlo, zhi, zl, zh, m);
                            store_pair(p.C, plo, phi, yl, yh, m);
                        }
                    } else if (EK == EK_DGELU) {
                        // dZ = dH * GELU'(z) (z = the Linear's saved pre-activation), and the
                        // column sums of the stored dZ: that Linear's bias gradient
                        const long o = (long)m * p.ldc + n;
                        const uint2 z2 = rb[qm][i];
                        const float z[4] = {__uint_as_float(z2.x << 16), __uint_as_float(z2.x & 0xffff0000u),
                                            __uint_as_float(z2.y << 16), __uint_as_float(z2.y & 0xffff0000u)};
                        const f32x2_t d0 = f32x2_t{a[0], a[1]} * gelu_erf_grad2(f32x2_t{z[0], z[1]});
                        const f32x2_t d1 = f32x2_t{a[2], a[3]} * gelu_erf_grad2(f32x2_t{z[2], z[3]});
                        const uint32_t lo = pack2bf(d0.x, d0.y), hi = pack2bf(d1.x, d1.y);
                        (void)o;
                        if ((i & 1) == 0) { plo = lo; phi = hi; }
                        else store_pair(p.C, plo, phi, lo, hi, m);
                        if (stats) {
                            const float t[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                                                __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                cs[e] += t[e];
                                cq[e] += t[e] * t[e];
                            }
                        }
                    } else if (EK == EK_F32) {
                        if (p.splits > 1) {
                            if constexpr (PB)   // the weight-gradient kernels' partials are always bf16
                                *reinterpret_cast<uint2*>((bf16_t*)p.C + split * p.split_stride + (long)m * p.ldc + n) =
                                    make_uint2(pack2bf(a[0], a[1]), pack2bf(a[2], a[3]));
                            else
                                *reinterpret_cast<f32x4*>((float*)p.C + split * p.split_stride + (long)m * p.ldc + n) = a;
                        } else {
                            f32x4* cp = reinterpret_cast<f32x4*>((float*)p.C + (long)m * p.ldc + n);
                            *cp = p.accumulate ? a + *cp : a;
                        }
                    } else {
                        float fin[4] = {0.f, 0.f, 0.f, 0.f};
                        direct4<PB>(p, m, n, a, split, fin);
                        if (stats && m < p.M) {
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                const float t = n + e < p.N ? bf2f(f2bf(fin[e])) : 0.f;
                                cs[e] += t;
                                cq[e] += t * t;
                            }
                        }
                    }
                }
            }
            if (stats) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    cs[e] = row16_sum(cs[e]);
                    cq[e] = row16_sum(cq[e]);
                }
                if (r16 == 0 && n < p.N) {
                    float* row = p.colstats + (long)(tm * 2 + wm) * 2 * p.N;
                    if (EK == EK_BF16) {
                        *reinterpret_cast<f32x4*>(row + n) = (f32x4){cs[0], cs[1], cs[2], cs[3]};
                        *reinterpret_cast<f32x4*>(row + p.N + n) = (f32x4){cq[0], cq[1], cq[2], cq[3]};
                    } else {
                        store4g(row + n, n + 3 < p.N, p.N - n, cs);
                        store4g(row + p.N + n, n + 3 < p.N, p.N - n, cq);
                    }
                }
            }
        }
}

// Row-contiguous variant of the plain bf16 register epilogue (EK_BF16, no residual / statistics):
// the packed tile goes through LDS one 128-row half at a time (64 KB, XOR-swizzled 16-byte chunks
// of 512-byte rows) and every store instruction then writes whole 128-byte lines -- the register
// epilogue's stores cover 32 bytes of a line each (two waves per line).  `stage` = 64 KB of LDS no
// DMA is writing; raw barriers (a __syncthreads fence would drain in-flight LDS-DMA).
__device__ __forceinline__ void epi_lds_bf16(const BigParams& p, f32x4 (&acc)[2][2][4][2], int m0, int n0, int wm,
                                             int wn, int lane, char* stage) {
    const int g4 = (lane >> 4) * 4, r16 = lane & 15;
    float bv[2][2][4];
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (p.bias) {
                const uint2 b2 = *reinterpret_cast<const uint2*>((const bf16_t*)p.bias + n0 + qn * 128 + wn * 32 + j * 16 + g4);
                bv[qn][j][0] = __uint_as_float(b2.x << 16);
                bv[qn][j][1] = __uint_as_float(b2.x & 0xffff0000u);
                bv[qn][j][2] = __uint_as_float(b2.y << 16);
                bv[qn][j][3] = __uint_as_float(b2.y & 0xffff0000u);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) bv[qn][j][e] = 0.f;
            }
        }
    const int rc = threadIdx.x & 31, rr = threadIdx.x >> 5;    // store side: 16 rows x 32 chunks per pass
#pragma unroll
    for (int qm = 0; qm < 2; ++qm) {
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const f32x4& a = acc[qm][qn][i][j];
                    const int r = wm * 64 + i * 16 + r16;
                    const int c = qn * 128 + wn * 32 + j * 16 + g4;
                    const int off = r * 512 + (((c >> 3) ^ (r & 15)) << 4) + (c & 7) * 2;
                    *reinterpret_cast<uint2*>(stage + off) =
                        make_uint2(pack2bf(a[0] + bv[qn][j][0], a[1] + bv[qn][j][1]),
                                   pack2bf(a[2] + bv[qn][j][2], a[3] + bv[qn][j][3]));
                }
        LGKM0();
        BARRIER();
        uint4 v[8];
#pragma unroll
        for (int ps = 0; ps < 8; ++ps) {
            const int r = ps * 16 + rr;
            v[ps] = *reinterpret_cast<const uint4*>(stage + r * 512 + ((rc ^ (r & 15)) << 4));
        }
#pragma unroll
        for (int ps = 0; ps < 8; ++ps)
            *reinterpret_cast<uint4*>((bf16_t*)p.C + (long)(m0 + qm * 128 + ps * 16 + rr) * p.ldc + n0 + rc * 8) = v[ps];
        LGKM0();
        BARRIER();      // every read of this half done before the next half (or a DMA) overwrites it
    }
}

// DIRECT: epilogue from registers (direct4) and, with it, a persistent grid: a
// block walks tiles blockIdx.x, +gridDim.x, ...; after a tile's last MFMA it
// stages the next tile's first K-tile, stores this tile from registers, then
// stages the rest of the prologue, so the result stores drain under the next
// tile's loads instead of in a chip-wide burst between waves of blocks.
// BNB: the BatchNorm-backward epilogue variant (its own instantiation, so the extra
// registers it needs never weigh on the other epilogues)
// EDGE = false (DDL_GEMM_LEAN=1): every tile is interior and the epilogue kind is one of the
// lean ones (M, N multiples of 256): the bounds-checked general epilogue is not compiled in.
// Its 64-bit per-site addresses are what spills (35-72 VGPRs of scratch in the persistent
// kernels); without it the NT kernel allocates spill-free -- but runs slower (see
// edge_split_enabled), so the spills are not on the interior tiles' critical path.
// N192: 256 x 192 tiles (register epilogue only): BERT's N = 768 / 2304 GEMMs have 192 / 576
// tiles of 256 x 256 on 256 CUs (one 75 %-full round / 2.25 rounds); 192-wide tiles make that
// 256 / 768 -- whole rounds.  The B operand is still staged as two 128-row halves (the rows
// past the tile's 192 are read but never multiplied: the weight panel is L2-resident), so the
// 8-phase schedule and its DMA counts are unchanged; quadrant qn = 1 runs one 16-column block
// per wave (8 MFMAs instead of 16 per phase).
template <int LA, int LB, bool KTAIL, bool DIRECT, bool BNB = false, bool EDGE = true, bool N192 = false>
__global__ __launch_bounds__(NTH, 1) void gemm_big_k(BigParams p) {
    static_assert(!N192 || (DIRECT && !BNB), "192-wide tiles: register epilogue only");
    constexpr int TBN = N192 ? 192 : TB;
    constexpr bool WGRAD = LA == KO && LB == KO;   // TN: weight gradients (split-K fp32 / accumulate)
    // B-fragment prefetch (DDL_PREFETCH_B1) where B is k-contiguous (NT, implicit-GEMM conv forward):
    // 8192^3 NT -32 % cycles, 4096^3 -20 %; NN (transposed B reads): 4096^3 +9 % in isolation but
    // +0.3 % on the BERT-base step (DDL_PREFETCH_B1_NN); never TN (the extra live range spilled its loop)
#ifndef DDL_PREFETCH_B1_NN
#define DDL_PREFETCH_B1_NN 1   // NN too: BERT-base same-box +0.3 % (9,024 vs 8,997 / 9,000, two pairs)
#endif
    constexpr bool PF_B1 = DDL_PREFETCH_B1 && (LB == KC || (DDL_PREFETCH_B1_NN && LA == KC && LB == KO));
    // (+16 bytes: the tile ticket.  One LDS object only: a second __shared__ variable
    // makes the compiler's LDS-DMA alias tracking wait vmcnt(0) before fragment reads)
    __shared__ __attribute__((aligned(16))) char smem[8 * HALF + 16];
    const int nwg = p.tiles_m * p.tiles_n;
    int tm, tn, m0, n0;
    // XCD-aware bijective remap: an XCD (blockIdx & 7) owns a contiguous range of
    // tile ids; a persistent block's later tiles keep its XCD (gridDim.x % 8 == 0)
    auto coords = [&](int bid, bool remap = true) {
        const int xcd = bid & 7, qn_ = nwg >> 3, rn = nwg & 7;
        const int wg = remap ? (xcd < rn ? xcd * (qn_ + 1) : rn * (qn_ + 1) + (xcd - rn) * qn_) + (bid >> 3) : bid;
        // grouped order: consecutive tiles (the ones an XCD runs together) cover a
        // GROUP_M x k block of tiles instead of one long row, so the A and B panels
        // they stream stay L2-resident at large M, N
        const int per_group = DDL_GROUP_M * p.tiles_n;
        const int grp = wg / per_group, first_m = grp * DDL_GROUP_M;
        const int gsz = min(p.tiles_m - first_m, DDL_GROUP_M);
        const int wl = wg - grp * per_group;
        tm = first_m + wl % gsz;
        tn = wl / gsz;
        m0 = tm * TB;
        n0 = tn * TBN;
    };
    // Tile order.  Static: block b walks tiles b, b + gridDim.x, ... (same XCD range).
    // Dynamic (p.sched, gridDim.x % 8 == 0): the first tile is static, every further one
    // a ticket from this XCD's counter, so a block that starts late (its CU held by a
    // concurrent RCCL collective, whose resident blocks leave no room for this kernel's
    // 256-VGPR waves) takes fewer tiles instead of extending the GEMM by its whole static
    // share.  Thread 0 asks for the ticket of the tile after next once a tile's
    // coordinates are known, before that tile's prologue loads, and publishes it through
    // LDS after the prologue wait that retired it (the main loop's barriers order the
    // publication before the read at the end of the tile).
    // (not in the BatchNorm-backward instantiations: their register budget has no room,
    // and their dgrad shapes have fewer tiles than CUs)
    constexpr bool DYN = DIRECT && !BNB;
    int& s_tick = *reinterpret_cast<int*>(smem + 8 * HALF);
    int tick = 0;
    auto ask = [&]() {
        if (DYN && p.sched && threadIdx.x == 0) tick = atomicAdd(p.sched + (blockIdx.x & 7) * SCHED_STRIDE, 1);
    };
    auto publish = [&]() {
        if (DYN && p.sched && threadIdx.x == 0) s_tick = tick;
    };
    int vt = blockIdx.x, split = blockIdx.y;
#ifdef DDL_GEMM_STAMPS
    int stamp_ti = 0;
#endif
    if (p.xsplit) {
        // split-K (one block per (tile, split), a 1-D grid): workgroups go to the XCDs round-robin,
        // so XCD x gets blocks x, x + 8, ...; they are given a CONTIGUOUS run of the split-major
        // (split, tile) order -- mostly one split's k-range over neighbouring tiles, whose A / B
        // panel rows then come from HBM once into that XCD's L2 and serve every tile that reads
        // them (with blockIdx.y = split, an XCD's blocks spread over all splits: the TN weight
        // gradients streamed ~5x their unique bytes at the HBM rate)
        const int n = nwg * p.splits, xcd = blockIdx.x & 7, qn_ = n >> 3, rn = n & 7;
        const int q = (xcd < rn ? xcd * (qn_ + 1) : rn * (qn_ + 1) + (xcd - rn) * qn_) + (int)(blockIdx.x >> 3);
        split = q / nwg;
        vt = q - split * nwg;
        coords(vt, false);
    } else {
        coords(vt);
    }
    ask();
    STAMP(0);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wm = w >> 2, wn = w & 3;
    const int nK_total = (p.K + BK - 1) / BK;
    const int kt0 = split * p.kt_per_split;
    const int kt_end = min(nK_total, kt0 + p.kt_per_split);
    const int nK = kt_end - kt0;              // may be odd: the last pair then skips its O half

    Stager<LA, true, KTAIL> sa;
    Stager<LB, false, KTAIL> sb;
    sa.init(p, m0);
    sb.init(p, n0, N192 && p.zero_b1);

    f32x4 acc[2][2][4][2];
    auto zero_acc = [&]() {
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[a][b][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    };
    zero_acc();

    bf16x8 fa[4][2], fb0[2][2], fb1[2][2];
    auto readA = [&](int buf, int qm) {
        const char* hb = smem + half_off(buf, 0, qm);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
#ifdef DDL_DIAG_A_ROWREADS
                // diagnostic builds only (wrong results): A fragments by row reads whatever the layout
                fa[i][kk] = frag<KC>(hb, wm * 64 + i * 16, kk);
#else
                fa[i][kk] = frag<LA>(hb, wm * 64 + i * 16, kk);
#endif
            }
    };
    auto readB = [&](int buf, int qn, bf16x8 (&fb)[2][2]) {
        const char* hb = smem + half_off(buf, 1, qn);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (N192 && qn && j) continue;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) fb[j][kk] = frag<LB>(hb, (N192 && qn) ? wn * 16 : wn * 32 + j * 16, kk);
        }
    };
    auto mma = [&](int qm, int qn, bf16x8 (&fb)[2][2]) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    if (!(N192 && qn && j)) acc[qm][qn][i][j] =
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][kk], fa[i][kk], acc[qm][qn][i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };

    // phases 1-4: the four quarter-products of the E buffer (tile kE); stO1
    // stages the last O half of tile kE+1, more stages tile kE+2 into E
    // phase-4 wait that retires tile O: normally VM6 (the three stages issued after O's
    // last half); right after a store-behind epilogue O was staged whole BEFORE the
    // tile's epilogue stores, so it retires with those stores still in flight: `hold`
    // = stores + 6 (a lower bound of the ops issued after O)
    auto vm_retire_o = [&](int hold) {
        if (hold == 22) asm volatile("s_waitcnt vmcnt(22)" ::: "memory");
        else if (hold == 30) asm volatile("s_waitcnt vmcnt(30)" ::: "memory");
        else if (hold == 38) asm volatile("s_waitcnt vmcnt(38)" ::: "memory");
        else VM6();
    };
#if DDL_DEEP_RETIRE == 1
    // Counted waits from the stage-issue history: bit s of `cm` = stage slot s (the DMA of
    // phase s + 1) of this iteration went out, `pm` = the previous iteration's slots (or the
    // prologue's: E -> slots 1-4, O A0 / B0 / B1 -> slots 5-7).  Stage order per iteration:
    // 1 O-A1(kO)  2 E-A0  3 E-B0  4 E-B1  5 E-A1 (kE+2)  6 O-A0  7 O-B0  8 O-B1 (kO+2).  A wait
    // that retires the half of slot t leaves the ops younger than it in flight: 2 per issued
    // slot after t (every wave issues 2 DMAs per half).  Half -> wait (the phase before its
    // first read): E-B1 phase 1, E-A1 phase 2, O-A0/B0 phase 4, O-B1 phase 5, O-A1 phase 6,
    // E-A0/B0 (next tile) phase 8.
    auto vm_younger = [&](int n) {
        switch (n) {
            case 10: VMN(10); break;
            case 8: VMN(8); break;
            case 6: VMN(6); break;
            case 4: VMN(4); break;
            case 2: VMN(2); break;
            default: VM0(); break;
        }
    };
    auto younger = [&](unsigned pm, unsigned cm, int t, int q) -> int {   // slots t+1 .. q
        const unsigned h = pm | (cm << 8);
        const unsigned m = ((1u << (q + 1)) - 1u) & ~((1u << (t + 1)) - 1u);
        return 2 * __builtin_popcount(h & m);
    };
    // fresh: the first pair after a store-behind epilogue -- E retired with the stores, O staged
    // whole before them: retired at phase 4 by `hold` (vm_retire_o), no per-half waits
    auto phasesE = [&](int kE, bool stO1, bool more, unsigned pm, unsigned& cm, bool fresh, int hold, bool hasO) {
        // phase 1: E (0,0)
        readA(0, 0);
        readB(0, 0, fb0);
        if (stO1) { sa.stage(p, smem, 1, 1, kE + 1); cm |= 1u; }
        if (!fresh) vm_younger(younger(pm, cm, 3, 8));          // E-B1(kE)
        READS_DONE_BARRIER();
        mma(0, 0, fb0);
        BARRIER();
        // phase 2: E (0,1)
        readB(0, 1, fb1);
        if (more) { sa.stage(p, smem, 0, 0, kE + 2); cm |= 2u; }
        if (!fresh) vm_younger(younger(pm, cm, 4, 9));          // E-A1(kE)
        READS_DONE_BARRIER();
        mma(0, 1, fb1);
        BARRIER();
        // phase 3: E (1,1)
        readA(0, 1);
        if (more) { sb.stage(p, smem, 0, 0, kE + 2); cm |= 4u; }
        READS_DONE_BARRIER();
        mma(1, 1, fb1);
        BARRIER();
        // phase 4: E (1,0); retire O-A0 / O-B0 (kE+1)
        if (more) { sb.stage(p, smem, 0, 1, kE + 2); cm |= 8u; }
        if (hasO) {
            if (!fresh) vm_younger(younger(pm, cm, 6, 11));
            else if (more) vm_retire_o(hold);
            else VM0();
        }
        BARRIER();
        mma(1, 0, fb0);
        BARRIER();
    };
#else
    auto phasesE = [&](int kE, bool stO1, bool more, int hold = 0, bool w2 = false) {
        // phase 1: E (0,0)
        readA(0, 0);
        readB(0, 0, fb0);
        if (stO1) sa.stage(p, smem, 1, 1, kE + 1);
        READS_DONE_BARRIER();
        if (PF_B1) readB(0, 1, fb1);   // phase 2's B fragments, under this phase's MFMAs
        mma(0, 0, fb0);
        BARRIER();
        // phase 2: E (0,1)
        if (!PF_B1) readB(0, 1, fb1);
        if (more) sa.stage(p, smem, 0, 0, kE + 2);
#if DDL_DEEP_RETIRE == 2
        // E-A1 (staged at the previous pair's phase 5) retired here, read in phase 3
        if (w2) { if (more) VMN(10); else VMN(8); }
#else
        (void)w2;
#endif
        READS_DONE_BARRIER();
        mma(0, 1, fb1);
        BARRIER();
        // phase 3: E (1,1)
        readA(0, 1);
        if (more) sb.stage(p, smem, 0, 0, kE + 2);
        READS_DONE_BARRIER();
        mma(1, 1, fb1);
        BARRIER();
        // phase 4: E (1,0); retire O(kE+1)
#if DDL_DEEP_RETIRE == 2
        // O-A0 / B0 / B1 only: O-A1 (staged at phase 1) is retired at phase 6
        if (more) { sb.stage(p, smem, 0, 1, kE + 2); if (hold) vm_retire_o(hold); else VMN(8); } else { VM0(); }
#else
        if (more) { sb.stage(p, smem, 0, 1, kE + 2); vm_retire_o(hold); } else { VM0(); }
#endif
        BARRIER();
        mma(1, 0, fb0);
        BARRIER();
    };

#endif

    // prologue, first part: E <- tile kt0 (all halves)
    auto prologueE = [&]() {
        sa.stage(p, smem, 0, 0, kt0);
        sb.stage(p, smem, 0, 0, kt0);
        sb.stage(p, smem, 0, 1, kt0);
        sa.stage(p, smem, 0, 1, kt0);
    };
    // second part: O <- tile kt0+1 (A0, B0, B1); E landed; wave groups staggered
    auto prologueO = [&]() {
        if (nK > 1) {
            sa.stage(p, smem, 1, 0, kt0 + 1);
            sb.stage(p, smem, 1, 0, kt0 + 1);
            sb.stage(p, smem, 1, 1, kt0 + 1);
#if DDL_DEEP_RETIRE == 1
            VMN(10);      // E-A0 / E-B0 only: E-B1 / E-A1 are retired at phases 1 / 2 (vm_younger)
#else
            VM6();
#endif
        } else {
            VM0();
        }
        BARRIER();
#if DDL_STAGGER
        // wave groups wm=0/1 run one barrier apart: one group's MFMA cluster
        // overlaps the other's LDS reads / DMA issue on the same SIMD
        if (wm == 1) BARRIER();
#endif
    };

    if (nK > 0) {
        prologueE();
        prologueO();
    }
    publish();
    STAMP(1);
    int hold_o = 0;     // != 0: the coming tile's O was staged before the previous tile's stores
    for (;;) {
        if (nK > 0) {
            const int pairs = nK / 2;
#if DDL_DEEP_RETIRE == 1
            unsigned pm = nK > 1 ? 0xFEu : 0x1Eu, cm = 0u;    // the prologue's slots (see vm_younger)
            for (int it = 0; it < pairs; ++it) {
                KSTAMP(it);
                const int kE = kt0 + 2 * it, kO = kE + 1;
                const bool more = kE + 2 < kt_end;
                const bool moreO = kO + 2 < kt_end;
                // first pair after a store-behind epilogue: O is already staged whole
                const bool fresh = !BNB && it == 0 && hold_o;
                phasesE(kE, !fresh, more, pm, cm, fresh, it == 0 ? hold_o : 0, true);
                // phase 5: O (0,0)
                readA(1, 0);
                readB(1, 0, fb0);
                if (more) { sa.stage(p, smem, 0, 1, kE + 2); cm |= 16u; }
                if (!fresh) vm_younger(younger(pm, cm, 7, 12));     // O-B1(kO)
                READS_DONE_BARRIER();
                mma(0, 0, fb0);
                BARRIER();
                // phase 6: O (0,1)
                readB(1, 1, fb1);
                if (moreO) { sa.stage(p, smem, 1, 0, kO + 2); cm |= 32u; }
                if (!fresh) vm_younger(younger(pm, cm, 8, 13));     // O-A1(kO)
                READS_DONE_BARRIER();
                mma(0, 1, fb1);
                BARRIER();
                // phase 7: O (1,1)
                readA(1, 1);
                if (moreO) { sb.stage(p, smem, 1, 0, kO + 2); cm |= 64u; }
                READS_DONE_BARRIER();
                mma(1, 1, fb1);
                BARRIER();
                // phase 8: O (1,0); retire E-A0 / E-B0 (kE+2)
                if (moreO) { sb.stage(p, smem, 1, 1, kO + 2); cm |= 128u; }
                if (more) vm_younger(younger(pm, cm, 10, 15));
                BARRIER();
                mma(1, 0, fb0);
                BARRIER();
                pm = cm;
                cm = 0u;
            }
            // odd tile count: the last E tile (its E-B1 / E-A1 retired at phases 1 / 2)
            if (nK & 1) phasesE(kt_end - 1, false, false, pm, cm, false, 0, false);
#else
            for (int it = 0; it < pairs; ++it) {
                KSTAMP(it);
                const int kE = kt0 + 2 * it, kO = kE + 1;
                const bool more = kE + 2 < kt_end;
                const bool moreO = kO + 2 < kt_end;
                // first pair after a store-behind epilogue: O is already staged whole
                if constexpr (BNB) phasesE(kE, true, more, 0, it > 0);
                else phasesE(kE, !(it == 0 && hold_o), more, it == 0 ? hold_o : 0, it > 0);
                // phase 5: O (0,0)
                readA(1, 0);
                readB(1, 0, fb0);
                if (more) sa.stage(p, smem, 0, 1, kE + 2);
                READS_DONE_BARRIER();
                if (PF_B1) readB(1, 1, fb1);   // O-B1 landed at phase 4
                mma(0, 0, fb0);
                BARRIER();
                // phase 6: O (0,1)
                if (!PF_B1) readB(1, 1, fb1);
                if (moreO) sa.stage(p, smem, 1, 0, kO + 2);
#if DDL_DEEP_RETIRE == 2
                if (BNB || !(it == 0 && hold_o)) {        // O-A1 (phase 1), read in phase 7
                    if (moreO) VMN(10);
                    else if (more) VMN(8);
                    else VM0();
                }
#endif
                READS_DONE_BARRIER();
                mma(0, 1, fb1);
                BARRIER();
                // phase 7: O (1,1)
                readA(1, 1);
                if (moreO) sb.stage(p, smem, 1, 0, kO + 2);
                READS_DONE_BARRIER();
                mma(1, 1, fb1);
                BARRIER();
                // phase 8: O (1,0); retire E(kE+2)
#if DDL_DEEP_RETIRE == 2
                // E-A0 / B0 / B1 only: E-A1 (phase 5) is retired at the next pair's phase 2
                if (moreO) { sb.stage(p, smem, 1, 1, kO + 2); VMN(8); } else { VM0(); }
#else
                if (moreO) { sb.stage(p, smem, 1, 1, kO + 2); VM6(); } else { VM0(); }
#endif
                BARRIER();
                mma(1, 0, fb0);
                BARRIER();
            }
            // odd tile count: the last E tile (fully landed: phase 8 waited vmcnt(0))
            if (nK & 1) phasesE(kt_end - 1, false, false);
#endif
#if DDL_STAGGER
            // realign the groups: after this barrier every wave has finished its
            // last MFMA and every fragment read, so the LDS buffers are free
            if (wm == 0) BARRIER();
#endif
        }
        STAMP(2);
        if (DIRECT) {
            // dynamic: ticket t of XCD x is its range's tile gridDim.x/8 + t, i.e. the
            // static-order id 8 * (gridDim.x/8 + t) + x
            const int vn = (DYN && p.sched) ? (int)((((gridDim.x >> 3) + s_tick) << 3) + (blockIdx.x & 7))
                                             : vt + (int)gridDim.x;
            const bool next = vn < nwg;
            const int m0c = m0, n0c = n0, tm_c = tm;
            const bool interior = !EDGE || (m0c + TB <= p.M && n0c + TBN <= p.N);
            // Store-behind: when this tile's epilogue issues a KNOWN number of vector-memory
            // ops (lean bf16 variant: one 8-byte store per site, +8 statistics stores), the
            // WHOLE next prologue (E and O halves) is issued first and only the E loads are
            // waited for -- vmcnt(6 + stores) -- so the stores drain under the next tile's
            // loads and MFMAs instead of being waited for (vmcnt retires in issue order).
            // Short-K tiles (1x1 convolutions: K = 64..256) are otherwise latency-bound on
            // load -> compute -> store-drain per tile.
            // (a residual's loads retire in order behind the next prologue's, so the counts
            // below stay upper bounds)
            // (not with 192-wide tiles: the store counts its vmcnt waits assume are the 256-wide ones)
            // whole-row stores through LDS (buffer O's 64 KB; the next prologue is issued after them)
            // (compiled in only with -DDDL_GEMM_EPI_LDS_CODE=1: its second prologue site raised the
            // register pressure enough to spill the KO operand loaders' row offsets inside the main
            // loop -- TN / NN 2x slower, profiles/gemm_spills_r04.md)
            const bool lds_epi = DDL_GEMM_EPI_LDS_CODE && !N192 && !BNB && p.epi_lds && interior && p.ek == EK_BF16 && !p.res && !p.colstats;
            const bool behind = !N192 && !lds_epi && next && nK > 0 && interior &&
                ((p.ek == EK_BF16 && (!p.bias || (p.behind_mask & BEHIND_BIAS)) &&
                  (!p.res || (p.behind_mask & BEHIND_RES))) ||
                 (p.ek == EK_GELU && (p.behind_mask & BEHIND_GELU)));
            if (next && !lds_epi) {
                coords(vn);
                ask();
                sa.init(p, m0);
                sb.init(p, n0, N192 && p.zero_b1);
                if (nK > 0) prologueE();
                if (behind && nK > 1) {
                    sa.stage(p, smem, 1, 0, kt0 + 1);
                    sb.stage(p, smem, 1, 0, kt0 + 1);
                    sb.stage(p, smem, 1, 1, kt0 + 1);
                    sa.stage(p, smem, 1, 1, kt0 + 1);   // all of O ahead of the stores (see vm_retire_o)
                }
            }
            // interior tiles take a lean variant (no bounds checks, one store per site);
            // edge tiles and the rarer epilogue options the general one
            if (BNB)   // checked on every tile: a lean interior twin spills (measured slower)
                epi_direct<EK_BNBC>(p, acc, m0c, n0c, tm_c, wm, wn, lane, split);
            else if (lds_epi) {
                epi_lds_bf16(p, acc, m0c, n0c, wm, wn, lane, smem + half_off(1, 0, 0));
                if (next) {
                    coords(vn);
                    ask();
                    sa.init(p, m0);
                    sb.init(p, n0);
                    if (nK > 0) prologueE();
                }
            } else if (interior && p.ek == EK_BF16)
                epi_direct<EK_BF16, N192, !WGRAD>(p, acc, m0c, n0c, tm_c, wm, wn, lane, split);
            else if (interior && p.ek == EK_F32)
                epi_direct<EK_F32, N192, true, WGRAD>(p, acc, m0c, n0c, tm_c, wm, wn, lane, split);
            else if (interior && p.ek == EK_GELU)
                epi_direct<EK_GELU, N192>(p, acc, m0c, n0c, tm_c, wm, wn, lane, split);
            else if (!WGRAD && interior && p.ek == EK_DGELU)   // (never a weight gradient's)
                epi_direct<EK_DGELU, N192>(p, acc, m0c, n0c, tm_c, wm, wn, lane, split);
            else if constexpr (EDGE)
                epi_direct<EK_GEN, N192, true, WGRAD>(p, acc, m0c, n0c, tm_c, wm, wn, lane, split);
            STAMP(3);
#ifdef DDL_GEMM_STAMPS
            ++stamp_ti;
            STAMP(0);
#endif
            if (!next) {
                if constexpr (DYN) break;    // the ticket slot's exit bookkeeping below the loop
                return;
            }
            zero_acc();
            hold_o = 0;
            vt = vn;
            if (nK > 0) {
                if (behind) {
                    // E landed once at most (O loads) + (epilogue stores) remain outstanding;
                    // GELU tiles store twice per site (output + pre-activation): the 6-bit
                    // counter's maximum is a stronger wait than needed, never a weaker one
                    // per wave: EK_BF16 16 pair stores (+8 statistics stores), EK_GELU 32;
                    // E retires with O (8 ops, nK > 1) and those stores younger than it
                    if (p.ek == EK_GELU) {
                        if (nK > 1) asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
                        else asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
                        hold_o = nK > 1 ? 38 : 0;
                    } else if (nK > 1) {
                        if (p.colstats) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
                        else asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
                        hold_o = p.colstats ? 30 : 22;
                    } else {
                        if (p.colstats) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
                        else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
                    }
                    BARRIER();
#if DDL_STAGGER
                    if (wm == 1) BARRIER();
#endif
                } else {
                    prologueO();
                }
            } else {
                BARRIER();
            }
            // on every path (the compiler's wait for the ticket then lands here, not in
            // the next main loop), after a barrier that follows every wave's read of s_tick
            publish();
            STAMP(1);
            continue;
        }
        break;
    }
    if constexpr (DYN) {
        if (p.sched && threadIdx.x == 0) {
            // the last block out re-arms the ticket slot for its next launch
            int* done = p.sched + 8 * SCHED_STRIDE;
            if (atomicAdd(done, 1) == (int)gridDim.x - 1) {
#pragma unroll 1
                for (int i = 0; i < 8; ++i) atomicExch(p.sched + i * SCHED_STRIDE, 0);
                atomicExch(done, 0);
            }
        }
        return;
    }

    // ---------------- LDS-staged epilogue (general: every epilogue option)
    // The accumulators go through LDS one 128x128 quarter at a time (fp32, rows
    // padded to 132 floats: the 16 rows a ds_write_b128 group touches land on
    // distinct bank quads).  Each thread then owns 8 consecutive columns of a
    // row, so the bias / residual / activation / store code exists once (not 32
    // unrolled copies -- the unrolled form cost ~10 us per tile in I-cache
    // misses) and global stores are row-contiguous.
    float* ep = reinterpret_cast<float*>(smem);
    const int g = lane >> 4;
    const bool partial = p.splits > 1;
    auto put = [&](f32x4 (&a)[4][2]) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                *reinterpret_cast<f32x4*>(ep + (wm * 64 + i * 16 + (lane & 15)) * EP_LD + wn * 32 + j * 16 + 4 * g) =
                    a[i][j];
    };
    // BN statistics: this thread always owns the same 8 columns (idx & 15) of a quarter
    float st_s[2][8], st_q[2][8];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int e = 0; e < 8; ++e) st_s[a][e] = st_q[a][e] = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        __syncthreads();
        put(acc[q >> 1][q & 1]);
        __syncthreads();
        const int mq = m0 + (q >> 1) * 128, nq = n0 + (q & 1) * 128;
#pragma unroll 1
        for (int it = 0; it < (128 * 16) / NTH; ++it) {
            const int idx = it * NTH + threadIdx.x;
            const int r = idx >> 4, c = (idx & 15) * 8;
            const int m = mq + r, n = nq + c;
            if (m >= p.M || n >= p.N) continue;
            float v[8];
            const f32x4 lo = *reinterpret_cast<const f32x4*>(ep + r * EP_LD + c);
            const f32x4 hi = *reinterpret_cast<const f32x4*>(ep + r * EP_LD + c + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) { v[e] = lo[e]; v[4 + e] = hi[e]; }
            if (p.colstats) {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float t = n + e < p.N ? bf2f(f2bf(v[e])) : 0.f;   // what BN will read
                    st_s[q & 1][e] += t;
                    st_q[q & 1][e] += t * t;
                }
            }
            if (partial) {
                if constexpr (WGRAD) {
                    bf16_t* dst = (bf16_t*)p.C + split * p.split_stride + (long)m * p.ldc + n;
                    store4g(dst, n + 3 < p.N, p.N - n, v);
                    if (n + 4 < p.N) store4g(dst + 4, n + 7 < p.N, p.N - n - 4, v + 4);
                } else {
                    float* dst = (float*)p.C + split * p.split_stride + (long)m * p.ldc + n;
                    store4g(dst, n + 3 < p.N, p.N - n, v);
                    if (n + 4 < p.N) store4g(dst + 4, n + 7 < p.N, p.N - n - 4, v + 4);
                }
                continue;
            }
            const long orow = out_row(p, m);
            epilogue4(p, orow, n, v);
            if (n + 4 < p.N) epilogue4(p, orow, n + 4, v + 4);
        }
    }
    if (p.colstats) {
        // lanes l, l^16, l^32, l^48 own the same columns; then 8 waves through LDS
        float* red = reinterpret_cast<float*>(smem + 96 * 1024);   // [8 waves][256 cols][2]
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float x = st_s[a][e], y = st_q[a][e];
                x += __shfl_xor(x, 16);
                y += __shfl_xor(y, 16);
                x += __shfl_xor(x, 32);
                y += __shfl_xor(y, 32);
                if (lane < 16) {
                    const int col = a * 128 + lane * 8 + e;
                    red[(w * 256 + col) * 2] = x;
                    red[(w * 256 + col) * 2 + 1] = y;
                }
            }
        __syncthreads();
        if (threadIdx.x < 256) {
            const int col = threadIdx.x, n = n0 + col;
            float x = 0.f, y = 0.f;
#pragma unroll
            for (int ww = 0; ww < 8; ++ww) {
                x += red[(ww * 256 + col) * 2];
                y += red[(ww * 256 + col) * 2 + 1];
            }
            if (n < p.N) {
                // partial rows are per 128 output rows (the direct epilogue writes one
                // per wave row): this tile's sums in row 2*tm, zeros in row 2*tm+1
                float* row = p.colstats + (long)tm * 4 * p.N;
                row[n] = x;
                row[p.N + n] = y;
                row[2 * p.N + n] = 0.f;
                row[3 * p.N + n] = 0.f;
            }
        }
    }
}

// Split-K: sum the partial slabs (fp32, or bf16 with p.part_bf16) + the epilogue; 4 consecutive
// columns per thread.
__global__ __launch_bounds__(256) void big_reduce_k(BigParams p, const float* __restrict__ part) {
    const long n4 = ((long)p.N + 3) / 4;
    const long total = (long)p.M * n4;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int m = (int)(i / n4);
        const int n = (int)(i - (long)m * n4) * 4;
        const bool full = n + 3 < p.N;
        const int nv = p.N - n;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        for (int s = 0; s < p.splits; ++s) {
            float t[4];
            if (p.part_bf16) load4g((const bf16_t*)part + s * p.split_stride + (long)m * p.ldc + n, full, nv, t);
            else load4g(part + s * p.split_stride + (long)m * p.ldc + n, full, nv, t);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += t[r];
        }
        epilogue4(p, out_row(p, m), n, v);
    }
}

// Split-K reduce, 8 consecutive columns per thread (N, ldc % 8 == 0): one 16-byte load per bf16 slab
// (two per fp32 slab), every split's load issued before the first sum, so a thread keeps the whole
// column group's reads in flight (the 4-column form issued one 8-byte load per split and waited for
// each in turn: ~3.4 TB/s on BERT's weight gradients)
__global__ __launch_bounds__(256) void big_reduce8_k(BigParams p, const float* __restrict__ part) {
    const long n8 = (long)p.N / 8;
    const long total = (long)p.M * n8;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int m = (int)(i / n8);
        const int n = (int)(i - (long)m * n8) * 8;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        const long off = (long)m * p.ldc + n;
        if (p.part_bf16) {
            // groups of 8 / 4 / 1 slabs, each group's loads unconditional (a per-slab "load if s <
            // splits" made the compiler branch around each load and wait for it)
            const bf16_t* pb = (const bf16_t*)part + off;
            auto add8 = [&](const uint4& r) {
                const uint32_t wds[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[2 * e] += __uint_as_float(wds[e] << 16);
                    v[2 * e + 1] += __uint_as_float(wds[e] & 0xffff0000u);
                }
            };
            int s = 0;
            for (; s + 8 <= p.splits; s += 8) {
                uint4 r[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) r[j] = *reinterpret_cast<const uint4*>(pb + (s + j) * p.split_stride);
#pragma unroll
                for (int j = 0; j < 8; ++j) add8(r[j]);
            }
            if (s + 4 <= p.splits) {
                uint4 r[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) r[j] = *reinterpret_cast<const uint4*>(pb + (s + j) * p.split_stride);
#pragma unroll
                for (int j = 0; j < 4; ++j) add8(r[j]);
                s += 4;
            }
            for (; s < p.splits; ++s) add8(*reinterpret_cast<const uint4*>(pb + s * p.split_stride));
        } else {
            for (int s = 0; s < p.splits; ++s) {
                float t[8];
                load8(part + s * p.split_stride + off, t);
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] += t[e];
            }
        }
        const long orow = out_row(p, m);
        epilogue4(p, orow, n, v);
        epilogue4(p, orow, n + 4, v + 4);
    }
}

// launch the split-K reduce: the 8-column form where it applies
void launch_reduce(const BigParams& p, const float* ws, hipStream_t st) {
    if (p.N % 8 == 0 && p.ldc % 8 == 0 && !p.row_remap) {
        const long total = (long)p.M * (p.N / 8);
        const int g = (int)std::min<long>(16384, (total + 255) / 256);
        big_reduce8_k<<<g, 256, 0, st>>>(p, ws);
    } else {
        const long total = (long)p.M * ((p.N + 3) / 4);
        const int g = (int)std::min<long>(16384, (total + 255) / 256);
        big_reduce_k<<<g, 256, 0, st>>>(p, ws);
    }
}

// ------------------------------------------------------------------ weight-gradient kernel ("wg")
// C[M, N] (+)= A^T B with A = [K][M] and B = [K][N] both k-outer: the TN weight gradients
// (dW = dY^T X over K = tokens / pixels).  The 8-wave kernel above reads a k-outer A operand with
// twice the transposed LDS reads of a row operand and, at two waves per SIMD (256 registers), has
// no registers to read ahead: each phase waits for its reads before its MFMAs
// (profiles/pmc_gemm_modes_r04.md: TN 5.0 K cycles per 64-deep k-tile vs NN 3.1 K).  Here 4 waves
// (one per SIMD, 512 registers each) own 128 x 64 of a 256 x 128 tile (acc 128 registers) and never
// wait for a read they just issued: tile t+1's fragments replace tile t's as soon as the MFMAs
// reading them have issued.  (128 x 128 per wave needs the
// whole 256-AGPR file for its accumulators and spilled them.)  Operands arrive by LDS-DMA in 32-deep
// k-tiles through a 4-stage ring (3 tiles in flight), in the swizzled k-outer image of the 8-wave
// kernel (frag<KO>).  Output: fp32 split-K partials; big_reduce_k sums them and applies accumulate
// and the output dtype (also for one split).
// Needs M % 256 == 0, N % 128 == 0, K % 128 == 0, lda / ldb % 8 == 0, ldc % 4 == 0, 16-byte aligned operands.
constexpr int WG_BK = 32, WG_ST = 4;
constexpr int WG_HALF = WG_BK * 256;     // bytes: 32 k-rows x 128 columns x 2 B

// (This file is compiled with -mllvm -amdgpu-mfma-vgpr-form, csrc/build.py: with the AGPR form the
// allocator gave each MFMA a destination other than its accumulator input and shuffled the
// accumulators through v_accvgpr moves around every MFMA of this kernel -- 2.7x its MFMA time.
// The 8-wave kernels' code is identical either way.)
// CW: B is the implicit im2col of an NHWC input (conv weight gradient, CONVW): reduction rows are
// output pixels, columns (tap, channel); a lane's 8 columns are one tap's 8 channels (C % 8 == 0),
// fixed for the whole reduction, so only the pixel is decomposed per DMA (padding: the zero page)
// NW: 4 waves (one per SIMD, 256 x 128 tiles, "wg") or 8 waves (two per SIMD, 256 x 256 tiles,
// "wg2": the 256 x 256 kernel's operand bytes per output, the second wave on each SIMD filling the
// first one's read / barrier gaps).  Every wave owns 128 x 64 (acc 128 registers).
// CONVW row table (4-wave kernel): the B operand's reduction rows are output pixels, and decomposing a
// row into (image, h, w) per DMA -- two divisions, the bounds and a 64-bit address per lane -- made the
// conv weight gradient's loop 2.6 VALU per MFMA against 0.4 for a plain TN GEMM (15-35 % slower than
// the same GEMM over a materialized im2col, profiles/wg_convw_r06.log).  The workgroup decomposes its
// split's rows ONCE into an LDS table behind the operand ring -- per row the element offset of its
// (h_off, w_off)-shifted corner pixel and the corner's (h, w) -- and a DMA then reads one 8-byte record:
// two adds, the bounds test, one 32-bit add and the zero-page select.
constexpr int WG_TBL_BYTES = 160 * 1024 - WG_ST * 3 * WG_HALF;   // 64 KB: 8192 rows
// table records are read by inline asm: a compiler-visible read of the LDS object -- even through a
// restrict-qualified pointer -- made its LDS-DMA alias tracking wait vmcnt(0), i.e. every in-flight
// operand tile, before each record (that version ran 1.5x SLOWER than the decomposing loader).  The
// caller waits lgkmcnt(0) itself before using the value.
__device__ __forceinline__ uint2 wg_row_rec(uint32_t lds_addr) {
    uint2 v;
    asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(lds_addr));
    return v;
}

template <bool CW, int NW, bool TBL = false>
__global__ __launch_bounds__(NW * 64, 1) void gemm_wg_k(BigParams p) {
    constexpr int WN = NW / 2, TNW = 64 * WN, BH = TNW / 128;   // waves along N, tile N, B halves
    constexpr int JW = 8 / NW;                                   // DMA instructions per wave per half
    constexpr int DMA = JW * (2 + BH);                           // ... per k-tile
    constexpr int RING = WG_ST * (2 + BH) * WG_HALF;
    static_assert(!TBL || (CW && RING + WG_TBL_BYTES <= 160 * 1024), "row table: CONVW, behind the ring");
    __shared__ __attribute__((aligned(16))) char smem[RING + (TBL ? WG_TBL_BYTES : 0)];   // one LDS object
    // stage s: A half 0, A half 1, B half 0 (, B half 1)
    auto wg_off = [](int s, int x, int h) { return (s * (2 + BH) + (x ? 2 + h : h)) * WG_HALF; };
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int wm = w / WN, wn = w % WN;
    // 1-D grid of (split, tile) blocks; XCD x (blocks x, x + 8, ...) runs a contiguous run of the
    // split-major order, so its blocks share k-rows of the A / B panels in its L2 (gemm_big_k xsplit)
    const int nwg = p.tiles_m * p.tiles_n;
    const int n = nwg * p.splits, xcd = blockIdx.x & 7, qn = n >> 3, rn = n & 7;
    const int q = (xcd < rn ? xcd * (qn + 1) : rn * (qn + 1) + (xcd - rn) * qn) + (int)(blockIdx.x >> 3);
    const int split = q / nwg, tile = q - split * nwg;
    const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
    const int m0 = tm * 256, n0 = tn * TNW;
    const int nkt = p.K / WG_BK;
    const int kt0 = split * p.kt_per_split;
    const int nt = min(nkt, kt0 + p.kt_per_split) - kt0;      // >= 1 (host)
    // DMA lanes: k-row krow0 (+4 j) of a 32-row half, 16-byte chunk c of its 128 columns, stored at
    // the swizzled slot l & 15 (for JW = 2, swz_ko ignores bit 2: the same c for both j)
    const int krow0 = (w * JW) * 4 + (l >> 4);
    const int c = (l & 15) ^ swz_ko(krow0);
    const bf16_t* ga = p.A + (long)krow0 * p.lda + m0 + 8 * c;
    const bf16_t* gb = p.B + (long)krow0 * p.ldb + n0 + 8 * c;
    int cdh[BH], cdw[BH], cci[BH], toff[BH];
#pragma unroll
    for (int h = 0; h < BH; ++h) {
        cdh[h] = cdw[h] = cci[h] = 0;
        if (CW) tap_of(p.cd, n0 + h * 128 + 8 * c, cdh[h], cdw[h], cci[h]);
        toff[h] = (cdh[h] * p.cd.W + cdw[h]) * p.cd.C + cci[h];   // the lane's tap / channel offset
    }
    if constexpr (TBL) {
        for (int r = threadIdx.x; r < nt * WG_BK; r += NW * 64) {
            const Pix x = decompose(p.cd, p.B, kt0 * WG_BK + r, p.K);
            const int corner = (int)(x.img - p.B) + (x.hb * p.cd.W + x.wb) * p.cd.C;
            *reinterpret_cast<uint2*>(smem + RING + r * 8) =
                make_uint2((uint32_t)corner, ((uint32_t)x.hb & 0xffffu) | ((uint32_t)x.wb << 16));
        }
        __syncthreads();
    }
    auto stage = [&](int kt, int st) {
        const long ka = (long)kt * WG_BK;
        if constexpr (TBL) {
            // every DMA's row record first, the A tiles' DMAs under the LDS reads, then the B DMAs
            uint2 rec[JW];
#pragma unroll
            for (int j = 0; j < JW; ++j)
                rec[j] = wg_row_rec((uint32_t)(uintptr_t)(smem + RING) + ((int)ka - kt0 * WG_BK + krow0 + j * 4) * 8);
#pragma unroll
            for (int j = 0; j < JW; ++j) {
                glds(ga + (ka + j * 4) * p.lda, smem + wg_off(st, 0, 0) + (w * JW + j) * 1024);
                glds(ga + (ka + j * 4) * p.lda + 128, smem + wg_off(st, 0, 1) + (w * JW + j) * 1024);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < JW; ++j)
#pragma unroll
                for (int h = 0; h < BH; ++h) {
                    const int hh = (int)(short)(rec[j].y & 0xffffu) + cdh[h], ww = ((int)rec[j].y >> 16) + cdw[h];
                    const bool ok = (unsigned)hh < (unsigned)p.cd.H && (unsigned)ww < (unsigned)p.cd.W;
                    glds(ok ? p.B + ((int)rec[j].x + toff[h]) : p.zero, smem + wg_off(st, 1, h) + (w * JW + j) * 1024);
                }
            return;
        }
#pragma unroll
        for (int j = 0; j < JW; ++j) {
            glds(ga + (ka + j * 4) * p.lda, smem + wg_off(st, 0, 0) + (w * JW + j) * 1024);
            glds(ga + (ka + j * 4) * p.lda + 128, smem + wg_off(st, 0, 1) + (w * JW + j) * 1024);
#pragma unroll
            for (int h = 0; h < BH; ++h) {
                if (CW) {
                    const Pix x = decompose(p.cd, p.B, (int)ka + krow0 + j * 4, p.K);
                    const int hh = x.hb + cdh[h], ww = x.wb + cdw[h];
                    const bool ok = (unsigned)hh < (unsigned)p.cd.H && (unsigned)ww < (unsigned)p.cd.W;
                    glds(ok ? x.img + ((long)hh * p.cd.W + ww) * p.cd.C + cci[h] : p.zero,
                         smem + wg_off(st, 1, h) + (w * JW + j) * 1024);
                } else {
                    glds(gb + (ka + j * 4) * p.ldb + h * 128, smem + wg_off(st, 1, h) + (w * JW + j) * 1024);
                }
            }
        }
    };
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // one set of fragments in registers (A: 8 row blocks, B: 4 column blocks); tile t+1's overwrite
    // tile t's as soon as the MFMAs that read them have issued: A rows 0-3 under the MFMAs of rows
    // 4-7, A rows 4-7 and B at the end of the tile, landing under the next tile's barrier
    bf16x8 fa[8], fb[4];
    auto readA = [&](int st, int i0) {
        const char* ha = smem + wg_off(st, 0, wm);
#pragma unroll
        for (int i = i0; i < i0 + 4; ++i) fa[i] = frag<KO>(ha, i * 16, 0);
    };
    auto readB = [&](int st) {
        const char* hb = smem + wg_off(st, 1, wn >> 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = frag<KO>(hb, (wn & 1) * 64 + j * 16, 0);
    };
    auto mma4 = [&](int i0) {
#pragma unroll
        for (int i = i0; i < i0 + 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    };
    // Branch-free steady state: every iteration stages a tile (past the last one it re-stages the
    // last, into the slot no longer read), waits, syncs and reads the next tile's fragments (past
    // the end: a stale slot, never used) -- accumulators crossing a branch were copied between
    // AGPRs and VGPRs (64 v_accvgpr_write + hazard nops per 16 MFMAs).
    const int ktl = kt0 + nt - 1;
    // prologue: tiles 0..2 in flight (two of them possibly re-stages of the last), tile 0 landed
    stage(kt0, 0);
    stage(min(kt0 + 1, ktl), 1);
    stage(min(kt0 + 2, ktl), 2);
    if constexpr (DMA == 6) VMN(12);
    else VMN(8);
    BARRIER();
    readB(0);
    readA(0, 0);
    readA(0, 4);
    // one k-tile per iteration: tile t+1 landed (tile t+2 may still be in flight) and made visible by
    // the barrier -- which also orders every wave's reads of tile t-1 (issued in the iteration before,
    // consumed by its MFMAs) before slot (t+3) % 4 = (t-1) % 4 is restaged.  One loop body, unrolled
    // by the 4 ring slots (nt % 4 == 0 by the host's split sizes): every LDS address is a loop-
    // invariant lane offset plus an immediate -- with a run-time slot each fragment read cost a VALU
    // add, and the loop's VALU overflowed the issue slots between MFMAs.
    auto iter = [&](int t, int sl) {
#ifndef DDL_DIAG_WG_NODMA   // diagnostic builds only (wrong results): no operand DMA after the prologue
        if constexpr (DMA == 6) VMN(6);
        else VMN(4);
#endif
        BARRIER();
        mma4(0);
        readA((sl + 1) & 3, 0);
#ifndef DDL_DIAG_WG_NODMA
        stage(min(kt0 + t + 3, ktl), (sl + 3) & 3);
#endif
        mma4(4);
        readA((sl + 1) & 3, 4);
        readB((sl + 1) & 3);
    };
#pragma unroll 1
    for (int t = 0; t < nt; t += 4) {
        iter(t, 0);
        iter(t + 1, 1);
        iter(t + 2, 2);
        iter(t + 3, 3);
    }
    VM0();      // no LDS-DMA may outlive the workgroup's LDS
    // partial tile: lane holds C[m][n .. n+3] of each 16 x 16 block (the MFMA layout); fp32, or
    // bf16 (p.part_bf16: half the slab bytes written here and read by the reduce)
    const int r16 = l & 15, g4 = (l >> 4) * 4;
    if (p.part_bf16) {
        bf16_t* out = (bf16_t*)p.C + (long)split * p.split_stride;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                *reinterpret_cast<uint2*>(out + (long)(m0 + wm * 128 + i * 16 + r16) * p.ldc + n0 + wn * 64 + j * 16 +
                                          g4) = make_uint2(pack2bf(acc[i][j][0], acc[i][j][1]),
                                                           pack2bf(acc[i][j][2], acc[i][j][3]));
    } else {
        float* out = (float*)p.C + (long)split * p.split_stride;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                *reinterpret_cast<f32x4*>(out + (long)(m0 + wm * 128 + i * 16 + r16) * p.ldc + n0 + wn * 64 + j * 16 + g4) =
                    acc[i][j];
    }
}

void fill_conv(ConvDesc& cd, const int* d) {
    cd.N = d[0]; cd.H = d[1]; cd.W = d[2]; cd.C = d[3]; cd.P = d[4]; cd.Q = d[5];
    cd.stride = d[6]; cd.h_off = d[7]; cd.w_off = d[8]; cd.h_step = d[9]; cd.w_step = d[10];
    cd.R = d[11]; cd.S = d[12]; cd.OH = d[13]; cd.OW = d[14]; cd.ostep = d[15]; cd.oa = d[16]; cd.ob = d[17];
    cd.fd_PQ = make_fastdiv((uint32_t)(cd.P * cd.Q));
    cd.fd_Q = make_fastdiv((uint32_t)cd.Q);
    cd.fd_C = make_fastdiv((uint32_t)cd.C);
    cd.fd_S = make_fastdiv((uint32_t)std::max(1, cd.S));
}

int num_cus() {
    static int n = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                     hipSuccess || v <= 0)
            v = 256;
        return v;
    }();
    return n;
}

// DDL_GEMM_DIRECT=0 forces the LDS-staged epilogue everywhere (A/B timing, tests)
bool direct_enabled() {
    static const bool on = [] {
        const char* e = getenv("DDL_GEMM_DIRECT");
        return !(e && e[0] == '0');
    }();
    return on;
}

// DDL_GEMM_LEAN=1 routes all-interior GEMMs to the variant without the general epilogue.
// Off by default: spill-free as it is (the NT kernel), it measured 1.9 % SLOWER on BERT-base
// same-box (8318-8333 vs 8473-8491 samples/s, 3 alternating runs each) -- the scratch the
// general epilogue costs sits off the interior tiles' path, and the allocation the lean
// variant gets in exchange schedules the main loop worse.
bool edge_split_enabled() {
    static const bool on = [] {
        const char* e = getenv("DDL_GEMM_LEAN");
        return e && e[0] == '1';
    }();
    return on;
}

// DDL_GEMM_XSPLIT=0: split-K grids as (tiles, splits) with blockIdx.y = split (A/B timing)
bool xsplit_enabled() {
    static const bool on = [] {
        const char* e = getenv("DDL_GEMM_XSPLIT");
        return !(e && e[0] == '0');
    }();
    return on;
}

// DDL_GEMM_DYNAMIC=0 keeps the static tile striding of the persistent grid (A/B timing)
bool dynamic_enabled() {
    static const bool on = [] {
        const char* e = getenv("DDL_GEMM_DYNAMIC");
        return !(e && e[0] == '0');
    }();
    return on;
}

// DDL_GEMM_PERSIST=0: one block per tile (grid = tiles) instead of one persistent block per CU (A/B)
bool persist_enabled() {
    static const bool on = [] {
        const char* e = getenv("DDL_GEMM_PERSIST");
        return !(e && e[0] == '0');
    }();
    return on;
}

// Tile-ticket slots of the persistent kernel, per device: SLOTS launches in flight at
// most (the launching stream orders the rest), each slot zero at launch and re-armed by
// the launch's last block.  Null while a stream is being captured before the first
// allocation (the kernel then strides statically).
int* sched_slot(hipStream_t st) {
    constexpr int SLOTS = 64, DEVS = 16;
    constexpr size_t SLOT_INTS = 9 * SCHED_STRIDE;
    static int* base[DEVS] = {};
    static unsigned next[DEVS] = {};
    static std::mutex mu;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= DEVS) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    if (!base[dev]) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
        int* b = nullptr;
        if (hipMalloc(&b, SLOTS * SLOT_INTS * sizeof(int)) != hipSuccess) return nullptr;
        if (hipMemsetAsync(b, 0, SLOTS * SLOT_INTS * sizeof(int), st) != hipSuccess) return nullptr;
        base[dev] = b;
    }
    return base[dev] + (size_t)(next[dev]++ % SLOTS) * SLOT_INTS;
}

// DDL_GEMM_BEHIND: BEHIND_* bits -- which register epilogues besides plain bf16 let
// their stores drain under the next tile's prologue.  Measured neutral (bias, GELU:
// profiles/epilogue_behind_ab.log) to -8 % (residual), so all off by default
int behind_mask() {
    static const int m = [] {
        const char* e = getenv("DDL_GEMM_BEHIND");
        return e ? atoi(e) : 0;
    }();
    return m;
}

// DDL_GEMM_PART_BF16=0: split-K partial slabs in fp32 (default bf16: each partial is a fp32 sum of
// its k-range rounded once; the reduce sums them in fp32 -- half the slab bytes on both sides)
bool part_bf16_enabled() {
    static const bool on = [] {
        const char* e = getenv("DDL_GEMM_PART_BF16");
        return !(e && e[0] == '0');
    }();
    return on;
}

// DDL_GEMM_ZB1=0: 256 x 192 NT tiles stage all 256 B rows (the 64 past the tile read, never used) (A/B)
bool zero_b1_enabled() {
    static const bool on = [] {
        const char* e = getenv("DDL_GEMM_ZB1");
        return !(e && e[0] == '0');
    }();
    return on;
}

// DDL_GEMM_EPI_LDS=1: plain bf16 interior tiles store whole rows through LDS (epi_lds_bf16)
bool epi_lds_enabled() {
    static const bool on = [] {
        const char* e = getenv("DDL_GEMM_EPI_LDS");
        return e && e[0] == '1';
    }();
    return on;
}

template <int LA, int LB>
int launch_big(BigParams& p, float* ws, long ws_elems, int splits, hipStream_t st, bool n192 = false) {
    p.behind_mask = behind_mask();
    p.epi_lds = epi_lds_enabled() ? 1 : 0;
    p.zero_b1 = zero_b1_enabled() ? 1 : 0;
    const int tbn = n192 ? 192 : TB;
    p.tiles_m = (p.M + TB - 1) / TB;
    p.tiles_n = (p.N + tbn - 1) / tbn;
    const int nk = (p.K + BK - 1) / BK;
    if (splits < 1) splits = 1;
    // the weight-gradient kernel's split-K partials are bf16 (compiled in): an fp32 output asks
    // for more than that, so it runs unsplit
    if (LA == KO && LB == KO && p.out_f32) splits = 1;
    if (splits > nk) splits = nk > 0 ? nk : 1;
    p.kt_per_split = nk > 0 ? (nk + splits - 1) / splits : 1;
    splits = nk > 0 ? (nk + p.kt_per_split - 1) / p.kt_per_split : 1;
    p.splits = splits;
    // weight gradients (TN): bf16 partial slabs, compiled in (epi_direct PB); the reduce reads them so
    p.part_bf16 = LA == KO && LB == KO && splits > 1 ? 1 : 0;
    if (splits > 1) {
        p.split_stride = (long)p.M * p.ldc;
        if (!ws || ws_elems < p.split_stride * splits) return -2;
    }
    BigParams kp = p;
    if (splits > 1) kp.C = ws;
    // KTAIL: per-chunk K checks; also selects the per-chunk tap decomposition for
    // convolutions whose channel count is not a multiple of 64
    const bool ktail = (p.K % BK) != 0 || ((LA == CONV || LB == CONVW) && (p.cd.C % BK) != 0);
    // register epilogue + persistent grid when the epilogue is one direct4 covers
    // (split-K partials always: the reduce kernel applies the real epilogue)
    const bool direct = direct_enabled() &&
        (splits > 1 || (!p.row_remap && (p.act == ACT_NONE || p.act == ACT_RELU || p.act == ACT_GELU ||
                                          (p.act == ACT_DGELU && p.aux) || p.act == ACT_BNB)));
    if (splits > 1 || (p.out_f32 && !p.bias && p.act == ACT_NONE))
        p.ek = (p.N % 4 == 0 && p.ldc % 4 == 0) ? EK_F32 : EK_GEN;
    else if (!p.out_f32 && !p.accumulate && p.act == ACT_NONE && (!p.bias || p.bias_bf16) && !p.row_remap)
        p.ek = (p.N % 8 == 0 && p.ldc % 8 == 0) ? EK_BF16 : EK_GEN;   // 16-byte pair stores
    else if (!p.out_f32 && !p.accumulate && p.act == ACT_GELU && (!p.bias || p.bias_bf16) && !p.row_remap && !p.res)
        p.ek = (p.N % 8 == 0 && p.ldc % 8 == 0) ? EK_GELU : EK_GEN;
    else if (!p.out_f32 && !p.accumulate && p.act == ACT_DGELU && p.aux && !p.bias && !p.row_remap && !p.res)
        p.ek = (p.N % 8 == 0 && p.ldc % 8 == 0 && !(LA == KO && LB == KO)) ? EK_DGELU : EK_GEN;   // 16-byte pair
        // stores; the weight-gradient (TN) kernels carry no dGELU epilogue (gemm_big_k WGRAD)
    else
        p.ek = EK_GEN;
    kp.ek = p.ek;
    // the LDS-staged epilogue sums BatchNorm statistics of the raw accumulator: dGELU
    // column sums exist on the register epilogue only
    if (p.colstats && p.act == ACT_DGELU && !direct) return -6;
    if (p.act == ACT_BNB && (!direct || splits > 1)) return -8;   // register epilogue only
    const int nwg = p.tiles_m * p.tiles_n;
    int gx = nwg;
    if (direct && splits == 1 && persist_enabled()) {
        // persistent: one block per CU walks tiles blockIdx.x, +gridDim.x, ...
        // (a multiple of 8, so a block's tiles stay on its XCD); split-K grids keep
        // one block per (tile, split) -- a capped grid would leave tiles for a second round
        const int cap = std::max(8, num_cus() & ~7);
        gx = std::min(nwg, cap);
        if (gx < nwg && p.act != ACT_BNB && dynamic_enabled()) kp.sched = sched_slot(st);
    }
    // split-K: a 1-D grid whose XCDs each run a contiguous (split, tile) range (gemm_big_k xsplit)
    kp.xsplit = splits > 1 && xsplit_enabled();
    const dim3 grid(kp.xsplit ? gx * splits : gx, kp.xsplit ? 1 : splits);
    if (direct) {
        if constexpr (LB == KC && (LA == KC || LA == CONV)) {   // dgrad operand layouts
            if (p.act == ACT_BNB) {
                if (ktail) hipLaunchKernelGGL((gemm_big_k<LA, LB, true, true, true>), grid, dim3(NTH), 0, st, kp);
                else hipLaunchKernelGGL((gemm_big_k<LA, LB, false, true, true>), grid, dim3(NTH), 0, st, kp);
                return (int)hipGetLastError();
            }
        }
        if (p.act == ACT_BNB) return -8;
        if (n192) {
            if constexpr (LA == KC && (LB == KC || LB == KO)) {   // Linear fwd / dgrad operand layouts
                if (ktail) hipLaunchKernelGGL((gemm_big_k<LA, LB, true, true, false, true, true>), grid, dim3(NTH), 0, st, kp);
                else hipLaunchKernelGGL((gemm_big_k<LA, LB, false, true, false, true, true>), grid, dim3(NTH), 0, st, kp);
            } else {
                return -9;
            }
        } else {
        // all tiles interior with a lean epilogue kind: the variant without the general epilogue
        const bool lean = p.M % TB == 0 && p.N % TB == 0 && p.ek != EK_GEN && edge_split_enabled();
        if (lean) {
            if (ktail) hipLaunchKernelGGL((gemm_big_k<LA, LB, true, true, false, false>), grid, dim3(NTH), 0, st, kp);
            else hipLaunchKernelGGL((gemm_big_k<LA, LB, false, true, false, false>), grid, dim3(NTH), 0, st, kp);
        } else if (ktail) {
            hipLaunchKernelGGL((gemm_big_k<LA, LB, true, true>), grid, dim3(NTH), 0, st, kp);
        } else {
            hipLaunchKernelGGL((gemm_big_k<LA, LB, false, true>), grid, dim3(NTH), 0, st, kp);
        }
        }
    } else {
        if (n192) return -9;    // 192-wide tiles: register epilogue only
        if (ktail) hipLaunchKernelGGL((gemm_big_k<LA, LB, true, false>), grid, dim3(NTH), 0, st, kp);
        else hipLaunchKernelGGL((gemm_big_k<LA, LB, false, false>), grid, dim3(NTH), 0, st, kp);
    }
    if (splits > 1) launch_reduce(p, ws, st);
    return (int)hipGetLastError();
}

}  // namespace

// mode: 0 = A KC, B KC (NT)   1 = A KC, B KO (NN)   2 = A KO, B KO (TN)
//       3 = A CONV, B KC      4 = A KO, B CONVW      | 32: 256 x 192 tiles (modes 0 / 1)
// Requirements: K % 8 == 0, leading dims % 8 == 0 (16-B chunks), zero points at >= 16 zero bytes.
DDL_API int ddl_gemm_big2(int mode, const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N,
                          int K, const void* bias, int bias_bf16, int act, void* aux, int out_f32, int splits,
                          float* workspace, long ws_elems, const int* conv, int row_remap, const void* res,
                          int accumulate, const void* zero, float* colstats, hipStream_t st) {
    if (M <= 0 || N <= 0) return 0;
    if (K % 8 || !zero) return -1;
    BigParams p{};
    p.A = (const bf16_t*)A; p.B = (const bf16_t*)B; p.lda = lda; p.ldb = ldb;
    p.C = C; p.ldc = ldc; p.M = M; p.N = N; p.K = K;
    p.bias = bias; p.bias_bf16 = bias_bf16; p.act = act; p.aux = (bf16_t*)aux;
    p.res = (const bf16_t*)res; p.accumulate = accumulate; p.out_f32 = out_f32;
    p.row_remap = row_remap; p.zero = (const bf16_t*)zero;
    p.colstats = colstats;
    // column statistics: plain bf16 outputs (BatchNorm) or dGELU outputs (the Linear's bias gradient)
    if (act == ACT_BNB) {
        const BnbArgs bn = ddl_take_bnb();
        if (!colstats || !aux || !bn.mean || !bn.istd || ldc != N || N % 8 || out_f32 || accumulate || splits > 1 ||
            bias || row_remap)
            return -8;
        p.bn_mask = bn.mask; p.bn_mean = bn.mean; p.bn_istd = bn.istd;
    } else if (colstats && (out_f32 || accumulate || splits > 1 || bias || (act && act != ACT_DGELU) || res)) {
        return -6;
    }
    if (conv) fill_conv(p.cd, conv);
    // mode flag 32: 256 x 192 tiles (N192 in gemm_big_k; NT / NN, register epilogue, no BN backward)
    const bool n192 = (mode & 32) != 0;
    mode &= ~32;
    if (n192 && (act == ACT_BNB || (mode != 0 && mode != 1))) return -9;
    switch (mode) {
        case 0: return launch_big<KC, KC>(p, workspace, ws_elems, splits, st, n192);
        case 1: return launch_big<KC, KO>(p, workspace, ws_elems, splits, st, n192);
        case 2: return launch_big<KO, KO>(p, workspace, ws_elems, splits, st);
        case 3: return launch_big<CONV, KC>(p, workspace, ws_elems, splits, st);
        default: return -1;   // conv wgrad (CONVW) stays on the 128x128 kernel (gemm.hip)
    }
}

// TN weight gradient on the 4-wave kernel (gemm_wg_k): C[M, N] (+)= A^T B, A = [K][M] (lda), B = [K][N]
// (ldb); fp32 partials in `workspace` (splits x M x ldc floats, also for one split), then the reduce
// applies accumulate / the output dtype.  Returns -1 when the shape is outside the kernel's contract.
// conv (nullable): the CONVW descriptor (as ddl_gemm_big2) -- B is then the NHWC input and C the
// weight gradient [Cout][R * S * Cin] (channel count % 8 == 0); zero: >= 16 zero bytes (padding taps)
// wide: 8 waves on 256 x 256 tiles ("wg2", N % 256 == 0) instead of 4 on 256 x 128 ("wg")
DDL_API int ddl_gemm_wgrad(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                           int out_f32, int splits, float* workspace, long ws_elems, int accumulate,
                           const int* conv, const void* zero, int wide, hipStream_t st) {
    if (M <= 0 || N <= 0) return 0;
    const int tnw = wide ? 256 : 128;
    if (M % 256 || N % tnw || K <= 0 || K % (4 * WG_BK) || lda % 8 || ldb % 8 || ldc % 4 || ldc < N ||
        ((uintptr_t)A & 15) || ((uintptr_t)B & 15) || (conv && (conv[3] % 8 || !zero)))
        return -1;
    BigParams p{};
    if (conv) fill_conv(p.cd, conv);
    p.zero = (const bf16_t*)zero;
    p.A = (const bf16_t*)A; p.B = (const bf16_t*)B; p.lda = lda; p.ldb = ldb;
    p.C = C; p.ldc = ldc; p.M = M; p.N = N; p.K = K;
    p.act = ACT_NONE; p.accumulate = accumulate; p.out_f32 = out_f32;
    p.tiles_m = M / 256;
    p.tiles_n = N / tnw;
    const int nkt = K / WG_BK;                    // a multiple of 4 (K % 128 == 0)
    if (splits < 1) splits = 1;
    if (splits > nkt / 4) splits = nkt / 4;
    p.kt_per_split = ((nkt + splits - 1) / splits + 3) & ~3;   // whole 4-tile rounds of the ring
    splits = (nkt + p.kt_per_split - 1) / p.kt_per_split;
    p.splits = splits;
    p.split_stride = (long)M * ldc;
    p.part_bf16 = !out_f32 && part_bf16_enabled() ? 1 : 0;
    // the row table: the split's rows fit behind the ring and every element offset fits 31 bits
    p.wg_tbl = conv && !wide && (long)p.kt_per_split * WG_BK * 8 <= WG_TBL_BYTES &&
               (long)conv[0] * conv[1] * conv[2] * conv[3] < (1L << 31) && conv[1] < 32768 && conv[2] < 32768;
    if (!workspace || ws_elems < p.split_stride * splits) return -2;
    BigParams kp = p;
    kp.C = workspace;
    const dim3 grid(p.tiles_m * p.tiles_n * splits);
    if (wide) {
        if (conv) hipLaunchKernelGGL((gemm_wg_k<true, 8>), grid, dim3(512), 0, st, kp);
        else hipLaunchKernelGGL((gemm_wg_k<false, 8>), grid, dim3(512), 0, st, kp);
    } else {
        if (conv && p.wg_tbl) hipLaunchKernelGGL((gemm_wg_k<true, 4, true>), grid, dim3(256), 0, st, kp);
        else if (conv) hipLaunchKernelGGL((gemm_wg_k<true, 4>), grid, dim3(256), 0, st, kp);
        else hipLaunchKernelGGL((gemm_wg_k<false, 4>), grid, dim3(256), 0, st, kp);
    }
    launch_reduce(p, workspace, st);
    return (int)hipGetLastError();
}
