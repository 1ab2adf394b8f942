// Dual-workgroup 256x128 bf16 GEMM for gfx950: the forward (NT: y = x W^T) and input-gradient
// (NN: dx = dy W) GEMMs of the transformer Linears at short reduction depth (K = 768 .. 3072) --
// kernel family K13 (reference workload: notebooks/cv/onnx_experiments.py:32,174,
// the BERT / ViT encoders).
//
// Why a second GEMM kernel next to the persistent 256x256 one (gemm_big.hip): there ONE workgroup
// owns a CU, so a tile's epilogue -- bias / GELU VALU work and the output stores -- runs with no MFMA
// work beside it, and the stores of every CU leave in one chip-wide burst at the HBM write rate
// (stamps: 3.5-4.2 us per 256x192 tile at ~6.6 TB/s chip-wide; the bias+GELU tile stores twice the
// bytes and ran 111 us against 83 us plain at 16384x3072x768).  A persistent block cannot hide them
// behind its next tile either: vmcnt retires loads and stores in issue order, so the next tile's
// operand waits wait out the stores.
//
// Here TWO workgroups share each CU (72 KB of LDS and <= 256 VGPRs per wave each): every SIMD runs
// one wave of each, and whatever one workgroup is doing that is not MFMA work -- its epilogue, its
// prologue loads, a barrier, an LDS read it waits for -- the other workgroup's wave fills with its
// MFMAs.  The two drift apart by themselves, so the output stores spread over the whole kernel.
//   * tile 256 x 128, 4 waves as 2 (M) x 2 (N), each 128 x 64 (8 x 4 accumulators of 16 x 16,
//     128 registers);
//   * operands by LDS-DMA (global_load_lds, 16 B per lane) in 32-deep k-stages through a 3-slot
//     ring (two stages in flight); A and a k-contiguous B (NT) as 16 x 32 subtiles of 1 KB with the
//     st_16x32 swizzle (gemm_big.hip swz_kc), a k-outer B (NN) as [32 k][128] rows of 256 B with the
//     XOR chunk swizzle (read by ds_read_b64_tr_b16);
//   * one barrier per stage: it publishes the stage every wave waited for and frees the slot the
//     stage after next is staged into;
//   * epilogue math from the MFMA layout (bias, residual, GELU with the pre-activation kept, dGELU,
//     column statistics), the bf16 tile through LDS and out as whole-row stores;
//   * one block per tile (no persistence: the next workgroup on a CU starts as soon as one ends,
//     with counters of its own), XCD-aware tile order (gemm_big.hip coords).
// Needs N % 128 == 0, K % 32 == 0, lda / ldb / ldc % 8 == 0, 16-byte aligned operands, operands and
// output under 2 GB; M is free (rows past M re-read row M - 1 and are not stored: buffer range checks).
#include "ddl_common.h"

#include <cstdlib>

namespace {

constexpr int TM = 256, TN = 128, DBK = 32, NST = 3, NTH = 256;
constexpr int A_BYTES = TM * DBK * 2;          // 16 KB: 16 subtiles of 16 rows x 32 k
constexpr int B_BYTES = TN * DBK * 2;          // 8 KB
constexpr int ST_BYTES = A_BYTES + B_BYTES;    // 24 KB per stage
constexpr int GROUP_M = 8;

enum { LKC = 0, LKO = 1, LCONV = 2 };
enum { E_BF16 = 0, E_GELU = 1, E_DGELU = 2, E_BNB = 3 };

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_v4;

struct DuoParams {
    const bf16_t* A;
    const bf16_t* B;
    long lda, ldb;
    bf16_t* C;
    long ldc;
    int M, N, K;
    const bf16_t* bias;     // [N] or null
    const bf16_t* res;      // E_BF16: residual [M][ldc] or null
    bf16_t* aux;            // E_GELU: pre-activation out; E_DGELU: pre-activation in
    float* colstats;        // [2 * tiles_m][2][N] partial column sums of the bf16 output, or null
    int tiles_m, tiles_n;
    // A = implicit im2col of an NHWC tensor (LCONV): rows are output pixels (n, p, q), columns
    // (r, s, c) with C % 32 == 0 (a 32-deep stage lies in one tap); input pixel (p * stride + h_off +
    // r * h_step, q * stride + w_off + s * w_step)
    int cN, cH, cW, cC, cP, cQ, cstride, h_off, w_off, h_step, w_step, cR, cS;
    FastDiv fd_PQ, fd_Q, fd_C, fd_S;
    // E_BNB: BatchNorm backward fused into the input gradient -- C = dz = (acc + res) * relu_mask,
    // colstats rows [sum dz | sum dz * xhat], xhat = (aux - mean) * istd
    const uint8_t* bn_mask;
    const float* bn_mean;
    const float* bn_istd;
    // split-K (weight gradients, LA = LB = LKO): block = (split, tile); splits > 1 write bf16 partial
    // tiles to ws[split][M][N] (duo_reduce_k sums them into C); accumulate: C += result
    int splits, kt_per_split;
    bf16_t* ws;
    int accumulate;
    int nt_store;       // DDL_DUO_NT bits (A/B timing): 1 = the pre-activation (aux) image, 2 = C, stored non-temporal
    const bf16_t* zero; // LCONV: 16 zero bytes (g_duo_zero), the source of padding pixels
};

__device__ __forceinline__ int swz_kc(int b) { return b ^ (((b >> 9) & 1) << 5); }
__device__ __forceinline__ int swz_ko(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }

__device__ __forceinline__ void glds(const bf16_t* g, char* dst) {
    // (default cache policy: the implicit-GEMM convolution re-reads every input pixel once per tap
    // -- the non-temporal policy cost ResNet-50 2 %, profiles/dma_nt_ab.log)
    __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)dst, 16, 0, 0);
}
__device__ __forceinline__ s16x4 ds_read_tr(lds_v4* __restrict__ p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(p);
}

// 16 x 32 fragment of a subtile image (rows on lane & 15, k chunk lane >> 4)
__device__ __forceinline__ bf16x8 frag_kc(const char* sub) {
    const int l = threadIdx.x & 63;
    return *reinterpret_cast<const bf16x8*>(sub + swz_kc((l & 15) * 64 + (l >> 4) * 16));
}
// 16 columns (cbase ..) x 32 k of a [32 k][128] k-outer image, transposed on read
__device__ __forceinline__ bf16x8 frag_ko(const char* img, int cbase) {
    const int l = threadIdx.x & 63;
    const int g = l >> 4, q = (l >> 2) & 3, pq = l & 3;
    const int chunk = (cbase + 4 * pq) >> 3;
    const int ra = 8 * g + q, rb = ra + 4;
    const char* pa = img + ra * 256 + ((chunk ^ swz_ko(ra)) << 4) + (pq & 1) * 8;
    const char* pb = img + rb * 256 + ((chunk ^ swz_ko(rb)) << 4) + (pq & 1) * 8;
    const s16x4 lo = ds_read_tr((lds_v4*)pa);
    const s16x4 hi = ds_read_tr((lds_v4*)pb);
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
}

#define BARRIER() __builtin_amdgcn_s_barrier()
#define VMN(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

// 16 zero bytes (static device storage is zero-initialised): the source of padding pixels.  An
// out-of-range LDS-DMA buffer load does not write its lane's LDS bytes (they keep stale data), so
// zeros must be loaded, not produced by the range check.
__device__ __attribute__((aligned(16))) uint4 g_duo_zero[1];

__device__ __forceinline__ float lo_f(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_f(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

template <int LA, int LB, int EK>
__global__ __launch_bounds__(NTH, 2) void gemm_duo_k(DuoParams p) {
    // one LDS object (a second __shared__ variable makes the compiler's LDS-DMA alias tracking
    // wait vmcnt(0) before the fragment reads)
    __shared__ __attribute__((aligned(16))) char smem[NST * ST_BYTES];
    // (wave index as a scalar: the LDS-DMA destinations below are then SGPR values for M0, not a
    // v_readfirstlane per DMA instruction)
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
    const int wm = w >> 1, wn = w & 1;

    // XCD-aware tile order: XCD x (blocks x, x + 8, ...) owns a contiguous range of tile ids,
    // walked GROUP_M row tiles at a time (the A / B panels its resident blocks read stay in its L2)
    int tm, tn, split = 0;
    {
        // with split-K the (split, tile) order is split-major, so an XCD's contiguous range is mostly
        // one split's k-range over neighbouring tiles (their A / B k-slices shared in its L2)
        const int nwg = p.tiles_m * p.tiles_n, n = nwg * p.splits, bid = blockIdx.x;
        const int xcd = bid & 7, qn = n >> 3, rn = n & 7;
        const int q = (xcd < rn ? xcd * (qn + 1) : rn * (qn + 1) + (xcd - rn) * qn) + (bid >> 3);
        split = q / nwg;
        const int wg = q - split * nwg;
        const int per_group = GROUP_M * p.tiles_n;
        const int grp = wg / per_group, first_m = grp * GROUP_M;
        const int gsz = min(p.tiles_m - first_m, GROUP_M);
        const int wl = wg - grp * per_group;
        tm = first_m + wl % gsz;
        tn = wl / gsz;
    }
    const int m0 = tm * TM, n0 = tn * TN;
    const int kbase = split * p.kt_per_split;                   // this block's first k-stage
    const int nt = min(p.K / DBK - kbase, p.kt_per_split);      // >= 1 (host)

    // DMA sources: buffer loads to LDS (per-lane 32-bit byte offsets, the k-stage as the scalar
    // offset); the convolution's A operand by global_load_lds (padding pixels from a zero page).
    // A: this wave's 4 subtiles (rows (4w + s) * 16 ..); B (KC): 2 subtiles (rows (2w + s) * 16 ..);
    // B (KO): 2 groups of 4 k-rows ((2w + s) * 4 + (l >> 4)), 16-byte chunk (l & 15) ^ its swizzle
    const int lb = swz_kc(l * 16);
    const int r_in = lb >> 6, kcol = ((lb >> 4) & 3) * 8;
    const long a_bytes = LA == LCONV ? (long)p.cN * p.cH * p.cW * p.cC * 2
                       : (LA == LKO ? (long)p.K * p.lda * 2 : (long)p.M * p.lda * 2);
    const __amdgpu_buffer_rsrc_t ars_op =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.A), 0, (int)a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t brs_op = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(p.B), 0, (int)((long)(LB == LKC ? p.N : p.K) * p.ldb * 2), 0x00020000);
    // A row offsets; LCONV: the lane's pixel of each subtile as a pointer to its (h_off, w_off)-shifted
    // corner + kcol, and a bit mask of the taps that land inside the image (host: R S <= 32; rows past
    // M: no tap).  The per-stage loader is then one bit test, one 64-bit add of the stage's uniform
    // tap offset and a select of the zero page -- it used to re-derive the pixel's full offset, bounds
    // checks and a 64-bit multiply-add per subtile and stage (136 VALU per two stages against 30 for
    // the NT loader: the 3x3 convolutions ran the same kernel ~35 % slower than plain NT GEMMs)
    int ao[4], bo[2];
    const bf16_t* abase[4];
    uint32_t vmask[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int m = m0 + (4 * w + s) * 16 + r_in;
        if (LA == LCONV) {
            const int mm = m < p.M ? m : 0;
            const int n = (int)fdiv((uint32_t)mm, p.fd_PQ);
            const int rem = mm - n * p.cP * p.cQ;
            const int pp = (int)fdiv((uint32_t)rem, p.fd_Q);
            const int qq = rem - pp * p.cQ;
            const int hb = pp * p.cstride + p.h_off, wb = qq * p.cstride + p.w_off;
            uint32_t mk = 0;
            if (m < p.M) {
                for (int rr = 0; rr < p.cR; ++rr)
                    for (int ss = 0; ss < p.cS; ++ss) {
                        const int hh = hb + rr * p.h_step, ww = wb + ss * p.w_step;
                        if ((unsigned)hh < (unsigned)p.cH && (unsigned)ww < (unsigned)p.cW) mk |= 1u << (rr * p.cS + ss);
                    }
            }
            vmask[s] = mk;
            abase[s] = p.A + ((long)(n * p.cH + hb) * p.cW + wb) * p.cC + kcol;
            ao[s] = 0;
        } else if (LA == LKO) {
            // k-outer A (weight gradients): two [32 k][128] halves; instruction u = 4w + s stages
            // k-rows 4 (u & 7) .. +3 of half u >> 3
            const int u = 4 * w + s, krow = (u & 7) * 4 + (l >> 4);
            ao[s] = (krow * (int)p.lda + m0 + (u >> 3) * 128 + 8 * ((l & 15) ^ swz_ko(krow))) * 2;
        } else {
            // rows past M re-read row M - 1 (never stored; excluded from the statistics)
            ao[s] = (min(m, p.M - 1) * (int)p.lda + kcol) * 2;
        }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        if (LB == LKC) {
            bo[s] = ((n0 + (2 * w + s) * 16 + r_in) * (int)p.ldb + kcol) * 2;
        } else {
            const int krow = (2 * w + s) * 4 + (l >> 4);
            bo[s] = (krow * (int)p.ldb + n0 + 8 * ((l & 15) ^ swz_ko(krow))) * 2;
        }
    }
    const int b_kstep = LB == LKC ? DBK * 2 : DBK * (int)p.ldb * 2;   // bytes per k-stage
    auto stage = [&](int kt, int slot) {
        kt += kbase;
        char* sb = smem + slot * ST_BYTES;
        if constexpr (LA == LKO) {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int u = 4 * w + s;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(ars_op, (lds_void*)(sb + (u >> 3) * 8192 + (u & 7) * 1024), 16,
                                                         ao[s], kt * DBK * (int)p.lda * 2, 0, 0);
            }
        } else if constexpr (LA == LCONV) {
            // the stage's tap (uniform): padding pixels and rows past M read the zero page
            const int k0 = kt * DBK;
            const int tap = (int)fdiv((uint32_t)k0, p.fd_C), ci = k0 - tap * p.cC;
            const int rr = (int)fdiv((uint32_t)tap, p.fd_S), ss = tap - rr * p.cS;
            const long toff = (long)(rr * p.h_step * p.cW + ss * p.w_step) * p.cC + ci;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const bool ok = (vmask[s] >> tap) & 1u;
                glds(ok ? abase[s] + toff : p.zero, sb + (4 * w + s) * 1024);
            }
        } else {
#pragma unroll
            for (int s = 0; s < 4; ++s)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(ars_op, (lds_void*)(sb + (4 * w + s) * 1024), 16, ao[s],
                                                         kt * (DBK * 2), 0, 0);
        }
#pragma unroll
        for (int s = 0; s < 2; ++s)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(brs_op, (lds_void*)(sb + A_BYTES + (2 * w + s) * 1024), 16, bo[s],
                                                     kt * b_kstep, 0, 0);
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    // Main loop, software-pipelined across the stage barrier: stage t's fragments are in registers
    // (F) when its MFMAs start; after the first 16 of them the wave waits for stage t + 1 (stage
    // t + 2 stays in flight: 6 DMAs per wave per stage), passes the barrier -- which also tells it
    // every wave has read slot t -- stages t + 3 into slot t, reads stage t + 1's fragments (G) and
    // issues the last 16 MFMAs of stage t under those reads.  Unrolled by two (F / G alternate), the
    // ring slot is a run-time value.
    bf16x8 fa0[8], fb0[4], fa1[8], fb1[4];
    auto read_frags = [&](int slot, bf16x8 (&fa)[8], bf16x8 (&fb)[4]) {
        const char* sb = smem + slot * ST_BYTES;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            fb[j] = LB == LKC ? frag_kc(sb + A_BYTES + (wn * 4 + j) * 1024) : frag_ko(sb + A_BYTES, wn * 64 + j * 16);
#pragma unroll
        for (int i = 0; i < 8; ++i) fa[i] = LA == LKO ? frag_ko(sb + wm * 8192, i * 16) : frag_kc(sb + (wm * 8 + i) * 1024);
    };
    auto mma_half = [&](int i0, bf16x8 (&fa)[8], bf16x8 (&fb)[4]) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = i0; i < i0 + 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };
    // prologue: stages 0, 1, 2 in flight, stage 0 landed and its fragments read
    stage(0, 0);
    if (nt > 1) stage(1, 1);
    if (nt > 2) stage(2, 2);
    if (nt > 2) VMN(12);
    else if (nt > 1) VMN(6);
    else VMN(0);
    BARRIER();
    read_frags(0, fa0, fb0);
    // one stage with fragments F; G receives stage t + 1's
    auto step = [&](int t, int slot, bf16x8 (&fa)[8], bf16x8 (&fb)[4], bf16x8 (&ga)[8], bf16x8 (&gb)[4]) {
        mma_half(0, fa, fb);
        if (t + 1 < nt) {
            if (t + 2 < nt) VMN(6);
            else VMN(0);
            // this wave's reads of slot t retired before the barrier that lets slot t be restaged
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            BARRIER();
            if (t + 3 < nt) stage(t + 3, slot);
            read_frags(slot == 2 ? 0 : slot + 1, ga, gb);
        }
        mma_half(4, fa, fb);
    };
    int slot = 0, t = 0;
#pragma unroll 1
    for (; t + 2 <= nt; t += 2) {
        const int s1 = slot == 2 ? 0 : slot + 1;
        step(t, slot, fa0, fb0, fa1, fb1);
        step(t + 1, s1, fa1, fb1, fa0, fb0);
        slot = s1 == 2 ? 0 : s1 + 1;
    }
    if (t < nt) step(t, slot, fa0, fb0, fa1, fb1);

    // ---------------- epilogue: acc[i][j] = rows m0 + wm*128 + i*16 + (l & 15), columns
    // n0 + wn*64 + j*16 + 4*(l >> 4) .. +3.  The finished bf16 tile goes through LDS (the operand ring
    // is free now: 64 KB image, rows of 256 B with the 16-byte chunks XOR-swizzled by row) and leaves
    // as whole-row stores -- every store instruction writes 4 rows x 256 B, i.e. whole 128-B lines,
    // where stores from the MFMA layout touch 32 rows x 32 B each (4x the lines per instruction for
    // the vector memory path).  Stores and the residual / pre-activation loads go through buffer
    // resources of M rows: rows past M are dropped (stores) or read as zeros.
    const int r16 = l & 15, g4 = (l >> 4) * 4;
    const int mw = m0 + wm * 128;
    const int nw = n0 + wn * 64;
    const uint32_t cbytes = (uint32_t)((long)p.M * p.ldc * 2);
    float bv[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (EK != E_DGELU && p.bias) {
            const uint2 b2 = *reinterpret_cast<const uint2*>(p.bias + nw + j * 16 + g4);
            bv[j][0] = lo_f(b2.x); bv[j][1] = hi_f(b2.x); bv[j][2] = lo_f(b2.y); bv[j][3] = hi_f(b2.y);
        } else {
            bv[j][0] = bv[j][1] = bv[j][2] = bv[j][3] = 0.f;
        }
    }
    // residual (E_BF16) / saved pre-activation (E_DGELU): every site's load goes out before the
    // first store (a load's wait would also wait out the stores issued before it)
    const bf16_t* pre = EK == E_BF16 ? p.res : (EK == E_DGELU ? (const bf16_t*)p.aux : nullptr);
    // E_BNB: BN mean / inverse std of the lane's 4 columns of each column block
    float bnm[4][4], bns[4][4];
    if (EK == E_BNB) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const f32x4 mv = *reinterpret_cast<const f32x4*>(p.bn_mean + nw + j * 16 + g4);
            const f32x4 sv = *reinterpret_cast<const f32x4*>(p.bn_istd + nw + j * 16 + g4);
#pragma unroll
            for (int e = 0; e < 4; ++e) { bnm[j][e] = mv[e]; bns[j][e] = sv[e]; }
        }
    }
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x2 rb[8][4];
    if (pre) {
        const __amdgpu_buffer_rsrc_t prs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(pre), 0, (int)cbytes, 0x00020000);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                rb[i][j] = __builtin_amdgcn_raw_buffer_load_b64(
                    prs, (int)(((long)(mw + i * 16 + r16) * p.ldc + nw + j * 16 + g4) * 2), 0, 0);
    }
    // tile image: row r (0..255) of 256 B, its 8-byte unit u (0..31) at r * 256 + ((u ^ (r & 15)) << 3).
    // An 8-byte swizzle, not a 16-byte one: a ds_write_b64 lane group is 16 lanes = 16 rows of ONE
    // 8-byte unit, banked over 128 B, so the 16 rows must land on 16 distinct 8-byte slots (the 16-byte
    // chunk swizzle gave 8: a 2-way conflict on every epilogue store, the 14-16 % LDS conflict rate of
    // the short-K NT kernels in profiles/pmc_bert.md / pmc_r50.md).  A 16-byte chunk c of row r then
    // sits whole at chunk c ^ ((r >> 1) & 7), its halves swapped when r is odd (store_image swaps back).
    const int wr0 = wm * 128 + r16;                    // this lane's image row for i = 0
    auto img_off = [&](int i, int j) {
        const int u = (wn * 8 + j * 2 + (l >> 5)) * 2 + ((l >> 4) & 1);
        return (wr0 + i * 16) * 256 + ((u ^ r16) << 3);
    };
    // every wave's last fragment reads of the ring are done (each waited lgkmcnt before its MFMAs)
    BARRIER();
    const bool stats = EK != E_GELU && p.colstats;
    u32x2 yk[8][4];                                    // GELU: the output, held while aux leaves
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc(EK == E_BNB ? (void*)p.aux : (void*)p.C, 0, (int)cbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rrs =
        __builtin_amdgcn_make_buffer_rsrc(EK == E_BNB && p.res ? (void*)p.res : (void*)p.C, 0, (int)cbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(
        EK == E_BNB && p.bn_mask ? (void*)p.bn_mask : (void*)p.C, 0, (int)(cbytes / 16), 0x00020000);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        float cs[4] = {0.f, 0.f, 0.f, 0.f}, cq[4] = {0.f, 0.f, 0.f, 0.f};
        // E_BNB: this column block's BN input, residual and mask bits of the 8 row blocks, loaded
        // together (rows past M read zeros)
        u32x2 bx[8], br[8];
        uint32_t bmk[8];
        if (EK == E_BNB) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int o = (mw + i * 16 + r16) * (int)p.ldc + nw + j * 16 + g4;
                bx[i] = __builtin_amdgcn_raw_buffer_load_b64(xrs, o * 2, 0, 0);
                br[i] = p.res ? __builtin_amdgcn_raw_buffer_load_b64(rrs, o * 2, 0, 0) : u32x2{0u, 0u};
                bmk[i] = p.bn_mask ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(mrs, o >> 3, 0, 0) >> (o & 4) : 0xfu;
            }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int m = mw + i * 16 + r16;
            const f32x4 a = acc[i][j];
            uint32_t lo, hi;
            if (EK == E_BF16) {
                float rv[4] = {0.f, 0.f, 0.f, 0.f};
                if (pre) { rv[0] = lo_f(rb[i][j][0]); rv[1] = hi_f(rb[i][j][0]); rv[2] = lo_f(rb[i][j][1]); rv[3] = hi_f(rb[i][j][1]); }
                lo = pack2bf(a[0] + bv[j][0] + rv[0], a[1] + bv[j][1] + rv[1]);
                hi = pack2bf(a[2] + bv[j][2] + rv[2], a[3] + bv[j][3] + rv[3]);
                *reinterpret_cast<uint2*>(smem + img_off(i, j)) = make_uint2(lo, hi);
            } else if (EK == E_GELU) {
                const float z[4] = {a[0] + bv[j][0], a[1] + bv[j][1], a[2] + bv[j][2], a[3] + bv[j][3]};
                const f32x2_t y0 = gelu_erf2(f32x2_t{z[0], z[1]}), y1 = gelu_erf2(f32x2_t{z[2], z[3]});
                lo = pack2bf(y0.x, y0.y);
                hi = pack2bf(y1.x, y1.y);
                yk[i][j] = u32x2{lo, hi};
                // the pre-activation leaves first (aux); without aux the output goes straight in
                *reinterpret_cast<uint2*>(smem + img_off(i, j)) =
                    p.aux ? make_uint2(pack2bf(z[0], z[1]), pack2bf(z[2], z[3])) : make_uint2(lo, hi);
            } else if (EK == E_BNB) {
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t rw = br[i][e >> 1];
                    const float rv = (e & 1) ? hi_f(rw) : lo_f(rw);
                    v[e] = ((bmk[i] >> e) & 1u) ? a[e] + rv : 0.f;
                }
                lo = pack2bf(v[0], v[1]);
                hi = pack2bf(v[2], v[3]);
                *reinterpret_cast<uint2*>(smem + img_off(i, j)) = make_uint2(lo, hi);
            } else {
                const u32x2 z2 = rb[i][j];
                const f32x2_t d0 = f32x2_t{a[0], a[1]} * gelu_erf_grad2(f32x2_t{lo_f(z2[0]), hi_f(z2[0])});
                const f32x2_t d1 = f32x2_t{a[2], a[3]} * gelu_erf_grad2(f32x2_t{lo_f(z2[1]), hi_f(z2[1])});
                lo = pack2bf(d0.x, d0.y);
                hi = pack2bf(d1.x, d1.y);
                *reinterpret_cast<uint2*>(smem + img_off(i, j)) = make_uint2(lo, hi);
            }
            if (stats) {
                const bool keep = m < p.M;                 // rows past M: not stored, not counted
                const float tv[4] = {keep ? lo_f(lo) : 0.f, keep ? hi_f(lo) : 0.f, keep ? lo_f(hi) : 0.f,
                                     keep ? hi_f(hi) : 0.f};
                if (EK == E_BNB) {
                    const float xv[4] = {lo_f(bx[i][0]), hi_f(bx[i][0]), lo_f(bx[i][1]), hi_f(bx[i][1])};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        cs[e] += tv[e];
                        cq[e] += tv[e] * (xv[e] - bnm[j][e]) * bns[j][e];
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        cs[e] += tv[e];
                        cq[e] += tv[e] * tv[e];
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
            if (r16 == 0) {
                // one partial row per 128 output rows (as the 256x256 kernel: row 2 tm + wm)
                float* row = p.colstats + (long)(tm * 2 + wm) * 2 * p.N;
                const int n = nw + j * 16 + g4;
                *reinterpret_cast<f32x4*>(row + n) = (f32x4){cs[0], cs[1], cs[2], cs[3]};
                *reinterpret_cast<f32x4*>(row + p.N + n) = (f32x4){cq[0], cq[1], cq[2], cq[3]};
            }
        }
    }
    // whole-row stores of the image: wave w takes rows 4 it + (l >> 4) of its 64-row quarter, lane
    // chunk l & 15 (16 B); 16 instructions per wave, each 4 rows x 256 B
    auto store_image = [&](bf16_t* dst, long ld, uint32_t bytes, bool acc_c, bool nt = false) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        BARRIER();
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)bytes, 0x00020000);
        const int c = l & 15;
        const bool odd = (l >> 4) & 1;                 // r & 1 for every it
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            const int r = w * 64 + it * 4 + (l >> 4);
            u32x4 v = *reinterpret_cast<const u32x4*>(smem + r * 256 + ((c ^ ((r >> 1) & 7)) << 4));
            if (odd) v = u32x4{v[2], v[3], v[0], v[1]};
            const int off = (int)(((long)(m0 + r) * ld + n0 + c * 8) * 2);
            if (acc_c) {   // C += result (weight gradients into their arena slot), summed in fp32
                const u32x4 o = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    v[e] = pack2bf(lo_f(v[e]) + lo_f(o[e]), hi_f(v[e]) + hi_f(o[e]));
            }
            if (nt) __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 2);   // cache policy: nt
            else __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
        }
    };
    if (p.splits > 1) {            // bf16 partial tile of this split
        store_image(p.ws + (long)split * p.M * p.N, p.N, (uint32_t)((long)p.M * p.N * 2), false);
        return;
    }
    if (EK == E_GELU && p.aux) {
        store_image(p.aux, p.ldc, cbytes, false, (p.nt_store & 1) != 0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        BARRIER();                                     // every image read done before it is rewritten
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                *reinterpret_cast<uint2*>(smem + img_off(i, j)) = make_uint2(yk[i][j][0], yk[i][j][1]);
    }
    store_image(p.C, p.ldc, cbytes, p.accumulate != 0, (p.nt_store & 2) != 0);
}

// split-K reduce of the weight-gradient path: C (+)= sum of the bf16 partial tiles, 8 columns per
// thread, slabs summed in split order in fp32 (groups of 4 loads in flight)
__global__ __launch_bounds__(256) void duo_reduce_k(const bf16_t* __restrict__ ws, bf16_t* __restrict__ C, long ldc,
                                                    int M, int N, int splits, int accumulate) {
    const long n8 = N / 8, total = (long)M * n8, slab = (long)M * N;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int m = (int)(i / n8), n = (int)(i - (long)m * n8) * 8;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        const bf16_t* pb = ws + (long)m * N + n;
        auto add = [&](const uint4& r) {
            const uint32_t wd[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) { v[2 * e] += lo_f(wd[e]); v[2 * e + 1] += hi_f(wd[e]); }
        };
        int s = 0;
        for (; s + 4 <= splits; s += 4) {
            uint4 r[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) r[j] = *reinterpret_cast<const uint4*>(pb + (s + j) * slab);
#pragma unroll
            for (int j = 0; j < 4; ++j) add(r[j]);
        }
        for (; s < splits; ++s) add(*reinterpret_cast<const uint4*>(pb + s * slab));
        bf16_t* cp = C + (long)m * ldc + n;
        if (accumulate) {
            float o[8];
            load8(cp, o);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += o[e];
        }
        store8(cp, v);
    }
}

template <int LA, int LB>
int launch(const DuoParams& p, int ek, hipStream_t st) {
    const dim3 grid(p.tiles_m * p.tiles_n), block(NTH);
    switch (ek) {
        case E_BF16: hipLaunchKernelGGL((gemm_duo_k<LA, LB, E_BF16>), grid, block, 0, st, p); break;
        case E_GELU: hipLaunchKernelGGL((gemm_duo_k<LA, LB, E_GELU>), grid, block, 0, st, p); break;
        case E_DGELU: hipLaunchKernelGGL((gemm_duo_k<LA, LB, E_DGELU>), grid, block, 0, st, p); break;
        default: hipLaunchKernelGGL((gemm_duo_k<LA, LB, E_BNB>), grid, block, 0, st, p); break;
    }
    return (int)hipGetLastError();
}

}  // namespace

// C[M, N] = A[M, K] op(B) (+ epilogue), bf16 in / out, fp32 accumulation, on 256 x 128 tiles with two
// workgroups per CU.  mode 0: NT (B = [N][K]), mode 1: NN (B = [K][N]), mode 3: A = the implicit im2col
// of an NHWC tensor (`conv`: the 18-int descriptor of ddl_gemm_big2, channel count % 32 == 0, no
// output row remap), B = [N][K] (a convolution forward / input gradient).
// act: 0 none (bias / residual optional), 1 GELU (bias optional; aux <- the pre-activation), 4 dGELU
// (aux = the pre-activation: C = acc * GELU'(aux); no bias / residual), 5 BatchNorm backward (side
// arguments from ddl_gemm_bnb; aux = the BN input, res optional, colstats required).  colstats
// (nullable, not with GELU): [2 * ceil(M / 256)][2][N] fp32, one row pair per 128 output rows.  Returns
// -1 for shapes outside the contract (N % 128, K % 32, ld % 8, 16-byte alignment, 2 GB extents), -2
// for an unsupported epilogue.
DDL_API int ddl_gemm_duo(int mode, const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N,
                         int K, const void* bias, int act, void* aux, const void* res, float* colstats, const int* conv,
                         hipStream_t st) {
    BnbArgs bn{};
    if (act == 5) bn = ddl_take_bnb();          // consumed by this call whatever happens next
    if (M <= 0 || N <= 0) return 0;
    if (mode != 0 && mode != 1 && mode != 3) return -1;
    if (mode == 3 && (!conv || conv[3] % 32 || conv[13] != conv[4] || conv[14] != conv[5] || conv[15] != 1 ||
                      conv[16] != 0 || conv[17] != 0 || K != conv[11] * conv[12] * conv[3] ||
                      conv[11] * conv[12] > 32))   // taps as one 32-bit validity mask per pixel
        return -1;
    if (N % TN || K % DBK || K <= 0 || lda % 8 || ldb % 8 || ldc % 8 || (mode != 3 && lda < K) || ldc < N ||
        (mode == 1 ? ldb < N : ldb < K) || ((uintptr_t)A & 15) || ((uintptr_t)B & 15) || ((uintptr_t)C & 15))
        return -1;
    int ek;
    if (act == 0) ek = E_BF16;
    else if (act == 1 && !res) ek = E_GELU;
    else if (act == 4 && aux && !bias && !res) ek = E_DGELU;
    else if (act == 5 && aux && !bias && colstats && bn.mean && bn.istd && ldc == N) ek = E_BNB;
    else return -2;
    if (ek == E_GELU && colstats) return -2;
    if ((res && ((uintptr_t)res & 7)) || (aux && ((uintptr_t)aux & 15)) || (bias && ((uintptr_t)bias & 7))) return -1;
    // 32-bit offsets: operand element offsets and output byte extents
    const long a_bytes = mode == 3 ? (long)conv[0] * conv[1] * conv[2] * conv[3] * 2 : (long)M * lda * 2;
    const long b_bytes = (long)(mode == 1 ? K : N) * ldb * 2, c_bytes = (long)M * ldc * 2;
    if (a_bytes >= (1L << 31) || b_bytes >= (1L << 31) || c_bytes >= (1L << 31)) return -1;
    DuoParams p{};
    p.A = (const bf16_t*)A; p.B = (const bf16_t*)B; p.lda = lda; p.ldb = ldb;
    p.C = (bf16_t*)C; p.ldc = ldc; p.M = M; p.N = N; p.K = K;
    p.bias = (const bf16_t*)bias; p.res = (const bf16_t*)res; p.aux = (bf16_t*)aux; p.colstats = colstats;
    p.bn_mask = bn.mask; p.bn_mean = bn.mean; p.bn_istd = bn.istd;
    p.splits = 1;
    // default 1: the pre-activation (read again only by the backward) leaves non-temporal --
    // BERT-base +0.25-0.35 % same-box (profiles/duo_nt_ab.log); the GELU output (the next GEMM's
    // operand) keeps the default policy
    static const int nt_bits = getenv("DDL_DUO_NT") ? atoi(getenv("DDL_DUO_NT")) : 1;
    p.nt_store = nt_bits;
    p.kt_per_split = K / DBK;
    p.tiles_m = (M + TM - 1) / TM;
    p.tiles_n = N / TN;
    if (mode == 3) {
        // the zero page's address on the current device (a __device__ symbol has one per device)
        static const bf16_t* zp[64] = {};
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -1;
        if (!zp[dev]) {
            void* a = nullptr;
            if (hipGetSymbolAddress(&a, HIP_SYMBOL(g_duo_zero)) != hipSuccess || !a) return -1;
            zp[dev] = (const bf16_t*)a;
        }
        p.zero = zp[dev];
        p.cN = conv[0]; p.cH = conv[1]; p.cW = conv[2]; p.cC = conv[3]; p.cP = conv[4]; p.cQ = conv[5];
        p.cstride = conv[6]; p.h_off = conv[7]; p.w_off = conv[8]; p.h_step = conv[9]; p.w_step = conv[10];
        p.cR = conv[11]; p.cS = conv[12];
        p.fd_PQ = make_fastdiv((uint32_t)(p.cP * p.cQ));
        p.fd_Q = make_fastdiv((uint32_t)p.cQ);
        p.fd_C = make_fastdiv((uint32_t)p.cC);
        p.fd_S = make_fastdiv((uint32_t)std::max(1, p.cS));
        return launch<LCONV, LKC>(p, ek, st);
    }
    return mode == 0 ? launch<LKC, LKC>(p, ek, st) : launch<LKC, LKO>(p, ek, st);
}

// TN weight gradient on the dual-workgroup kernel: C[M, N] (+)= A^T B, A = [K][M] (lda), B = [K][N] (ldb),
// bf16 C, split-K over `splits` (bf16 partial tiles in `ws`, ws_elems >= splits * M * N when splits > 1;
// then duo_reduce_k).  Needs M % 256 == 0, N % 128 == 0, K % 32 == 0, 8-element leading dimensions,
// 16-byte aligned operands, operands under 2 GB.  Returns the split count used, or -1.
DDL_API int ddl_gemm_duo_tn(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                            int splits, int accumulate, void* ws, long ws_elems, hipStream_t st) {
    if (M <= 0 || N <= 0) return 0;
    if (M % TM || N % TN || K % DBK || K <= 0 || lda % 8 || ldb % 8 || ldc % 8 || lda < M || ldb < N || ldc < N ||
        ((uintptr_t)A & 15) || ((uintptr_t)B & 15) || ((uintptr_t)C & 15))
        return -1;
    if ((long)K * lda * 2 >= (1L << 31) || (long)K * ldb * 2 >= (1L << 31) || (long)M * ldc * 2 >= (1L << 31)) return -1;
    const int nkt = K / DBK;
    if (splits < 1) splits = 1;
    if (splits > nkt) splits = nkt;
    DuoParams p{};
    p.A = (const bf16_t*)A; p.B = (const bf16_t*)B; p.lda = lda; p.ldb = ldb;
    p.C = (bf16_t*)C; p.ldc = ldc; p.M = M; p.N = N; p.K = K;
    p.tiles_m = M / TM;
    p.tiles_n = N / TN;
    p.kt_per_split = (nkt + splits - 1) / splits;
    splits = (nkt + p.kt_per_split - 1) / p.kt_per_split;
    p.splits = splits;
    p.accumulate = accumulate;
    if (splits > 1) {
        if (!ws || ws_elems < (long)splits * M * N || ((uintptr_t)ws & 15) || (long)splits * M * N * 2 >= (1L << 31))
            return -1;
        p.ws = (bf16_t*)ws;
    }
    const dim3 grid(p.tiles_m * p.tiles_n * splits);
    hipLaunchKernelGGL((gemm_duo_k<LKO, LKO, E_BF16>), grid, dim3(NTH), 0, st, p);
    if (splits > 1) {
        const long total = (long)M * (N / 8);
        const int g = (int)std::min<long>(16384, (total + 255) / 256);
        duo_reduce_k<<<g, 256, 0, st>>>(p.ws, p.C, ldc, M, N, splits, accumulate);
    }
    const int rc = (int)hipGetLastError();
    return rc ? -rc - 1 : splits;
}
