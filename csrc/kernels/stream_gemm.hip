// Streaming NT GEMM with the weight operand resident in REGISTERS, for the memory-bound 1x1
// convolutions of ResNet stage 2 (and any (N, K) with N * K <= 64 Ki elements):
//   C[M, N] = A[M, K] . B[N, K]^T,  (N, K) = (512, 128) or (128, 512), bf16, fp32 accumulate,
// with the epilogues those convolutions need: BatchNorm statistics of the output (forward), the
// BatchNorm-backward reduction of the next layer (dgrad, EPI_BNB), that plus the block-input
// residual (EPI_RESBNB).
//
// Why a kernel of its own: these GEMMs move ~10x more bytes than their MFMA time (200704 x 512 x
// 128: 4 MFLOP against ~100 KB of HBM traffic per 32-row tile), and the general 128-row kernels --
// B restaged for every tile, epilogue operands loaded after the MFMAs, no overlap of one tile's
// stores with the next tile's loads -- ran them at 2.5-3.1 TB/s (profiles/gemm_trace_r50.md).  The
// stage-1 streaming kernel (skinny_gemm.hip) keeps B in LDS, which at stage 2 (128 KB of B) no
// longer leaves room for the double-buffered tiles.  Here:
//   * 8 wave64 (two per SIMD) each own N/8 output columns; a wave's B fragments for ALL of K
//     (N/8 x K bf16 = 64 VGPRs) are loaded once per workgroup and stay in registers, so LDS holds
//     only the streamed images;
//   * a persistent workgroup walks a contiguous chunk of 32-row tiles; everything the NEXT tile
//     reads -- its A rows, its epilogue operand (residual or BatchNorm input) and its ReLU-mask
//     bytes -- is in flight by LDS-DMA into the other half of double-buffered images while the
//     current tile computes (the RESBNB BatchNorm input rides in registers, a tile ahead);
//   * the epilogue writes the bf16 result into the tile's C image (in place over its operand)
//     and the tile leaves as whole rows, 1 KB of contiguous bytes per store instruction;
//   * every wave issues a fixed number of DMA and store instructions per tile, so "the next tile
//     landed" is a counted vmcnt that never waits out the stores;
//   * BatchNorm sums accumulate in registers over all of a workgroup's tiles; a wave owns whole
//     columns, so each workgroup writes one partial row with no cross-wave reduction.
// Reference behaviour: torchvision Bottleneck 1x1 convolutions under cuDNN.
#include "ddl_common.h"

#include <algorithm>

namespace {

constexpr int NW = 8, NTH = NW * 64;
enum Epi { EPI_PLAIN = 0, EPI_BNB = 2, EPI_RESBNB = 3 };

typedef __attribute__((address_space(3))) void lds_void;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct StParams {
    const bf16_t* A;
    const bf16_t* B;
    bf16_t* C;
    long M;
    int tiles, chunk;
    float* colstats;       // [gridDim.x][2][N] or null
    const bf16_t* res;     // EPI_RESBNB
    const bf16_t* aux;     // EPI_BNB / EPI_RESBNB: BatchNorm input (same layout as C)
    const uint8_t* mask;   // ReLU bit mask of the BatchNorm output (null: all kept)
    const float* mean;
    const float* istd;
    uint32_t c_bytes;
};

__device__ __forceinline__ void glds(const void* g, char* dst, int bytes) {
    if (bytes == 16) __builtin_amdgcn_global_load_lds(g, (lds_void*)dst, 16, 0, 2);   // nt: streamed once
    else __builtin_amdgcn_global_load_lds(g, (lds_void*)dst, 4, 0, 0);
}
__device__ __forceinline__ bf16x8 ds_read16(uint32_t addr) {
    bf16x8 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
    return v;
}
__device__ __forceinline__ uint2 ds_read8(uint32_t addr) {
    uint2 v;
    asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(addr));
    return v;
}
__device__ __forceinline__ uint32_t ds_read32(uint32_t addr) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(addr));
    return v;
}
__device__ __forceinline__ void ds_write8(uint32_t addr, uint2 v) {
    asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(v) : "memory");
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

// swizzled [rows][W] bf16 image: 16-byte chunk c of row r sits at chunk c ^ (r & swm): the 16
// rows a ds_read_b128 lane group touches land on 16 distinct 16-byte slots of the bank row
template <int W>
constexpr int swm() { return W / 8 >= 16 ? 15 : W / 8 - 1; }

// NROWS rows of W bf16 columns (row stride LD elements) into a swizzled [NROWS][W] LDS image by
// LDS-DMA: a fixed (compile-time) number of 1 KB instructions per wave, so the waits can count them
template <int W, int NROWS, long LD = W>
__device__ __forceinline__ void dma_rows(const bf16_t* src, long row0, long rows_valid, char* dst, int wv, int lane,
                                         long ld = LD) {
    constexpr int CPR = W / 8;                    // 16-byte chunks per row
    constexpr int RPI = CPR >= 64 ? 1 : 64 / CPR; // rows per 1 KB wave instruction
    constexpr int IPR = CPR >= 64 ? CPR / 64 : 1; // instructions per row (W > 512)
    constexpr int NINST = NROWS * IPR / RPI;
    static_assert(NINST % NW == 0, "instructions split evenly over the waves");
#pragma unroll
    for (int qq = 0; qq < NINST / NW; ++qq) {
        const int q = qq * NW + wv;
        const int r = (q / IPR) * RPI + (CPR >= 64 ? 0 : lane / CPR);
        const int cl = CPR >= 64 ? (q % IPR) * 64 + lane : lane % CPR;
        const int c = cl ^ (r & swm<W>());
        const long gr = min(row0 + r, rows_valid - 1);   // rows past the end: any valid row
        glds(src + gr * ld + c * 8, dst + q * 1024, 16);
    }
}

// NT = the whole output width, NB = the column slab one workgroup owns (NT / NB slabs; the slabs of
// one row chunk are workgroups b, b + 8, ... -- one XCD under round-robin placement, so they share
// the chunk's A rows in its L2: speed only, never correctness)
template <int NT, int NB, int K, int TM, int EPI>
__global__ __launch_bounds__(NTH, 1) void stream_gemm_k(StParams p) {
    constexpr bool BNB = EPI == EPI_BNB || EPI == EPI_RESBNB;
    constexpr int NSLAB = NT / NB;
    constexpr int CW = NB / NW;                   // columns per wave
    constexpr int NCF = CW / 16;                  // 16-column fragments per wave
    constexpr int KK = K / 32;                    // 32-deep k-steps
    constexpr int TI = TM / 16;                   // 16-row fragments per tile
    static_assert(NCF >= 1 && CW % 16 == 0 && TM % 16 == 0 && NT % NB == 0, "shape");
    constexpr int ABYTES = TM * K * 2, CBYTES = TM * NB * 2;
    constexpr int NCIMG = EPI == EPI_PLAIN ? 1 : 2;
    constexpr int MWPR = NB / 32;                 // mask words per row of the slab
    constexpr int MINST = BNB ? (TM * MWPR + 63) / 64 : 0;   // 4-byte-per-lane DMA instructions
    constexpr int MS = MINST * 256 > 1024 ? MINST * 256 : 1024;
    constexpr int OFF_A = 0, OFF_C = 2 * ABYTES, OFF_M = OFF_C + NCIMG * CBYTES;
    constexpr int LDS = OFF_M + (BNB ? 2 * MS : 0);
    static_assert(LDS <= 160 * 1024, "LDS");
    constexpr int SPW = CBYTES / 1024 / NW;       // store instructions per wave per tile (1 KB each)
    static_assert(SPW >= 1 && CBYTES % (1024 * NW) == 0, "stores split evenly over the waves");
    __shared__ __attribute__((aligned(16))) char smem[LDS];
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, r16 = lane & 15;
    // workgroup -> (column slab, row chunk)
    const int slab = NSLAB > 1 ? (int)((blockIdx.x >> 3) % NSLAB) : 0;
    const int chunk = NSLAB > 1 ? (int)((blockIdx.x & 7) + 8 * (blockIdx.x / (8 * NSLAB))) : (int)blockIdx.x;
    const int n0 = slab * NB;                     // the slab's first output column
    const int cl0 = wv * CW;                      // this wave's first column inside the slab
    const int cb = n0 + cl0;                      // ... in the output
    const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
    const __amdgpu_buffer_rsrc_t crs = rsrc(p.C, p.c_bytes);
    const bf16_t* eop = EPI == EPI_RESBNB ? p.res : p.aux;

    const int t0 = chunk * p.chunk, t1 = min(p.tiles, t0 + p.chunk);
    auto prefetch = [&](int t, int buf) {
        dma_rows<K, TM>(p.A, (long)t * TM, p.M, smem + OFF_A + buf * ABYTES, wv, lane);
        if constexpr (EPI != EPI_PLAIN)
            dma_rows<NB, TM, NT>(eop + n0, (long)t * TM, p.M, smem + OFF_C + buf * CBYTES, wv, lane);
        if constexpr (BNB) {
            // the slab's TM x NB/8 mask bytes as 4-byte-per-lane DMA instructions (a row's NB/8 bytes
            // are contiguous, rows NT/8 apart); every wave issues the same ones (identical data)
#pragma unroll
            for (int k = 0; k < MINST; ++k) {
                const int wi = k * 64 + lane, row = min(wi / MWPR, TM - 1), wc = wi % MWPR;
                const long r = min((long)t * TM + row, p.M - 1);
                const uint8_t* src = p.mask ? p.mask + r * (NT / 8) + n0 / 8 + 4 * wc : (const uint8_t*)p.A;
                glds(src, smem + OFF_M + buf * MS + k * 256, 4);
            }
        }
    };
    // EPI_RESBNB: this lane's BN-input values (rows 16 i + r16, columns cb + 16 j + 4 g ..+3) of
    // tile t, one tile ahead in registers (two sets alternating per tile; see skinny_gemm.hip)
    uint2 xa[TI][NCF], xb[TI][NCF];
    auto prefetch_x = [&](int t, uint2 (&dst)[TI][NCF]) {
#pragma unroll
        for (int i = 0; i < TI; ++i) {
            const long row = min((long)t * TM + 16 * i + r16, p.M - 1);
#pragma unroll
            for (int j = 0; j < NCF; ++j)
                dst[i][j] = *reinterpret_cast<const uint2*>(p.aux + row * NT + cb + 16 * j + 4 * g);
        }
    };
    // the wave's B fragments for the whole reduction: lane holds B[cb + 16 j + r16][32 kk + 8 g .. +7]
    bf16x8 breg[NCF][KK];
#pragma unroll
    for (int j = 0; j < NCF; ++j)
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
            breg[j][kk] = *reinterpret_cast<const bf16x8*>(p.B + (long)(cb + 16 * j + r16) * K + 32 * kk + 8 * g);
    if (t0 < t1) {
        prefetch(t0, 0);
        if constexpr (EPI == EPI_RESBNB) prefetch_x(t0, xa);
    }

    // A fragment offsets in the tile image (kernel constants)
    uint32_t aoff[TI][KK];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
#pragma unroll
        for (int i = 0; i < TI; ++i) {
            const int r = 16 * i + r16;
            aoff[i][kk] = r * (K * 2) + (((kk * 4 + g) ^ (r & swm<K>())) << 4);
        }
    // C-tile image (the slab: [TM][NB]) offset of this lane's 4 columns in row 16 i + r16, block j
    auto coff = [&](int i, int j) -> uint32_t {
        const int row = 16 * i + r16, c = (cl0 + 16 * j) / 8 + (g >> 1);
        return row * (NB * 2) + ((c ^ (row & swm<NB>())) << 4) + (g & 1) * 8;
    };

    float st_s[NCF][4], st_q[NCF][4];
#pragma unroll
    for (int j = 0; j < NCF; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) st_s[j][e] = st_q[j][e] = 0.f;

    auto tile = [&](const int t, uint2 (&xc)[TI][NCF], uint2 (&xn)[TI][NCF]) __attribute__((always_inline)) {
        const int buf = (t - t0) & 1;
        // the previous tile's stores (SPW per wave) may stay in flight; everything older -- this
        // tile's DMA (and register prefetch) issued at the previous tile's top -- has landed
        if constexpr (EPI == EPI_RESBNB) __builtin_amdgcn_s_waitcnt(0xF70 | SPW);   // vmcnt(SPW), compiler-visible
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(SPW) : "memory");
        __builtin_amdgcn_s_barrier();
        // the next tile's loads (none after the last tile: LDS-DMA still landing when the
        // workgroup exits would write into the LDS of the next workgroup on this CU)
        if (t + 1 < t1) prefetch(t + 1, buf ^ 1);
        // unconditional (a clamped row past the last tile): the same number of loads on every
        // path lets the compiler's wait before the first use of xc leave these in flight
        if constexpr (EPI == EPI_RESBNB) prefetch_x(t + 1, xn);

        const uint32_t abase = lds0 + OFF_A + buf * ABYTES;
        f32x4 acc[TI][NCF];
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < NCF; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
            bf16x8 af[TI];
#pragma unroll
            for (int i = 0; i < TI; ++i) af[i] = ds_read16(abase + aoff[i][kk]);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < NCF; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(breg[j][kk], af[i], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }

        // ---- epilogue: lane holds C[m0 + 16 i + r16][cb + 16 j + 4 g .. + 3]
        const long m0 = (long)t * TM;
        const uint32_t cimg = lds0 + OFF_C + (EPI == EPI_PLAIN ? 0 : buf * CBYTES);
        // (raw words: nothing may touch an asm ds_read's result before the lgkmcnt wait below)
        uint32_t mraw[TI][NCF];
        if constexpr (BNB) {
#pragma unroll
            for (int i = 0; i < TI; ++i) {
                const uint32_t rowm = lds0 + OFF_M + buf * MS + (16 * i + r16) * (NB / 8) + cl0 / 8;
#pragma unroll
                for (int j = 0; j < NCF; ++j)   // fragment j's 16 columns = 2 mask bytes at rowm + 2 j
                    mraw[i][j] = p.mask ? ds_read32((rowm + 2 * j) & ~3u) : ~0u;
            }
        }
        uint2 ev[TI][NCF];
        if constexpr (EPI != EPI_PLAIN) {
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < NCF; ++j) ev[i][j] = ds_read8(cimg + coff(i, j));
        }
        // the asm reads are invisible to the compiler's waits: nothing may use their
        // results above this wait (sched_barrier: ALU would otherwise move up)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < TI; ++i) {
            const bool ok = m0 + 16 * i + r16 < p.M;
#pragma unroll
            for (int j = 0; j < NCF; ++j) {
                float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                float xv[4] = {0.f, 0.f, 0.f, 0.f};
                if constexpr (EPI != EPI_PLAIN) {
                    xv[0] = __uint_as_float(ev[i][j].x << 16);
                    xv[1] = __uint_as_float(ev[i][j].x & 0xffff0000u);
                    xv[2] = __uint_as_float(ev[i][j].y << 16);
                    xv[3] = __uint_as_float(ev[i][j].y & 0xffff0000u);
                }
                if constexpr (EPI == EPI_RESBNB) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] += xv[e];      // + residual
                    xv[0] = __uint_as_float(xc[i][j].x << 16);      // the BN input for the statistics
                    xv[1] = __uint_as_float(xc[i][j].x & 0xffff0000u);
                    xv[2] = __uint_as_float(xc[i][j].y << 16);
                    xv[3] = __uint_as_float(xc[i][j].y & 0xffff0000u);
                }
                if constexpr (BNB) {
                    // bytes (rowm + 2 j), +1 sit at bits 0-15 or 16-31 of the word; columns 4 g .. +3
                    const uint32_t bits = mraw[i][j] >> (((cl0 / 8 + 2 * j) & 2) * 8 + 4 * g);
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = ((bits >> e) & 1u) ? v[e] : 0.f;
                }
                const uint32_t lo = pack2bf(v[0], v[1]), hi = pack2bf(v[2], v[3]);
                ds_write8(cimg + coff(i, j), make_uint2(lo, hi));
                if (ok) {
                    const float tq[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                                         __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        st_s[j][e] += tq[e];
                        st_q[j][e] += BNB ? tq[e] * xv[e] : tq[e] * tq[e];
                    }
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        // stores of the slab's rows: each instruction writes 1 KB (whole slab rows, NB * 2 bytes each)
        constexpr int CPR = NB * 2 / 16;                       // 16-byte chunks per slab row
        constexpr int RPI = CPR >= 64 ? 1 : 64 / CPR;
        constexpr int IPR = CPR >= 64 ? CPR / 64 : 1;
#pragma unroll
        for (int qq = 0; qq < SPW; ++qq) {
            const int q = qq * NW + wv;
            const int row = (q / IPR) * RPI + (CPR >= 64 ? 0 : lane / CPR);
            const int c = CPR >= 64 ? (q % IPR) * 64 + lane : lane % CPR;
            const u32x4 d = __builtin_bit_cast(u32x4, ds_read16(cimg + row * (NB * 2) + ((c ^ (row & swm<NB>())) << 4)));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            const long grow = m0 + row;
            const uint32_t off = grow < p.M ? (uint32_t)((grow * NT + n0 + c * 8) * 2) : 0x80000000u;
            __builtin_amdgcn_raw_buffer_store_b128(d, crs, (int)off, 0, 0);
        }
    };
    // B, the first tile's operands (and BN input): vmcnt(0), visible to the compiler's own
    // wait tracking (the register B fragments must not look outstanding inside the loop)
    __builtin_amdgcn_s_waitcnt(0xF70);
    if constexpr (EPI == EPI_RESBNB) {
        for (int t = t0; t < t1; t += 2) {
            tile(t, xa, xb);
            if (t + 1 < t1) tile(t + 1, xb, xa);
        }
    } else {
        for (int t = t0; t < t1; ++t) tile(t, xa, xb);
    }

    if (p.colstats) {
        // a wave owns its columns: lanes r16 == 0 hold the column sums after the row reduction;
        // statistics row = this workgroup's row chunk (the NSLAB slab workgroups fill its columns)
#pragma unroll
        for (int j = 0; j < NCF; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float a = row16_sum(st_s[j][e]), b = row16_sum(st_q[j][e]);
                const int col = cb + 16 * j + 4 * g + e;
                if constexpr (BNB) b = (b - p.mean[col] * a) * p.istd[col];   // sum dz * xhat
                if (r16 == 0) {
                    p.colstats[(long)chunk * 2 * NT + col] = a;
                    p.colstats[(long)chunk * 2 * NT + NT + col] = b;
                }
            }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// returns the number of statistics rows (row chunks)
template <int NT, int NB, int K, int TM, int EPI>
int launch(const StParams& p0, int grid, hipStream_t st) {
    StParams p = p0;
    constexpr int NSLAB = NT / NB;
    // one workgroup per CU (LDS + 8 waves): 256 / NSLAB row chunks, a multiple of 8 per slab set
    int chunks = grid > 0 ? grid : 256 / NSLAB;
    p.tiles = (int)((p.M + TM - 1) / TM);
    chunks = std::min(chunks, p.tiles);
    if (NSLAB > 1) chunks = std::max(8, chunks / 8 * 8);
    p.chunk = (p.tiles + chunks - 1) / chunks;
    if (NSLAB == 1) chunks = (p.tiles + p.chunk - 1) / p.chunk;
    hipLaunchKernelGGL((stream_gemm_k<NT, NB, K, TM, EPI>), dim3(chunks * NSLAB), dim3(NTH), 0, st, p);
    return chunks;
}

}  // namespace

// C[M, N] = A[M, K] B[N, K]^T for (N, K) = (512, 128), (128, 512) (ResNet stage 2, B whole in
// registers) or (1024, 256), (256, 1024) (stage 3, B in column slabs of 256 / 128 over workgroups),
// bf16, row-major contiguous.  Epilogue: aux (the BatchNorm input, same layout as C) -> the
// BatchNorm backward: C = (acc [+ res]) * relu_mask, colstats rows [sum C | sum C * (aux - mean) *
// istd] (res only for the wide outputs N = 512 / 1024); otherwise colstats (nullable) rows
// [sum C | sum C^2].  Returns the number of statistics rows written (0 without colstats; at most
// 256), -1 when not covered (nothing launched), -2 - hipError.
DDL_API int ddl_stream_gemm(const void* A, const void* B, void* C, long M, int N, int K, float* colstats,
                            const void* res, const void* aux, const uint8_t* mask, const float* mean,
                            const float* istd, int grid, hipStream_t stream) {
    if (M < 1 || M * (long)N * 2 >= (1l << 31)) return -1;
    const bool w512 = N == 512 && K == 128, w128 = N == 128 && K == 512;
    const bool w1024 = N == 1024 && K == 256, w256 = N == 256 && K == 1024;
    if (!w512 && !w128 && !w1024 && !w256) return -1;
    if (res && !aux) return -1;
    if (res && (w128 || w256)) return -1;
    if (aux && (!mean || !istd)) return -1;
    StParams p{};
    p.A = (const bf16_t*)A;
    p.B = (const bf16_t*)B;
    p.C = (bf16_t*)C;
    p.M = M;
    p.colstats = colstats;
    p.res = (const bf16_t*)res;
    p.aux = (const bf16_t*)aux;
    p.mask = mask;
    p.mean = mean;
    p.istd = istd;
    p.c_bytes = (uint32_t)(M * N * 2);
    int g;
    if (w512) {
        if (res) g = launch<512, 512, 128, 32, EPI_RESBNB>(p, grid, stream);
        else if (aux) g = launch<512, 512, 128, 32, EPI_BNB>(p, grid, stream);
        else g = launch<512, 512, 128, 64, EPI_PLAIN>(p, grid, stream);
    } else if (w128) {
        if (aux) g = launch<128, 128, 512, 32, EPI_BNB>(p, grid, stream);
        else g = launch<128, 128, 512, 64, EPI_PLAIN>(p, grid, stream);
    } else if (w1024) {
        if (res) g = launch<1024, 256, 256, 32, EPI_RESBNB>(p, grid, stream);
        else if (aux) g = launch<1024, 256, 256, 32, EPI_BNB>(p, grid, stream);
        else g = launch<1024, 256, 256, 64, EPI_PLAIN>(p, grid, stream);
    } else {
        if (aux) g = launch<256, 128, 1024, 32, EPI_BNB>(p, grid, stream);
        else g = launch<256, 128, 1024, 32, EPI_PLAIN>(p, grid, stream);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return -2 - (int)e;
    return colstats ? g : 0;
}

// ====================================================================== streaming weight gradient
// C[M, N] (+)= A^T B with A = [K][M], B = [K][N] (k-outer: the TN weight gradient dW = dY^T X of a
// 1x1 convolution, K = pixels) for the memory-bound ResNet shapes M, N in {64 .. 512}, M * N <=
// 64 Ki.  The general kernels tile the OUTPUT (128 x 64 / 256 x 128) and split K, so every operand
// row is streamed once per output tile it feeds and the split-K slabs are wide: they ran these at
// 1.8-2.6 TB/s (tuner timings in bench.py's log).  Here each workgroup (8 waves, one per CU) owns
// the WHOLE M x N output over a contiguous range of K rows:
//   * A and B rows stream through an LDS ring of 32-row slots by LDS-DMA, R - 1 slots in flight
//     (~100 KB per CU), in the swizzled k-outer image of gemm_big.hip (128-column panels of
//     256-byte rows, read by ds_read_b64_tr_b16);
//   * every operand byte is read once; the only extra traffic is one bf16 partial of M x N per
//     workgroup (32 MB at 512 x 128 against 256 MB of operands), summed by wgrad_reduce_k.
namespace {

constexpr int WS_ROWS = 32;                      // K rows per ring slot
constexpr int PANEL = WS_ROWS * 256;             // one 128-column panel of a slot: 8 KB

__device__ __forceinline__ int swz_ko2(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }

typedef __attribute__((address_space(3))) s16x4 lds_s4;
__device__ __forceinline__ s16x4 ds_read_tr4(lds_s4* __restrict__ p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(p);
}

// 16 columns (rbase .. +15 of a panel) x 32 k-rows as an MFMA operand fragment: lane holds column
// rbase + (lane & 15), k = 8 (lane >> 4) .. +7 (two transposed reads of 4 rows each)
__device__ __forceinline__ bf16x8 frag_ko(const char* panel, int rbase, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, pq = lane & 3;
    const int col = rbase + 4 * pq, chunk = col >> 3;
    const int ra = 8 * g + q, rb = ra + 4;
    const s16x4 lo = ds_read_tr4((lds_s4*)(panel + ra * 256 + ((chunk ^ swz_ko2(ra)) << 4) + (pq & 1) * 8));
    const s16x4 hi = ds_read_tr4((lds_s4*)(panel + rb * 256 + ((chunk ^ swz_ko2(rb)) << 4) + (pq & 1) * 8));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
}

struct WgParams {
    const bf16_t* A;     // [K][lda]
    const bf16_t* B;     // [K][ldb]
    long lda, ldb;
    long K;
    int rows_per_blk;    // multiple of WS_ROWS
    bf16_t* part;        // [gridDim.x][M][N]
    const bf16_t* zero;  // >= 16 zero bytes
};

// wave grid: WM waves along M x (8 / WM) along N, picked to minimise fragment reads per MFMA
template <int M, int N>
constexpr int wg_wm() {
    int best = 1, cost = 1 << 30;
    for (int wm = 1; wm <= 8; wm *= 2) {
        const int wn = 8 / wm;
        if (M % (16 * wm) || N % (16 * wn)) continue;
        const int c = M / wm / 16 + N / wn / 16;
        if (c < cost) { cost = c; best = wm; }
    }
    return best;
}

template <int M, int N>
__global__ __launch_bounds__(512, 1) void stream_wgrad_k(WgParams p) {
    constexpr int PA = M >= 128 ? M / 128 : 1, PB = N >= 128 ? N / 128 : 1;
    constexpr int SLOT = (PA + PB) * PANEL;
    constexpr int R = (150 * 1024) / SLOT < 8 ? (150 * 1024) / SLOT : 8;   // ring slots
    static_assert(R >= 3, "ring");
    constexpr int WM = wg_wm<M, N>(), WN = 8 / WM;
    constexpr int TMW = M / WM, TNW = N / WN, FI = TMW / 16, FJ = TNW / 16;
    constexpr int DPW = PA + PB;                 // DMA instructions per wave per slot
    __shared__ __attribute__((aligned(16))) char smem[R * SLOT];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm = w / WN, wn = w % WN;
    const long k0 = (long)blockIdx.x * p.rows_per_blk;
    const long k1 = min(p.K, k0 + p.rows_per_blk);
    const int nsteps = (int)((k1 - k0 + WS_ROWS - 1) / WS_ROWS);

    // DMA of slot s <- k rows [k0 + 32 t, +32): panel instruction q (0..7) covers rows 4q .. 4q+3;
    // wave w issues panel (w) of A then B (round-robin over the PA + PB panels x 8 instructions)
    auto stage = [&](int t, int s) {
        char* base = smem + s * SLOT;
#pragma unroll
        for (int d = 0; d < DPW; ++d) {
            const int inst = d * 8 + w;              // 0 .. 8 (PA + PB) - 1
            const int pnl = inst >> 3, q = inst & 7;
            const int row = 4 * q + (lane >> 4);
            const int c = (lane & 15) ^ swz_ko2(row);  // data chunk this lane's slot holds
            const long k = k0 + (long)t * WS_ROWS + row;
            const bool isA = pnl < PA;
            const int col = (isA ? pnl : pnl - PA) * 128 + 8 * c;
            const bool ok = k < k1 && col < (isA ? M : N);
            const bf16_t* src = ok ? (isA ? p.A + k * p.lda + col : p.B + k * p.ldb + col) : p.zero;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(base + pnl * PANEL + q * 1024), 16, 0, 2);
        }
    };
    f32x4 acc[FI][FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // prologue: R - 1 slots in flight
#pragma unroll
    for (int t = 0; t < R - 1; ++t)
        if (t < nsteps) stage(t, t);
    for (int t = 0; t < nsteps; ++t) {
        // slot t landed: the younger ones (t + 1 .. t + R - 2, issued if they exist) may stay in flight
        const int younger = min(R - 2, nsteps - 1 - t);
        switch (younger) {
            case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
            case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPW) : "memory"); break;
            case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * DPW) : "memory"); break;
            case 3: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * DPW) : "memory"); break;
            case 4: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * DPW) : "memory"); break;
            case 5: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 * DPW) : "memory"); break;
            default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 * DPW) : "memory"); break;
        }
        // (every wave's reads of slot t - 1 completed before this barrier: lgkmcnt(0) below)
        __builtin_amdgcn_s_barrier();
        if (t + R - 1 < nsteps) stage(t + R - 1, (t + R - 1) % R);
        const char* base = smem + (t % R) * SLOT;
        bf16x8 fa[FI], fb[FJ];
#pragma unroll
        for (int i = 0; i < FI; ++i) {
            const int r = wm * TMW + 16 * i;
            fa[i] = frag_ko(base + (r >> 7) * PANEL, r & 127, lane);
        }
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
            const int r = wn * TNW + 16 * j;
            fb[j] = frag_ko(base + (PA + (r >> 7)) * PANEL, r & 127, lane);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < FI; ++i)
#pragma unroll
            for (int j = 0; j < FJ; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    // lane holds C[wm TMW + 16 i + (lane & 15)][wn TNW + 16 j + 4 g .. +3]: one 8-byte bf16 store each
    bf16_t* out = p.part + (long)blockIdx.x * M * N;
    const int g4 = (lane >> 4) * 4, r16 = lane & 15;
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j)
            *reinterpret_cast<uint2*>(out + (long)(wm * TMW + 16 * i + r16) * N + wn * TNW + 16 * j + g4) =
                make_uint2(pack2bf(acc[i][j][0], acc[i][j][1]), pack2bf(acc[i][j][2], acc[i][j][3]));
}

// C[m][n] (+)= sum over the G bf16 partials: 64 output quads x 4 partial lanes per workgroup
__global__ __launch_bounds__(256) void wgrad_reduce_k(const bf16_t* __restrict__ part, int G, int M, int N,
                                                      bf16_t* __restrict__ C, long ldc, int accumulate) {
    __shared__ f32x4 red[256];
    const int quad = blockIdx.x * 64 + (threadIdx.x & 63), gl = threadIdx.x >> 6;
    const int nq = M * N / 4;
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    if (quad < nq) {
        const bf16_t* src = part + (long)quad * 4;
        int gg = gl;
        for (; gg + 28 < G; gg += 32) {
            uint2 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const uint2*>(src + (long)(gg + 4 * u) * M * N);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s[0] += __uint_as_float(v[u].x << 16);
                s[1] += __uint_as_float(v[u].x & 0xffff0000u);
                s[2] += __uint_as_float(v[u].y << 16);
                s[3] += __uint_as_float(v[u].y & 0xffff0000u);
            }
        }
        for (; gg < G; gg += 4) {
            const uint2 v = *reinterpret_cast<const uint2*>(src + (long)gg * M * N);
            s[0] += __uint_as_float(v.x << 16);
            s[1] += __uint_as_float(v.x & 0xffff0000u);
            s[2] += __uint_as_float(v.y << 16);
            s[3] += __uint_as_float(v.y & 0xffff0000u);
        }
    }
    red[threadIdx.x] = s;
    __syncthreads();
    if (gl != 0 || quad >= nq) return;
    const f32x4 t = red[threadIdx.x] + red[threadIdx.x + 64] + red[threadIdx.x + 128] + red[threadIdx.x + 192];
    const int m = quad * 4 / N, n = quad * 4 - m * N;
    bf16_t* dst = C + (long)m * ldc + n;
    float o[4] = {t[0], t[1], t[2], t[3]};
    if (accumulate) {
        float a[4];
        load4(dst, a);
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] += a[e];
    }
    store4(dst, o);
}

template <int M, int N>
int launch_wgrad(const WgParams& p0, int G, bf16_t* C, long ldc, int accumulate, hipStream_t st) {
    WgParams p = p0;
    hipLaunchKernelGGL((stream_wgrad_k<M, N>), dim3(G), dim3(512), 0, st, p);
    hipLaunchKernelGGL(wgrad_reduce_k, dim3((M * N / 4 + 63) / 64), dim3(256), 0, st, (const bf16_t*)p.part, G, M, N, C,
                       ldc, accumulate);
    return (int)hipGetLastError();
}

}  // namespace

// TN weight gradient C[M, N] (+)= A^T B, A = [K][lda], B = [K][ldb] bf16 (lda, ldb % 8 == 0, 16-byte
// aligned), C bf16 (ldc % 4 == 0), M, N in {64, 128, 256, 512} with M * N <= 65536.  workspace:
// >= ddl_stream_wgrad_ws(M, N) bf16 elements (the workgroups' partials); zero: >= 16 zero bytes.
// Returns -1 when the shape is not covered (nothing launched).
DDL_API long ddl_stream_wgrad_ws(int M, int N) { return 256L * M * N; }

DDL_API int ddl_stream_wgrad(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, long K,
                             int accumulate, void* workspace, long ws_elems, const void* zero, int grid,
                             hipStream_t st) {
    auto pow2 = [](int v) { return v == 64 || v == 128 || v == 256 || v == 512; };
    if (!pow2(M) || !pow2(N) || (long)M * N > 65536 || K < WS_ROWS || lda % 8 || ldb % 8 || ldc % 4 || lda < M ||
        ldb < N || ((uintptr_t)A & 15) || ((uintptr_t)B & 15) || !zero)
        return -1;
    const int G = grid > 0 ? std::min(grid, 256) : 256;
    if (!workspace || ws_elems < (long)G * M * N) return -2;
    WgParams p{};
    p.A = (const bf16_t*)A;
    p.B = (const bf16_t*)B;
    p.lda = lda;
    p.ldb = ldb;
    p.K = K;
    const long steps = (K + WS_ROWS - 1) / WS_ROWS;
    p.rows_per_blk = (int)((steps + G - 1) / G) * WS_ROWS;
    p.part = (bf16_t*)workspace;
    p.zero = (const bf16_t*)zero;
    // blocks past the end of K (K small against the grid) write zero partials: every partial is summed
    bf16_t* c = (bf16_t*)C;
#define WGR(m, n) if (M == m && N == n) return launch_wgrad<m, n>(p, G, c, ldc, accumulate, st)
    WGR(64, 64); WGR(64, 128); WGR(64, 256); WGR(64, 512);
    WGR(128, 64); WGR(128, 128); WGR(128, 256); WGR(128, 512);
    WGR(256, 64); WGR(256, 128); WGR(256, 256);
    WGR(512, 64); WGR(512, 128);
#undef WGR
    return -1;
}
