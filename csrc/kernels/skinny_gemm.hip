// Streaming GEMM for the short-reduction, memory-bound 1x1 convolutions of ResNet stage 1:
//   C[M, N] = A[M, K] . B[N, K]^T,  (N, K) = (256, 64) or (64, 256), bf16, fp32 accumulate,
// with the epilogues those convolutions need (BatchNorm statistics of the output, a
// residual, or the BatchNorm-backward reduction of the next layer).
//
// These GEMMs move ~8x more bytes than they spend in MFMA time (802816 x 256 x 64:
// 0.2 us of MFMA and ~3 us of memory per 64-row tile per CU), so the general 128/256-row
// kernels -- B staged again for every tile, epilogue operands loaded after the MFMAs,
// 16-byte pair stores that each touch 32 rows x 32 B -- ran them at 3-4 TB/s.  Here a
// persistent workgroup keeps
//   * B (32 KB) resident in LDS for its whole life, and
//   * everything the NEXT 64-row tile reads -- its A tile, its epilogue operand
//     (residual or BatchNorm input) and ReLU-mask bytes -- in flight by LDS-DMA into
//     the other half of double-buffered LDS images while the current tile computes;
// the epilogue writes the bf16 result into the tile's C image (in place over its
// operand) and the tile leaves as whole rows, 1 KB of contiguous bytes per store
// instruction (raw buffer stores: rows past M are dropped by the range check).  Every
// wave issues a fixed number of DMA and store instructions per tile, so "the next tile
// landed" is a counted vmcnt that never waits out the stores.  BatchNorm statistics
// accumulate in registers over all of a workgroup's tiles: one partial row per workgroup.
// Reference behaviour: the 1x1 convolutions of torchvision's Bottleneck under cuDNN
// (SURVEY.md §2.3 K1/K2).
#include "ddl_common.h"

#include <algorithm>
#include <cstdlib>

namespace {

constexpr int TM = 64, NT = 256;
// EPI_RESBNB (N = 256): residual added, then the BatchNorm backward as EPI_BNB -- the
// BN input is register-prefetched a tile ahead (its LDS image would not fit beside the
// residual's), the mask comes by LDS-DMA
enum Epi { EPI_PLAIN = 0, EPI_RES = 1, EPI_BNB = 2, EPI_RESBNB = 3 };
template <int EPI>
constexpr bool is_bnb() { return EPI == EPI_BNB || EPI == EPI_RESBNB; }
template <int N>
constexpr int mask_stride() { return TM * N / 8 > 1024 ? TM * N / 8 : 1024; }   // bytes per mask image

typedef __attribute__((address_space(3))) void lds_void;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct SkParams {
    const bf16_t* A;
    const bf16_t* B;
    bf16_t* C;
    long M;
    int tiles, chunk;
    float* colstats;       // [gridDim.x][2][N] or null
    const bf16_t* res;     // EPI_RES
    const bf16_t* aux;     // EPI_BNB: BatchNorm input (same layout as C)
    const uint8_t* mask;   // EPI_BNB: ReLU bit mask of the BatchNorm output (null: all kept)
    const float* mean;
    const float* istd;
    uint32_t c_bytes;
};

__device__ __forceinline__ void glds(const bf16_t* g, char* dst) {
    __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)dst, 16, 0, 2);   // nt: streamed once
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

// swizzled [rows][K] bf16 image: 16-byte chunk c of row r at chunk c ^ (r & SWM)
template <int K>
constexpr int swm() { return K == 64 ? 7 : 15; }

// NROWS rows of a [rows][K] bf16 matrix into a swizzled LDS image by LDS-DMA: a fixed
// (compile-time) number of 1 KB instructions per wave, so the waits can count them
template <int K, int NROWS>
__device__ __forceinline__ void dma_rows(const bf16_t* src, long row0, long rows_valid, char* dst, int wv, int lane) {
    constexpr int CPR = K / 8;                    // 16-byte chunks per row
    constexpr int RPI = 64 / CPR;                 // rows per 1 KB wave instruction
    constexpr int NINST = NROWS / RPI;
    static_assert(NINST % 4 == 0, "instructions split evenly over the 4 waves");
#pragma unroll
    for (int qq = 0; qq < NINST / 4; ++qq) {
        const int q = qq * 4 + wv;
        const int r = q * RPI + lane / CPR;
        const int c = (lane % CPR) ^ (r & swm<K>());
        const long gr = min(row0 + r, rows_valid - 1);   // rows past the end: any valid row
        glds(src + gr * K + c * 8, dst + q * 1024);
    }
}

template <int N, int K, int EPI>
__global__ __launch_bounds__(NT) void skinny_gemm_k(SkParams p) {
    constexpr int NCF = N / 64;                   // 16-column fragments per wave
    constexpr int KK = K / 32;
    constexpr int ABYTES = TM * K * 2, BBYTES = N * K * 2, CBYTES = TM * N * 2;
    // LDS: B | A x2 | C-tile images: PLAIN one staging image; RES / BNB the epilogue
    // operand (residual / BN input) x2, which the epilogue overwrites in place with the
    // output | BNB: ReLU-mask images x2 (1 KB each)
    constexpr int OFF_A = BBYTES, OFF_C = OFF_A + 2 * ABYTES;
    constexpr int NCIMG = EPI == EPI_PLAIN ? 1 : 2;
    constexpr int OFF_M = OFF_C + NCIMG * CBYTES;
    constexpr int MS = mask_stride<N>();
    constexpr int LDS = OFF_M + (is_bnb<EPI>() ? 2 * MS : 0);
    __shared__ __attribute__((aligned(16))) char smem[LDS];
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, r16 = lane & 15;
    const int cb = wv * 16 * NCF;                 // this wave's first column
    const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
    const __amdgpu_buffer_rsrc_t crs = rsrc(p.C, p.c_bytes);
    const bf16_t* eop = (EPI == EPI_RES || EPI == EPI_RESBNB) ? p.res : p.aux;

    const int t0 = blockIdx.x * p.chunk, t1 = min(p.tiles, t0 + p.chunk);
    // everything a tile reads comes in by LDS-DMA, one tile ahead: A, the epilogue operand,
    // the mask.  Each wave issues a fixed number of DMA instructions per tile, then its
    // stores, so "this tile's DMA landed" is vmcnt(stores of the previous tile).  (A tile
    // is only ever waited for by the tile that prefetched it + 1, which exists.)
    auto prefetch = [&](int t, int buf) {
        dma_rows<K, TM>(p.A, (long)t * TM, p.M, smem + OFF_A + buf * ABYTES, wv, lane);
        if constexpr (EPI != EPI_PLAIN) dma_rows<N, TM>(eop, (long)t * TM, p.M, smem + OFF_C + buf * CBYTES, wv, lane);
        if constexpr (is_bnb<EPI>()) {
            // 64 rows x N/8 mask bytes (512 B / 2 KB) as 4-byte-per-lane DMA instructions (the
            // mask ends on a dword: clamping never misplaces a valid row's bytes); every
            // wave issues the same ones (identical data)
            const long byte0 = (long)t * TM * (N / 8), last = p.M * (N / 8) - 4;
#pragma unroll
            for (int k = 0; k < TM * N / 8 / 256; ++k) {
                const long b = min(byte0 + (long)(k * 64 + lane) * 4, last);
                const uint8_t* src = p.mask ? p.mask + b : (const uint8_t*)p.A;
                __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(smem + OFF_M + buf * MS + k * 256), 4, 0,
                                                 0);
            }
        }
    };
    // EPI_RESBNB: this lane's BN-input values (rows 16 i + r16, columns cb + 16 j + 4 g ..+3)
    // of tile t, loaded one tile ahead into registers (issued with the DMAs, so the counted
    // wait at the top of the tile that uses them covers them too)
    // Two register sets, alternating per tile (the tile loop is unrolled by two for this
    // epilogue): no copies, and the compiler's wait before a set's first use only covers the
    // loads issued before it, not the stores behind them.
    uint2 xa[4][NCF], xb[4][NCF];
    auto prefetch_x = [&](int t, uint2 (&dst)[4][NCF]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const long row = min((long)t * TM + 16 * i + r16, p.M - 1);
#pragma unroll
            for (int j = 0; j < NCF; ++j)
                dst[i][j] = *reinterpret_cast<const uint2*>(p.aux + row * N + cb + 16 * j + 4 * g);
        }
    };
    dma_rows<K, N>(p.B, 0, N, smem, wv, lane);
    if (t0 < t1) {
        prefetch(t0, 0);
        if constexpr (EPI == EPI_RESBNB) prefetch_x(t0, xa);
    }

    // per-lane fragment byte offsets (kernel constants)
    uint32_t aoff[4][KK], boff[NCF][KK];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = 16 * i + r16;
            aoff[i][kk] = r * (K * 2) + (((kk * 4 + g) ^ (r & swm<K>())) << 4);
        }
#pragma unroll
        for (int j = 0; j < NCF; ++j) {
            const int r = cb + 16 * j + r16;
            boff[j][kk] = lds0 + r * (K * 2) + (((kk * 4 + g) ^ (r & swm<K>())) << 4);
        }
    }
    // C-tile image offset of this lane's 4 columns in row 16 i + r16, column block j
    auto coff = [&](int i, int j) -> uint32_t {
        const int row = 16 * i + r16, c = (cb + 16 * j) / 8 + (g >> 1);
        return row * (N * 2) + ((c ^ (row & swm<N>())) << 4) + (g & 1) * 8;
    };

    float st_s[NCF][4], st_q[NCF][4];
#pragma unroll
    for (int j = 0; j < NCF; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) st_s[j][e] = st_q[j][e] = 0.f;
    float bmu[NCF][4] = {}, bis[NCF][4] = {};
    if constexpr (is_bnb<EPI>()) {
#pragma unroll
        for (int j = 0; j < NCF; ++j) {
            load4(p.mean + cb + 16 * j + 4 * g, bmu[j]);
            load4(p.istd + cb + 16 * j + 4 * g, bis[j]);
        }
    }

    auto tile = [&](const int t, uint2 (&xc)[4][NCF], uint2 (&xn)[4][NCF]) __attribute__((always_inline)) {
        const int buf = (t - t0) & 1;
        if constexpr (EPI == EPI_RESBNB) {
            // the builtin (not asm) form: the compiler sees that the register-prefetched BN
            // input (older than the previous tile's stores) has landed and adds no vmcnt(0)
            // of its own before its first use (gfx9 encoding: vmcnt[3:0], expcnt 7, lgkmcnt 15)
            // (unconditional: the first tile's vmcnt(0) is issued before the loop)
            __builtin_amdgcn_s_waitcnt(0xF70 | (2 * NCF));
        } else {
            if (t == t0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NCF) : "memory");   // the previous tile's stores
        }
        __builtin_amdgcn_s_barrier();
        // the next tile's loads (none after the last tile: LDS-DMA still landing when the
        // workgroup exits would write into the LDS of the next workgroup on this CU)
        if (t + 1 < t1) prefetch(t + 1, buf ^ 1);
        // unconditional (a clamped row past the last tile): the same number of loads on every
        // path lets the compiler's wait before the first use of xc leave these in flight
        if constexpr (EPI == EPI_RESBNB) prefetch_x(t + 1, xn);

        const uint32_t abase = lds0 + OFF_A + buf * ABYTES;
        f32x4 acc[4][NCF];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NCF; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
            bf16x8 af[4], bfr[NCF];
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i] = ds_read16(abase + aoff[i][kk]);
#pragma unroll
            for (int j = 0; j < NCF; ++j) bfr[j] = ds_read16(boff[j][kk]);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < NCF; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }

        // ---- epilogue: lane holds C[m0 + 16 i + r16][cb + 16 j + 4 g .. + 3]; the bf16
        // result goes into the C-tile image (in place over the epilogue operand), then out
        // as whole rows
        const long m0 = (long)t * TM;
        const uint32_t cimg = lds0 + OFF_C + (EPI == EPI_PLAIN ? 0 : buf * CBYTES);
        // mask words of this lane's row: bits of columns (cb & ~31) + 32 w + 0..31
        uint32_t mwords[4][2] = {{~0u, ~0u}, {~0u, ~0u}, {~0u, ~0u}, {~0u, ~0u}};
        if constexpr (is_bnb<EPI>()) {
            if (p.mask) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t a = lds0 + OFF_M + buf * MS + (16 * i + r16) * (N / 8) + (cb & ~31) / 8;
                    if constexpr (NCF > 2) {
                        const uint2 w2 = ds_read8(a);
                        mwords[i][0] = w2.x;
                        mwords[i][1] = w2.y;
                    } else {
                        mwords[i][0] = ds_read32(a);
                    }
                }
            }
        }
        uint2 ev[4][NCF];
        if constexpr (EPI != EPI_PLAIN) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < NCF; ++j) ev[i][j] = ds_read8(cimg + coff(i, j));
        }
        // the asm reads are invisible to the compiler's waits: nothing may use their
        // results above this wait (sched_barrier: ALU would otherwise move up)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
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
                if constexpr (EPI == EPI_RES || EPI == EPI_RESBNB) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] += xv[e];
                }
                if constexpr (EPI == EPI_RESBNB) {   // the BN input for the statistics
                    xv[0] = __uint_as_float(xc[i][j].x << 16);
                    xv[1] = __uint_as_float(xc[i][j].x & 0xffff0000u);
                    xv[2] = __uint_as_float(xc[i][j].y << 16);
                    xv[3] = __uint_as_float(xc[i][j].y & 0xffff0000u);
                }
                if constexpr (is_bnb<EPI>()) {
                    const uint32_t bits = mwords[i][(((cb & 31) + 16 * j) >> 5)] >> (((cb + 16 * j) & 16) + 4 * g);
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = ((bits >> e) & 1u) ? v[e] : 0.f;
                }
                const uint32_t lo = pack2bf(v[0], v[1]), hi = pack2bf(v[2], v[3]);
                ds_write8(cimg + coff(i, j), make_uint2(lo, hi));
                if (EPI != EPI_RES && ok) {
                    const float tq[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                                         __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        st_s[j][e] += tq[e];
                        st_q[j][e] += is_bnb<EPI>() ? tq[e] * xv[e] : tq[e] * tq[e];
                    }
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        // whole-row stores: each instruction writes 1 KB (2 or 8 rows); 2 NCF per wave
        constexpr int RPI = 1024 / (N * 2), CPR = N * 2 / 16;
#pragma unroll
        for (int qq = 0; qq < 2 * NCF; ++qq) {
            const int q = qq * 4 + wv;
            const int row = q * RPI + lane / CPR, c = lane % CPR;
            const u32x4 d = __builtin_bit_cast(u32x4, ds_read16(cimg + row * (N * 2) + ((c ^ (row & swm<N>())) << 4)));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            const long grow = m0 + row;
            const uint32_t off = grow < p.M ? (uint32_t)((grow * N + c * 8) * 2) : 0x80000000u;
            __builtin_amdgcn_raw_buffer_store_b128(d, crs, (int)off, 0, 0);
        }
    };
    if constexpr (EPI == EPI_RESBNB) {
        __builtin_amdgcn_s_waitcnt(0xF70);      // B, the first tile's operands and BN input
        for (int t = t0; t < t1; t += 2) {
            tile(t, xa, xb);
            if (t + 1 < t1) tile(t + 1, xb, xa);
        }
    } else {
        for (int t = t0; t < t1; ++t) tile(t, xa, xb);
    }

    if (EPI != EPI_RES && p.colstats) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        float* red = reinterpret_cast<float*>(smem);
        for (int t = tid; t < 2 * N; t += NT) red[t] = 0.f;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < NCF; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float a = row16_sum(st_s[j][e]), b = row16_sum(st_q[j][e]);
                if constexpr (is_bnb<EPI>()) b = (b - bmu[j][e] * a) * bis[j][e];   // sum dz * xhat
                if (r16 == 0) {
                    const int col = cb + 16 * j + 4 * g + e;
                    atomicAdd(&red[col], a);
                    atomicAdd(&red[N + col], b);
                }
            }
        __syncthreads();
        for (int t = tid; t < 2 * N; t += NT) p.colstats[(long)blockIdx.x * 2 * N + t] = red[t];
    }
}

template <int N, int K, int EPI>
int launch(const SkParams& p0, int grid, hipStream_t st) {
    SkParams p = p0;
    constexpr int lds = N * K * 2 + 2 * TM * K * 2 + (EPI == EPI_PLAIN ? 1 : 2) * TM * N * 2 +
                        (is_bnb<EPI>() ? 2 * mask_stride<N>() : 0);
    const int per_cu = std::max(1, std::min(4, (160 * 1024) / lds));
    int g = grid > 0 ? grid : 256 * per_cu;
    g = std::min(g, p.tiles);
    p.chunk = (p.tiles + g - 1) / g;
    g = (p.tiles + p.chunk - 1) / p.chunk;
    hipLaunchKernelGGL((skinny_gemm_k<N, K, EPI>), dim3(g), dim3(NT), 0, st, p);
    return g;
}

}  // namespace

// C[M, N] = A[M, K] B[N, K]^T for (N, K) = (256, 64) or (64, 256), bf16, all row-major
// contiguous.  Epilogue: res (N = 256 only): C += res; aux (N = 64, or N = 256 with res):
// the BatchNorm backward -- C = (acc [+ res]) * relu_mask, colstats rows
// [sum C | sum C * (aux - mean) * istd];
// otherwise colstats (nullable) rows [sum C | sum C^2].  Returns the number of statistics
// rows written (0 without colstats), -1 when not covered (nothing launched), -2 - hipError.
DDL_API int ddl_skinny_gemm(const void* A, const void* B, void* C, long M, int N, int K, float* colstats,
                            const void* res, const void* aux, const uint8_t* mask, const float* mean,
                            const float* istd, int grid, hipStream_t stream) {
    if (M < 1 || M * (long)N * 2 >= (1l << 31)) return -1;
    const bool n256 = N == 256 && K == 64, n64 = N == 64 && K == 256;
    if (!n256 && !n64) return -1;
    if (res && !n256) return -1;
    if (aux && (!mean || !istd || (n256 && !res))) return -1;
    SkParams p{};
    p.A = (const bf16_t*)A;
    p.B = (const bf16_t*)B;
    p.C = (bf16_t*)C;
    p.M = M;
    p.tiles = (int)((M + TM - 1) / TM);
    p.colstats = colstats;
    p.res = (const bf16_t*)res;
    p.aux = (const bf16_t*)aux;
    p.mask = mask;
    p.mean = mean;
    p.istd = istd;
    p.c_bytes = (uint32_t)(M * N * 2);
    int g;
    if (n256) g = res ? (aux ? launch<256, 64, EPI_RESBNB>(p, grid, stream) : launch<256, 64, EPI_RES>(p, grid, stream))
                      : launch<256, 64, EPI_PLAIN>(p, grid, stream);
    else g = aux ? launch<64, 256, EPI_BNB>(p, grid, stream) : launch<64, 256, EPI_PLAIN>(p, grid, stream);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return -2 - (int)e;
    return (colstats && (!res || aux)) ? g : 0;
}
