// The ResNet stem (7x7 / stride-2 conv of the RGB image, 64 channels) as direct kernels on its
// space-to-depth form (ops/_native_conv.py _StemConvS2D): the stride-1 4x4 convolution of
// xs [N, P + 3, Q + 3, 16] (2x2 pixel blocks, 16 channels) with ws [64][4][4][16] giving
// y [N, P, Q, 64].  Forward (stem_fwd_k) and weight gradient (stem_wgrad_k); the image needs no
// input gradient.
//
// ---- forward
// The implicit GEMM (M = 3.2M pixels, N = 64, K = 256) ran at ~285 us against ~90 us of HBM
// traffic (y 411 MB + xs 108 MB): 64-wide tiles re-stage the weights per tile and gather every
// xs pixel 16 times.  stem_fwd_k keeps the weight in registers (each wave: 8 k-steps x 2
// 16-channel blocks of A fragments) and is persistent over output row quads (n, p0), 8 waves
// (two per SIMD) per workgroup:
//   * a stage holds xs rows p0 .. p0 + 6 (7 rows of 128 pixel slots x 32 B, plus a zero-page
//     filler row: 4 LDS-DMA instructions per wave; 3-slot ring, two stages in flight); the
//     16-byte halves of a pixel are swapped on odd 8-pixel groups so a fragment read (16
//     consecutive pixels, one half) is conflict-free at any tap shift;
//   * wave w computes output row p0 + (w & 3), channels 32 (w >> 2) .. +31: per 16-pixel block,
//     8 ds_read_b128 (tap pair x channel half = one 32-deep k-step) and 16 v_mfma_f32_16x16x32_bf16
//     with the weight as the A operand, so a lane ends with 8 consecutive channels of one pixel:
//     one 16-byte store, 64 contiguous bytes per pixel per instruction (the weight rows are
//     permuted to make them consecutive);
//   * optional BatchNorm statistics of the stored (bf16-rounded) output: per-lane sums over the
//     workgroup's pixels, one [2][64] partial row per workgroup (the contract of conv3x3.hip).
//
// ---- weight gradient
//   dWs[k][r][s][c] = sum over (n, p, q) of dy[n][p][q][k] * xs[n][p + r][q + s][c].
// As an implicit GEMM this is 64 x 256 x N*P*Q (3.2M pixels at batch 256): the CONVW kernel
// gathers the 16 taps of every pixel (16 x 512 B of xs per 16 pixels) and split-K-reduces
// 64 x 256 slabs -- it ran at ~320 us against ~90 us of HBM traffic (dy 411 MB + xs 108 MB).
//
// Here each workgroup (8 waves, one workgroup per CU: 144 KB of LDS) is persistent over a run of
// output row pairs (n, p0), p0 even:
//   * a stage holds dy rows p0, p0 + 1 (2 Q pixels x 128 B, one contiguous block of HBM) and
//     xs rows p0 .. p0 + 4 (5 x (Q + 3) x 32 B, contiguous too), brought in by LDS-DMA as 48
//     1-KB wave instructions (6 per wave, zero-page filler past the data), two stages in
//     flight in a 3-slot ring;
//   * the 16 taps are 16 shifted fragment reads of the same xs rows (no im2col): a 32-deep
//     k-step is two 16-pixel segments (ds_read_b64_tr_b16 "lo" = segment 2ks, "hi" = 2ks + 1),
//     a tap (r, s) is the byte offset (r (Q + 3) + s) * 32 into the row block;
//   * wave w owns taps (w >> 1, 2 (w & 1) + {0, 1}) (2 taps x 16 channels) for all 64 output
//     channels: 2 x 4 v_mfma_f32_16x16x32_bf16 tiles per k-step, accumulated over all its tiles;
//   * dy images use a 16-byte chunk swizzle c ^ 2 ((row >> 1) & 3), which spreads a segment's
//     16 rows over all 32-byte bank slots twice (a conflict-free transposed read); xs reads
//     are 512 contiguous bytes per instruction, conflict-free unswizzled;
//   * one fp32 partial [64][256] per workgroup; stem_wgrad_reduce_k sums them and writes the
//     gradient straight in the stem weight's layout [64][R][S][C] (the inverse space-to-depth
//     of the tap/channel index), accumulating into the gradient sink.
// Reference behaviour: the stem conv of torchvision's resnet50 (reference: SURVEY.md §2.3 --
// the cuDNN weight-gradient kernel under loss.backward()).
#include "ddl_common.h"

namespace {

constexpr int SK = 64;                 // output channels
constexpr int SC = 16;                 // space-to-depth channels
constexpr int NWV = 8;                 // waves per workgroup (two per SIMD)
constexpr int NT = 64 * NWV;
constexpr int NI = 6;                  // LDS-DMA instructions per wave per stage (weight gradient)
constexpr int STAGE = NWV * NI * 1024; // 48 KB
constexpr int XS_OFF = 28672;          // xs block offset in a stage (dy block: 2 Q x 128 B, Q <= 112)
constexpr int NSTAGE = 3;

typedef __attribute__((address_space(3))) void lds_void;

__device__ uint4 g_stem_zero[2];       // zero page for the filler lanes (never written)

struct StemWParams {
    const bf16_t* xs;      // [N, P + 3, Q + 3, 16]
    const bf16_t* dy;      // [N, P, Q, 64]
    float* part;           // [gridDim.x][64][256]
    int P, tiles, chunk;   // tiles = N * P / 2 row pairs; [b * chunk, (b + 1) * chunk) per workgroup
};

__device__ __forceinline__ int dswz(int row) { return 2 * ((row >> 1) & 3); }

// transposing LDS read the compiler does not track: the caller places the lgkmcnt waits
__device__ __forceinline__ s16x4 ds_read_tr(uint32_t addr) {
    s16x4 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
    return v;
}
__device__ __forceinline__ bf16x8 tr_frag(uint32_t a, uint32_t b) {
    const s16x4 lo = ds_read_tr(a), hi = ds_read_tr(b);
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
}

template <int QS>
__global__ __launch_bounds__(NT, 1) void stem_wgrad_k(StemWParams p) {
    constexpr int Q = 16 * QS, WX = Q + 3;
    constexpr int DYCH = 16 * Q;         // 16-byte chunks of dy per tile
    constexpr int XSCH = 10 * WX;        // 16-byte chunks of xs per tile (5 rows)
    static_assert(DYCH * 16 <= XS_OFF && XS_OFF + XSCH * 16 <= STAGE, "stage layout");
    __shared__ __attribute__((aligned(16))) char smem[NSTAGE * STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, q4 = (lane >> 2) & 3, pq = lane & 3;
    const int HP = p.P >> 1, HX = p.P + 3;
    const int t0 = blockIdx.x * p.chunk, nt = min(p.tiles, t0 + p.chunk) - t0;

    // chunk u = 64 d + lane of wave instruction d = wv + 8 k lands at stage byte 16 u
    auto stage = [&](int T, int slot) {
        const int n = T / HP, p0 = (T - n * HP) * 2;
        const bf16_t* dyt = p.dy + ((long)n * p.P + p0) * Q * SK;
        const bf16_t* xst = p.xs + ((long)n * HX + p0) * WX * SC;
        char* base = smem + slot * STAGE;
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const int d = wv + NWV * k, u = d * 64 + lane;
            const bf16_t* src = (const bf16_t*)g_stem_zero;
            if (u < DYCH) {
                const int row = u >> 3;
                src = dyt + row * SK + (((u & 7) ^ dswz(row)) << 3);
            } else if (u >= XS_OFF / 16 && u < XS_OFF / 16 + XSCH) {
                src = xst + (u - XS_OFF / 16) * 8;
            }
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(base + d * 1024), 16, 0, 2);   // nt
        }
    };

    // per-lane tr-read offsets.  dy (B operand, columns = output channels): segment row 4 g + q4,
    // chunk 2 i + (pq >> 1) swizzled (the swizzle only sees row bits 1..2: the same for the hi
    // segment, +16 rows, and every k-step, +32 rows).  xs (A operand, columns = the 16 channels
    // of one tap): pixel 4 g + q4 of the segment, 8 pq bytes in; wave w: tap row w >> 1, tap
    // columns 2 (w & 1) + {0, 1}.
    uint32_t ao[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = 4 * g + q4;
        ao[i] = r * 128 + (((2 * i + (pq >> 1)) ^ dswz(r)) << 4) + (pq & 1) * 8;
    }
    const uint32_t bo = XS_OFF + (4 * g + q4) * 32 + pq * 8 + (wv >> 1) * WX * 32 + 2 * (wv & 1) * 32;

    f32x4 acc[2][4];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[s][i] = (f32x4){0.f, 0.f, 0.f, 0.f};

    const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
    if (nt > 0) stage(t0, 0);
    if (nt > 1) stage(t0 + 1, 1);
    for (int T = 0; T < nt; ++T) {
        // this tile's stage landed (the next one, if issued, may stay in flight)
        if (T + 1 < nt) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // every wave's reads of the slot recycled below finished before this barrier (lgkmcnt(0)
        // ahead of the last k-step's MFMAs)
        __builtin_amdgcn_s_barrier();
        if (T + 2 < nt) stage(t0 + T + 2, (T + 2) % NSTAGE);
        const uint32_t sb = lds0 + (T % NSTAGE) * STAGE;
        bf16x8 fa[2][2], fb[2][4];
        auto read_ks = [&](int ks, bf16x8 (&a)[2], bf16x8 (&b)[4]) {
            const uint32_t da = sb + ks * 4096;
#pragma unroll
            for (int i = 0; i < 4; ++i) b[i] = tr_frag(da + ao[i], da + ao[i] + 2048);
            // segment starts (pixel 32 ks and 32 ks + 16 of the row pair) in the xs row block
            const int pa = 32 * ks, pb = pa + 16;
            const int ra = pa / Q, rb = pb / Q;
            const uint32_t xa = sb + bo + (ra * WX + pa - ra * Q) * 32;
            const uint32_t xb = sb + bo + (rb * WX + pb - rb * Q) * 32;
#pragma unroll
            for (int s = 0; s < 2; ++s) a[s] = tr_frag(xa + s * 32, xb + s * 32);
        };
        read_ks(0, fa[0], fb[0]);
#pragma unroll
        for (int ks = 0; ks < QS; ++ks) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            const int c = ks & 1;
            if (ks + 1 < QS) read_ks(ks + 1, fa[c ^ 1], fb[c ^ 1]);
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    acc[s][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[c][s], fb[c][i], acc[s][i], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    // lane holds dWs[k = 16 i + (lane & 15)][tap 2 wv + s][channels 4 g .. 4 g + 3]
    float* out = p.part + (long)blockIdx.x * SK * 256 + (lane & 15) * 256 + (2 * wv) * 16 + 4 * g;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) *reinterpret_cast<f32x4*>(out + i * 16 * 256 + s * 16) = acc[s][i];
}

// dw[k][rr][ss][c] (+)= sum_b part[b][k][col], col = tap (rr / 2, ss / 2) * 16 + space-to-depth
// channel ((rr & 1) * 2 + (ss & 1)) * 4 + c.  Block: 64 columns of one k x 4 partial groups.
__global__ __launch_bounds__(256) void stem_wgrad_reduce_k(const float* __restrict__ part, int G, void* out, int R,
                                                           int S, int C, int out_f32, int accumulate) {
    __shared__ float red[4][64];
    const int t = threadIdx.x & 63, bg = threadIdx.x >> 6;
    const int k = blockIdx.x >> 2, col = (blockIdx.x & 3) * 64 + t;
    const float* src = part + (long)k * 256 + col;
    float s0 = 0.f, s1 = 0.f;
    int b = bg;
    for (; b + 4 < G; b += 8) {
        s0 += src[(long)b * SK * 256];
        s1 += src[(long)(b + 4) * SK * 256];
    }
    if (b < G) s0 += src[(long)b * SK * 256];
    red[bg][t] = s0 + s1;
    __syncthreads();
    if (bg != 0) return;
    const float v = red[0][t] + red[1][t] + red[2][t] + red[3][t];
    const int tap = col >> 4, sub = (col >> 2) & 3, c = col & 3;
    const int rr = 2 * (tap >> 2) + (sub >> 1), ss = 2 * (tap & 3) + (sub & 1);
    if (rr >= R || ss >= S || c >= C) return;
    const long o = (((long)k * R + rr) * S + ss) * C + c;
    if (out_f32) {
        float* d = (float*)out + o;
        *d = accumulate ? *d + v : v;
    } else {
        bf16_t* d = (bf16_t*)out + o;
        *d = f2bf(accumulate ? bf2f(*d) + v : v);
    }
}

template <int QS>
void launch_stem(const StemWParams& p, int g, hipStream_t st) {
    hipLaunchKernelGGL(stem_wgrad_k<QS>, dim3(g), dim3(NT), 0, st, p);
}

// ====================================================================== forward
constexpr int FROW = 4096;             // LDS row image: 128 pixel slots x 32 B
constexpr int FROWS = 8;               // xs rows per stage: 4 output rows + 3, and a zero-page filler row
constexpr int FSTAGE = FROWS * FROW;   // 32 KB
constexpr int FNI = FSTAGE / 1024 / NWV;   // LDS-DMA instructions per wave per stage (4)

struct StemFParams {
    const bf16_t* xs;      // [N, P + 3, Q + 3, 16]
    const bf16_t* w;       // [64][256] (tap-major, 16 channels per tap)
    bf16_t* y;             // [N, P, Q, 64]
    float* colstats;       // [gridDim.x][2][64] or null
    int P, tiles, chunk;   // tiles = N * P / 4 row quads
};

// untracked 16-byte LDS read with a compile-time offset (a per-lane base + immediates keeps the
// 8 x QS fragment addresses of a tile out of the register file)
template <int OFF>
__device__ __forceinline__ bf16x8 ds_read16(uint32_t addr) {
    bf16x8 v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
    return v;
}
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

template <int QS, bool STATS>
__global__ __launch_bounds__(NT, 1) void stem_fwd_k(StemFParams p) {
    constexpr int Q = 16 * QS, WX = Q + 3;
    constexpr int NST = QS;              // 16-byte stores per wave per tile
    static_assert(WX <= 128, "row image");
    __shared__ __attribute__((aligned(16))) char smem[NSTAGE * FSTAGE];
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, r16 = lane & 15;
    const int orow = wv & 3, ch = wv >> 2;   // wave: output row p0 + orow, channels 32 ch .. + 31
    const int QP = p.P >> 2, HX = p.P + 3;
    const int t0 = blockIdx.x * p.chunk, nt = min(p.tiles, t0 + p.chunk) - t0;

    // weight fragments (A operand): row m of channel block j (of the wave's half) is output channel
    // 32 ch + 8 (m >> 2) + 4 j + (m & 3); k-step t covers taps 2t, 2t + 1 (g >> 1) and channel half g & 1
    bf16x8 wf[8][2];
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int c = 32 * ch + 8 * (r16 >> 2) + 4 * j + (r16 & 3);
            wf[t][j] = *reinterpret_cast<const bf16x8*>(p.w + c * 256 + (2 * t + (g >> 1)) * 16 + 8 * (g & 1));
        }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // chunk u = 64 d + lane (d = wv + 8 k) of a stage: row u >> 8, pixel slot (u >> 1) & 127, stored
    // half u & 1 = data half ^ bit 3 of the slot; row 7 is a zero-page filler (4 instructions per wave)
    auto stage = [&](int T, int slot) {
        const int n = T / QP, p0 = (T - n * QP) * 4;
        const bf16_t* xst = p.xs + ((long)n * HX + p0) * WX * SC;
        char* base = smem + slot * FSTAGE;
#pragma unroll
        for (int k = 0; k < FNI; ++k) {
            const int d = wv + NWV * k, u = d * 64 + lane;
            const int row = u >> 8, px = (u >> 1) & 127, h = (u & 1) ^ ((px >> 3) & 1);
            const bf16_t* src = px < WX && row < 7 ? xst + (row * WX + px) * SC + 8 * h : (const bf16_t*)g_stem_zero;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(base + d * 1024), 16, 0, 2);   // nt
        }
    };
    // B fragment (pixels = columns): lane reads pixel 16 mb + r16 + s of tap row r, s = 2 (t & 1) +
    // (g >> 1), data half g & 1 -- the stored half depends on bit 3 of r16 + s only
    uint32_t off[2];
#pragma unroll
    for (int tp = 0; tp < 2; ++tp) {
        const int x = r16 + 2 * tp + (g >> 1);
        off[tp] = x * 32 + (((g & 1) ^ ((x >> 3) & 1)) << 4);
    }

    float st_s[2][4], st_q[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) st_s[j][e] = st_q[j][e] = 0.f;

    const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
    if (nt > 0) stage(t0, 0);
    if (nt > 1) stage(t0 + 1, 1);
    for (int T = 0; T < nt; ++T) {
        // this tile's stage landed; the next stage and the previous tile's stores may stay in flight
        const bool nxt = T + 1 < nt, prv = T > 0;
        if (nxt && prv) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(FNI + NST) : "memory");
        else if (nxt) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(FNI) : "memory");
        else if (prv) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (T + 2 < nt) stage(t0 + T + 2, (T + 2) % NSTAGE);
        const int TT = t0 + T, n = TT / QP, p0 = (TT - n * QP) * 4;
        bf16_t* yrow = p.y + (((long)n * p.P + p0 + orow) * Q + r16) * SK + 32 * ch + 8 * g;
        const uint32_t rb = lds0 + (T % NSTAGE) * FSTAGE + orow * FROW;
        const uint32_t ra[2] = {rb + off[0], rb + off[1]};
        bf16x8 fb[2][8];
        auto read_mb = [&](auto mbc, bf16x8 (&b)[8]) {
            constexpr int mb = decltype(mbc)::value;
            static_for<0, 8>([&](auto tc) {
                constexpr int t = decltype(tc)::value;
                b[t] = ds_read16<(t >> 1) * FROW + mb * 512>(ra[t & 1]);
            });
        };
        read_mb(std::integral_constant<int, 0>{}, fb[0]);
        static_for<0, QS>([&](auto mbc) {
            constexpr int mb = decltype(mbc)::value;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            constexpr int c = mb & 1;
            if constexpr (mb + 1 < QS) read_mb(std::integral_constant<int, mb + 1>{}, fb[c ^ 1]);
            f32x4 acc[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int t = 0; t < 8; ++t)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t][j], fb[c][t], acc[j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            // lane: pixel 16 mb + r16, channels 32 ch + 8 g + 4 j + e
            uint32_t pk[2][2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                pk[j][0] = pack2bf(acc[j][0], acc[j][1]);
                pk[j][1] = pack2bf(acc[j][2], acc[j][3]);
                if constexpr (STATS) {
                    const float v[4] = {__uint_as_float(pk[j][0] << 16), __uint_as_float(pk[j][0] & 0xffff0000u),
                                        __uint_as_float(pk[j][1] << 16), __uint_as_float(pk[j][1] & 0xffff0000u)};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        st_s[j][e] += v[e];
                        st_q[j][e] += v[e] * v[e];
                    }
                }
            }
            bf16_t* dst = yrow + mb * 16 * SK;
            *reinterpret_cast<uint4*>(dst) = make_uint4(pk[0][0], pk[0][1], pk[1][0], pk[1][1]);
            __builtin_amdgcn_sched_barrier(0);
        });
    }
    if constexpr (STATS) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // per-row slots summed in row order (LDS float atomics from four waves would make the
        // statistics -- and training -- differ run to run in the last bits)
        float* red = reinterpret_cast<float*>(smem);   // [output row][2][64]
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float a = row16_sum(st_s[j][e]), b = row16_sum(st_q[j][e]);
                if (r16 == 0) {
                    const int col = 32 * ch + 8 * g + 4 * j + e;
                    red[orow * 2 * SK + col] = a;
                    red[orow * 2 * SK + SK + col] = b;
                }
            }
        __syncthreads();
        if (tid < 2 * SK)
            p.colstats[(long)blockIdx.x * 2 * SK + tid] = ((red[tid] + red[2 * SK + tid]) + red[4 * SK + tid]) + red[6 * SK + tid];
    }
}

template <int QS>
void launch_stem_fwd(const StemFParams& p, int g, hipStream_t st) {
    if (p.colstats) hipLaunchKernelGGL((stem_fwd_k<QS, true>), dim3(g), dim3(NT), 0, st, p);
    else hipLaunchKernelGGL((stem_fwd_k<QS, false>), dim3(g), dim3(NT), 0, st, p);
}

}  // namespace

// Stem forward on the space-to-depth operands: y [N, P, Q, 64] = the 4x4 stride-1 convolution of
// xs [N, P + 3, Q + 3, 16] with w [64][4][4][16] (bf16, contiguous, 16-byte aligned), P % 4 == 0,
// Q % 16 == 0, 16 <= Q <= 112.  colstats (optional): [grid][2][64] floats, the BatchNorm sums of y.
// Returns the statistics rows written (0 without colstats), -1 when the shape is not covered
// (nothing launched), or -2 - hipError.
DDL_API int ddl_stem_fwd(const void* xs, const void* w, void* y, int N, int P, int Q, int K, float* colstats,
                         int grid, hipStream_t stream) {
    if (K != SK || N < 1 || P < 4 || P % 4 || Q % 16 || Q < 16 || Q > 112 || ((uintptr_t)xs & 15) ||
        ((uintptr_t)w & 15) || ((uintptr_t)y & 15))
        return -1;
    StemFParams p{};
    p.xs = (const bf16_t*)xs;
    p.w = (const bf16_t*)w;
    p.y = (bf16_t*)y;
    p.colstats = colstats;
    p.P = P;
    p.tiles = N * (P / 4);
    int g = grid > 0 ? grid : 256;
    g = std::min(g, p.tiles);
    p.chunk = (p.tiles + g - 1) / g;
    g = (p.tiles + p.chunk - 1) / p.chunk;
    switch (Q / 16) {
        case 1: launch_stem_fwd<1>(p, g, stream); break;
        case 2: launch_stem_fwd<2>(p, g, stream); break;
        case 3: launch_stem_fwd<3>(p, g, stream); break;
        case 4: launch_stem_fwd<4>(p, g, stream); break;
        case 5: launch_stem_fwd<5>(p, g, stream); break;
        case 6: launch_stem_fwd<6>(p, g, stream); break;
        default: launch_stem_fwd<7>(p, g, stream); break;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return -2 - (int)e;
    return colstats ? g : 0;
}

// Stem weight gradient from the space-to-depth operands: xs [N, P + 3, Q + 3, 16], dy [N, P, Q, 64]
// (bf16, contiguous, 16-byte aligned), P even, Q % 16 == 0, 16 <= Q <= 112.  dw: the stem weight's
// gradient [64][R][S][C] (R, S <= 8, C <= 4; bf16 or fp32; accumulate: +=).  ws: >= grid * 64 * 256
// floats (grid <= 0: 256).  Returns 0, -1 when the shape is not covered (nothing launched), or
// -2 - hipError.
DDL_API long ddl_stem_wgrad_ws(int grid) { return (long)(grid > 0 ? grid : 256) * SK * 256; }

DDL_API int ddl_stem_wgrad(const void* xs, const void* dy, void* dw, int N, int P, int Q, int K, int R, int S, int C,
                           float* ws, long ws_elems, int accumulate, int out_f32, int grid, hipStream_t stream) {
    if (K != SK || N < 1 || P < 2 || P % 2 || Q % 16 || Q < 16 || Q > 112 || R < 1 || R > 8 || S < 1 || S > 8 ||
        C < 1 || C > 4 || ((uintptr_t)xs & 15) || ((uintptr_t)dy & 15) || !ws)
        return -1;
    StemWParams p{};
    p.xs = (const bf16_t*)xs;
    p.dy = (const bf16_t*)dy;
    p.P = P;
    p.tiles = N * (P / 2);
    int g = grid > 0 ? grid : 256;
    g = std::min(g, p.tiles);
    p.chunk = (p.tiles + g - 1) / g;
    g = (p.tiles + p.chunk - 1) / p.chunk;
    if (ws_elems < (long)g * SK * 256) return -1;
    p.part = ws;
    switch (Q / 16) {
        case 1: launch_stem<1>(p, g, stream); break;
        case 2: launch_stem<2>(p, g, stream); break;
        case 3: launch_stem<3>(p, g, stream); break;
        case 4: launch_stem<4>(p, g, stream); break;
        case 5: launch_stem<5>(p, g, stream); break;
        case 6: launch_stem<6>(p, g, stream); break;
        default: launch_stem<7>(p, g, stream); break;
    }
    hipLaunchKernelGGL(stem_wgrad_reduce_k, dim3(SK * 4), dim3(256), 0, stream, (const float*)ws, g, dw, R, S, C,
                       out_f32, accumulate);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -2 - (int)e;
}

// ------------------------------------------------------------------ space-to-depth transforms
// The stem's stride-2 conv runs as a stride-1 conv of the image's 2x2 space-to-depth transform
// (ops/_native_conv.py _StemConvS2D).  These build the transformed input / weight in ONE pass each
// (ATen took a pad + a permuted copy for each: four launches and two full-size intermediates).
namespace {
// xs[n][i][j][(dy * 2 + dx) * 4 + c] = x[n][2i + dy - pad][2j + dx - pad][c] (0 outside, c >= C);
// one thread per output pixel: 4 input pixels of C <= 4 channels -> 32 bytes, two 16-byte stores
__global__ __launch_bounds__(256) void s2d_input_k(const bf16_t* __restrict__ x, int N, int H, int W, int C, int pad,
                                                   bf16_t* __restrict__ xs, int Hs, int Ws) {
    const long total = (long)N * Hs * Ws;
    for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
        const int j = (int)(t % Ws);
        const long r = t / Ws;
        const int i = (int)(r % Hs), n = (int)(r / Hs);
        uint16_t v[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int h = 2 * i + (q >> 1) - pad, w = 2 * j + (q & 1) - pad;
            const bool in = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
            const bf16_t* src = x + (((long)n * H + (in ? h : 0)) * W + (in ? w : 0)) * C;
#pragma unroll
            for (int c = 0; c < 4; ++c) v[q * 4 + c] = (in && c < C) ? src[c] : (uint16_t)0;
        }
        uint4* dst = reinterpret_cast<uint4*>(xs + t * 16);
        dst[0] = make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16), v[6] | (v[7] << 16));
        dst[1] = make_uint4(v[8] | (v[9] << 16), v[10] | (v[11] << 16), v[12] | (v[13] << 16), v[14] | (v[15] << 16));
    }
}

// ws[k][r2][s2][(dy * 2 + dx) * 4 + c] = w[k][2 r2 + dy][2 s2 + dx][c] (0 past R / S / C)
__global__ __launch_bounds__(256) void s2d_weight_k(const bf16_t* __restrict__ w, int K, int R, int S, int C,
                                                    bf16_t* __restrict__ ws, int R2, int S2) {
    const long total = (long)K * R2 * S2 * 16;
    for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
        const int ch = (int)(t & 15), c = ch & 3, q = ch >> 2;
        const long r = t >> 4;
        const int s2 = (int)(r % S2), r2 = (int)((r / S2) % R2), k = (int)(r / ((long)S2 * R2));
        const int rr = 2 * r2 + (q >> 1), ss = 2 * s2 + (q & 1);
        ws[t] = (rr < R && ss < S && c < C) ? w[(((long)k * R + rr) * S + ss) * C + c] : (bf16_t)0;
    }
}
}  // namespace

DDL_API int ddl_s2d_input(const void* x, int N, int H, int W, int C, int pad, void* xs, int Hs, int Ws,
                          hipStream_t st) {
    if (C > 4 || C < 1 || 2 * Hs < H + 2 * pad || 2 * Ws < W + 2 * pad) return -1;
    const long total = (long)N * Hs * Ws;
    const int grid = (int)std::min<long>((total + 255) / 256, 8192);
    s2d_input_k<<<grid, 256, 0, st>>>((const bf16_t*)x, N, H, W, C, pad, (bf16_t*)xs, Hs, Ws);
    DDL_RETURN_LAUNCH();
}

DDL_API int ddl_s2d_weight(const void* w, int K, int R, int S, int C, void* ws, int R2, int S2, hipStream_t st) {
    if (C > 4 || C < 1 || 2 * R2 < R || 2 * S2 < S) return -1;
    const long total = (long)K * R2 * S2 * 16;
    s2d_weight_k<<<(int)std::min<long>((total + 255) / 256, 4096), 256, 0, st>>>((const bf16_t*)w, K, R, S, C,
                                                                                 (bf16_t*)ws, R2, S2);
    DDL_RETURN_LAUNCH();
}
