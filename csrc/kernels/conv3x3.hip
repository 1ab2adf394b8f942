// Direct 3x3 / stride-1 / pad-1 convolution for 64 -> 64 channels, NHWC bf16, on MFMA
// (ResNet stage-1 bottleneck conv2: forward, and its input gradient as the same
// convolution of dy with the flipped, transposed weight).
//
// Why not the implicit GEMM (gemm.hip CONV mode): with N = 64 output channels the
// GEMM runs 128x64 tiles that gather every input pixel nine times (once per tap)
// through registers, K = 576 is only nine K-steps, and each tile re-stages the
// whole weight -- the 56x56x64 convs ran at 330-460 TF, far from both the MFMA and
// the HBM limit.  Here each workgroup is persistent over a run of output row pairs:
//
//   * the whole weight [9 taps][64 out][64 in] (72 KB) is staged in LDS once;
//   * input rows live in a 6-slot LDS ring (plus one zero row for the padding
//     rows), each row image [66 px][64 ch] with zero pad columns; consecutive row
//     pairs of an image share two of their four input rows, so each tile brings
//     in only its two new rows (LDS-DMA, one tile ahead, overlapped with the
//     current tile's MFMAs) -- every input byte crosses HBM once;
//   * the 9 taps are 9 shifted fragment reads of the same LDS rows (no im2col);
//   * tile = 2 output rows x 64 pixel slots (W <= 64) x 64 channels; 4 waves as
//     2 (rows) x 2 (32-channel halves), each 4 x 2 v_mfma_f32_16x16x32_bf16 tiles;
//   * epilogue: bf16 out through 16-byte pair stores (v_permlane16_swap) as raw
//     buffer stores -- slots past W / H are dropped by the buffer range check, so
//     every wave issues the same 4 stores per tile and the next tile's wait for its
//     prefetched rows is a counted vmcnt(4) that never waits out those stores;
//   * BatchNorm statistics of the stored output (forward) or the BatchNorm-backward
//     reduction (dgrad: dz = (acc + res) * relu_mask, sums of dz and dz * xhat)
//     accumulate in registers over all the workgroup's tiles: one partial row per
//     workgroup instead of one per 128-pixel tile.
// Reference behaviour: the convolutions of torchvision's Bottleneck
// (reference: SURVEY.md §2.3 K1/K2 -- cuDNN implicit-GEMM convs under resnet50()).
#include "ddl_common.h"

#include <cstdlib>

namespace {

constexpr int CH = 64;                     // C_in == C_out
constexpr int NT = 256;
constexpr int PXS = 66;                    // pixel slots of a row image: pad, W <= 64, pad
constexpr int ROWB = PXS * CH * 2;         // 8448 B
constexpr int NRING = 6, ZSLOT = 6, NSLOT = 7;
constexpr int WBYTES = 9 * CH * CH * 2;    // 72 KB
constexpr int LDS_BYTES = WBYTES + NSLOT * ROWB;
constexpr int STORES_PER_TILE = 4;         // pair stores per wave per tile (vmcnt accounting)

typedef __attribute__((address_space(3))) void lds_void;

struct C3Params {
    const bf16_t* x;        // [N, H, W, 64]
    const bf16_t* w;        // [64 out][3][3][64 in]
    bf16_t* y;              // [N, H, W, 64]
    int N, H, W, HP;        // HP = row pairs per image
    int tiles, chunk;       // tiles = N * HP; tiles [b * chunk, (b + 1) * chunk) per workgroup
    float* colstats;        // [gridDim.x][2][64] or null
    const bf16_t* res;      // BNB: added before the mask (may be null)
    const bf16_t* aux;      // BNB: BatchNorm input (xhat = (aux - mean) * istd)
    const uint8_t* mask;    // BNB: ReLU bit mask (null: all kept)
    const float* mean;
    const float* istd;
    int has_res, has_mask;  // BNB: res / mask given (otherwise they point at aux, loaded and ignored)
    uint32_t y_bytes;
    int dbg;                // DDL_CONV3X3_DBG bits (timing experiments only): 1 no stores, 2 no row DMA, 4 no MFMA, 8 no epilogue
};

// 16-byte chunk swizzle of a 128-byte LDS row: chunk ^ (row & 7).  ds_read_b128 banks
// 16-lane groups (4 x 16 B = 256 B per LDS cycle); a fragment read covers 16 consecutive
// rows starting at ANY row (the tap shift s moves it), and r & 7 keeps every such group
// conflict-free, where the GEMM kernels' (r >> 1) & 7 is 2-way for odd starts.
__device__ __forceinline__ int swz(int row) { return row & 7; }

// LDS fragment read the compiler does not track (the caller places the lgkmcnt waits)
__device__ __forceinline__ bf16x8 ds_read16(uint32_t addr) {
    bf16x8 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
    return v;
}

__device__ __forceinline__ void glds(const bf16_t* g, char* dst) {
    __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)dst, 16, 0, 2);   // nt: rows are staged once
}

// LDS-DMA of input row h of image n into ring slot `slot`: W/8 wave instructions of
// 1 KB (8 pixels x 8 chunks), spread over the 4 waves; the chunk swizzle is applied on
// the source address so the DMA image stays lane-linear.
__device__ __forceinline__ void issue_row(const C3Params& p, char* smem, int n, int h, int slot, int wv, int lane) {
    char* base = smem + WBYTES + slot * ROWB + 128;    // pixel slot 1 = w 0
    const bf16_t* src = p.x + ((long)n * p.H + h) * p.W * CH;
    const int nq = p.W >> 3;
    for (int q = wv; q < nq; q += 4) {
        const int px = q * 8 + (lane >> 3);            // w
        const int c = (lane & 7) ^ swz(px + 1);
        glds(src + px * CH + c * 8, base + q * 1024);
    }
}

template <bool BNB>
__global__ __launch_bounds__(NT, 1) void conv3x3_k(C3Params p) {
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wv & 1, wn = wv >> 1;      // wave-uniform
    const int g = lane >> 4, r16 = lane & 15;

    // zero the row slots (pad columns and the zero row stay zero: the DMA writes only
    // the W interior pixels), then the weight image by DMA
    for (int i = tid; i < NSLOT * ROWB / 16; i += NT)
        reinterpret_cast<uint4*>(smem + WBYTES)[i] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    for (int q = wv; q < 72; q += 4) {                 // 1 KB = 8 weight rows of one tap
        const int t = q >> 3, k = (q & 7) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ swz(k);
        glds(p.w + ((long)k * 9 + t) * CH + c * 8, smem + q * 1024);
    }

    // BNB: this lane's BatchNorm mean / inverse std (fixed columns for the whole kernel)
    float bn_mu[2][4] = {}, bn_is[2][4] = {};
    if constexpr (BNB) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            load4(p.mean + wn * 32 + j * 16 + 4 * g, bn_mu[j]);
            load4(p.istd + wn * 32 + j * 16 + 4 * g, bn_is[j]);
        }
    }
    // per-lane LDS fragment offsets (kernel constants): A by (tap column s, k-half, pixel
    // block) relative to a row image, B absolute for (k-half, channel block) of tap 0
    const uint32_t lds_base = (uint32_t)(uintptr_t)smem;
    uint32_t aoff[3][2][4], boff[2][2];
#pragma unroll
    for (int sh = 0; sh < 3; ++sh)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int px = i * 16 + r16 + sh;
                aoff[sh][kk][i] = px * 128 + (((kk * 4 + g) ^ swz(px)) << 4);
            }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int k = wn * 32 + j * 16 + r16;
            boff[kk][j] = lds_base + k * 128 + (((kk * 4 + g) ^ swz(k)) << 4);
        }
    float st_s[2][4], st_q[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) st_s[j][r] = st_q[j][r] = 0.f;

    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(p.y, 0, (int)p.y_bytes, 0x00020000);
    const int t0 = blockIdx.x * p.chunk, t1 = min(p.tiles, t0 + p.chunk);
    int sl[4] = {ZSLOT, ZSLOT, ZSLOT, ZSLOT};
    int ptr = 0;
    bool pref = false;       // this tile's rows were prefetched by the previous tile
    bool counted = false;    // ... and the previous tile issued exactly STORES_PER_TILE stores per wave
    for (int T = t0; T < t1; ++T) {
        const int n = T / p.HP, h0 = (T - n * p.HP) * 2;
        if (!pref) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();             // every wave is past the previous tile
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int h = h0 - 1 + r;
                if (h < 0 || h >= p.H) { sl[r] = ZSLOT; continue; }
                sl[r] = ptr;
                ptr = ptr == NRING - 1 ? 0 : ptr + 1;
                issue_row(p, smem, n, h, sl[r], wv, lane);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if (counted) {
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // STORES_PER_TILE
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        // rows landed everywhere, old slots free.  A bare s_barrier: __syncthreads() would
        // also wait out this wave's output stores (vmcnt(0)), which the counted wait avoids
        __builtin_amdgcn_s_barrier();
        // prefetch the next row pair's two new rows (same image only)
        int nsl[4] = {sl[2], sl[3], ZSLOT, ZSLOT};
        const bool npref = T + 1 < t1 && h0 + 2 < p.H;   // next tile = (n, h0 + 2)
        if (npref) {
#pragma unroll
            for (int r = 2; r < 4; ++r) {
                const int h = h0 + 1 + r;
                if (h >= p.H) continue;
                nsl[r] = ptr;
                ptr = ptr == NRING - 1 ? 0 : ptr + 1;
                if (!(p.dbg & 2)) issue_row(p, smem, n, h, nsl[r], wv, lane);
            }
        }

        // BNB: this tile's epilogue operands (BN input, residual, ReLU mask) go in flight
        // now, under the MFMAs (clamped addresses for slots past W / H)
        const int h = h0 + wm;
        const bool hok = h < p.H;
        const long rowpix = ((long)n * p.H + (hok ? h : 0)) * p.W;
        uint2 xr[4][2], rr[4][2];
        uint32_t mb[4];      // ReLU mask bits of this wave's 32 columns, one dword per pixel block
        if constexpr (BNB) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int w = min(i * 16 + r16, p.W - 1);
                    const long o = (rowpix + w) * CH + wn * 32 + j * 16 + 4 * g;
                    // unconditional loads (the launcher points absent operands at aux; the
                    // flags select afterwards): a load under a branch gets waited at the join
                    xr[i][j] = *reinterpret_cast<const uint2*>(p.aux + o);
                    rr[i][j] = *reinterpret_cast<const uint2*>(p.res + o);
                    if (j == 0)   // bits picked after the MFMAs
                        mb[i] = *reinterpret_cast<const uint32_t*>(p.mask + (((rowpix + w) * CH + wn * 32) >> 3));
                }
        }

        // ---- 9 taps x 2 k-halves of MFMA from LDS
        f32x4 acc[4][2];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
        // input rows h0 + wm - 1 .. h0 + wm + 1 of this wave (selects: no dynamic private indexing)
        const int srow[3] = {wm ? sl[1] : sl[0], wm ? sl[2] : sl[1], wm ? sl[3] : sl[2]};
        // step q = (tap r*3+s, k-half kk), 18 per tile.  Fragment reads run two steps ahead
        // (three register sets) and each is issued in an MFMA's shadow, one per MFMA.  The
        // reads are inline asm with hand-placed counted waits (lgkmcnt(6) before step q:
        // step q + 1's six stay in flight): the compiler's own accounting put lgkmcnt(0)
        // in front of every other MFMA group, exposing the LDS latency of the reads
        // issued just before it.
        const uint32_t rb0 = lds_base + WBYTES + srow[0] * ROWB, rb1 = lds_base + WBYTES + srow[1] * ROWB,
                       rb2 = lds_base + WBYTES + srow[2] * ROWB;
        auto read_k = [&](int q, int k, bf16x8 (&af)[4], bf16x8 (&bfr)[2]) {
            const int tap = q >> 1, kk = q & 1, r = tap / 3, sh = tap - r * 3;
            if (k < 4) af[k] = ds_read16((r == 0 ? rb0 : r == 1 ? rb1 : rb2) + aoff[sh][kk][k]);
            else bfr[k - 4] = ds_read16(boff[kk][k - 4] + tap * (CH * CH * 2));
        };
        bf16x8 fa[3][4], fb[3][2];
#pragma unroll
        for (int k = 0; k < 6; ++k) read_k(0, k, fa[0], fb[0]);
#pragma unroll
        for (int k = 0; k < 6; ++k) read_k(1, k, fa[1], fb[1]);
#pragma unroll
        for (int q = 0; q < 18; ++q) {
            if (p.dbg & 4) break;
            if (q + 1 < 18) asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
            else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            const int c = q % 3, n2 = (q + 2) % 3;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int i = k >> 1, j = k & 1;
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[c][j], fa[c][i], acc[i][j], 0, 0, 0);
                if (k < 6 && q + 2 < 18) read_k(q + 2, k, fa[n2], fb[n2]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }

        // nothing that consumes the epilogue loads may be scheduled into the MFMA stream:
        // its wait would also wait out the row prefetch issued before those loads
        __builtin_amdgcn_sched_barrier(0);

        if (p.dbg & 8) { counted = false; sl[0] = nsl[0]; sl[1] = nsl[1]; sl[2] = nsl[2]; sl[3] = nsl[3]; pref = npref; continue; }
        // ---- epilogue: lane holds out[pixel (h0 + wm, 16 i + r16)][channels nb + 4 g .. + 3]
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int nb = wn * 32 + j * 16;
            uint32_t plo = 0, phi = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int w = i * 16 + r16;
                const bool ok = hok && w < p.W;
                float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                float xv[4] = {0.f, 0.f, 0.f, 0.f};
                if constexpr (BNB) {
                    const uint2 x2 = xr[i][j], r2 = p.has_res ? rr[i][j] : make_uint2(0u, 0u);
                    const uint32_t mbits = p.has_mask ? mb[i] >> (j * 16 + 4 * g) : 0xfu;
                    xv[0] = __uint_as_float(x2.x << 16);
                    xv[1] = __uint_as_float(x2.x & 0xffff0000u);
                    xv[2] = __uint_as_float(x2.y << 16);
                    xv[3] = __uint_as_float(x2.y & 0xffff0000u);
                    const float rv[4] = {__uint_as_float(r2.x << 16), __uint_as_float(r2.x & 0xffff0000u),
                                         __uint_as_float(r2.y << 16), __uint_as_float(r2.y & 0xffff0000u)};
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = ((mbits >> e) & 1u) ? v[e] + rv[e] : 0.f;
                }
                const uint32_t lo = pack2bf(v[0], v[1]), hi = pack2bf(v[2], v[3]);
                if (ok) {
                    const float t[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                                        __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        st_s[j][e] += t[e];
                        st_q[j][e] += BNB ? t[e] * xv[e] : t[e] * t[e];   // BNB: sum dz*x, centred at the end
                    }
                }
                if ((i & 1) == 0) { plo = lo; phi = hi; continue; }
                // pair store of row blocks (i - 1, i): odd lane rows (g = 1, 3) take block i
                const auto xs = __builtin_amdgcn_permlane16_swap(plo, lo, false, false);
                const auto ys = __builtin_amdgcn_permlane16_swap(phi, hi, false, false);
                const int ws = (lane & 16) ? w : w - 16;
                const bool sok = hok && ws < p.W;
                const uint32_t off = sok && !(p.dbg & 1) ? (uint32_t)(((rowpix + ws) * CH + nb + (lane >> 5) * 8) * 2) : 0x80000000u;
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 d = {xs[0], ys[0], xs[1], ys[1]};
                __builtin_amdgcn_raw_buffer_store_b128(d, yrs, (int)off, 0, 0);
            }
        }
        sl[0] = nsl[0]; sl[1] = nsl[1]; sl[2] = nsl[2]; sl[3] = nsl[3];
        pref = npref;
        counted = true;
    }

    // ---- one statistics row per workgroup: 16 lanes per column group (DPP), then the two row waves
    if (p.colstats) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        float* red = reinterpret_cast<float*>(smem);
        for (int t = tid; t < 2 * CH; t += NT) red[t] = 0.f;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float a = row16_sum(st_s[j][e]), b = row16_sum(st_q[j][e]);
                if constexpr (BNB) b = (b - bn_mu[j][e] * a) * bn_is[j][e];   // sum dz*(x-mean)*istd
                if (r16 == 0) {
                    const int col = wn * 32 + j * 16 + 4 * g + e;
                    atomicAdd(&red[col], a);
                    atomicAdd(&red[CH + col], b);
                }
            }
        __syncthreads();
        if (tid < 2 * CH) p.colstats[(long)blockIdx.x * 2 * CH + tid] = red[tid];
    }
}


// ======================================================================= weight gradient
// dW[k][r][s][c] = sum over output pixels p of dy[p][k] * x[p + (r - 1, s - 1)][c], as
// dW^T (rows (tap, c), columns k) on MFMA with the pixels as the reduction: the same
// persistent row-pair walk as the forward, x rows in the LDS ring, the tile's two dy
// rows in a double-buffered LDS image, both fed one tile ahead by LDS-DMA.  Fragments
// are k-major reads (ds_read_b64_tr_b16) of those images -- the 9 taps are 9 pixel
// shifts of the same x rows.  Wave w owns channels 16w..16w+15 of every tap and all 64
// k: 9 x 4 accumulator tiles (144 AGPRs) summed over all the workgroup's tiles, then one
// fp32 partial [576][64] per workgroup, reduced (and transposed) by conv3x3_wgrad_reduce_k.
// (The implicit GEMM ran this as a 64 x 576 x 802816 split-K CONVW GEMM at ~290 TF.)
constexpr int DYB = 2 * 64 * 128;                 // one dy tile image: 2 rows x 64 pixel slots
constexpr int WG_LDS = NSLOT * ROWB + 2 * DYB;    // x ring + zero row, two dy images

struct C3WParams {
    const bf16_t* x;       // [N, H, W, 64] conv input
    const bf16_t* dy;      // [N, H, W, 64] output gradient
    float* part;           // [gridDim.x][576][64]
    int N, H, W, HP, tiles, chunk;
    int dbg;
};

// transposing LDS read (ds_read_b64_tr_b16) the compiler does not track: the caller waits
// (lgkmcnt) by hand -- tracked reads drew lgkmcnt(0) waits in the middle of the MFMA stream
__device__ __forceinline__ s16x4 ds_read_tr(uint32_t addr) {
    s16x4 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
    return v;
}
// k-major fragment (rows = the image's columns) from the two tr reads at LDS addresses a, b
__device__ __forceinline__ bf16x8 tr_frag(uint32_t a, uint32_t b) {
    const s16x4 lo = ds_read_tr(a), hi = ds_read_tr(b);
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
}

// dy rows h0, h0 + 1 of image n into dy image `buf` (pixel slot swizzle: slot & 7)
__device__ __forceinline__ void issue_dy(const C3WParams& p, char* smem, int n, int h0, int buf, int wv, int lane) {
    char* base = smem + NSLOT * ROWB + buf * DYB;
    const int nq = p.W >> 3;
    for (int rr = 0; rr < 2; ++rr) {
        if (h0 + rr >= p.H) continue;      // stays zero (cleared when the buffer is recycled)
        const bf16_t* src = p.dy + ((long)n * p.H + h0 + rr) * p.W * CH;
        for (int q = wv; q < nq; q += 4) {
            const int px = q * 8 + (lane >> 3);
            const int c = (lane & 7) ^ (px & 7);
            glds(src + px * CH + c * 8, base + rr * 8192 + q * 1024);
        }
    }
}

__device__ __forceinline__ void issue_xrow(const C3WParams& p, char* smem, int n, int h, int slot, int wv, int lane) {
    char* base = smem + slot * ROWB + 128;
    const bf16_t* src = p.x + ((long)n * p.H + h) * p.W * CH;
    const int nq = p.W >> 3;
    for (int q = wv; q < nq; q += 4) {
        const int px = q * 8 + (lane >> 3);
        const int c = (lane & 7) ^ swz(px + 1);
        glds(src + px * CH + c * 8, base + q * 1024);
    }
}

__global__ __launch_bounds__(NT, 1) void conv3x3_wgrad_k(C3WParams p) {
    __shared__ __attribute__((aligned(16))) char smem[WG_LDS];
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, q4 = (lane >> 2) & 3, pq = lane & 3;
    for (int i = tid; i < WG_LDS / 16; i += NT) reinterpret_cast<uint4*>(smem)[i] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();

    // per-lane tr-read byte offsets (kernel constants; the step / row parts are scalar).
    // x (A, rows = channels 16 wv + .., k = pixels): image row (pixel slot)
    //   hw * 32 + s + 8 g + q4 (+ 4), column chunk 2 wv + (pq >> 1); the swizzle (slot & 7)
    //   depends on s but not on hw (32 | hw * 32).
    // dy (B, rows = k, k = pixels): slot (ks >> 1) * 64 + (ks & 1) * 32 + 8 g + q4 (+ 4).
    uint32_t xo[3][2], dyo[4][2];
#pragma unroll
    for (int sh = 0; sh < 3; ++sh)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int ra = sh + 8 * g + q4 + 4 * e;
            xo[sh][e] = ra * 128 + (((2 * wv + (pq >> 1)) ^ swz(ra)) << 4) + (pq & 1) * 8;
        }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int slot = 8 * g + q4 + 4 * e;
            dyo[j][e] = slot * 128 + (((2 * j + (pq >> 1)) ^ (slot & 7)) << 4) + (pq & 1) * 8;
        }

    f32x4 acc[9][4];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[t][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    const int t0 = blockIdx.x * p.chunk, t1 = min(p.tiles, t0 + p.chunk);
    int sl[4] = {ZSLOT, ZSLOT, ZSLOT, ZSLOT};
    int ptr = 0;
    bool pref = false;
    for (int T = t0; T < t1; ++T) {
        const int n = T / p.HP, h0 = (T - n * p.HP) * 2;
        const int buf = (T - t0) & 1;
        if (!pref) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int h = h0 - 1 + r;
                if (h < 0 || h >= p.H) { sl[r] = ZSLOT; continue; }
                sl[r] = ptr;
                ptr = ptr == NRING - 1 ? 0 : ptr + 1;
                issue_xrow(p, smem, n, h, sl[r], wv, lane);
            }
            issue_dy(p, smem, n, h0, buf, wv, lane);
            if (h0 + 1 >= p.H)      // odd H: the missing second dy row must read as zeros
                for (int i = tid; i < 8192 / 16; i += NT)
                    reinterpret_cast<uint4*>(smem + NSLOT * ROWB + buf * DYB + 8192)[i] = make_uint4(0u, 0u, 0u, 0u);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        // prefetch the next tile: its two new x rows and its dy rows (other dy image; a
        // missing second row -- odd H -- is cleared instead)
        int nsl[4] = {sl[2], sl[3], ZSLOT, ZSLOT};
        const bool npref = T + 1 < t1 && h0 + 2 < p.H;
        if (npref) {
#pragma unroll
            for (int r = 2; r < 4; ++r) {
                const int h = h0 + 1 + r;
                if (h >= p.H) continue;
                nsl[r] = ptr;
                ptr = ptr == NRING - 1 ? 0 : ptr + 1;
                if (!(p.dbg & 2)) issue_xrow(p, smem, n, h, nsl[r], wv, lane);
            }
            if (h0 + 3 >= p.H)
                for (int i = tid; i < 8192 / 16; i += NT)
                    reinterpret_cast<uint4*>(smem + NSLOT * ROWB + (buf ^ 1) * DYB + 8192)[i] = make_uint4(0u, 0u, 0u, 0u);
            if (!(p.dbg & 2)) issue_dy(p, smem, n, h0 + 2, buf ^ 1, wv, lane);
        }

        // 4 pixel k-steps of 32 (row ks >> 1, columns (ks & 1) * 32 ..): 9 taps x 4 k-blocks;
        // step ks + 1's fragments are read under step ks's MFMAs
        const uint32_t lds_base = (uint32_t)(uintptr_t)smem;
        const uint32_t dyb = lds_base + NSLOT * ROWB + buf * DYB;
        const uint32_t xb[4] = {lds_base + sl[0] * ROWB, lds_base + sl[1] * ROWB, lds_base + sl[2] * ROWB,
                                lds_base + sl[3] * ROWB};
        bf16x8 fx[2][9], fd[2][4];
        auto read_ks = [&](int ks, bf16x8 (&ax)[9], bf16x8 (&ad)[4]) {
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const int r = t / 3, sh = t - r * 3;
                const uint32_t rb = xb[(ks >> 1) + r] + (ks & 1) * 32 * 128;
                ax[t] = tr_frag(rb + xo[sh][0], rb + xo[sh][1]);
            }
            const uint32_t db = dyb + ks * 32 * 128;
#pragma unroll
            for (int j = 0; j < 4; ++j) ad[j] = tr_frag(db + dyo[j][0], db + dyo[j][1]);
        };
        read_ks(0, fx[0], fd[0]);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            if (p.dbg & 4) break;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // step ks's reads
            __builtin_amdgcn_sched_barrier(0);
            const int c = ks & 1;
            if (ks + 1 < 4) read_ks(ks + 1, fx[c ^ 1], fd[c ^ 1]);
#pragma unroll
            for (int t = 0; t < 9; ++t)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fd[c][j], fx[c][t], acc[t][j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        sl[0] = nsl[0]; sl[1] = nsl[1]; sl[2] = nsl[2]; sl[3] = nsl[3];
        pref = npref;
    }
    // partial dW^T of this workgroup: rows (tap, c = 16 wv + r16), 4 consecutive k per lane
    const int c = 16 * wv + (lane & 15);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            *reinterpret_cast<f32x4*>(p.part + (((long)blockIdx.x * 9 + t) * 64 + c) * 64 + j * 16 + 4 * g) = acc[t][j];
}

// out[k][m] (+)= sum_b part[b][m][k], m = tap * 64 + c (576 rows), k < 64.  Block: 2 rows
// of m x 16 k-quads x 8 slab groups, combined through LDS.
__global__ __launch_bounds__(256) void conv3x3_wgrad_reduce_k(const float* __restrict__ part, int nparts, void* out,
                                                               int out_f32, int accumulate) {
    __shared__ f32x4 red[8][32];
    const int t = threadIdx.x, quad = t & 15, mr = (t >> 4) & 1, grp = t >> 5;
    const int m = blockIdx.x * 2 + mr;
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
    int b = grp;
    for (; b + 8 < nparts; b += 16) {
        s0 += *reinterpret_cast<const f32x4*>(part + ((long)b * 576 + m) * 64 + 4 * quad);
        s1 += *reinterpret_cast<const f32x4*>(part + ((long)(b + 8) * 576 + m) * 64 + 4 * quad);
    }
    if (b < nparts) s0 += *reinterpret_cast<const f32x4*>(part + ((long)b * 576 + m) * 64 + 4 * quad);
    red[grp][t & 31] = s0 + s1;
    __syncthreads();
    if (grp == 0) {
        f32x4 v = red[0][t];
#pragma unroll
        for (int i = 1; i < 8; ++i) v += red[i][t];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const long o = (long)(4 * quad + e) * 576 + m;
            if (out_f32) {
                float* d = (float*)out + o;
                *d = accumulate ? *d + v[e] : v[e];
            } else {
                bf16_t* d = (bf16_t*)out + o;
                *d = f2bf(accumulate ? bf2f(*d) + v[e] : v[e]);
            }
        }
    }
}
}  // namespace

// Direct 3x3 stride-1 pad-1 conv, 64 -> 64 channels, W in [49, 64] with W % 8 == 0.
// BNB (aux != null): the BatchNorm-backward epilogue (see gemm.hip Params::bn_mask).
// Returns the number of statistics rows written to colstats (one per workgroup; 0 when
// colstats is null), -1 when the shape is not covered (nothing launched), or -2 - hipError.
DDL_API int ddl_conv3x3(const void* x, const void* w, void* y, int N, int H, int W, int C, int K, float* colstats,
                        const void* res, const void* aux, const uint8_t* mask, const float* mean, const float* istd,
                        int grid, hipStream_t stream) {
    if (C != CH || K != CH || W % 8 != 0 || W < 49 || W > 64 || H < 1 || N < 1) return -1;
    const long ybytes = (long)N * H * W * CH * 2;
    if (ybytes >= (1l << 31)) return -1;
    if (aux && (!mean || !istd)) return -1;
    C3Params p{};
    p.x = (const bf16_t*)x;
    p.w = (const bf16_t*)w;
    p.y = (bf16_t*)y;
    p.N = N; p.H = H; p.W = W; p.HP = (H + 1) / 2;
    p.tiles = N * p.HP;
    int g = grid > 0 ? grid : 256;
    g = std::min(g, p.tiles);
    p.chunk = (p.tiles + g - 1) / g;
    g = (p.tiles + p.chunk - 1) / p.chunk;
    p.colstats = colstats;
    p.aux = (const bf16_t*)aux;
    p.has_res = res != nullptr;
    p.has_mask = mask != nullptr;
    p.res = res ? (const bf16_t*)res : p.aux;
    p.mask = mask ? mask : (const uint8_t*)aux;
    p.mean = mean;
    p.istd = istd;
    p.y_bytes = (uint32_t)ybytes;
    static const int dbg = getenv("DDL_CONV3X3_DBG") ? atoi(getenv("DDL_CONV3X3_DBG")) : 0;
    p.dbg = dbg;
    if (aux) hipLaunchKernelGGL(conv3x3_k<true>, dim3(g), dim3(NT), 0, stream, p);
    else hipLaunchKernelGGL(conv3x3_k<false>, dim3(g), dim3(NT), 0, stream, p);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return -2 - (int)e;
    return colstats ? g : 0;
}

// Weight gradient of the direct 3x3 conv (same shape coverage as ddl_conv3x3): dw [64][3][3][64]
// (bf16 or fp32, accumulate: +=).  ws: >= grid * 576 * 64 floats (grid <= 0: 256).
// Returns 0, -1 when the shape is not covered (nothing launched), or -2 - hipError.
DDL_API int ddl_conv3x3_wgrad(const void* x, const void* dy, void* dw, int N, int H, int W, int C, int K, float* ws,
                              long ws_elems, int accumulate, int out_f32, int grid, hipStream_t stream) {
    if (C != CH || K != CH || W % 8 != 0 || W < 49 || W > 64 || H < 1 || N < 1) return -1;
    C3WParams p{};
    p.x = (const bf16_t*)x;
    p.dy = (const bf16_t*)dy;
    p.N = N; p.H = H; p.W = W; p.HP = (H + 1) / 2;
    p.tiles = N * p.HP;
    int g = grid > 0 ? grid : 256;
    g = std::min(g, p.tiles);
    p.chunk = (p.tiles + g - 1) / g;
    g = (p.tiles + p.chunk - 1) / p.chunk;
    if (ws_elems < (long)g * 576 * 64) return -1;
    p.part = ws;
    static const int dbg = getenv("DDL_CONV3X3_DBG") ? atoi(getenv("DDL_CONV3X3_DBG")) : 0;
    p.dbg = dbg;
    hipLaunchKernelGGL(conv3x3_wgrad_k, dim3(g), dim3(NT), 0, stream, p);
    hipLaunchKernelGGL(conv3x3_wgrad_reduce_k, dim3(288), dim3(256), 0, stream, (const float*)ws, g, dw, out_f32,
                       accumulate);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -2 - (int)e;
}
