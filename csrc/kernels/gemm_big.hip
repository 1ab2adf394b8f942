// Large-tile bf16 GEMM for gfx950: C[M,N] = A[M,K] . B[N,K]^T (+bias)(act), the
// "NT" shape of every Linear forward (and of dgrad once W^T is materialised).
//
// Structure (the CDNA4 256x256 8-phase schedule):
//   * block tile 256x256, BK = 64, 8 wave64 (512 threads) as 2 (M) x 4 (N);
//     each wave owns a 128x64 output tile held as four 64x32 quadrants
//     (8 v_mfma_f32_16x16x32_bf16 accumulators each = 128 accumulator VGPRs);
//   * operands reach LDS by global_load_lds (LDS-DMA, 16 B per lane, no VGPR
//     staging); a K-tile is four 16 KB half-tiles (A rows 0-127 / 128-255,
//     B rows 0-127 / 128-255), two LDS buffers = 128 KB;
//   * every K-tile is computed in 4 phases, one quadrant each:
//       {ds_read the new fragments, issue one half-tile prefetch,
//        s_barrier, lgkmcnt(0), 16 MFMA (setprio 1), s_barrier};
//     the prefetch stays in flight across barriers (counted vmcnt(6) twice per
//     2 K-tiles, never vmcnt(0) in steady state), 3 half-tiles ahead;
//   * wave quadrants are interleaved (rows wm*64 and 128+wm*64, cols wn*32 and
//     128+wn*32) so each phase reads exactly one A half and/or one B half, which
//     is what lets a half-tile be restaged one phase after its last read;
//   * LDS images are 16x32 subtiles of 1 KB with the st_16x32 swizzle (byte bit
//     5 ^= bit 9) applied on the glds SOURCE address and on the ds_read, so the
//     DMA image stays lane-linear and fragment reads are conflict-free;
//   * XCD-aware bijective block remap; bias / GELU / ReLU / tanh epilogue from
//     the fp32 accumulators (GELU also stores the pre-activation for backward).
// Requirements (checked by the host): K % 128 == 0, lda/ldb % 8 == 0, 16-B aligned.
#include "ddl_common.h"

namespace {

constexpr int TB = 256, BK = 64, NTH = 512;
constexpr int HALF = 128 * 64 * 2;   // 16 KB half-tile

typedef __attribute__((address_space(3))) void lds_void;

struct BigParams {
    const bf16_t* A;
    const bf16_t* B;
    long lda, ldb;
    bf16_t* C;
    long ldc;
    int M, N, K;
    const void* bias;
    int bias_bf16;
    int act;
    bf16_t* aux;
    int accumulate;
    int tiles_m, tiles_n;
};

__device__ __forceinline__ int half_off(int buf, int x, int h) { return ((buf * 2 + x) * 2 + h) * HALF; }

__device__ __forceinline__ int swz(int b) { return b ^ (((b >> 9) & 1) << 5); }

// Issue the LDS-DMA of half-tile h of operand x (0 = A, 1 = B) for K-tile kt into buffer buf.
__device__ __forceinline__ void stage(const BigParams& p, char* smem, int buf, int x, int h, int kt, int r0tile) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const bf16_t* base = x ? p.B : p.A;
    const long ld = x ? p.ldb : p.lda;
    const int rows = x ? p.N : p.M;
    const int lb = swz(l * 16);           // logical byte this lane's DMA slot holds
    const int r = lb >> 6, c = (lb >> 4) & 3;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int sub = w * 2 + j;       // 16 subtiles of 16 rows x 32 k
        const int rb = sub >> 1, kb = sub & 1;
        int row = r0tile + h * 128 + rb * 16 + r;
        row = row < rows ? row : rows - 1;
        const bf16_t* g = base + (long)row * ld + (long)kt * BK + kb * 32 + c * 8;
        __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)(smem + half_off(buf, x, h) + sub * 1024), 16, 0, 0);
    }
}

__device__ __forceinline__ bf16x8 frag(const char* smem, int buf, int x, int h, int rb, int kb) {
    const int l = threadIdx.x & 63;
    const int pb = swz((l & 15) * 64 + (l >> 4) * 16);
    return *reinterpret_cast<const bf16x8*>(smem + half_off(buf, x, h) + (rb * 2 + kb) * 1024 + pb);
}

#define BARRIER() __builtin_amdgcn_s_barrier()
#define LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
#define VM6() asm volatile("s_waitcnt vmcnt(6)" ::: "memory")
#define VM0() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")

__device__ __forceinline__ float act_fn(float v, int act) {
    switch (act) {
        case 1: return gelu_erf(v);
        case 2: return fmaxf(v, 0.f);
        case 3: return tanhf(v);
        default: return v;
    }
}

__global__ __launch_bounds__(NTH, 2) void gemm_big_k(BigParams p) {
    __shared__ __attribute__((aligned(16))) char smem[8 * HALF];
    const int nwg = p.tiles_m * p.tiles_n;
    const int bid = blockIdx.x;
    const int xcd = bid & 7, qn_ = nwg >> 3, rn = nwg & 7;
    const int wg = (xcd < rn ? xcd * (qn_ + 1) : rn * (qn_ + 1) + (xcd - rn) * qn_) + (bid >> 3);
    const int tm = wg / p.tiles_n, tn = wg - tm * p.tiles_n;
    const int m0 = tm * TB, n0 = tn * TB;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wm = w >> 2, wn = w & 3;
    const int nK = p.K / BK;

    f32x4 acc[2][2][4][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[a][b][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    bf16x8 fa[4][2], fb0[2][2], fb1[2][2];

    auto readA = [&](int buf, int qm) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) fa[i][kk] = frag(smem, buf, 0, qm, wm * 4 + i, kk);
    };
    auto readB = [&](int buf, int qn, bf16x8 (&fb)[2][2]) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) fb[j][kk] = frag(smem, buf, 1, qn, wn * 2 + j, kk);
    };
    auto mma = [&](int qm, int qn, bf16x8 (&fb)[2][2]) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[qm][qn][i][j] =
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][kk], fa[i][kk], acc[qm][qn][i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };

    // ---------------- prologue: E <- K-tile 0 (all halves), O <- K-tile 1 (A0, B0, B1)
    stage(p, smem, 0, 0, 0, 0, m0);
    stage(p, smem, 0, 1, 0, 0, n0);
    stage(p, smem, 0, 1, 1, 0, n0);
    stage(p, smem, 0, 0, 1, 0, m0);
    stage(p, smem, 1, 0, 0, 1, m0);
    stage(p, smem, 1, 1, 0, 1, n0);
    stage(p, smem, 1, 1, 1, 1, n0);
    VM6();
    BARRIER();

    for (int it = 0; it < nK / 2; ++it) {
        const int kE = 2 * it, kO = kE + 1;
        const bool stE = kE + 2 < nK, stO = kO + 2 < nK;
        // ---- phase 1: E, quadrant (0,0)
        readA(0, 0);
        readB(0, 0, fb0);
        stage(p, smem, 1, 0, 1, kO, m0);
        BARRIER(); LGKM0();
        mma(0, 0, fb0);
        BARRIER();
        // ---- phase 2: E, (0,1)
        readB(0, 1, fb1);
        if (stE) stage(p, smem, 0, 0, 0, kE + 2, m0);
        BARRIER(); LGKM0();
        mma(0, 1, fb1);
        BARRIER();
        // ---- phase 3: E, (1,1)
        readA(0, 1);
        if (stE) stage(p, smem, 0, 1, 0, kE + 2, n0);
        BARRIER(); LGKM0();
        mma(1, 1, fb1);
        BARRIER();
        // ---- phase 4: E, (1,0); retire O(kO)
        if (stE) { stage(p, smem, 0, 1, 1, kE + 2, n0); VM6(); } else { VM0(); }
        BARRIER();
        mma(1, 0, fb0);
        BARRIER();
        // ---- phase 5: O, (0,0)
        readA(1, 0);
        readB(1, 0, fb0);
        if (stE) stage(p, smem, 0, 0, 1, kE + 2, m0);
        BARRIER(); LGKM0();
        mma(0, 0, fb0);
        BARRIER();
        // ---- phase 6: O, (0,1)
        readB(1, 1, fb1);
        if (stO) stage(p, smem, 1, 0, 0, kO + 2, m0);
        BARRIER(); LGKM0();
        mma(0, 1, fb1);
        BARRIER();
        // ---- phase 7: O, (1,1)
        readA(1, 1);
        if (stO) stage(p, smem, 1, 1, 0, kO + 2, n0);
        BARRIER(); LGKM0();
        mma(1, 1, fb1);
        BARRIER();
        // ---- phase 8: O, (1,0); retire E(kE+2)
        if (stO) { stage(p, smem, 1, 1, 1, kO + 2, n0); VM6(); } else { VM0(); }
        BARRIER();
        mma(1, 0, fb0);
        BARRIER();
    }

    // ---------------- epilogue: lane holds C[m][n..n+3]
    const int g = lane >> 4;
#pragma unroll
    for (int qm = 0; qm < 2; ++qm)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = m0 + qm * 128 + wm * 64 + i * 16 + (lane & 15);
            if (m >= p.M) continue;
#pragma unroll
            for (int qn = 0; qn < 2; ++qn)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int n = n0 + qn * 128 + wn * 32 + j * 16 + 4 * g;
                    if (n >= p.N) continue;
                    float v[4] = {acc[qm][qn][i][j][0], acc[qm][qn][i][j][1], acc[qm][qn][i][j][2],
                                  acc[qm][qn][i][j][3]};
                    const bool full = n + 3 < p.N;
                    if (p.bias) {
                        float bv[4] = {0.f, 0.f, 0.f, 0.f};
                        if (full) {
                            if (p.bias_bf16) load4((const bf16_t*)p.bias + n, bv);
                            else load4((const float*)p.bias + n, bv);
                        } else {
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                if (n + r < p.N)
                                    bv[r] = p.bias_bf16 ? bf2f(((const bf16_t*)p.bias)[n + r]) : ((const float*)p.bias)[n + r];
                        }
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] += bv[r];
                    }
                    if (p.act) {
                        if (p.aux) {
                            bf16_t* ap = p.aux + (long)m * p.ldc + n;
                            if (full) store4(ap, v);
                            else {
#pragma unroll
                                for (int r = 0; r < 4; ++r) if (n + r < p.N) ap[r] = f2bf(v[r]);
                            }
                        }
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] = act_fn(v[r], p.act);
                    }
                    bf16_t* cp = p.C + (long)m * p.ldc + n;
                    if (p.accumulate) {
                        float o[4] = {0.f, 0.f, 0.f, 0.f};
                        if (full) load4(cp, o);
                        else {
#pragma unroll
                            for (int r = 0; r < 4; ++r) if (n + r < p.N) o[r] = bf2f(cp[r]);
                        }
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] += o[r];
                    }
                    if (full) store4(cp, v);
                    else {
#pragma unroll
                        for (int r = 0; r < 4; ++r) if (n + r < p.N) cp[r] = f2bf(v[r]);
                    }
                }
        }
}

}  // namespace

DDL_API int ddl_gemm_big_supported(int M, int N, int K, long lda, long ldb) {
    return K > 0 && K % 128 == 0 && lda % 8 == 0 && ldb % 8 == 0 && M > 0 && N > 0;
}

// C = A . B^T (+bias)(act: 0 none, 1 gelu (aux <- pre-activation), 2 relu, 3 tanh); bf16 in/out
DDL_API int ddl_gemm_big(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                         const void* bias, int bias_bf16, int act, void* aux, int accumulate, hipStream_t st) {
    if (!ddl_gemm_big_supported(M, N, K, lda, ldb)) return -1;
    BigParams p{};
    p.A = (const bf16_t*)A; p.B = (const bf16_t*)B; p.lda = lda; p.ldb = ldb;
    p.C = (bf16_t*)C; p.ldc = ldc; p.M = M; p.N = N; p.K = K;
    p.bias = bias; p.bias_bf16 = bias_bf16; p.act = act; p.aux = (bf16_t*)aux;
    p.accumulate = accumulate;
    p.tiles_m = (M + TB - 1) / TB;
    p.tiles_n = (N + TB - 1) / TB;
    hipLaunchKernelGGL(gemm_big_k, dim3(p.tiles_m * p.tiles_n), dim3(NTH), 0, st, p);
    return (int)hipGetLastError();
}
