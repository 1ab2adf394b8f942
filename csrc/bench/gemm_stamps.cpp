// Per-tile timeline of the 256x256 GEMM (diagnostic; not part of the library).
//
// Includes csrc/kernels/gemm_big.hip with -DDDL_GEMM_STAMPS: waves 0 and 4 of every block
// record s_memrealtime (100 MHz) and s_memtime at tile start, main-loop start, main-loop
// end and epilogue-issued.  Prints, per shape: hipEvent time, the spans of those phases
// averaged over blocks (first tile / later tiles), block start / end skew and the clock.
//
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -DDDL_GEMM_STAMPS -I csrc/include \
//            -ffp-contract=fast -munsafe-fp-atomics csrc/bench/gemm_stamps.cpp -o build/gemm_stamps
//   run:   build/gemm_stamps [mode M N K]...
#include "../kernels/gemm_big.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

BnbArgs ddl_take_bnb() { return BnbArgs{nullptr, nullptr, nullptr}; }

int main(int argc, char** argv) {
    struct Case { int mode, M, N, K; };
    std::vector<Case> cases;
    if (argc > 1) {
        for (int i = 1; i + 3 < argc; i += 4) cases.push_back({atoi(argv[i]), atoi(argv[i + 1]), atoi(argv[i + 2]), atoi(argv[i + 3])});
    } else {
        cases = {{0, 16384, 768, 768}, {0, 16384, 3072, 768}, {0, 16384, 2304, 768}, {0, 16384, 768, 3072},
                 {1, 16384, 768, 768}, {1, 16384, 3072, 768}, {0, 8192, 8192, 8192}};
    }
    void *A, *B, *C, *Z;
    const long maxe = 8192L * 8192;
    hipMalloc(&A, maxe * 2);
    hipMalloc(&B, maxe * 2);
    hipMalloc(&C, maxe * 2);
    hipMalloc(&Z, 256);
    std::vector<uint16_t> hA(maxe);   // A and B hold the same random bf16 data
    {
        std::vector<uint16_t>& h = hA;
        uint32_t s = 12345;
        for (auto& v : h) {
            s = s * 1664525u + 1013904223u;
            const float f = ((s >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;
            uint32_t u;
            memcpy(&u, &f, 4);
            v = (uint16_t)(u >> 16);
        }
        hipMemcpy(A, h.data(), h.size() * 2, hipMemcpyHostToDevice);
        hipMemcpy(B, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    }
    hipMemset(Z, 0, 256);
    const long nst = 4096L * STAMP_TILES * 2 * 8;
    unsigned long long* dst;
    hipMalloc(&dst, nst * 8);
    hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &dst, sizeof(dst));
    const long nks = 4096L * 32;
    unsigned long long* kdst;
    hipMalloc(&kdst, nks * 8);
    hipMemcpyToSymbol(HIP_SYMBOL(g_kstamps), &kdst, sizeof(kdst));
    std::vector<unsigned long long> hk(nks);
    void* flush = nullptr;
    if (getenv("COLD")) hipMalloc(&flush, 512L << 20);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<unsigned long long> h(nst);
    for (const Case& c : cases) {
        const int M = c.M, N = c.N, K = c.K;
        const int lay = c.mode & 31;       // | 32: 256 x 192 tiles (NT / NN)
        const long lda = lay == 2 ? M : K;
        const long ldb = lay == 0 ? K : N;
        auto run = [&] {
            int r = ddl_gemm_big2(c.mode, A, lda, B, ldb, C, N, M, N, K, nullptr, 0, 0, nullptr, 0, 1, nullptr, 0,
                                  nullptr, 0, nullptr, 0, Z, nullptr, 0);
            if (r) printf("launch error %d\n", r);
        };
        for (int i = 0; i < 5; ++i) run();
        hipEventRecord(e0, 0);
        const int it = 20;
        for (int i = 0; i < it; ++i) run();
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= it;
        hipMemset(dst, 0, nst * 8);
        hipMemset(kdst, 0, nks * 8);
        if (flush) hipMemset(flush, 1, 512L << 20);   // COLD=1: evict L2 / Infinity Cache before the stamped run
        run();
        hipDeviceSynchronize();
        hipMemcpy(h.data(), dst, nst * 8, hipMemcpyDeviceToHost);
        hipMemcpy(hk.data(), kdst, nks * 8, hipMemcpyDeviceToHost);
        {   // correctness: sampled outputs against a double-precision host reference
            std::vector<uint16_t> hc((size_t)M * N);
            hipMemcpy(hc.data(), C, hc.size() * 2, hipMemcpyDeviceToHost);
            auto f = [](uint16_t v) { uint32_t u = (uint32_t)v << 16; float x; memcpy(&x, &u, 4); return (double)x; };
            uint32_t r = 777;
            int bad = 0;
            double worst = 0;
            for (int t = 0; t < 512; ++t) {
                r = r * 1664525u + 1013904223u;
                const int m = (int)((r >> 8) % (uint32_t)M);
                r = r * 1664525u + 1013904223u;
                const int n = (int)((r >> 8) % (uint32_t)N);
                double ref = 0;
                for (int k = 0; k < K; ++k) {
                    const double a = f(hA[(lay == 2 ? (size_t)k * M + m : (size_t)m * K + k)]);
                    const double b = f(hA[(lay == 0 ? (size_t)n * K + k : (size_t)k * N + n)]);
                    ref += a * b;
                }
                const double got = f(hc[(size_t)m * N + n]);
                const double err = fabs(got - ref), tol = 0.02 * sqrt((double)K) + fabs(ref) / 128.0;
                worst = std::max(worst, err / tol);
                if (err > tol) ++bad;
            }
            printf("   check: %d / 512 sampled outputs off (worst err / tol %.3f)%s\n", bad, worst, bad ? "  *** MISMATCH ***" : "");
        }
        const int tbn = (c.mode & 32) ? 192 : 256;
        const int tiles = ((M + 255) / 256) * ((N + tbn - 1) / tbn);
        const int grid = std::min(tiles, 256);
        // phases per wave group (0: waves 0-3, 1: waves 4-7)
        double sum[2][2][3] = {}, cnt[2][2] = {};
        unsigned long long t0 = ~0ull, t1 = 0, s_min = ~0ull, s_max = 0, e_min = ~0ull, e_max = 0;
        double clk_num = 0, clk_den = 0;
        int max_ti = 0;
        for (int b = 0; b < grid; ++b) {
            unsigned long long bend = 0;
            for (int g = 0; g < 2; ++g) {
                for (int ti = 0; ti < STAMP_TILES; ++ti) {
                    const unsigned long long* d = h.data() + (((long)b * STAMP_TILES + ti) * 2 + g) * 8;
                    if (!d[0] || !d[6]) continue;   // tile not run
                    max_ti = std::max(max_ti, ti + 1);
                    const int f = ti ? 1 : 0;
                    for (int k = 0; k < 3; ++k) sum[g][f][k] += (double)(d[2 * k + 2] - d[2 * k]);
                    cnt[g][f] += 1;
                    t0 = std::min(t0, d[0]);
                    t1 = std::max(t1, d[6]);
                    if (ti == 0) { s_min = std::min(s_min, d[0]); s_max = std::max(s_max, d[0]); }
                    bend = std::max(bend, d[6]);
                    clk_num += (double)(d[7] - d[1]);
                    clk_den += (double)(d[6] - d[0]);
                }
            }
            if (bend) { e_min = std::min(e_min, bend); e_max = std::max(e_max, bend); }
        }
        const double us = 0.01;   // 100 MHz ticks
        printf("mode=%d M=%d N=%d K=%d tiles=%d grid=%d  event %.1f us (%.0f TF)  stamped span %.1f us  max tiles/block %d"
               "  clock %.2f GHz\n",
               c.mode, M, N, K, tiles, grid, ms * 1e3, 2.0 * M * N * K / ms / 1e9, (t1 - t0) * us, max_ti,
               clk_den > 0 ? clk_num / clk_den * 0.1 : 0.0);
        printf("   block start skew %.2f us, block end skew %.2f us\n", (s_max - s_min) * us, (e_max - e_min) * us);
        {   // first tile: time of each k-tile pair (iteration it -> it+1), mean over blocks
            const int pairs = std::min(32, ((K + 63) / 64) / 2);
            printf("   first-tile k-pair times (us):");
            for (int it = 0; it < pairs; ++it) {
                double sm = 0;
                int n = 0;
                for (int b = 0; b < grid; ++b) {
                    const unsigned long long* d = h.data() + ((long)b * STAMP_TILES) * 2 * 8;
                    const unsigned long long a = hk[(long)b * 32 + it];
                    const unsigned long long z = it + 1 < pairs ? hk[(long)b * 32 + it + 1] : d[4];   // loop end
                    if (a && z > a) { sm += (double)(z - a); ++n; }
                }
                printf(" %.2f", n ? sm / n * 0.01 : 0.0);
            }
            printf("\n");
        }
        for (int g = 0; g < 2; ++g)
            for (int f = 0; f < 2; ++f)
                if (cnt[g][f] > 0)
                    printf("   waves %d-%d %s tiles (%4.0f): prologue %.2f us  main loop %.2f us  epilogue %.2f us\n",
                           4 * g, 4 * g + 3, f ? "later" : "first", cnt[g][f], sum[g][f][0] / cnt[g][f] * us,
                           sum[g][f][1] / cnt[g][f] * us, sum[g][f][2] / cnt[g][f] * us);
    }
    return 0;
}
