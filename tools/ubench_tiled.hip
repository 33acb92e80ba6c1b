// ubench_tiled.hip -- diagnostic build of the tiled build path (not product code).
// Includes the product kernels with NB_DIAG_STOP wired to a device constant, and
// times, for the C2 workload (10M x 16B keys, m = 95,850,584, k = 7):
//   * bin kernel configurations (keys/thread x threads/block) and tile sizes,
//     each stopped after phase 1 / 2 / 3 / full, to price every phase;
//   * tile kernel configurations (threads x loads in flight).
#include <hip/hip_runtime.h>
__constant__ int g_diag_stop;
// stop 11: phase 1 without the LDS count atomics (hashing + index generation)
#define NB_DIAG_STOP(phase) (g_diag_stop == (phase) || ((phase) == 1 && g_diag_stop == 11))
#define NB_DIAG_NOCOUNT (g_diag_stop == 11)
__constant__ int g_stagger_blocks;  // blocks [lo, 2*lo) sleep ~g_stagger_cycles at start
__constant__ int g_stagger_cycles;
#define NB_DIAG_PROLOGUE()                                                              \
    do {                                                                                \
        if (g_stagger_blocks && blockIdx.x >= (unsigned)g_stagger_blocks &&             \
            blockIdx.x < 2u * g_stagger_blocks) {                                       \
            const long long t0 = clock64();                                             \
            while (clock64() - t0 < g_stagger_cycles) __builtin_amdgcn_s_sleep(8);      \
        }                                                                               \
    } while (0)
#include "../nasp-key-value-engine_amd/csrc/bloom_kernels.hip"

#include <cstdio>
#include <cstring>

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e = (x);                                                 \
        if (e != hipSuccess) {                                              \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                        \
        }                                                                   \
    } while (0)

__global__ void k_fill(uint64_t *p, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        uint64_t x = i + 0x9E3779B97F4A7C15ull;
        x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
        x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
        p[i] = x ^ (x >> 31);
    }
}

struct Ev {
    hipEvent_t a, b;
    Ev() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
};

static void set_stop(int s) { CK(hipMemcpyToSymbol(HIP_SYMBOL(g_diag_stop), &s, sizeof s)); }
static void set_stagger(int blocks, int cycles) {
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stagger_blocks), &blocks, sizeof blocks));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stagger_cycles), &cycles, sizeof cycles));
}

static size_t g_lds_pad = 0;  // extra dynamic LDS (forces fewer blocks per CU)

template <int KPT, typename E, int KR = 0>
static float time_bin(const uint8_t *keys, uint64_t n, const FilterConsts &c, TileCfg tc,
                      TileScratch sc, void *buckets, int stop) {
    constexpr int NT = kBinThreads;
    constexpr uint64_t kpb = (uint64_t)KPT * NT;
    const size_t lds = (size_t)bin_sort_offset_words(tc.T) * 4 + kpb * c.k * 4 + g_lds_pad;
    auto kern = bloom_bin_kernel<0, kFixed16, KPT, E, NT, false, KR>;
    if (lds > 160 * 1024) return -1.f;
    allow_lds(kern, lds);
    set_stop(stop);
    Ev ev;
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        CK(hipMemset(sc.gcur, 0, kCurWords * 4));
        CK(hipEventRecord(ev.a));
        hipLaunchKernelGGL(kern, dim3((uint32_t)((n + kpb - 1) / kpb)), dim3(NT), lds, 0, keys,
                           nullptr, 16u, n, c, tc, sc, (E *)buckets);
        CK(hipEventRecord(ev.b));
        CK(hipEventSynchronize(ev.b));
        float ms;
        CK(hipEventElapsedTime(&ms, ev.a, ev.b));
        best = std::min(best, ms);
    }
    set_stop(0);
    return best;
}

template <typename E, int UN>
static float time_tile(const uint8_t *keys, uint64_t n, const FilterConsts &c, TileCfg tc,
                       TileScratch sc, void *buckets, uint64_t *words) {
    auto kern = bloom_tile_or_kernel<E, true, kTileThreads, UN>;
    const size_t lds = ((size_t)1 << (tc.ts - 3)) + (2 * kShards + 1) * 4;
    allow_lds(kern, lds);
    const uint64_t nwords = ((uint64_t)c.fm.m + 63) / 64;
    Ev ev;
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        time_bin<kBinKPT, E>(keys, n, c, tc, sc, buckets, 0);
        CK(hipEventRecord(ev.a));
        hipLaunchKernelGGL(kern, dim3(tc.T), dim3(kTileThreads), lds, 0, tc, sc, (const E *)buckets,
                           words, nwords);
        CK(hipEventRecord(ev.b));
        CK(hipEventSynchronize(ev.b));
        float ms;
        CK(hipEventElapsedTime(&ms, ev.a, ev.b));
        best = std::min(best, ms);
    }
    return best;
}

int main(int argc, char **argv) {
    const bool pmc = argc > 1 && !strcmp(argv[1], "pmc");  // one dispatch per stop, for counters
    const uint64_t n = 10000000;
    const uint32_t m = 95850584, k = 7;
    uint8_t *keys;
    uint64_t *words;
    CK(hipMalloc(&keys, n * 16 + 64));
    CK(hipMalloc(&words, ((uint64_t)m + 63) / 64 * 8));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(keys), 2 * n);
    FilterConsts c = nb::make_consts(m, k, 17027509906831645879ull, 0);
    nb::set_fixed_len(c, 16);
    void *buckets;
    TileScratch sc;
    uint32_t *zeroed;
    const size_t zb = (kCurWords + kMaxTiles + 2 * (((size_t)m + 63) / 64)) * 4;
    CK(hipMalloc(&zeroed, zb));
    CK(hipMemset(zeroed, 0, zb));
    sc.gcur = zeroed;
    sc.spill_flag = zeroed + kCurWords;
    sc.spill32 = zeroed + kCurWords + kMaxTiles;
    CK(hipMalloc(&buckets, (size_t)n * k * 4 * 2 + (1 << 26)));
    if (pmc) {
        TileCfg tc;
        tc.ts = 16;
        tc.T = (uint32_t)(((uint64_t)m + (1ull << 16) - 1) >> 16);
        tc.G = 8;
        double e = (double)n * k / ((double)tc.T * tc.G);
        tc.cap = ((uint32_t)(e + 8 * std::sqrt(e) + 64) + 7) & ~7u;
        constexpr int NT = kBinThreads;
        constexpr uint64_t kpb = (uint64_t)kBinKPT * NT;
        const size_t lds = (size_t)bin_sort_offset_words(tc.T) * 4 + kpb * c.k * 4;
        auto kern = bloom_bin_kernel<0, kFixed16, kBinKPT, uint16_t, NT, false, 8>;
        allow_lds(kern, lds);
        // dispatch order: stop 11, 1, 2, 3, 0 (full), then the tile kernel
        for (int stop : {11, 1, 2, 3, 0}) {
            set_stop(stop);
            CK(hipMemset(sc.gcur, 0, kCurWords * 4));
            hipLaunchKernelGGL(kern, dim3((uint32_t)((n + kpb - 1) / kpb)), dim3(NT), lds, 0, keys,
                               nullptr, 16u, n, c, tc, sc, (uint16_t *)buckets);
            CK(hipDeviceSynchronize());
        }
        set_stop(0);
        auto tk = bloom_tile_or_kernel<uint16_t, true>;
        const size_t tl = ((size_t)1 << (tc.ts - 3)) + (2 * kShards + 1) * 4;
        allow_lds(tk, tl);
        hipLaunchKernelGGL(tk, dim3(tc.T), dim3(kTileThreads), tl, 0, tc, sc, (const uint16_t *)buckets,
                           words, ((uint64_t)m + 63) / 64);
        CK(hipDeviceSynchronize());
        printf("pmc mode done\n");
        return 0;
    }
    {
        TileCfg tc;
        tc.ts = 16;
        tc.T = (uint32_t)(((uint64_t)m + (1ull << 16) - 1) >> 16);
        tc.G = 8;
        double e = (double)n * k / ((double)tc.T * tc.G);
        tc.cap = ((uint32_t)(e + 8 * std::sqrt(e) + 64) + 7) & ~7u;
        for (size_t pad : {(size_t)0, (size_t)70 * 1024}) {
            g_lds_pad = pad;
            printf("ts=16 T=%u G=8 u16 lds_pad=%zu (%s block/CU): p1 %.4f p12 %.4f p123 %.4f full %.4f ms\n",
                   tc.T, pad, pad ? "1" : "2",
                   time_bin<kBinKPT, uint16_t>(keys, n, c, tc, sc, buckets, 1),
                   time_bin<kBinKPT, uint16_t>(keys, n, c, tc, sc, buckets, 2),
                   time_bin<kBinKPT, uint16_t>(keys, n, c, tc, sc, buckets, 3),
                   time_bin<kBinKPT, uint16_t>(keys, n, c, tc, sc, buckets, 0));
        }
        g_lds_pad = 0;
        printf("rank mode (KR=8): p1-nocount %.4f p1 %.4f p12 %.4f p123 %.4f full %.4f ms\n",
               time_bin<kBinKPT, uint16_t, 8>(keys, n, c, tc, sc, buckets, 11),
               time_bin<kBinKPT, uint16_t, 8>(keys, n, c, tc, sc, buckets, 1),
               time_bin<kBinKPT, uint16_t, 8>(keys, n, c, tc, sc, buckets, 2),
               time_bin<kBinKPT, uint16_t, 8>(keys, n, c, tc, sc, buckets, 3),
               time_bin<kBinKPT, uint16_t, 8>(keys, n, c, tc, sc, buckets, 0));
        printf("tile kernel: %.4f ms\n", time_tile<uint16_t, kTileUnroll>(keys, n, c, tc, sc, buckets, words));
        printf("tile kernel unroll 1/4/8: %.4f %.4f %.4f ms\n",
               time_tile<uint16_t, 1>(keys, n, c, tc, sc, buckets, words),
               time_tile<uint16_t, 4>(keys, n, c, tc, sc, buckets, words),
               time_tile<uint16_t, 8>(keys, n, c, tc, sc, buckets, words));
        // desynchronise the two resident blocks per CU: blocks [lo, 2lo) start late
        for (int lo : {256, 512})
            for (int cyc : {4000, 8000, 16000, 24000}) {
                set_stagger(lo, cyc);
                printf("stagger lo=%d cycles=%d: full %.4f ms\n", lo, cyc,
                       time_bin<kBinKPT, uint16_t, 8>(keys, n, c, tc, sc, buckets, 0));
            }
        set_stagger(0, 0);
    }
    CK(hipDeviceSynchronize());
    return 0;
}
