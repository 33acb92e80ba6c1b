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
#include <vector>

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

// The product's C2 configuration: choose_tiles + the packed-entry capacity of
// launch_tiled (three 21-bit in-tile offsets per 64-bit word).
static TileCfg c2_tiles(uint64_t n, uint32_t m, uint32_t k) {
    TileCfg tc = choose_tiles(m, n, k);
    constexpr uint64_t kpb = (uint64_t)kBinKPT * kBinThreads;
    const uint64_t nblk = (n + kpb - 1) / kpb, bps = (nblk + tc.G - 1) / tc.G;
    const uint64_t capw = ((uint64_t)tc.cap + 2 * bps + 2) / 3;
    tc.cap = (uint32_t)((capw + 7) & ~7ull);
    return tc;
}

static const uint64_t *g_offsets = nullptr;  // set: variable-length keys (C3)

template <int KPT, typename E, int KR>
static float time_bin_packed(const uint8_t *keys, uint64_t n, const FilterConsts &c, TileCfg tc,
                             TileScratch sc, void *buckets, int stop) {
    constexpr int NT = kBinThreads;
    constexpr uint64_t kpb = (uint64_t)KPT * NT;
    size_t sort = kpb * c.k * 4 + (size_t)tc.T * 8;
    if (g_offsets) sort = std::max<size_t>(sort, stage_lds_bytes(NT));
    const size_t lds = (size_t)bin_sort_offset_words(tc.T) * 4 + sort + g_lds_pad;
    auto kern = g_offsets ? bloom_bin_kernel<0, kOffsets, KPT, E, NT, true, KR>
                          : bloom_bin_kernel<0, kFixed16, KPT, E, NT, false, KR>;
    allow_lds(kern, lds);
    set_stop(stop);
    Ev ev;
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CK(hipMemset(sc.gcur, 0, kCurWords * 4));
        CK(hipEventRecord(ev.a));
        hipLaunchKernelGGL(kern, dim3((uint32_t)((n + kpb - 1) / kpb)), dim3(NT), lds, 0, keys,
                           g_offsets, g_offsets ? 0u : 16u, n, c, tc, sc, (E *)buckets);
        CK(hipEventRecord(ev.b));
        CK(hipEventSynchronize(ev.b));
        float ms;
        CK(hipEventElapsedTime(&ms, ev.a, ev.b));
        best = std::min(best, ms);
    }
    set_stop(0);
    return best;
}

// C5's pass-1 bin kernel (one 200M-key pass of 32-byte keys, k = 10, m = 2^32-1,
// Pack5 entries into 2^25-bit super tiles, as launch_two_level configures it), one
// dispatch per phase stop for per-phase counters (tools/pmc_phase.sh c5).
static int c5_pmc() {
    const uint64_t n = 200000000;
    const uint32_t m = 0xFFFFFFFFu, k = 10;
    constexpr int NT = kBinThreads, KPT = 1;
    constexpr uint64_t kpb = (uint64_t)KPT * NT;
    uint8_t *keys;
    CK(hipMalloc(&keys, n * 32 + 64));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(keys), n * 4);
    FilterConsts c = nb::make_consts(m, k, 17027509906831645879ull, 0);
    nb::set_fixed_len(c, 32);
    TileCfg t1 = super_tiles(choose_tiles(m, n, k), m, n, k, 5);
    const uint64_t nblk = (n + kpb - 1) / kpb, bps = (nblk + t1.G - 1) / t1.G;
    const uint64_t capu = ((uint64_t)t1.cap + 4 * bps + 4) / 5;
    t1.cap = (uint32_t)((capu + 7) & ~7ull);
    void *buckets;
    CK(hipMalloc(&buckets, (size_t)t1.T * t1.G * t1.cap * 16));
    TileScratch sc;
    uint32_t *zeroed;
    const size_t zb = (kCurWords + kMaxTiles + 2 * (((size_t)m + 63) / 64)) * 4;
    CK(hipMalloc(&zeroed, zb));
    CK(hipMemset(zeroed, 0, zb));
    sc.gcur = zeroed;
    sc.spill_flag = zeroed + kCurWords;
    sc.spill32 = zeroed + kCurWords + kMaxTiles;
    const size_t lds = (size_t)bin_sort_offset_words(t1.T) * 4 + kpb * k * 4 + (size_t)t1.T * 16;
    auto kern = bloom_bin_kernel<0, kFixed32, KPT, Pack5, NT, false, 16>;
    allow_lds(kern, lds);
    printf("C5 pass 1: ts=%u T=%u G=%u cap=%u units\n", t1.ts, t1.T, t1.G, t1.cap);
    for (int stop : {11, 1, 2, 3, 0}) {
        set_stop(stop);
        CK(hipMemset(sc.gcur, 0, kCurWords * 4));
        hipLaunchKernelGGL(kern, dim3((uint32_t)nblk), dim3(NT), lds, 0, keys, nullptr, 32u, n, c, t1,
                           sc, (Pack5 *)buckets);
        CK(hipDeviceSynchronize());
    }
    set_stop(0);
    printf("pmc dispatches: stops 11 1 2 3 0\n");
    return 0;
}

int main(int argc, char **argv) {
    // argv[1]: c2 (default), c4 (the 100M-key shard) or c3 (100M keys of 8-64 bytes);
    // c5 (pmc only): C5's pass-1 bin kernel; argv[2] == "intmod": integer remainders;
    // "c3 product": C3's phase stops in the product configuration
    if (argc > 1 && !strcmp(argv[1], "c5")) return c5_pmc();
    const bool c4 = argc > 1 && !strcmp(argv[1], "c4"), c3 = argc > 1 && !strcmp(argv[1], "c3");
    const uint64_t n = (c4 || c3) ? 100000000 : 10000000;
    const uint32_t m = (c4 || c3) ? 958505838u : 95850584u, k = 7;
    uint8_t *keys;
    uint64_t *words;
    uint64_t key_bytes = n * 16;
    if (c3) {  // lengths 8 + (splitmix(i) mod 57), offsets by a host scan
        std::vector<uint64_t> offs(n + 1, 0);
        for (uint64_t i = 0; i < n; ++i) {
            uint64_t x = i * 0x9E3779B97F4A7C15ull + 0x1EA5;
            x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
            x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
            offs[i + 1] = offs[i] + 8 + (x ^ (x >> 31)) % 57;
        }
        key_bytes = offs[n];
        uint64_t *d_offs;
        CK(hipMalloc(&d_offs, (n + 1) * 8));
        CK(hipMemcpy(d_offs, offs.data(), (n + 1) * 8, hipMemcpyHostToDevice));
        g_offsets = d_offs;
    }
    CK(hipMalloc(&keys, key_bytes + 64));
    CK(hipMalloc(&words, ((uint64_t)m + 63) / 64 * 8));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(keys),
                       (key_bytes + 7) / 8);
    FilterConsts c = nb::make_consts(m, k, 17027509906831645879ull, 0);
    if (!c3) nb::set_fixed_len(c, 16);
    if (argc > 2 && !strcmp(argv[2], "intmod")) c.fm.fp = 0;
    void *buckets;
    TileScratch sc;
    uint32_t *zeroed;
    const size_t zb = (kCurWords + kMaxTiles + 2 * (((size_t)m + 63) / 64)) * 4;
    CK(hipMalloc(&zeroed, zb));
    CK(hipMemset(zeroed, 0, zb));
    sc.gcur = zeroed;
    sc.spill_flag = zeroed + kCurWords;
    sc.spill32 = zeroed + kCurWords + kMaxTiles;
    CK(hipMalloc(&buckets, (size_t)n * k * 4 + (1 << 28)));
    const TileCfg tc = c2_tiles(n, m, k);
    if (argc > 2 && !strcmp(argv[2], "pmc")) {
        // one dispatch per stop (11 = hash only, 1 = + count, 2 = + scan/reservations,
        // 3 = + placement, 0 = full), in that order, for per-phase counters
        for (int stop : {11, 1, 2, 3, 0}) {
            set_stop(stop);
            constexpr uint64_t kpb = (uint64_t)kBinKPT * kBinThreads;
            size_t sort = kpb * c.k * 4 + (size_t)tc.T * 8;
            if (g_offsets) sort = std::max<size_t>(sort, stage_lds_bytes(kBinThreads));
            const size_t lds = (size_t)bin_sort_offset_words(tc.T) * 4 + sort;
            auto kern = g_offsets ? bloom_bin_kernel<0, kOffsets, kBinKPT, uint64_t, kBinThreads, true, 8>
                                  : bloom_bin_kernel<0, kFixed16, kBinKPT, uint64_t, kBinThreads, false, 8>;
            allow_lds(kern, lds);
            CK(hipMemset(sc.gcur, 0, kCurWords * 4));
            hipLaunchKernelGGL(kern, dim3((uint32_t)((n + kpb - 1) / kpb)), dim3(kBinThreads), lds, 0,
                               keys, g_offsets, g_offsets ? 0u : 16u, n, c, tc, sc, (uint64_t *)buckets);
            CK(hipDeviceSynchronize());
        }
        set_stop(0);
        printf("pmc dispatches: stops 11 1 2 3 0\n");
        return 0;
    }
    if (c3 && argc > 2 && !strcmp(argv[2], "product")) {
        // C3 in the product's configuration (launch_tiled: counted tiles, k = 7
        // exact, shard-major buckets): phase stops of the
        // staged bin kernel after a settle, then the tile kernel
        TileCfg p2 = choose_tiles(m, n, k), ct;
        if (!counted_tiles(m, n, k, p2, &ct)) ct = p2;
        constexpr int NT = kBinThreads, KPT = kBinKPT;
        constexpr uint64_t kpb = (uint64_t)KPT * NT;
        {
            const uint64_t nblk = (n + kpb - 1) / kpb, bps = (nblk + ct.G - 1) / ct.G;
            const uint64_t capw = ((uint64_t)ct.cap + 2 * bps + 2) / 3;
            ct.cap = (uint32_t)((capw + 7) & ~7ull);
        }
        TileScratch scz = sc;
        scz.zero_words = words;
        const size_t sort = std::max<size_t>(kpb * c.k * 4 + (size_t)ct.T * 8, stage_lds_bytes(NT));
        const size_t lds = (size_t)bin_sort_offset_words(ct.T) * 4 + sort;
        auto kern = bloom_bin_kernel<0, kOffsets, KPT, uint64_t, NT, true, 7, 7>;
        allow_lds(kern, lds);
        auto tile = bloom_tile_or_kernel<uint64_t, true>;
        const size_t tlds = (size_t)ct.w64 * 8 + (2 * kShards + 1) * 4;
        allow_lds(tile, tlds);
        printf("C3 product: T=%u mul=%u cap=%u words, %s buckets, bin LDS %zu B\n", ct.T, ct.mul, ct.cap,
               "shard-major", lds);
        auto bin = [&]() {
            hipLaunchKernelGGL(kern, dim3((uint32_t)((n + kpb - 1) / kpb)), dim3(NT), lds, 0, keys, g_offsets, 0u,
                               n, c, ct, scz, (uint64_t *)buckets);
        };
        auto tl = [&]() {
            hipLaunchKernelGGL(tile, dim3(ct.T), dim3(kTileThreads), tlds, 0, ct, sc, (const uint64_t *)buckets,
                               words, ((uint64_t)m + 63) / 64);
        };
        for (int r = 0; r < 20; ++r) {  // settle the clock
            bin();
            tl();
        }
        CK(hipDeviceSynchronize());
        const char *names[] = {"stage+hash+indices (stop 11)", "+count atomics (stop 1)", "+scan/reserve (stop 2)",
                               "+placement (stop 3)", "full bin kernel (stop 0)"};
        const int stops[] = {11, 1, 2, 3, 0};
        Ev ev;
        for (int i = 0; i < 5; ++i) {
            set_stop(stops[i]);
            float best = 1e30f, sum = 0;
            for (int r = 0; r < 7; ++r) {
                CK(hipMemset(sc.gcur, 0, kCurWords * 4));
                CK(hipEventRecord(ev.a));
                bin();
                CK(hipEventRecord(ev.b));
                CK(hipEventSynchronize(ev.b));
                float ms;
                CK(hipEventElapsedTime(&ms, ev.a, ev.b));
                best = std::min(best, ms);
                if (r >= 2) sum += ms;
            }
            printf("phase stop %-30s best %.4f  mean(5) %.4f ms\n", names[i], best, sum / 5);
        }
        set_stop(0);
        CK(hipMemset(sc.gcur, 0, kCurWords * 4));
        float best = 1e30f;
        for (int r = 0; r < 6; ++r) {
            bin();
            CK(hipEventRecord(ev.a));
            tl();
            CK(hipEventRecord(ev.b));
            CK(hipEventSynchronize(ev.b));
            float ms;
            CK(hipEventElapsedTime(&ms, ev.a, ev.b));
            best = std::min(best, ms);
        }
        printf("tile kernel: best %.4f ms\n", best);
        return 0;
    }
    printf("%s packed: ts=%u T=%u G=%u cap=%u words\n", c3 ? "C3" : c4 ? "C4" : "C2", tc.ts, tc.T, tc.G, tc.cap);
    for (size_t pad : {(size_t)0, (size_t)96 * 1024}) {
        g_lds_pad = pad;
        printf("%s block/CU: p1-nocount %.4f p1 %.4f p12 %.4f p123 %.4f full %.4f ms\n", pad ? "1" : "2",
               time_bin_packed<kBinKPT, uint64_t, 8>(keys, n, c, tc, sc, buckets, 11),
               time_bin_packed<kBinKPT, uint64_t, 8>(keys, n, c, tc, sc, buckets, 1),
               time_bin_packed<kBinKPT, uint64_t, 8>(keys, n, c, tc, sc, buckets, 2),
               time_bin_packed<kBinKPT, uint64_t, 8>(keys, n, c, tc, sc, buckets, 3),
               time_bin_packed<kBinKPT, uint64_t, 8>(keys, n, c, tc, sc, buckets, 0));
    }
    g_lds_pad = 0;
    {
        auto kern = bloom_tile_or_kernel<uint64_t, true>;
        const size_t lds = ((size_t)1 << (tc.ts - 3)) + (2 * kShards + 1) * 4;
        allow_lds(kern, lds);
        Ev ev;
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            time_bin_packed<kBinKPT, uint64_t, 8>(keys, n, c, tc, sc, buckets, 0);
            CK(hipEventRecord(ev.a));
            hipLaunchKernelGGL(kern, dim3(tc.T), dim3(kTileThreads), lds, 0, tc, sc,
                               (const uint64_t *)buckets, words, ((uint64_t)m + 63) / 64);
            CK(hipEventRecord(ev.b));
            CK(hipEventSynchronize(ev.b));
            float ms;
            CK(hipEventElapsedTime(&ms, ev.a, ev.b));
            best = std::min(best, ms);
        }
        printf("tile kernel: %.4f ms\n", best);
    }
    for (int lo : {256, 512})
        for (int cyc : {8000, 30000, 60000}) {
            set_stagger(lo, cyc);
            printf("stagger lo=%d cycles=%d: full %.4f ms\n", lo, cyc,
                   time_bin_packed<kBinKPT, uint64_t, 8>(keys, n, c, tc, sc, buckets, 0));
        }
    set_stagger(0, 0);
    CK(hipDeviceSynchronize());
    return 0;
}
