// ubench_c4.hip -- diagnostic build of C4's tiled build (not product code).
// Includes the product kernels with NB_DIAG_STOP wired to a device constant and
// measures, on C4's shard (100M x 16 B keys, k = 7, m = 958,505,838) with the
// bin-kernel instantiation the product launches for it (768 threads x 3 keys,
// packed 21-bit entries, KX = 7):
//   1. phase stops of the bin kernel (11 = hash + indices only, 1 = + LDS count
//      atomics, 2 = + scan / reservations, 3 = + placement, 0 = full) and the tile
//      kernel alone -- the measured floors behind DESIGN.md's ceiling section;
//   2. which CUs a CU-masked stream's blocks land on (XCC / SE / CU ids);
//   3. the tile kernel and the bin kernel restricted to x CUs by a stream CU mask;
//   4. a chunked pipeline: bin kernels on (256 - x) CUs beside tile kernels on x
//      CUs, checked bit for bit against the one-shot build.
//   5. power-of-two (915) vs counted (768) tiles, one-shot builds interleaved.
//   6. cstops: phase stops in the product configuration (counted tiles, shard-major
//      buckets).  (Round 4's `layout` mode -- tile-major vs shard-major buckets -- went
//      with the tile-major layout in round 5; profiles/r04_c4_layout.txt is its output.)
// usage: ubench_c4 [all|stops|cstops|tiles|mask|pipe]
#include <hip/hip_runtime.h>
__constant__ int g_diag_stop;
#define NB_DIAG_STOP(phase) (g_diag_stop == (phase) || ((phase) == 1 && g_diag_stop == 11))
#define NB_DIAG_NOCOUNT (g_diag_stop == 11)
#include "../nasp-key-value-engine_amd/csrc/bloom_kernels.hip"

#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <vector>

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t ck_ = (x);                                                 \
        if (ck_ != hipSuccess) {                                            \
            printf("HIP error %s at %d\n", hipGetErrorString(ck_), __LINE__); \
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

// where a block runs: XCC id (HW_REG_XCC_ID = 20) and HW_ID (reg 4: cu [11:8],
// sh [12], se [15:13]); each block holds its CU ~20 us so the grid spreads out
__global__ void k_where(uint32_t *out) {
    extern __shared__ uint32_t pad[];
    if (threadIdx.x == 0) {
        const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 15u;
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        pad[0] = hw;
        out[blockIdx.x] = xcc << 16 | ((hw >> 8) & 0x1fffu);
        const long long t0 = clock64();
        while (clock64() - t0 < 40000) __builtin_amdgcn_s_sleep(8);
    }
}

constexpr int kNT = kBinThreads16Wide, kKPT = 3;
constexpr uint64_t kKPB = (uint64_t)kNT * kKPT;
constexpr uint64_t kN = 100000000;
constexpr uint32_t kM = 958505838u, kK = 7;
#define BIN bloom_bin_kernel<0, kFixed16, kKPT, uint64_t, kNT, false, 7, 7>

struct Setup {
    uint8_t *keys;
    uint64_t *words, *words_ref;
    FilterConsts c;
    uint32_t *zeroed[2];
    TileScratch sc[2];
    uint64_t *bk[2];
    size_t zb;
};

static void set_stop(int s) { CK(hipMemcpyToSymbol(HIP_SYMBOL(g_diag_stop), &s, sizeof s)); }

// launch_tiled's packed configuration for `chunk` keys
static TileCfg c4_tiles(uint64_t chunk) {
    TileCfg tc = choose_tiles(kM, chunk, kK);
    const uint64_t nblk = (chunk + kKPB - 1) / kKPB, bps = (nblk + tc.G - 1) / tc.G;
    const uint64_t capw = ((uint64_t)tc.cap + 2 * bps + 2) / 3;
    tc.cap = (uint32_t)((capw + 7) & ~7ull);
    return tc;
}
static size_t bin_lds_of(const TileCfg &tc) {
    return (size_t)bin_sort_offset_words(tc.T) * 4 + kKPB * kK * 4 + (size_t)tc.T * 8;
}
static size_t tile_lds_of(const TileCfg &tc) { return ((size_t)1 << (tc.ts - 3)) + (2 * kShards + 1) * 4; }

static void launch_bin(Setup &s, int q, const TileCfg &tc, uint64_t first, uint64_t cn, hipStream_t st) {
    hipLaunchKernelGGL(BIN, dim3((uint32_t)((cn + kKPB - 1) / kKPB)), dim3(kNT), bin_lds_of(tc), st,
                       s.keys + first * 16, nullptr, 16u, cn, s.c, tc, s.sc[q], s.bk[q]);
}
template <int UNROLL = kTileUnroll>
static void launch_tile(Setup &s, int q, const TileCfg &tc, bool ow, uint64_t *words, hipStream_t st) {
    auto k = ow ? bloom_tile_or_kernel<uint64_t, true, kTileThreads, UNROLL>
                : bloom_tile_or_kernel<uint64_t, false, kTileThreads, UNROLL>;
    hipLaunchKernelGGL(k, dim3(tc.T), dim3(kTileThreads), tile_lds_of(tc), st, tc, s.sc[q], s.bk[q], words,
                       ((uint64_t)kM + 63) / 64);
}

// wait for a stream with a deadline: a CU mask that selects no usable CU would
// leave the launch pending forever -- report it and leave without tearing down
static void wait_or_die(hipStream_t s, const char *what, double secs = 5.0) {
    const auto t0 = std::chrono::steady_clock::now();
    while (true) {
        const hipError_t q = hipStreamQuery(s);
        if (q == hipSuccess) return;
        if (q != hipErrorNotReady) { printf("HIP error %s waiting for %s\n", hipGetErrorString(q), what); _exit(4); }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > secs) {
            printf("TIMEOUT: %s did not complete in %.0f s\n", what, secs);
            _exit(3);
        }
        usleep(200);
    }
}

struct Ev {
    hipEvent_t a, b;
    Ev() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    float ms() { float t; CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&t, a, b)); return t; }
};

static std::vector<uint32_t> mask_bits(int x, int mode) {
    std::vector<uint32_t> m(8, 0);  // 256 CUs
    if (mode == 0) {                // low x bits
        for (int i = 0; i < x; ++i) m[i / 32] |= 1u << (i % 32);
    } else {                        // high x bits (the complement of mode 0 at 256 - x)
        for (int i = 256 - x; i < 256; ++i) m[i / 32] |= 1u << (i % 32);
    }
    return m;
}
static hipStream_t masked_stream(int x, int mode) {
    hipStream_t s;
    if (x >= 256) { CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking)); return s; }
    std::vector<uint32_t> m = mask_bits(x, mode);
    CK(hipExtStreamCreateWithCUMask(&s, 8, m.data()));
    return s;
}

static void where(int x, int mode) {
    hipStream_t s = masked_stream(x, mode);
    const int nb = 4096;
    uint32_t *d;
    CK(hipMalloc(&d, nb * 4));
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(k_where),
                           hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024));
    hipLaunchKernelGGL(k_where, dim3(nb), dim3(64), 100 * 1024, s, d);
    wait_or_die(s, "k_where on a masked stream");
    std::vector<uint32_t> h(nb);
    CK(hipMemcpy(h.data(), d, nb * 4, hipMemcpyDeviceToHost));
    std::map<uint32_t, int> cu;
    int per_xcc[16] = {0};
    for (uint32_t v : h) cu[v]++;
    for (auto &kv : cu) per_xcc[kv.first >> 16]++;
    printf("mask x=%3d mode=%d: %zu distinct CUs; per XCC:", x, mode, cu.size());
    for (int i = 0; i < 8; ++i) printf(" %d", per_xcc[i]);
    printf("\n");
    CK(hipFree(d));
    CK(hipStreamDestroy(s));
}

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const char *what = argc > 1 ? argv[1] : "all";
    const bool all = !strcmp(what, "all");
    Setup s;
    CK(hipMalloc(&s.keys, kN * 16 + 64));
    const uint64_t nwords = ((uint64_t)kM + 63) / 64;
    CK(hipMalloc(&s.words, nwords * 8));
    CK(hipMalloc(&s.words_ref, nwords * 8));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(s.keys), kN * 2);
    s.c = nb::make_consts(kM, kK, 17027509906831645879ull, 0);
    nb::set_fixed_len(s.c, 16);
    s.zb = (kCurWords + kFlagWords + kSuperCurWords + 2 * (((size_t)kM + 63) / 64)) * 4;
    const TileCfg tfull = c4_tiles(kN);
    for (int q = 0; q < 2; ++q) {
        CK(hipMalloc(&s.zeroed[q], s.zb));
        CK(hipMemset(s.zeroed[q], 0, s.zb));
        s.sc[q].gcur = s.zeroed[q];
        s.sc[q].spill_flag = s.zeroed[q] + kCurWords;
        s.sc[q].spill32 = s.zeroed[q] + kCurWords + kFlagWords + kSuperCurWords;
        CK(hipMalloc(&s.bk[q], (size_t)tfull.T * tfull.G * tfull.cap * 8));
    }
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(BIN), hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)bin_lds_of(tfull)));
    for (auto k : {bloom_tile_or_kernel<uint64_t, true, kTileThreads, 4>,
                   bloom_tile_or_kernel<uint64_t, false, kTileThreads, 4>,
                   bloom_tile_or_kernel<uint64_t, true, kTileThreads, 8>,
                   bloom_tile_or_kernel<uint64_t, false, kTileThreads, 8>,
                   bloom_tile_or_kernel<uint64_t, true, kTileThreads, 16>,
                   bloom_tile_or_kernel<uint64_t, false, kTileThreads, 16>})
        CK(hipFuncSetAttribute(reinterpret_cast<const void *>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)tile_lds_of(tfull)));
    printf("C4: n=%llu m=%u k=%u ts=%u T=%u G=%u cap=%u words, bin LDS %zu B\n", (unsigned long long)kN, kM, kK,
           tfull.ts, tfull.T, tfull.G, tfull.cap, bin_lds_of(tfull));
    hipStream_t s0;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    // reference filter (one-shot build, the product's sequence)
    set_stop(0);
    for (int r = 0; r < 3; ++r) {  // warm-up (clocks) + reference
        launch_bin(s, 0, tfull, 0, kN, s0);
        launch_tile(s, 0, tfull, true, s.words_ref, s0);
    }
    CK(hipStreamSynchronize(s0));

    if (all || !strcmp(what, "stops")) {
        // per-dispatch durations of back-to-back builds (clock drift within a process)
        Ev ev[24];
        for (int r = 0; r < 24; ++r) {
            CK(hipEventRecord(ev[r].a, s0));
            launch_bin(s, 0, tfull, 0, kN, s0);
            CK(hipEventRecord(ev[r].b, s0));
            launch_tile(s, 0, tfull, true, s.words, s0);
        }
        printf("bin dispatches back to back (ms):");
        for (int r = 0; r < 24; ++r) printf(" %.3f", ev[r].ms());
        printf("\n");
        const char *names[] = {"hash+indices (stop 11)", "+count atomics (stop 1)", "+scan/reserve (stop 2)",
                               "+placement (stop 3)", "full bin kernel (stop 0)"};
        const int stops[] = {11, 1, 2, 3, 0};
        for (int i = 0; i < 5; ++i) {
            set_stop(stops[i]);
            float best = 1e30f, sum = 0;
            for (int r = 0; r < 7; ++r) {
                CK(hipMemsetAsync(s.sc[0].gcur, 0, kCurWords * 4, s0));
                Ev e;
                CK(hipEventRecord(e.a, s0));
                launch_bin(s, 0, tfull, 0, kN, s0);
                CK(hipEventRecord(e.b, s0));
                const float t = e.ms();
                best = std::min(best, t);
                if (r >= 2) sum += t;
            }
            printf("phase stop %-26s best %.4f  mean(5) %.4f ms\n", names[i], best, sum / 5);
        }
        set_stop(0);
        CK(hipMemsetAsync(s.sc[0].gcur, 0, kCurWords * 4, s0));
        // the tile kernel on the same buckets (it resets the cursors: rebuild each time)
        for (int unroll : {4, 8, 16}) {
            float best = 1e30f, sum = 0;
            for (int r = 0; r < 6; ++r) {
                launch_bin(s, 0, tfull, 0, kN, s0);
                Ev e;
                CK(hipEventRecord(e.a, s0));
                if (unroll == 4) launch_tile<4>(s, 0, tfull, true, s.words, s0);
                else if (unroll == 8) launch_tile<8>(s, 0, tfull, true, s.words, s0);
                else launch_tile<16>(s, 0, tfull, true, s.words, s0);
                CK(hipEventRecord(e.b, s0));
                const float t = e.ms();
                best = std::min(best, t);
                if (r >= 1) sum += t;
            }
            printf("tile kernel unroll %2d: best %.4f  mean(5) %.4f ms\n", unroll, best, sum / 5);
        }
    }

    if (all || !strcmp(what, "cstops")) {
        // the product's configuration: counted tiles (768), shard-major buckets; phase
        // stops of the bin kernel and the tile kernel alone
        TileCfg p2 = choose_tiles(kM, kN, kK), ct;
        if (!counted_tiles(kM, kN, kK, p2, &ct)) { printf("counted tiles: policy declined\n"); return 1; }
        {
            const uint64_t nblk = (kN + kKPB - 1) / kKPB, bps = (nblk + ct.G - 1) / ct.G;
            const uint64_t capw = ((uint64_t)ct.cap + 2 * bps + 2) / 3;
            ct.cap = (uint32_t)((capw + 7) & ~7ull);
        }
        CK(hipFuncSetAttribute(reinterpret_cast<const void *>(BIN), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)std::max(bin_lds_of(tfull), bin_lds_of(ct))));
        CK(hipFuncSetAttribute(reinterpret_cast<const void *>(bloom_tile_or_kernel<uint64_t, true, kTileThreads, 4>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)(ct.w64 * 8 + (2 * kShards + 1) * 4)));
        TileScratch sc = s.sc[0];
        sc.zero_words = s.words;
        auto bin = [&](const TileCfg &tc) {
            hipLaunchKernelGGL(BIN, dim3((uint32_t)((kN + kKPB - 1) / kKPB)), dim3(kNT), bin_lds_of(tc), s0,
                               s.keys, nullptr, 16u, kN, s.c, tc, sc, s.bk[0]);
        };
        auto tile = [&](const TileCfg &tc) {
            hipLaunchKernelGGL((bloom_tile_or_kernel<uint64_t, true, kTileThreads, 4>), dim3(tc.T),
                               dim3(kTileThreads), (size_t)tc.w64 * 8 + (2 * kShards + 1) * 4, s0, tc, s.sc[0],
                               s.bk[0], s.words, nwords);
        };
        printf("product config: counted T=%u, shard-major buckets\n", ct.T);
        for (int r = 0; r < 20; ++r) {  // settle the clock
            bin(ct);
            tile(ct);
        }
        CK(hipStreamSynchronize(s0));
        if (!strcmp(what, "cstops") || all) {
            const char *names[] = {"hash+indices (stop 11)", "+count atomics (stop 1)", "+scan/reserve (stop 2)",
                                   "+placement (stop 3)", "full bin kernel (stop 0)"};
            const int stops[] = {11, 1, 2, 3, 0};
            for (int i = 0; i < 5; ++i) {
                set_stop(stops[i]);
                float best = 1e30f, sum = 0;
                for (int r = 0; r < 7; ++r) {
                    CK(hipMemsetAsync(s.sc[0].gcur, 0, kCurWords * 4, s0));
                    Ev e;
                    CK(hipEventRecord(e.a, s0));
                    bin(ct);
                    CK(hipEventRecord(e.b, s0));
                    const float t = e.ms();
                    best = std::min(best, t);
                    if (r >= 2) sum += t;
                }
                printf("phase stop %-26s best %.4f  mean(5) %.4f ms\n", names[i], best, sum / 5);
            }
            set_stop(0);
            CK(hipMemsetAsync(s.sc[0].gcur, 0, kCurWords * 4, s0));
            float best = 1e30f, sum = 0;
            for (int r = 0; r < 6; ++r) {
                bin(ct);
                Ev e;
                CK(hipEventRecord(e.a, s0));
                tile(ct);
                CK(hipEventRecord(e.b, s0));
                const float t = e.ms();
                best = std::min(best, t);
                if (r >= 1) sum += t;
            }
            printf("tile kernel: best %.4f  mean(5) %.4f ms\n", best, sum / 5);
        }
    }

    if (all || !strcmp(what, "tiles")) {
        // power-of-two tiles (915) vs counted tiles (768: three tile-kernel rounds),
        // one-shot builds interleaved, both checked against the reference filter
        TileCfg p2 = choose_tiles(kM, kN, kK), ct;
        if (!counted_tiles(kM, kN, kK, p2, &ct)) { printf("counted tiles: policy declined\n"); return 1; }
        {
            const uint64_t nblk = (kN + kKPB - 1) / kKPB, bps = (nblk + ct.G - 1) / ct.G;
            const uint64_t capw = ((uint64_t)ct.cap + 2 * bps + 2) / 3;
            ct.cap = (uint32_t)((capw + 7) & ~7ull);
        }
        CK(hipFuncSetAttribute(reinterpret_cast<const void *>(BIN), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)std::max(bin_lds_of(tfull), bin_lds_of(ct))));
        for (auto k : {bloom_tile_or_kernel<uint64_t, true, kTileThreads, 4>})
            CK(hipFuncSetAttribute(reinterpret_cast<const void *>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)(ct.w64 * 8 + (2 * kShards + 1) * 4)));
        printf("counted: T=%u mul=%u w64=%u cap=%u, tile LDS %u B, bin LDS %zu B\n", ct.T, ct.mul, ct.w64, ct.cap,
               ct.w64 * 8 + (2 * kShards + 1) * 4, bin_lds_of(ct));
        float bb[2] = {1e30f, 1e30f}, tt[2] = {1e30f, 1e30f}, sum[2] = {0, 0};
        for (int r = 0; r < 8; ++r)
            for (int v = 0; v < 2; ++v) {
                const TileCfg &tc = v ? ct : tfull;
                TileScratch sc = s.sc[0];
                sc.zero_words = v ? s.words : nullptr;
                CK(hipMemsetAsync(s.words, 0xA5, nwords * 8, s0));
                Ev e, f;
                CK(hipEventRecord(e.a, s0));
                hipLaunchKernelGGL(BIN, dim3((uint32_t)((kN + kKPB - 1) / kKPB)), dim3(kNT), bin_lds_of(tc), s0,
                                   s.keys, nullptr, 16u, kN, s.c, tc, sc, s.bk[0]);
                CK(hipEventRecord(e.b, s0));
                CK(hipEventRecord(f.a, s0));
                hipLaunchKernelGGL((bloom_tile_or_kernel<uint64_t, true, kTileThreads, 4>), dim3(tc.T),
                                   dim3(kTileThreads), (size_t)tc.w64 * 8 + (2 * kShards + 1) * 4, s0, tc,
                                   s.sc[0], s.bk[0], s.words, nwords);
                CK(hipEventRecord(f.b, s0));
                const float b = e.ms(), t = f.ms();
                bb[v] = std::min(bb[v], b);
                tt[v] = std::min(tt[v], t);
                if (r >= 2) sum[v] += b + t;
                if (r == 7) {
                    std::vector<uint64_t> a(nwords), ref(nwords);
                    CK(hipMemcpy(a.data(), s.words, nwords * 8, hipMemcpyDeviceToHost));
                    CK(hipMemcpy(ref.data(), s.words_ref, nwords * 8, hipMemcpyDeviceToHost));
                    printf("%s tiles: %s\n", v ? "counted" : "pow2", a == ref ? "bit-exact" : "MISMATCH");
                }
            }
        for (int v = 0; v < 2; ++v)
            printf("%s tiles (T=%u): bin best %.4f, tile best %.4f, build mean(6) %.4f ms\n", v ? "counted" : "pow2",
                   v ? ct.T : tfull.T, bb[v], tt[v], sum[v] / 6);
    }

    if (all || !strcmp(what, "mask")) {
        {
            hipStream_t d;
            CK(hipStreamCreateWithFlags(&d, hipStreamNonBlocking));
            uint32_t m[16] = {0};
            CK(hipExtStreamGetCUMask(d, 16, m));
            int bits = 0;
            printf("default stream CU mask:");
            for (int i = 0; i < 16; ++i) { printf(" %08x", m[i]); bits += __builtin_popcount(m[i]); }
            printf("  (%d bits)\n", bits);
            CK(hipStreamDestroy(d));
        }
        for (int x : {32, 64, 128}) {
            where(x, 0);
            where(x, 1);
        }
        where(224, 0);
        // the tile kernel on x CUs (unroll 4 / 16) and the bin kernel on x CUs
        for (int x : {32, 64, 128, 256}) {
            hipStream_t sm = masked_stream(x, 1);
            float t4 = 1e30f, t16 = 1e30f;
            for (int r = 0; r < 3; ++r) {
                launch_bin(s, 0, tfull, 0, kN, s0);
                CK(hipStreamSynchronize(s0));
                Ev e;
                CK(hipEventRecord(e.a, sm));
                launch_tile<4>(s, 0, tfull, true, s.words, sm);
                CK(hipEventRecord(e.b, sm));
                wait_or_die(sm, "tile kernel on a masked stream");
                t4 = std::min(t4, e.ms());
                launch_bin(s, 0, tfull, 0, kN, s0);
                CK(hipStreamSynchronize(s0));
                Ev f;
                CK(hipEventRecord(f.a, sm));
                launch_tile<16>(s, 0, tfull, true, s.words, sm);
                CK(hipEventRecord(f.b, sm));
                wait_or_die(sm, "tile kernel on a masked stream");
                t16 = std::min(t16, f.ms());
            }
            printf("tile kernel on %3d CUs: unroll 4 %.4f ms, unroll 16 %.4f ms\n", x, t4, t16);
            CK(hipStreamDestroy(sm));
        }
        for (int x : {256, 224, 192}) {
            hipStream_t sm = masked_stream(x, 0);
            float best = 1e30f;
            for (int r = 0; r < 4; ++r) {
                Ev e;
                CK(hipEventRecord(e.a, sm));
                launch_bin(s, 0, tfull, 0, kN, sm);
                CK(hipEventRecord(e.b, sm));
                wait_or_die(sm, "bin kernel on a masked stream");
                best = std::min(best, e.ms());
                launch_tile(s, 0, tfull, true, s.words, sm);
            }
            CK(hipStreamSynchronize(sm));
            printf("bin kernel on %3d CUs: %.4f ms\n", x, best);
            CK(hipStreamDestroy(sm));
        }
    }

    if (all || !strcmp(what, "pipe")) {
        // baseline: one-shot build (bin + tile) on the full chip
        float base = 1e30f;
        for (int r = 0; r < 5; ++r) {
            Ev e;
            CK(hipEventRecord(e.a, s0));
            launch_bin(s, 0, tfull, 0, kN, s0);
            launch_tile(s, 0, tfull, true, s.words, s0);
            CK(hipEventRecord(e.b, s0));
            base = std::min(base, e.ms());
        }
        printf("one-shot build: %.4f ms\n", base);
        hipEvent_t ev_bin[2], ev_tile[2], ev_go;
        for (int q = 0; q < 2; ++q) {
            CK(hipEventCreateWithFlags(&ev_bin[q], hipEventDisableTiming));
            CK(hipEventCreateWithFlags(&ev_tile[q], hipEventDisableTiming));
        }
        CK(hipEventCreateWithFlags(&ev_go, hipEventDisableTiming));
        for (int C : {2, 4, 8})
            for (int x : {32, 48, 64, 96}) {
                const uint64_t chunk = (kN / C + kKPB - 1) / kKPB * kKPB;
                const TileCfg tc = c4_tiles(chunk);
                hipStream_t sb = masked_stream(256 - x, 0), stl = masked_stream(x, 1), sfull;
                CK(hipStreamCreateWithFlags(&sfull, hipStreamNonBlocking));
                float best = 1e30f;
                bool ok = true;
                for (int r = 0; r < 4; ++r) {
                    CK(hipMemsetAsync(s.words, 0xA5, nwords * 8, s0));
                    Ev e;
                    CK(hipEventRecord(e.a, s0));
                    CK(hipEventRecord(ev_go, s0));
                    for (hipStream_t t : {sb, stl, sfull}) CK(hipStreamWaitEvent(t, ev_go, 0));
                    int c = 0;
                    for (uint64_t first = 0; first < kN; first += chunk, ++c) {
                        const uint64_t cn = std::min(chunk, kN - first);
                        const int q = c & 1;
                        const bool last = first + cn >= kN;
                        hipStream_t bs = c == 0 ? sfull : sb;  // the first bin kernel on all CUs
                        if (c >= 2) CK(hipStreamWaitEvent(bs, ev_tile[q], 0));  // buckets q free
                        launch_bin(s, q, tc, first, cn, bs);
                        CK(hipEventRecord(ev_bin[q], bs));
                        hipStream_t ts = last ? sfull : stl;  // the last tile kernel on all CUs
                        CK(hipStreamWaitEvent(ts, ev_bin[q], 0));
                        if (c >= 1) CK(hipStreamWaitEvent(ts, ev_tile[q ^ 1], 0));  // tiles in order
                        launch_tile(s, q, tc, c == 0, s.words, ts);
                        CK(hipEventRecord(ev_tile[q], ts));
                    }
                    CK(hipStreamWaitEvent(s0, ev_tile[(c - 1) & 1], 0));
                    CK(hipEventRecord(e.b, s0));
                    wait_or_die(s0, "the chunked pipeline", 10.0);
                    best = std::min(best, e.ms());
                    if (r == 3) {
                        std::vector<uint64_t> a(nwords), b(nwords);
                        CK(hipMemcpy(a.data(), s.words, nwords * 8, hipMemcpyDeviceToHost));
                        CK(hipMemcpy(b.data(), s.words_ref, nwords * 8, hipMemcpyDeviceToHost));
                        ok = a == b;
                    }
                }
                printf("pipeline C=%d chunks, tile CUs x=%2d: %.4f ms  %s\n", C, x, best,
                       ok ? "bit-exact" : "MISMATCH");
                CK(hipStreamDestroy(sb));
                CK(hipStreamDestroy(stl));
                CK(hipStreamDestroy(sfull));
            }
    }
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
