// ubench_occ.hip -- round 5: C4's bin kernel at three resident blocks per CU (DESIGN
// §10.1 of round 4: "a third resident block once the per-block LDS drops"; diagnostic,
// not product code).  Includes the product kernels; the variants run the product's
// bin-kernel body (BinPhase1 + the packed two-tile tail) with other block shapes and
// launch bounds, on C4's shard (100M x 16 B keys, k = 7, m = 958,505,838, counted
// tiles, shard-major buckets), interleaved after a 25-build settle, every build
// checked bit for bit against the product's:
//   prod     768 threads x 3 keys (2 304 keys, 77 KB LDS, two blocks per CU)
//   k2n768   768 x 2 (1 536 keys, 55 KB): two blocks per CU (the control)
//   k2n640   640 x 2 (1 280 keys, 48 KB): three blocks per CU, 8 waves per SIMD
//   k2n704   704 x 2 (1 408 keys, 52 KB): three blocks per CU, 9 waves per SIMD
//   k2n512   512 x 2 (1 024 keys, 41 KB): three blocks per CU, 6 waves per SIMD
// usage: ubench_occ [rounds] [variants]
#include <hip/hip_runtime.h>

#include "../nasp-key-value-engine_amd/csrc/bloom_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t ck_ = (x);                                                 \
        if (ck_ != hipSuccess) {                                              \
            printf("HIP error %s at %d\n", hipGetErrorString(ck_), __LINE__); \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

namespace {

// the product's packed bin kernel body with its own launch bounds (MINW waves per SIMD)
template <int KPT, int NT, int MINW>
__global__ __launch_bounds__(NT, MINW) void bin_occ_kernel(const uint8_t *__restrict__ keys, uint64_t n,
                                                           FilterConsts c, TileCfg tc, TileScratch sc,
                                                           uint64_t *__restrict__ buckets) {
    extern __shared__ uint32_t lds[];
    const uint32_t T = tc.T, tid = threadIdx.x;
    uint32_t *cnt = lds;
    uint32_t *wave_sums = lds + 2 * T;
    uint32_t *sorted = lds + bin_sort_offset_words(T);
    if (sc.zero_words && tid == 0)
        for (uint32_t t = blockIdx.x + 1; t < T; t += gridDim.x) {
            const uint64_t b = tile_start(t, tc.mul);
            if (b & 63) sc.zero_words[b >> 6] = 0;
        }
    const uint64_t base = (uint64_t)blockIdx.x * (KPT * NT);
    BinPhase1<NB_FLAVOR_LIBSTDCXX, kFixed16, KPT, NT, false, 7, 7> ph;
    ph.run(keys, nullptr, 16u, n, c, tc.mul, T, cnt, sorted, wave_sums + NT / 64 + 1, base);
    bin_tail_two_tiles<NT, KPT, 7, uint64_t, 7>(lds, bin_sort_offset_words(T), tc, sc, buckets, base, n, c.k,
                                               ph.ridx, ph.rank);
}

}  // namespace
__global__ void k_fill(uint64_t *p, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        uint64_t x = i + 0x9E3779B97F4A7C15ull;
        x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
        x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
        p[i] = x ^ (x >> 31);
    }
}

constexpr int kNT = kBinThreads16Wide, kKPT = 3;
constexpr uint64_t kKPB = (uint64_t)kNT * kKPT;
constexpr uint64_t kN = 100000000;
constexpr uint32_t kM = 958505838u, kK = 7;
#define BIN bloom_bin_kernel<0, kFixed16, kKPT, uint64_t, kNT, false, 7, 7>
struct Var {
    const char *name;
    const void *fn;
    int nt, kpt;
};
const Var kVars[] = {
    {"prod", reinterpret_cast<const void *>(BIN), kNT, kKPT},
    {"k2n768", reinterpret_cast<const void *>(bin_occ_kernel<2, 768, 6>), 768, 2},
    {"k2n640", reinterpret_cast<const void *>(bin_occ_kernel<2, 640, 8>), 640, 2},
    {"k2n704", reinterpret_cast<const void *>(bin_occ_kernel<2, 704, 9>), 704, 2},
    {"k2n512", reinterpret_cast<const void *>(bin_occ_kernel<2, 512, 6>), 512, 2},
};
constexpr int kNV = sizeof(kVars) / sizeof(kVars[0]);

struct Ev {
    hipEvent_t a, b;
    Ev() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    ~Ev() { (void)hipEventDestroy(a); (void)hipEventDestroy(b); }
    float ms() { float t; CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&t, a, b)); return t; }
};

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int rounds = argc > 1 ? atoi(argv[1]) : 10;
    const std::string want = argc > 2 ? argv[2] : "prod,k2n768,k2n640,k2n704,k2n512";
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t *keys;
    uint64_t *words, *words_ref, *bk;
    uint32_t *zeroed;
    CK(hipMalloc(&keys, kN * 16 + 64));
    const uint64_t nwords = ((uint64_t)kM + 63) / 64;
    CK(hipMalloc(&words, nwords * 8));
    CK(hipMalloc(&words_ref, nwords * 8));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(keys), kN * 2);
    FilterConsts c = nb::make_consts(kM, kK, 17027509906831645879ull, 0);
    nb::set_fixed_len(c, 16);
    const size_t zb = (kCurWords + kFlagWords + kSuperCurWords + 2 * nwords) * 4;
    TileScratch sc;
    CK(hipMalloc(&zeroed, zb));
    CK(hipMemset(zeroed, 0, zb));
    sc.gcur = zeroed;
    sc.spill_flag = zeroed + kCurWords;
    sc.spill32 = zeroed + kCurWords + kFlagWords + kSuperCurWords;
    sc.zero_words = nullptr;
    // the product's tiling for C4; capacity in words for the most runs any variant makes
    TileCfg p2 = choose_tiles(kM, kN, kK), ct;
    if (!counted_tiles(kM, kN, kK, p2, &ct)) { printf("counted tiles: policy declined\n"); return 1; }
    {
        const uint64_t blocks = (kN + 1024 - 1) / 1024;
        const uint64_t bps = (blocks + ct.G - 1) / ct.G + 2;
        const uint64_t capw = ((uint64_t)ct.cap + 2 * bps + 2) / 3;
        ct.cap = (uint32_t)((capw + 7) & ~7ull);
    }
    CK(hipMalloc(&bk, (size_t)ct.T * ct.G * ct.cap * 8));
    // the product's LDS formula: run tables, the sort area, <= 2 pad slots per run
    auto lds_of = [&](const Var &v) {
        return (size_t)bin_sort_offset_words(ct.T) * 4 + (size_t)v.nt * v.kpt * kK * 4 + (size_t)ct.T * 8;
    };
    const size_t tile_lds = (size_t)ct.w64 * 8 + (2 * kShards + 1) * 4;
    for (const Var &v : kVars) {
        CK(hipFuncSetAttribute(v.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_of(v)));
        printf("%s: %d threads x %d keys, LDS %zu B\n", v.name, v.nt, v.kpt, lds_of(v));
    }
    for (const void *k : {reinterpret_cast<const void *>(bloom_tile_or_kernel<uint64_t, true>),
                          reinterpret_cast<const void *>(bloom_tile_or_kernel<uint64_t, false>)})
        CK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)tile_lds));
    printf("C4: n=%llu m=%u k=%u T=%u G=%u cap=%u words, tile LDS %zu B, CUs %d\n", (unsigned long long)kN, kM, kK,
           ct.T, ct.G, ct.cap, tile_lds, cus);
    hipStream_t s0;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    auto bin_k = [&](int v, uint64_t *zw) {
        TileScratch s = sc;
        s.zero_words = zw;
        const Var &q = kVars[v];
        const uint64_t kpb = (uint64_t)q.nt * q.kpt;
        const dim3 grid((uint32_t)((kN + kpb - 1) / kpb));
        if (v == 0)
            hipLaunchKernelGGL(BIN, grid, dim3(kNT), lds_of(q), s0, keys, nullptr, 16u, kN, c, ct, s, bk);
        else if (v == 1)
            hipLaunchKernelGGL((bin_occ_kernel<2, 768, 6>), grid, dim3(768), lds_of(q), s0, keys, kN, c, ct, s, bk);
        else if (v == 2)
            hipLaunchKernelGGL((bin_occ_kernel<2, 640, 8>), grid, dim3(640), lds_of(q), s0, keys, kN, c, ct, s, bk);
        else if (v == 3)
            hipLaunchKernelGGL((bin_occ_kernel<2, 704, 9>), grid, dim3(704), lds_of(q), s0, keys, kN, c, ct, s, bk);
        else
            hipLaunchKernelGGL((bin_occ_kernel<2, 512, 6>), grid, dim3(512), lds_of(q), s0, keys, kN, c, ct, s, bk);
        CK(hipGetLastError());
    };
    auto tile_k = [&](uint64_t *w) {
        hipLaunchKernelGGL((bloom_tile_or_kernel<uint64_t, true>), dim3(ct.T), dim3(kTileThreads), tile_lds, s0, ct, sc,
                           bk, w, nwords);
        CK(hipGetLastError());
    };
    auto build = [&](int v, uint64_t *w) {
        bin_k(v, w);
        tile_k(w);
    };
    build(0, words_ref);
    CK(hipStreamSynchronize(s0));
    for (int r = 0; r < 25; ++r) build(0, words);
    CK(hipStreamSynchronize(s0));
    std::vector<int> vs;
    for (int v = 0; v < kNV; ++v)
        if (("," + want + ",").find(std::string(",") + kVars[v].name + ",") != std::string::npos) vs.push_back(v);
    std::vector<float> tb[kNV], tt[kNV];
    bool ok[kNV];
    for (bool &o : ok) o = true;
    std::vector<uint64_t> a(nwords), ref(nwords);
    CK(hipMemcpy(ref.data(), words_ref, nwords * 8, hipMemcpyDeviceToHost));
    for (int r = 0; r < rounds; ++r)
        for (int v : vs) {
            CK(hipMemsetAsync(words, 0xA5, nwords * 8, s0));
            Ev e, f;
            CK(hipEventRecord(e.a, s0));
            bin_k(v, words);
            CK(hipEventRecord(e.b, s0));
            CK(hipEventRecord(f.a, s0));
            tile_k(words);
            CK(hipEventRecord(f.b, s0));
            tb[v].push_back(e.ms());
            tt[v].push_back(f.ms());
            if (r == 0 || r == rounds - 1) {
                CK(hipStreamSynchronize(s0));
                CK(hipMemcpy(a.data(), words, nwords * 8, hipMemcpyDeviceToHost));
                ok[v] = ok[v] && a == ref;
            }
        }
    for (int v : vs) {
        std::vector<float> x = tb[v], y = tt[v];
        std::sort(x.begin(), x.end());
        std::sort(y.begin(), y.end());
        double sb = 0, st = 0;
        for (float q : tb[v]) sb += q;
        for (float q : tt[v]) st += q;
        printf("%s: bin min %.4f med %.4f mean %.4f | tile min %.4f med %.4f | build mean %.4f ms  %s\n", kVars[v].name,
               x[0], x[x.size() / 2], sb / x.size(), y[0], y[y.size() / 2], (sb + st) / x.size(),
               ok[v] ? "bit-exact" : "MISMATCH");
    }
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
