// ubench_r05.hip -- round-5 experiments on C4's bin kernel (diagnostic, not product
// code).  Includes the product kernels and measures, on C4's shard (100M x 16 B keys,
// k = 7, m = 958,505,838) in the product configuration (counted tiles, shard-major
// buckets, 768 threads x 3 keys, packed 21-bit entries), interleaved after a settle:
//   prod    the product bin kernel (one batch of 2 304 keys per block)
//   pers    a persistent grid (2 blocks per CU) looping over batches, no offset
//   pofs    the same, the second half of the grid starting with a half batch, so
//           the two blocks sharing a CU run half a batch out of phase (one hashes --
//           VALU -- while the other sorts -- LDS)
//   s2, s4  the build in 2 / 4 key chunks: every bin kernel on one stream, every tile
//           kernel on a second, high-priority stream (chunk i's tile kernel beside
//           chunk i+1's bin kernel; no CU masks -- the dispatcher interleaves the two
//           kernels' workgroups as CUs free up), two bucket sets alternating
// Each build is checked bit for bit against the product's one-shot build.
// usage: ubench_r05 [rounds] [variants, e.g. prod,s2,s4]
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

// Persistent packed bin kernel: block b handles (b >= H: the half batch b - H of the
// keys [0, H * half)), then the full batches R1 + j * kpb for j = b, b + P, ...
template <int FLAVOR, int LAYOUT, int KPT, typename ENTRY, int NT, bool STAGE, int KR, int KX, bool OFFSET>
__global__ __launch_bounds__(NT, NB_BIN_MIN_WAVES(NT)) void bin_persist_kernel(
    const uint8_t *__restrict__ keys, const uint64_t *__restrict__ offsets, uint32_t key_len,
    uint64_t n, FilterConsts c, TileCfg tc, TileScratch sc, ENTRY *__restrict__ buckets) {
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
    constexpr uint64_t kpb = (uint64_t)KPT * NT, half = kpb / 2;
    const uint32_t P = gridDim.x, H = OFFSET ? P / 2 : 0, b = blockIdx.x;
    const uint64_t R1 = (uint64_t)H * half;
    constexpr int kR = KR > 0 ? KR : 1;
    bool first = true;
    auto body = [&](uint64_t base, uint64_t end) {
        if (!first) __syncthreads();  // the previous batch's write-out has read the LDS
        first = false;
        BinPhase1<FLAVOR, LAYOUT, KPT, NT, STAGE, KR, KX> ph;
        ph.run(keys, offsets, key_len, end, c, tc.mul, T, cnt, sorted, wave_sums + NT / 64 + 1, base);
        bin_tail_two_tiles<NT, KPT, kR, ENTRY, KX>(lds, bin_sort_offset_words(T), tc, sc, buckets, base, end,
                                                   c.k, ph.ridx, ph.rank);
    };
    if (OFFSET && b >= H) {
        const uint64_t s = (uint64_t)(b - H) * half;
        if (s < n) body(s, min(s + half, n));
    }
    for (uint64_t j = b; R1 + j * kpb < n; j += P) body(R1 + j * kpb, min(R1 + (j + 1) * kpb, n));
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
#define PERS bin_persist_kernel<0, kFixed16, kKPT, uint64_t, kNT, false, 7, 7, false>
#define POFS bin_persist_kernel<0, kFixed16, kKPT, uint64_t, kNT, false, 7, 7, true>

struct Ev {
    hipEvent_t a, b;
    Ev() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    ~Ev() { (void)hipEventDestroy(a); (void)hipEventDestroy(b); }
    float ms() { float t; CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&t, a, b)); return t; }
};

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int rounds = argc > 1 ? atoi(argv[1]) : 10;
    const std::string want = argc > 2 ? argv[2] : "prod,pers,pofs,s2,s4";
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t *keys;
    uint64_t *words, *words_ref, *bk[2];
    uint32_t *zeroed[2];
    CK(hipMalloc(&keys, kN * 16 + 64));
    const uint64_t nwords = ((uint64_t)kM + 63) / 64;
    CK(hipMalloc(&words, nwords * 8));
    CK(hipMalloc(&words_ref, nwords * 8));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(keys), kN * 2);
    FilterConsts c = nb::make_consts(kM, kK, 17027509906831645879ull, 0);
    nb::set_fixed_len(c, 16);
    const size_t zb = (kCurWords + kFlagWords + kSuperCurWords + 2 * nwords) * 4;
    TileScratch sc[2];
    for (int q = 0; q < 2; ++q) {
        CK(hipMalloc(&zeroed[q], zb));
        CK(hipMemset(zeroed[q], 0, zb));
        sc[q].gcur = zeroed[q];
        sc[q].spill_flag = zeroed[q] + kCurWords;
        sc[q].spill32 = zeroed[q] + kCurWords + kFlagWords + kSuperCurWords;
        sc[q].zero_words = nullptr;
    }
    // the product's tiling for C4; capacity in words for the most runs any variant makes
    TileCfg p2 = choose_tiles(kM, kN, kK), ct;
    if (!counted_tiles(kM, kN, kK, p2, &ct)) { printf("counted tiles: policy declined\n"); return 1; }
    const uint32_t P = 2 * (uint32_t)cus;
    {
        const uint64_t items = (kN + kKPB - 1) / kKPB + P;  // full batches + the half batches
        const uint64_t bps = (items + ct.G - 1) / ct.G + 2;
        const uint64_t capw = ((uint64_t)ct.cap + 2 * bps + 2) / 3;
        ct.cap = (uint32_t)((capw + 7) & ~7ull);
    }
    for (int q = 0; q < 2; ++q) CK(hipMalloc(&bk[q], (size_t)ct.T * ct.G * ct.cap * 8));
    const size_t bin_lds = (size_t)bin_sort_offset_words(ct.T) * 4 + kKPB * kK * 4 + (size_t)ct.T * 8;
    const size_t tile_lds = (size_t)ct.w64 * 8 + (2 * kShards + 1) * 4;
    for (const void *k : {reinterpret_cast<const void *>(BIN), reinterpret_cast<const void *>(PERS),
                          reinterpret_cast<const void *>(POFS)})
        CK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bin_lds));
    for (const void *k : {reinterpret_cast<const void *>(bloom_tile_or_kernel<uint64_t, true>),
                          reinterpret_cast<const void *>(bloom_tile_or_kernel<uint64_t, false>)})
        CK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)tile_lds));
    printf("C4: n=%llu m=%u k=%u T=%u G=%u cap=%u words, bin LDS %zu B, tile LDS %zu B, CUs %d, P %u\n",
           (unsigned long long)kN, kM, kK, ct.T, ct.G, ct.cap, bin_lds, tile_lds, cus, P);
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipStreamCreateWithPriority(&s1, hipStreamNonBlocking, hi));
    hipEvent_t ev_bin[2], ev_tile[2];
    for (int q = 0; q < 2; ++q) {
        CK(hipEventCreateWithFlags(&ev_bin[q], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&ev_tile[q], hipEventDisableTiming));
    }
    auto bin_k = [&](int v, int q, uint64_t first, uint64_t cn, uint64_t *zw, hipStream_t st) {
        TileScratch s = sc[q];
        s.zero_words = zw;
        const uint8_t *kk = keys + first * 16;
        if (v == 1)
            hipLaunchKernelGGL(PERS, dim3(P), dim3(kNT), bin_lds, st, kk, nullptr, 16u, cn, c, ct, s, bk[q]);
        else if (v == 2)
            hipLaunchKernelGGL(POFS, dim3(P), dim3(kNT), bin_lds, st, kk, nullptr, 16u, cn, c, ct, s, bk[q]);
        else
            hipLaunchKernelGGL(BIN, dim3((uint32_t)((cn + kKPB - 1) / kKPB)), dim3(kNT), bin_lds, st, kk,
                               nullptr, 16u, cn, c, ct, s, bk[q]);
        CK(hipGetLastError());
    };
    auto tile_k = [&](int q, bool ow, uint64_t *w, hipStream_t st) {
        auto k = ow ? bloom_tile_or_kernel<uint64_t, true> : bloom_tile_or_kernel<uint64_t, false>;
        hipLaunchKernelGGL(k, dim3(ct.T), dim3(kTileThreads), tile_lds, st, ct, sc[q], bk[q], w, nwords);
        CK(hipGetLastError());
    };
    // one build of variant v into w (all work ends on s0)
    auto build = [&](int v, uint64_t *w) {
        if (v <= 2) {
            bin_k(v, 0, 0, kN, w, s0);
            tile_k(0, true, w, s0);
            return;
        }
        const int C = v == 3 ? 2 : 4;
        const uint64_t chunk = (kN / C + kKPB - 1) / kKPB * kKPB;
        CK(hipEventRecord(ev_tile[1], s0));  // s1 starts after everything on s0
        CK(hipStreamWaitEvent(s1, ev_tile[1], 0));
        int i = 0;
        for (uint64_t first = 0; first < kN; first += chunk, ++i) {
            const uint64_t cn = std::min(chunk, kN - first);
            const int q = i & 1;
            if (i >= 2) CK(hipStreamWaitEvent(s0, ev_tile[q], 0));  // buckets q free
            bin_k(0, q, first, cn, i == 0 ? w : nullptr, s0);
            CK(hipEventRecord(ev_bin[q], s0));
            CK(hipStreamWaitEvent(s1, ev_bin[q], 0));
            tile_k(q, i == 0, w, s1);
            CK(hipEventRecord(ev_tile[q], s1));
        }
        CK(hipStreamWaitEvent(s0, ev_tile[(i - 1) & 1], 0));
    };
    // reference (product) filter, then settle the clock
    build(0, words_ref);
    CK(hipStreamSynchronize(s0));
    for (int r = 0; r < 25; ++r) build(0, words);
    CK(hipStreamSynchronize(s0));
    const char *names[] = {"prod", "pers", "pofs", "s2", "s4"};
    std::vector<int> vs;
    for (int v = 0; v < 5; ++v)
        if (("," + want + ",").find(std::string(",") + names[v] + ",") != std::string::npos) vs.push_back(v);
    std::vector<float> tb[5], tt[5];
    bool ok[5] = {true, true, true, true, true};
    std::vector<uint64_t> a(nwords), ref(nwords);
    CK(hipMemcpy(ref.data(), words_ref, nwords * 8, hipMemcpyDeviceToHost));
    for (int r = 0; r < rounds; ++r)
        for (int v : vs) {
            CK(hipMemsetAsync(words, 0xA5, nwords * 8, s0));
            Ev e, f;
            CK(hipEventRecord(e.a, s0));
            if (v <= 2) {
                bin_k(v, 0, 0, kN, words, s0);
                CK(hipEventRecord(e.b, s0));
                CK(hipEventRecord(f.a, s0));
                tile_k(0, true, words, s0);
                CK(hipEventRecord(f.b, s0));
                tb[v].push_back(e.ms());
                tt[v].push_back(f.ms());
            } else {
                build(v, words);
                CK(hipEventRecord(e.b, s0));
                tb[v].push_back(e.ms());
                tt[v].push_back(0.f);
            }
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
        if (v <= 2)
            printf("%s: bin min %.4f med %.4f mean %.4f | tile min %.4f med %.4f | build mean %.4f ms  %s\n",
                   names[v], x[0], x[x.size() / 2], sb / x.size(), y[0], y[y.size() / 2], (sb + st) / x.size(),
                   ok[v] ? "bit-exact" : "MISMATCH");
        else
            printf("%s: build min %.4f med %.4f mean %.4f ms  %s\n", names[v], x[0], x[x.size() / 2], sb / x.size(),
                   ok[v] ? "bit-exact" : "MISMATCH");
    }
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
