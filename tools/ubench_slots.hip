// ubench_slots.hip -- round 5, VERDICT r04 item 1: the bin kernel with fixed-capacity
// slot ranges per tile (diagnostic, not product code).  Includes the product kernels and
// measures, on C4's shard (100M x 16 B keys, k = 7, m = 958,505,838) with the product's
// counted tiles and shard-major buckets, interleaved after a 25-build settle:
//   prod      the product bin kernel (768 threads x 3 keys; count -> scan -> reserve ->
//             place -> write-out)
//   slotsA    slot ranges, 768 threads x 2 keys (1 536 keys, ~14 indices per tile), C = 25
//             slots per tile (76.8 KB, two blocks per CU)
//   slotsB    slot ranges, 512 threads x 2 keys (1 024 keys, ~9.3 per tile), C = 15
//             (46 KB, three blocks per CU)
//   slotsA_stop1 / slotsA_stop2  diagnostics: slotsA stopped after phase 1 (count + slot
//             stores) / with reservations and word packing but no bucket stores (their
//             filters are not expected to match)
// A slot kernel's counter of tile t starts at t C, so the count atomic returns the
// index's slot: the index is stored there at once -- no scan, no run-start read, no
// placement pass.  Indices past a tile's C slots go to a small LDS overflow list (past
// that, to the spill bitmap the tile kernel folds).  Then thread t owns tile t: one
// reservation atomic, and the run's packed words (three 21-bit offsets, pads = copies
// of the first entry, the product's bucket format) written from its slots.  The tile
// kernel is the product's.  Every build is checked bit for bit against the product's.
// usage: ubench_slots [rounds] [variants, e.g. prod,slotsA,slotsB]
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

constexpr uint32_t kOvf = 256;  // LDS overflow list (entries)

template <uint32_t C>
__host__ __device__ constexpr size_t slots_lds_bytes(uint32_t T) {
    return ((size_t)T + 4 + kOvf + (size_t)T * C) * 4;
}

__device__ __forceinline__ void spill_entry(const TileScratch &sc, const TileCfg &tc, uint32_t v) {
    __hip_atomic_fetch_or(sc.spill32 + (v >> 5), 1u << (v & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sc.spill_flag[__umulhi(v, tc.fmul)] = 1u;
}

// STOP (diagnostic): 0 full kernel; 1 return after phase 1 (count + slot stores);
// 2 reservations and word packing but no bucket stores
template <int KPT, int NT, uint32_t C, int MINB, int STOP = 0>
__global__ __launch_bounds__(NT, MINB *NT / 256) void bin_slots_kernel(
    const uint8_t *__restrict__ keys, uint64_t n, FilterConsts c, TileCfg tc, TileScratch sc,
    uint64_t *__restrict__ buckets) {
    constexpr int K = 7;
    extern __shared__ uint32_t lds[];
    const uint32_t T = tc.T, tid = threadIdx.x;
    uint32_t *cnt = lds;                 // [T]: t C + count
    uint32_t *ovn = lds + T;             // overflow count
    uint32_t *ovl = lds + T + 4;         // [kOvf]
    uint32_t *slots = ovl + kOvf;        // [T][C]
    if (sc.zero_words && tid == 0)  // counted tiles, overwrite (as the product's bin kernel)
        for (uint32_t t = blockIdx.x + 1; t < T; t += gridDim.x) {
            const uint64_t b = tile_start(t, tc.mul);
            if (b & 63) sc.zero_words[b >> 6] = 0;
        }
    const uint64_t base = (uint64_t)blockIdx.x * (KPT * NT);
    KeyBatch<NB_FLAVOR_LIBSTDCXX, kFixed16, KPT> kb;
    kb.load(keys, nullptr, base + tid, NT, n);
    for (uint32_t t = tid; t < T; t += NT) cnt[t] = t * C;
    if (tid == 0) *ovn = 0u;
    __syncthreads();
    uint32_t ridx[KPT][K], ret[KPT][K];
    uint64_t h1[KPT], h2[KPT];
#pragma unroll
    for (int p = 0; p < KPT; ++p) kb.hash(c, keys, 16u, base + (uint64_t)p * NT + tid, p, &h1[p], &h2[p]);
#pragma unroll
    for (int p = 0; p < KPT; ++p) {
        if (base + (uint64_t)p * NT + tid < n) {
            IndexGen g;
            g.start(h1[p], h2[p], c);
#pragma unroll
            for (int j = 0; j < K; ++j) {
                if (j) g.next(c);
                ridx[p][j] = g.r;
                ret[p][j] = atomicAdd(&cnt[__umulhi(g.r, tc.mul)], 1u);
            }
        }
    }
    bool any_over = false;
#pragma unroll
    for (int p = 0; p < KPT; ++p) {
        if (base + (uint64_t)p * NT + tid < n) {
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const uint32_t r = ridx[p][j], s = ret[p][j];
                const bool over = s - __umulhi(r, tc.mul) * C >= C;
                any_over |= over;
                if (!over) slots[s] = r;
            }
        }
    }
    if (any_over) {  // rare: the lane's indices past their tile's slots
#pragma unroll
        for (int p = 0; p < KPT; ++p) {
            if (base + (uint64_t)p * NT + tid < n) {
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    const uint32_t r = ridx[p][j], s = ret[p][j];
                    if (s - __umulhi(r, tc.mul) * C >= C) {
                        const uint32_t o = atomicAdd(ovn, 1u);
                        if (o < kOvf) ovl[o] = r;
                        else spill_entry(sc, tc, r);
                    }
                }
            }
        }
    }
    __syncthreads();
    if (STOP == 1) return;
    // write-out: thread t owns tile t
    const uint32_t shard = blockIdx.x & (tc.G - 1);
    uint32_t *cur = sc.gcur + (size_t)shard * T;
    const uint32_t msk = (1u << tc.ts) - 1, hb = tc.ts - 11;
    const uint32_t no = min(*ovn, kOvf);
    for (uint32_t t = tid; t < T; t += NT) {
        const uint32_t h = cnt[t] - t * C;
        if (h == 0) continue;
        const uint32_t *sl = slots + t * C;
        uint32_t hr = h;
        if (h > C) {  // count the tile's entries in the overflow list
            hr = C;
            for (uint32_t o = 0; o < no; ++o) hr += __umulhi(ovl[o], tc.mul) == t;
        }
        const uint32_t w = (hr + 2) / 3;
        const uint32_t g = atomicAdd(&cur[t], w);
        uint64_t *dst = buckets + (size_t)bucket_region(tc, t, shard) * tc.cap + g;
        const uint32_t e0 = sl[0];
        if (h <= C && g + w <= tc.cap) {
            for (uint32_t q = 0; q < w; ++q) {
                const uint32_t i = 3 * q;
                const uint32_t a = sl[i], b = i + 1 < h ? sl[i + 1] : e0, d = i + 2 < h ? sl[i + 2] : e0;
                const uint32_t lo = (a & msk) | (b << 21);
                const uint32_t hi = __builtin_amdgcn_ubfe(b, 11, hb) | ((d & msk) << 10);
                if (STOP != 2 || (lo ^ hi) == 0x12345678u) dst[q] = (uint64_t)hi << 32 | lo;
            }
        } else {  // slow path: overflow-list entries and / or a full bucket
            uint32_t o = 0;
            auto entry = [&](uint32_t i) -> uint32_t {
                if (i < min(h, C)) return sl[i];
                while (__umulhi(ovl[o], tc.mul) != t) ++o;  // the (i - C)-th match, in order
                return ovl[o++];
            };
            for (uint32_t q = 0; q < w; ++q) {
                const uint32_t i = 3 * q;
                const uint32_t a = entry(i), b = i + 1 < hr ? entry(i + 1) : e0, d = i + 2 < hr ? entry(i + 2) : e0;
                if (g + q < tc.cap) {
                    const uint32_t lo = (a & msk) | (b << 21);
                    const uint32_t hi = __builtin_amdgcn_ubfe(b, 11, hb) | ((d & msk) << 10);
                    dst[q] = (uint64_t)hi << 32 | lo;
                } else {
                    spill_entry(sc, tc, a);
                    spill_entry(sc, tc, b);
                    spill_entry(sc, tc, d);
                }
            }
        }
    }
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
#define SLOTA bin_slots_kernel<2, 768, 25, 2>
#define SLOTB bin_slots_kernel<2, 512, 15, 3>
#define SLOTA1 bin_slots_kernel<2, 768, 25, 2, 1>
#define SLOTA2 bin_slots_kernel<2, 768, 25, 2, 2>
constexpr uint64_t kKPB_A = 2 * 768, kKPB_B = 2 * 512;

struct Ev {
    hipEvent_t a, b;
    Ev() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    ~Ev() { (void)hipEventDestroy(a); (void)hipEventDestroy(b); }
    float ms() { float t; CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&t, a, b)); return t; }
};

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int rounds = argc > 1 ? atoi(argv[1]) : 10;
    const std::string want = argc > 2 ? argv[2] : "prod,slotsA,slotsB";
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
        const uint64_t blocks = (kN + kKPB_B - 1) / kKPB_B;
        const uint64_t bps = (blocks + ct.G - 1) / ct.G + 2;
        const uint64_t capw = ((uint64_t)ct.cap + 2 * bps + 2) / 3;
        ct.cap = (uint32_t)((capw + 7) & ~7ull);
    }
    CK(hipMalloc(&bk, (size_t)ct.T * ct.G * ct.cap * 8));
    const size_t bin_lds = (size_t)bin_sort_offset_words(ct.T) * 4 + kKPB * kK * 4 + (size_t)ct.T * 8;
    const size_t lds_a = slots_lds_bytes<25>(ct.T), lds_b = slots_lds_bytes<15>(ct.T);
    const size_t tile_lds = (size_t)ct.w64 * 8 + (2 * kShards + 1) * 4;
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(BIN), hipFuncAttributeMaxDynamicSharedMemorySize, (int)bin_lds));
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(SLOTA), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_a));
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(SLOTB), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_b));
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(SLOTA1), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_a));
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(SLOTA2), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_a));
    for (const void *k : {reinterpret_cast<const void *>(bloom_tile_or_kernel<uint64_t, true>),
                          reinterpret_cast<const void *>(bloom_tile_or_kernel<uint64_t, false>)})
        CK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)tile_lds));
    printf("C4: n=%llu m=%u k=%u T=%u G=%u cap=%u words, LDS prod %zu / slotsA %zu / slotsB %zu B, tile %zu B, CUs %d\n",
           (unsigned long long)kN, kM, kK, ct.T, ct.G, ct.cap, bin_lds, lds_a, lds_b, tile_lds, cus);
    hipStream_t s0;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    auto bin_k = [&](int v, uint64_t *zw) {
        TileScratch s = sc;
        s.zero_words = zw;
        if (v == 1)
            hipLaunchKernelGGL(SLOTA, dim3((uint32_t)((kN + kKPB_A - 1) / kKPB_A)), dim3(768), lds_a, s0, keys, kN, c,
                               ct, s, bk);
        else if (v == 3)
            hipLaunchKernelGGL(SLOTA1, dim3((uint32_t)((kN + kKPB_A - 1) / kKPB_A)), dim3(768), lds_a, s0, keys, kN, c,
                               ct, s, bk);
        else if (v == 4)
            hipLaunchKernelGGL(SLOTA2, dim3((uint32_t)((kN + kKPB_A - 1) / kKPB_A)), dim3(768), lds_a, s0, keys, kN, c,
                               ct, s, bk);
        else if (v == 2)
            hipLaunchKernelGGL(SLOTB, dim3((uint32_t)((kN + kKPB_B - 1) / kKPB_B)), dim3(512), lds_b, s0, keys, kN, c,
                               ct, s, bk);
        else
            hipLaunchKernelGGL(BIN, dim3((uint32_t)((kN + kKPB - 1) / kKPB)), dim3(kNT), bin_lds, s0, keys, nullptr,
                               16u, kN, c, ct, s, bk);
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
    const char *names[] = {"prod", "slotsA", "slotsB", "slotsA_stop1", "slotsA_stop2"};
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
        printf("%s: bin min %.4f med %.4f mean %.4f | tile min %.4f med %.4f | build mean %.4f ms  %s\n", names[v],
               x[0], x[x.size() / 2], sb / x.size(), y[0], y[y.size() / 2], (sb + st) / x.size(),
               ok[v] ? "bit-exact" : "MISMATCH");
    }
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
