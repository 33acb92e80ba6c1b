// bloom_kernels.hip -- gfx950 (CDNA4, wave64) kernels of the SSTable Bloom-filter
// build/probe path, and the C ABI declared in include/nasp_bloom.h.
//
// Reference behaviour reproduced bit for bit (see bloom_math.h for the math):
//   BloomFilter::add             BloomFilter.cpp:82-86   -> bloom_build_kernel
//   BloomFilter::possiblyContains BloomFilter.cpp:67-80  -> bloom_probe_kernel
//   hash closure                 BloomFilter.cpp:57-62   -> key_hashes / for_each_index
//
// Kernel structure (one lane per key; integer/byte work, no MFMA):
//   1. read the key's bytes as 8-byte little-endian words (fixed 16-byte keys:
//      one 16-byte load per lane, fully coalesced; variable-length keys: aligned
//      8-byte loads + funnel shifts);
//   2. h1 and h2 in one pass over those words (h2's seed prefix is pre-mixed);
//   3. two reciprocal remainders, then k incremental indices;
//   4. set bits with no-return 32-bit agent-scope atomic OR (the filter is a
//      little-endian u64 word array; u32 halves alias the same bit positions).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/nasp_bloom.h"
#include "bloom_math.h"

using nb::FilterConsts;

namespace {

enum Layout : int { kOffsets = 0, kFixedStride = 1, kFixed16 = 2 };

constexpr int kBlock = 256;

// --------------------------------------------------------------- hashing ----
// The word-stream hashing (lsx_*, fnv_consume, hash_aligned_words) lives in
// bloom_math.h so the host test (tests/cpp/test_math.cpp) runs the same code.
using nb::LsxState;

template <int FLAVOR>
__device__ __forceinline__ void key_hashes_ptr(const FilterConsts &c, const uint8_t *p,
                                               uint32_t len, uint64_t *h1, uint64_t *h2) {
    const uintptr_t addr = reinterpret_cast<uintptr_t>(p);
    const uint32_t a = (uint32_t)(addr & 7);
    const uint64_t *q = reinterpret_cast<const uint64_t *>(addr - a);
    nb::hash_aligned_words<FLAVOR>(c, [q](uint32_t j) { return q[j]; }, a, len, h1, h2);
}

// Fixed 16-byte keys, 16-byte aligned: one dwordx4 load per lane.
template <int FLAVOR>
__device__ __forceinline__ void key_hashes_16(const FilterConsts &c, const uint8_t *keys,
                                              uint64_t i, uint64_t *h1, uint64_t *h2) {
    const ulonglong2 kv = reinterpret_cast<const ulonglong2 *>(keys)[i];
    if (FLAVOR == NB_FLAVOR_MSVC_FNV1A) {
        uint64_t f1 = nb::kFnvBasis, f2 = c.fnv_pre;
        nb::fnv_consume(f1, f2, kv.x, 8);
        nb::fnv_consume(f1, f2, kv.y, 8);
        *h1 = f1;
        *h2 = f2;
    } else {
        LsxState s;
        nb::lsx_begin(c, s, 16);
        nb::lsx_consume(c, s, 0, kv.x, 16);
        nb::lsx_consume(c, s, 1, kv.y, 16);
        nb::lsx_end(c, s, 16, h1, h2);
    }
}

template <int FLAVOR, int LAYOUT>
__device__ __forceinline__ void hashes_of(const FilterConsts &c, const uint8_t *keys,
                                          const uint64_t *offsets, uint32_t key_len,
                                          uint64_t i, uint64_t *h1, uint64_t *h2) {
    if (LAYOUT == kFixed16) {
        key_hashes_16<FLAVOR>(c, keys, i, h1, h2);
    } else if (LAYOUT == kFixedStride) {
        key_hashes_ptr<FLAVOR>(c, keys + i * key_len, key_len, h1, h2);
    } else {
        uint64_t b = offsets[i], e = offsets[i + 1];
        key_hashes_ptr<FLAVOR>(c, keys + b, (uint32_t)(e - b), h1, h2);
    }
}

// ------------------------------------------------------------- kernels ----

// Index stream of one key: r_0 = h1 mod m, then r_{j+1} = r_j + (h2 mod m) with a
// -(2^64 mod m) correction whenever the 64-bit x_j = h1 + j*h2 wraps.
struct IndexGen {
    uint64_t x, h2;
    uint32_t r, s;
    __device__ __forceinline__ void start(uint64_t h1_, uint64_t h2_, const FilterConsts &c) {
        x = h1_;
        h2 = h2_;
        r = nb::mod64(h1_, c.fm);
        s = nb::mod64(h2_, c.fm);
    }
    __device__ __forceinline__ void next(const FilterConsts &c) {
        const uint64_t nx = x + h2;
        r = nb::addmod(r, s, c.fm.m);
        if (nx < x) r = nb::submod(r, c.c64, c.fm.m);
        x = nx;
    }
};

// Path A ("atomic"): one lane per key, k no-return agent-scope atomic ORs.
// Bounded by the chip's atomic request rate (~27 G/s measured, tools/ubench.hip),
// used for k > 16, for filters too large for the tiled path, and for tiny batches.
template <int FLAVOR, int LAYOUT>
__global__ __launch_bounds__(kBlock) void bloom_build_atomic_kernel(
    const uint8_t *__restrict__ keys, const uint64_t *__restrict__ offsets, uint32_t key_len,
    uint64_t n, FilterConsts c, uint32_t *__restrict__ words32) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        uint64_t h1, h2;
        hashes_of<FLAVOR, LAYOUT>(c, keys, offsets, key_len, i, &h1, &h2);
        IndexGen g;
        g.start(h1, h2, c);
        for (uint32_t j = 0; j < c.k; ++j) {
            if (j) g.next(c);
            __hip_atomic_fetch_or(words32 + (g.r >> 5), 1u << (g.r & 31), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <int FLAVOR, int LAYOUT>
__global__ __launch_bounds__(kBlock) void bloom_probe_kernel(
    const uint8_t *__restrict__ keys, const uint64_t *__restrict__ offsets, uint32_t key_len,
    uint64_t n, FilterConsts c, const uint32_t *__restrict__ words32, uint8_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        uint64_t h1, h2;
        hashes_of<FLAVOR, LAYOUT>(c, keys, offsets, key_len, i, &h1, &h2);
        IndexGen g;
        g.start(h1, h2, c);
        uint8_t hit = 1;
        for (uint32_t j = 0; j < c.k; ++j) {
            if (j) g.next(c);
            if (!((words32[g.r >> 5] >> (g.r & 31)) & 1u)) { hit = 0; break; }
        }
        out[i] = hit;
    }
}


// Path B ("tiled"): the filter is cut into T tiles of 2^ts bits.
//   bin kernel : hash KPB keys per block, rank every index inside its tile with
//                an LDS counter, counting-sort the block's indices in LDS, reserve
//                a run per tile in that tile's global bucket (one contiguous-lane
//                atomicAdd per tile per block), and write the runs out coalesced.
//   tile kernel: one block per tile: OR the tile's bucket into a zeroed LDS copy
//                (ds_or, ~1.4 T ops/s chip-wide), then OR the tile into the filter
//                words with coalesced 8-byte loads/stores.
// Buckets hold the full 32-bit index.  A bucket that would exceed its capacity
// (only for pathological inputs, e.g. massively duplicated keys) spills the extra
// indices straight into the filter with atomic ORs, so results never depend on it.
struct TileCfg {
    uint32_t ts;     // log2 bits per tile
    uint32_t T;      // number of tiles = ceil(m / 2^ts)
    uint32_t cap;    // bucket capacity (entries) per tile, multiple of 4
};

constexpr int kBinThreads = 512;
constexpr int kTileThreads = 1024;

// Exclusive scan of hist[0..T) into S[0..T); returns the total.  blockDim = kBinThreads.
__device__ uint32_t block_exclusive_scan(const uint32_t *hist, uint32_t *S, uint32_t T,
                                         uint32_t *wave_sums) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t per = (T + kBinThreads - 1) / kBinThreads;
    const uint32_t b = min(tid * per, T), e = min(b + per, T);
    uint32_t local = 0;
    for (uint32_t t = b; t < e; ++t) local += hist[t];
    uint32_t incl = local;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t v = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += v;
    }
    if (lane == 63) wave_sums[wid] = incl;
    __syncthreads();
    if (wid == 0) {
        uint32_t w = lane < kBinThreads / 64 ? wave_sums[lane] : 0;
        uint32_t wi = w;
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            uint32_t v = __shfl_up(wi, d, 64);
            if (lane >= (uint32_t)d) wi += v;
        }
        if (lane < kBinThreads / 64) wave_sums[lane] = wi - w;  // exclusive wave offsets
        if (lane == kBinThreads / 64 - 1) wave_sums[kBinThreads / 64] = wi;  // total
    }
    __syncthreads();
    uint32_t run = wave_sums[wid] + incl - local;
    for (uint32_t t = b; t < e; ++t) {
        S[t] = run;
        run += hist[t];
    }
    return wave_sums[kBinThreads / 64];
}

template <int FLAVOR, int LAYOUT, int KPT, int KMAX>
__global__ __launch_bounds__(kBinThreads) void bloom_bin_kernel(
    const uint8_t *__restrict__ keys, const uint64_t *__restrict__ offsets, uint32_t key_len,
    uint64_t n, FilterConsts c, TileCfg tc, uint32_t *__restrict__ gcur,
    uint32_t *__restrict__ buckets, uint32_t *__restrict__ words32) {
    extern __shared__ uint32_t lds[];
    const uint32_t T = tc.T;
    uint32_t *hist = lds;              // [T]
    uint32_t *S = hist + T;            // [T] block-local run starts
    uint32_t *G = S + T;               // [T] global run starts (bucket positions)
    uint32_t *wave_sums = G + T;       // [kBinThreads/64 + 1]
    uint32_t *sorted = wave_sums + 32; // [KPB * k]
    const uint32_t tid = threadIdx.x;
    for (uint32_t t = tid; t < T; t += kBinThreads) hist[t] = 0;
    __syncthreads();

    // phase 1: hash, indices, in-tile ranks (kept in registers)
    uint32_t idx[KPT][KMAX], rnk[KPT][KMAX];
    const uint64_t base = (uint64_t)blockIdx.x * (KPT * kBinThreads);
#pragma unroll
    for (int p = 0; p < KPT; ++p) {
        const uint64_t i = base + (uint64_t)p * kBinThreads + tid;
        if (i < n) {
            uint64_t h1, h2;
            hashes_of<FLAVOR, LAYOUT>(c, keys, offsets, key_len, i, &h1, &h2);
            IndexGen g;
            g.start(h1, h2, c);
#pragma unroll
            for (int j = 0; j < KMAX; ++j) {
                if ((uint32_t)j < c.k) {
                    if (j) g.next(c);
                    idx[p][j] = g.r;
                    rnk[p][j] = atomicAdd(&hist[g.r >> tc.ts], 1u);
                }
            }
        }
    }
    __syncthreads();

    // phase 2: block-local run starts and global reservations
    const uint32_t total = block_exclusive_scan(hist, S, T, wave_sums);
    for (uint32_t t = tid; t < T; t += kBinThreads) {
        const uint32_t h = hist[t];
        G[t] = h ? atomicAdd(&gcur[t], h) : 0u;
    }
    __syncthreads();

    // phase 3: counting-sort the block's indices by tile
#pragma unroll
    for (int p = 0; p < KPT; ++p) {
        const uint64_t i = base + (uint64_t)p * kBinThreads + tid;
        if (i < n) {
#pragma unroll
            for (int j = 0; j < KMAX; ++j)
                if ((uint32_t)j < c.k) sorted[S[idx[p][j] >> tc.ts] + rnk[p][j]] = idx[p][j];
        }
    }
    __syncthreads();

    // phase 4: coalesced write-out of the runs (spill beyond capacity)
    for (uint32_t j = tid; j < total; j += kBinThreads) {
        const uint32_t v = sorted[j];
        const uint32_t t = v >> tc.ts;
        const uint32_t pos = G[t] + (j - S[t]);
        if (pos < tc.cap)
            buckets[(size_t)t * tc.cap + pos] = v;
        else
            __hip_atomic_fetch_or(words32 + (v >> 5), 1u << (v & 31), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ __launch_bounds__(kTileThreads) void bloom_tile_or_kernel(
    TileCfg tc, uint32_t *__restrict__ gcur, const uint32_t *__restrict__ buckets,
    uint64_t *__restrict__ words, uint64_t nwords) {
    extern __shared__ uint32_t tile[];
    const uint32_t t = blockIdx.x, tid = threadIdx.x;
    const uint32_t tile_words32 = 1u << (tc.ts - 5);
    const uint32_t mask = (1u << tc.ts) - 1;
    for (uint32_t w = tid; w < tile_words32; w += kTileThreads) tile[w] = 0;
    __syncthreads();
    const uint32_t cnt = min(gcur[t], tc.cap);
    const uint32_t *e = buckets + (size_t)t * tc.cap;
    const uint4 *e4 = reinterpret_cast<const uint4 *>(e);
    for (uint32_t q = tid; q < cnt / 4; q += kTileThreads) {
        const uint4 v = e4[q];
        atomicOr(&tile[(v.x & mask) >> 5], 1u << (v.x & 31));
        atomicOr(&tile[(v.y & mask) >> 5], 1u << (v.y & 31));
        atomicOr(&tile[(v.z & mask) >> 5], 1u << (v.z & 31));
        atomicOr(&tile[(v.w & mask) >> 5], 1u << (v.w & 31));
    }
    for (uint32_t q = (cnt & ~3u) + tid; q < cnt; q += kTileThreads) {
        const uint32_t v = e[q];
        atomicOr(&tile[(v & mask) >> 5], 1u << (v & 31));
    }
    __syncthreads();
    if (tid == 0) gcur[t] = 0;  // the workspace invariant: cursors are zero between builds
    const uint64_t w0 = (uint64_t)t << (tc.ts - 6);
    const uint32_t tile_words64 = tile_words32 / 2;
    const uint64_t *tile64 = reinterpret_cast<const uint64_t *>(tile);
    for (uint32_t w = tid; w < tile_words64; w += kTileThreads) {
        const uint64_t gw = w0 + w;
        if (gw < nwords) {
            const uint64_t v = tile64[w];
            if (v) words[gw] |= v;
        }
    }
}

__global__ __launch_bounds__(kBlock) void or_merge_kernel(uint64_t *__restrict__ dst,
                                                          const uint64_t *__restrict__ src,
                                                          uint64_t nwords, uint32_t nsrc,
                                                          uint64_t src_stride) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x; w < nwords; w += stride) {
        uint64_t v = dst[w];
        for (uint32_t s = 0; s < nsrc; ++s) v |= src[s * src_stride + w];
        dst[w] = v;
    }
}

// ------------------------------------------------------------ host side ----

thread_local std::string g_last_error;

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

#define NB_HIP(expr)                                                                    \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(NB_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_));   \
    } while (0)

uint32_t grid_for(uint64_t n) {
    uint64_t g = (n + kBlock - 1) / kBlock;
    const uint64_t cap = 256ull * 64;  // 256 CUs x 64 blocks: grid-stride beyond that
    return (uint32_t)std::max<uint64_t>(1, std::min(g, cap));
}

int check_common(uint64_t n, uint32_t m, int flavor, const void *keys, const void *words) {
    if (flavor != NB_FLAVOR_LIBSTDCXX && flavor != NB_FLAVOR_MSVC_FNV1A)
        return fail(NB_ERR_ARG, "unknown flavor");
    if (n && m == 0) return fail(NB_ERR_ARG, "m == 0 with keys (reference divides by zero)");
    if (n && (!keys || !words)) return fail(NB_ERR_ARG, "NULL keys or words");
    return NB_OK;
}

// Per-(device, stream) scratch of the tiled path: tile cursors (kept zero between
// builds by the tile kernel) and the bucket array.
struct Workspace {
    int dev = -1;
    hipStream_t st = nullptr;
    uint32_t *gcur = nullptr;
    size_t gcur_cap = 0;     // entries
    uint32_t *buckets = nullptr;
    size_t bucket_cap = 0;   // entries
};
std::mutex g_ws_mu;
std::vector<Workspace *> g_ws;

int get_ws(hipStream_t st, Workspace **out) {
    int dev = 0;
    NB_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_ws_mu);
    for (Workspace *w : g_ws)
        if (w->dev == dev && w->st == st) { *out = w; return NB_OK; }
    Workspace *w = new Workspace;
    w->dev = dev;
    w->st = st;
    g_ws.push_back(w);
    *out = w;
    return NB_OK;
}

int ws_reserve(Workspace &w, uint32_t T, size_t entries) {
    if (T > w.gcur_cap || entries > w.bucket_cap) NB_HIP(hipStreamSynchronize(w.st));
    if (T > w.gcur_cap) {
        if (w.gcur) NB_HIP(hipFree(w.gcur));
        w.gcur = nullptr;
        w.gcur_cap = 0;
        const size_t want = std::max<size_t>(T, 4096);
        NB_HIP(hipMalloc(&w.gcur, want * 4));
        NB_HIP(hipMemset(w.gcur, 0, want * 4));
        w.gcur_cap = want;
    }
    if (entries > w.bucket_cap) {
        if (w.buckets) NB_HIP(hipFree(w.buckets));
        w.buckets = nullptr;
        w.bucket_cap = 0;
        const size_t want = entries + entries / 8;
        NB_HIP(hipMalloc(&w.buckets, want * 4));
        w.bucket_cap = want;
    }
    return NB_OK;
}

TileCfg choose_tiles(uint32_t m, uint64_t n_chunk, uint32_t k) {
    TileCfg tc;
    uint32_t ts = 12;  // floor(log2(m / 256)) clamped to [12, 20]: >= 256 tiles when possible
    while (ts < 20 && ((uint64_t)m >> (ts + 1)) >= 256) ++ts;
    tc.ts = ts;
    tc.T = (uint32_t)(((uint64_t)m + (1ull << ts) - 1) >> ts);
    const double e = (double)n_chunk * k / tc.T;
    uint64_t cap = (uint64_t)(e + 8.0 * std::sqrt(e) + 64.0);
    cap = (cap + 63) & ~63ull;
    tc.cap = (uint32_t)std::min<uint64_t>(cap, 0xFFFFFFC0ull);
    return tc;
}

enum class BuildPath { kAuto, kAtomic, kTiled };

BuildPath path_override() {
    const char *e = std::getenv("NB_BUILD_PATH");
    if (!e) return BuildPath::kAuto;
    if (!std::strcmp(e, "atomic")) return BuildPath::kAtomic;
    if (!std::strcmp(e, "tiled")) return BuildPath::kTiled;
    return BuildPath::kAuto;
}

uint64_t chunk_keys() {
    const char *e = std::getenv("NB_CHUNK_KEYS");
    uint64_t v = e ? std::strtoull(e, nullptr, 10) : 0;
    return v ? v : (1ull << 27);
}

template <class K>
int allow_lds(K kernel, size_t bytes) {
    if (bytes > 64 * 1024)
        NB_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    return NB_OK;
}

template <int FLAVOR, int LAYOUT>
int launch_atomic(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                  const FilterConsts &c, uint64_t *words, hipStream_t st) {
    hipLaunchKernelGGL((bloom_build_atomic_kernel<FLAVOR, LAYOUT>), dim3(grid_for(n)),
                       dim3(kBlock), 0, st, keys, offsets, key_len, n, c,
                       reinterpret_cast<uint32_t *>(words));
    NB_HIP(hipGetLastError());
    return NB_OK;
}

template <int FLAVOR, int LAYOUT, int KPT, int KMAX>
int launch_tiled(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                 const FilterConsts &c, uint64_t *words, hipStream_t st) {
    constexpr uint64_t kpb = (uint64_t)KPT * kBinThreads;
    const uint64_t chunk = std::min<uint64_t>(n, std::max<uint64_t>(kpb, chunk_keys()));
    const TileCfg tc = choose_tiles(c.fm.m, chunk, c.k);
    Workspace *ws;
    int rc;
    if ((rc = get_ws(st, &ws))) return rc;
    if ((rc = ws_reserve(*ws, tc.T, (size_t)tc.T * tc.cap))) return rc;
    const size_t bin_lds = (3ull * tc.T + 32 + kpb * c.k) * 4;
    const size_t tile_lds = (size_t)1 << (tc.ts - 3);
    auto bin = bloom_bin_kernel<FLAVOR, LAYOUT, KPT, KMAX>;
    if ((rc = allow_lds(bin, bin_lds)) || (rc = allow_lds(bloom_tile_or_kernel, tile_lds))) return rc;
    const uint64_t nwords = ((uint64_t)c.fm.m + 63) / 64;
    uint32_t *w32 = reinterpret_cast<uint32_t *>(words);
    for (uint64_t done = 0; done < n; done += chunk) {
        const uint64_t cn = std::min(chunk, n - done);
        const uint8_t *ck = offsets ? keys : keys + done * key_len;
        const uint64_t *co = offsets ? offsets + done : nullptr;
        hipLaunchKernelGGL(bin, dim3((uint32_t)((cn + kpb - 1) / kpb)), dim3(kBinThreads), bin_lds,
                           st, ck, co, key_len, cn, c, tc, ws->gcur, ws->buckets, w32);
        NB_HIP(hipGetLastError());
        hipLaunchKernelGGL(bloom_tile_or_kernel, dim3(tc.T), dim3(kTileThreads), tile_lds, st, tc,
                           ws->gcur, ws->buckets, words, nwords);
        NB_HIP(hipGetLastError());
    }
    return NB_OK;
}

template <int FLAVOR, int LAYOUT>
int launch_build_l(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                   const FilterConsts &c, uint64_t *words, hipStream_t st) {
    BuildPath p = path_override();
    if (p == BuildPath::kAuto) {
        const TileCfg tc = choose_tiles(c.fm.m, n, c.k);
        const bool ok = c.k <= 16 && tc.T <= 2048 && n >= 4096;
        p = ok ? BuildPath::kTiled : BuildPath::kAtomic;
    }
    if (p == BuildPath::kTiled && c.k <= 16 && choose_tiles(c.fm.m, 1, c.k).T <= 2048) {
        if (c.k <= 8) return launch_tiled<FLAVOR, LAYOUT, 4, 8>(keys, offsets, key_len, n, c, words, st);
        return launch_tiled<FLAVOR, LAYOUT, 2, 16>(keys, offsets, key_len, n, c, words, st);
    }
    return launch_atomic<FLAVOR, LAYOUT>(keys, offsets, key_len, n, c, words, st);
}

template <int FLAVOR>
int launch_build_f(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                   const FilterConsts &c, uint64_t *words, hipStream_t st) {
    if (!offsets && key_len == 16 && (reinterpret_cast<uintptr_t>(keys) & 15) == 0)
        return launch_build_l<FLAVOR, kFixed16>(keys, offsets, key_len, n, c, words, st);
    if (!offsets)
        return launch_build_l<FLAVOR, kFixedStride>(keys, offsets, key_len, n, c, words, st);
    return launch_build_l<FLAVOR, kOffsets>(keys, offsets, key_len, n, c, words, st);
}

template <int FLAVOR>
int launch_probe_f(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                   const FilterConsts &c, const uint64_t *words, uint8_t *out, hipStream_t st) {
    dim3 grid(grid_for(n)), block(kBlock);
    const uint32_t *w32 = reinterpret_cast<const uint32_t *>(words);
    if (!offsets && key_len == 16 && (reinterpret_cast<uintptr_t>(keys) & 15) == 0)
        hipLaunchKernelGGL((bloom_probe_kernel<FLAVOR, kFixed16>), grid, block, 0, st, keys,
                           offsets, key_len, n, c, w32, out);
    else if (!offsets)
        hipLaunchKernelGGL((bloom_probe_kernel<FLAVOR, kFixedStride>), grid, block, 0, st, keys,
                           offsets, key_len, n, c, w32, out);
    else
        hipLaunchKernelGGL((bloom_probe_kernel<FLAVOR, kOffsets>), grid, block, 0, st, keys,
                           offsets, key_len, n, c, w32, out);
    NB_HIP(hipGetLastError());
    return NB_OK;
}

int launch_build(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                 uint32_t m, uint32_t k, uint64_t seed, int flavor, uint64_t *words,
                 hipStream_t st) {
    if (n == 0 || k == 0) return NB_OK;
    FilterConsts c = nb::make_consts(m, k, seed, (uint32_t)flavor);
    return flavor == NB_FLAVOR_MSVC_FNV1A
               ? launch_build_f<NB_FLAVOR_MSVC_FNV1A>(keys, offsets, key_len, n, c, words, st)
               : launch_build_f<NB_FLAVOR_LIBSTDCXX>(keys, offsets, key_len, n, c, words, st);
}

int launch_probe(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                 uint32_t m, uint32_t k, uint64_t seed, int flavor, const uint64_t *words,
                 uint8_t *out, hipStream_t st) {
    if (n == 0) return NB_OK;
    if (k == 0) {  // no hash closures: possiblyContains answers true
        NB_HIP(hipMemsetAsync(out, 1, n, st));
        return NB_OK;
    }
    FilterConsts c = nb::make_consts(m, k, seed, (uint32_t)flavor);
    return flavor == NB_FLAVOR_MSVC_FNV1A
               ? launch_probe_f<NB_FLAVOR_MSVC_FNV1A>(keys, offsets, key_len, n, c, words, out, st)
               : launch_probe_f<NB_FLAVOR_LIBSTDCXX>(keys, offsets, key_len, n, c, words, out, st);
}

// Per-device cached scratch for the host-buffer entry points.
struct DevScratch {
    std::mutex mu;
    bool init = false;
    hipStream_t stream = nullptr;
    void *buf[4] = {nullptr, nullptr, nullptr, nullptr};  // keys, offsets, words, out
    size_t cap[4] = {0, 0, 0, 0};
};

constexpr int kMaxDev = 64;
DevScratch g_dev[kMaxDev];

int ensure(DevScratch &d, int slot, size_t bytes) {
    if (bytes <= d.cap[slot]) return NB_OK;
    if (d.buf[slot]) NB_HIP(hipFree(d.buf[slot]));
    d.buf[slot] = nullptr;
    d.cap[slot] = 0;
    size_t want = std::max<size_t>(bytes + 64, d.cap[slot] * 3 / 2);
    NB_HIP(hipMalloc(&d.buf[slot], want));
    d.cap[slot] = want;
    return NB_OK;
}

int open_device(int device, DevScratch **out) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        return fail(NB_ERR_NODEV, "no HIP device visible");
    if (device < 0 || device >= count || device >= kMaxDev)
        return fail(NB_ERR_ARG, "device index out of range");
    NB_HIP(hipSetDevice(device));
    DevScratch &d = g_dev[device];
    if (!d.init) {
        NB_HIP(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
        d.init = true;
    }
    *out = &d;
    return NB_OK;
}

inline size_t nwords_of(uint32_t m) { return ((size_t)m + 63) / 64; }

size_t keys_bytes(const uint64_t *offsets, uint32_t key_len, uint64_t n) {
    return offsets ? (size_t)offsets[n] : (size_t)n * key_len;
}

}  // namespace

// =================================================================== C ABI ==

extern "C" {

int nb_abi_version(void) { return NB_ABI_VERSION; }

int nb_device_count(void) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) return 0;
    return c;
}

const char *nb_last_error(void) { return g_last_error.c_str(); }

int nb_shutdown(void) {
    {
        std::lock_guard<std::mutex> lk(g_ws_mu);
        for (Workspace *w : g_ws) {
            (void)hipSetDevice(w->dev);
            (void)hipStreamSynchronize(w->st);
            if (w->gcur) (void)hipFree(w->gcur);
            if (w->buckets) (void)hipFree(w->buckets);
            delete w;
        }
        g_ws.clear();
    }
    for (int i = 0; i < kMaxDev; ++i) {
        DevScratch &d = g_dev[i];
        std::lock_guard<std::mutex> lk(d.mu);
        if (!d.init) continue;
        (void)hipSetDevice(i);
        for (int s = 0; s < 4; ++s) {
            if (d.buf[s]) (void)hipFree(d.buf[s]);
            d.buf[s] = nullptr;
            d.cap[s] = 0;
        }
        (void)hipStreamDestroy(d.stream);
        d.stream = nullptr;
        d.init = false;
    }
    return NB_OK;
}

static uint32_t x86_double_to_u32(double v) { return (uint32_t)(uint64_t)(int64_t)v; }

uint32_t nb_size_of_bitset(uint32_t n, double p) {
    const double ln2 = std::log(2.0);
    return x86_double_to_u32(std::ceil(-(double)n * std::log(p) / (ln2 * ln2)));
}

uint32_t nb_num_hashes(uint32_t n, uint32_t m) {
    uint32_t k = x86_double_to_u32(std::round(((double)m / (double)n) * std::log(2.0)));
    return k == 0 ? 1 : k;
}

uint64_t nb_seed_from_time(uint32_t time_const);  // defined in bloom_host.cpp

int nb_build(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
             uint32_t m, uint32_t k, uint64_t h2_seed, int flavor, uint64_t *words, int device) {
    int rc = check_common(n, m, flavor, keys, words);
    if (rc || n == 0 || k == 0) return rc;
    DevScratch *d;
    if ((rc = open_device(device, &d))) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    const size_t kb = keys_bytes(offsets, key_len, n);
    const size_t wb = nwords_of(m) * 8;
    if ((rc = ensure(*d, 0, kb + 16)) || (offsets && (rc = ensure(*d, 1, (n + 1) * 8))) ||
        (rc = ensure(*d, 2, wb)))
        return rc;
    NB_HIP(hipMemcpyAsync(d->buf[0], keys, kb, hipMemcpyHostToDevice, d->stream));
    if (offsets)
        NB_HIP(hipMemcpyAsync(d->buf[1], offsets, (n + 1) * 8, hipMemcpyHostToDevice, d->stream));
    NB_HIP(hipMemcpyAsync(d->buf[2], words, wb, hipMemcpyHostToDevice, d->stream));
    rc = launch_build((const uint8_t *)d->buf[0], offsets ? (const uint64_t *)d->buf[1] : nullptr,
                      key_len, n, m, k, h2_seed, flavor, (uint64_t *)d->buf[2], d->stream);
    if (rc) return rc;
    NB_HIP(hipMemcpyAsync(words, d->buf[2], wb, hipMemcpyDeviceToHost, d->stream));
    NB_HIP(hipStreamSynchronize(d->stream));
    return NB_OK;
}

int nb_probe(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
             uint32_t m, uint32_t k, uint64_t h2_seed, int flavor, const uint64_t *words,
             uint8_t *out, int device) {
    if (n == 0) return NB_OK;
    if (!out) return fail(NB_ERR_ARG, "NULL out");
    if (k == 0) {
        std::memset(out, 1, n);
        return NB_OK;
    }
    int rc = check_common(n, m, flavor, keys, words);
    if (rc) return rc;
    DevScratch *d;
    if ((rc = open_device(device, &d))) return rc;
    std::lock_guard<std::mutex> lk(d->mu);
    const size_t kb = keys_bytes(offsets, key_len, n);
    const size_t wb = nwords_of(m) * 8;
    if ((rc = ensure(*d, 0, kb + 16)) || (offsets && (rc = ensure(*d, 1, (n + 1) * 8))) ||
        (rc = ensure(*d, 2, wb)) || (rc = ensure(*d, 3, n)))
        return rc;
    NB_HIP(hipMemcpyAsync(d->buf[0], keys, kb, hipMemcpyHostToDevice, d->stream));
    if (offsets)
        NB_HIP(hipMemcpyAsync(d->buf[1], offsets, (n + 1) * 8, hipMemcpyHostToDevice, d->stream));
    NB_HIP(hipMemcpyAsync(d->buf[2], words, wb, hipMemcpyHostToDevice, d->stream));
    rc = launch_probe((const uint8_t *)d->buf[0], offsets ? (const uint64_t *)d->buf[1] : nullptr,
                      key_len, n, m, k, h2_seed, flavor, (const uint64_t *)d->buf[2],
                      (uint8_t *)d->buf[3], d->stream);
    if (rc) return rc;
    NB_HIP(hipMemcpyAsync(out, d->buf[3], n, hipMemcpyDeviceToHost, d->stream));
    NB_HIP(hipStreamSynchronize(d->stream));
    return NB_OK;
}

int nb_build_device(const uint8_t *d_keys, const uint64_t *d_offsets, uint32_t key_len,
                    uint64_t n, uint32_t m, uint32_t k, uint64_t h2_seed, int flavor,
                    uint64_t *d_words, void *stream) {
    int rc = check_common(n, m, flavor, d_keys, d_words);
    if (rc) return rc;
    return launch_build(d_keys, d_offsets, key_len, n, m, k, h2_seed, flavor, d_words,
                        (hipStream_t)stream);
}

int nb_probe_device(const uint8_t *d_keys, const uint64_t *d_offsets, uint32_t key_len,
                    uint64_t n, uint32_t m, uint32_t k, uint64_t h2_seed, int flavor,
                    const uint64_t *d_words, uint8_t *d_out, void *stream) {
    if (n && !d_out) return fail(NB_ERR_ARG, "NULL out");
    if (k == 0) return launch_probe(d_keys, d_offsets, key_len, n, m, k, h2_seed, flavor,
                                    d_words, d_out, (hipStream_t)stream);
    int rc = check_common(n, m, flavor, d_keys, d_words);
    if (rc) return rc;
    return launch_probe(d_keys, d_offsets, key_len, n, m, k, h2_seed, flavor, d_words, d_out,
                        (hipStream_t)stream);
}

int nb_or_merge_device(uint64_t *d_dst, const uint64_t *d_src, uint64_t nwords, uint32_t nsrc,
                       uint64_t src_stride, void *stream) {
    if (nwords == 0 || nsrc == 0) return NB_OK;
    if (!d_dst || !d_src) return fail(NB_ERR_ARG, "NULL buffer");
    hipLaunchKernelGGL(or_merge_kernel, dim3(grid_for(nwords)), dim3(kBlock), 0,
                       (hipStream_t)stream, d_dst, d_src, nwords, nsrc, src_stride);
    NB_HIP(hipGetLastError());
    return NB_OK;
}

}  // extern "C"
