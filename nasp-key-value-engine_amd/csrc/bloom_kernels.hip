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
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/nasp_bloom.h"
#include "bloom_math.h"
#include "nb_knobs.h"

using nb::FilterConsts;

size_t nb_internal_frame_header(uint32_t m, uint32_t k, double p, uint32_t time_const,
                                uint64_t h2_seed, int framing, uint8_t *out);  // bloom_host.cpp

namespace {

// kFixed16 / kFixed32: 16- / 32-byte keys at a 16-byte-aligned base, loaded as
// dwordx4 vectors straight into registers (no LDS stage)
enum Layout : int { kOffsets = 0, kFixedStride = 1, kFixed16 = 2, kFixed32 = 3 };
constexpr bool vec_layout(int l) { return l == kFixed16 || l == kFixed32; }

constexpr int kBlock = 256;

// --------------------------------------------------------------- hashing ----
// The word-stream hashing (lsx_*, fnv_consume, hash_aligned_words) lives in
// bloom_math.h so the host test (tests/cpp/test_math.cpp) runs the same code.
using nb::LsxState;

template <int FLAVOR, bool FIXED_LEN>
__device__ __forceinline__ void key_hashes_ptr(const FilterConsts &c, const uint8_t *p,
                                               uint32_t len, uint64_t *h1, uint64_t *h2) {
    const uintptr_t addr = reinterpret_cast<uintptr_t>(p);
    const uint32_t a = (uint32_t)(addr & 7);
    const uint64_t *q = reinterpret_cast<const uint64_t *>(addr - a);
    auto load = [q](uint32_t j) { return q[j]; };
    nb::hash_aligned_words<FLAVOR, decltype(load), FIXED_LEN>(c, load, a, len, h1, h2);
}

// libstdc++ hashes of a 16-byte key with PREM = D % 8 leftover seed digits, as
// straight-line code: h2's stream is the PREM digits ++ the key, i.e. two whole
// words spliced with constant funnel shifts and (PREM > 0) a PREM-byte tail --
// the same words lsx_begin_fixed/lsx_consume/lsx_end feed, without their
// run-time shift amounts and branches.
template <int PREM>
__device__ __forceinline__ void lsx16(const FilterConsts &c, const ulonglong2 &kv, uint64_t *h1,
                                      uint64_t *h2) {
    uint64_t h = nb::lsx_init(16);
    h = nb::lsx_round(h, kv.x);
    h = nb::lsx_round(h, kv.y);
    *h1 = nb::lsx_final(h);
    uint64_t g = c.h2_init_fixed;
    if (PREM == 0) {
        g = nb::lsx_round(g, kv.x);
        g = nb::lsx_round(g, kv.y);
    } else {
        constexpr int r8 = 8 * PREM;
        g = nb::lsx_round(g, c.pre_tail | (kv.x << r8));
        g = nb::lsx_round(g, (kv.x >> (64 - r8)) | (kv.y << r8));
        g = nb::lsx_tail(g, kv.y >> (64 - r8));
    }
    *h2 = nb::lsx_final(g);
}

// Fixed 16-byte keys, 16-byte aligned: one dwordx4 load per lane.
#ifndef NB_PREM_SPECIALIZE
#define NB_PREM_SPECIALIZE 1
#endif
template <int FLAVOR>
__device__ __forceinline__ void hash16(const FilterConsts &c, const ulonglong2 &kv, uint64_t *h1,
                                       uint64_t *h2) {
    if (FLAVOR == NB_FLAVOR_MURMUR3_X64_128) {
        nb::mm3_x64_128([&](uint32_t j) { return j ? kv.y : kv.x; }, 16, c.mm3_seed, h1, h2);
    } else if (FLAVOR == NB_FLAVOR_MSVC_FNV1A) {
        uint64_t f1 = nb::kFnvBasis, f2 = c.fnv_pre;
        nb::fnv_consume(f1, f2, kv.x, 8);
        nb::fnv_consume(f1, f2, kv.y, 8);
        *h1 = f1;
        *h2 = f2;
    } else if (!NB_PREM_SPECIALIZE) {
        LsxState s;
        nb::lsx_begin_fixed(c, s, 16);
        nb::lsx_consume(c, s, 0, kv.x, 16);
        nb::lsx_consume(c, s, 1, kv.y, 16);
        nb::lsx_end(c, s, 16, h1, h2);
    } else {
        switch (c.prem) {  // kernel-uniform: a scalar branch
            case 0: lsx16<0>(c, kv, h1, h2); break;
            case 1: lsx16<1>(c, kv, h1, h2); break;
            case 2: lsx16<2>(c, kv, h1, h2); break;
            case 3: lsx16<3>(c, kv, h1, h2); break;
            case 4: lsx16<4>(c, kv, h1, h2); break;
            case 5: lsx16<5>(c, kv, h1, h2); break;
            case 6: lsx16<6>(c, kv, h1, h2); break;
            default: lsx16<7>(c, kv, h1, h2); break;
        }
    }
}

template <int FLAVOR>
__device__ __forceinline__ void key_hashes_16(const FilterConsts &c, const uint8_t *keys,
                                              uint64_t i, uint64_t *h1, uint64_t *h2) {
    hash16<FLAVOR>(c, reinterpret_cast<const ulonglong2 *>(keys)[i], h1, h2);
}

// 32-byte keys (C5's shape): four words in registers; h2's stream words are the
// seed-prefix splice of consecutive key words (bloom_math.h lsx_splice, prefix
// class PC of D % 8), then the D % 8 leftover bytes as the tail.
template <int PC>
__device__ __forceinline__ void lsx32(const FilterConsts &c, const uint64_t (&w)[4], uint64_t *h1,
                                      uint64_t *h2) {
    uint64_t h = nb::lsx_init(32), g = c.h2_init_fixed;
    const uint32_t p = c.prem;
    uint64_t kwp = PC ? c.pre_tail << (64 - 8 * p) : 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        h = nb::lsx_round(h, w[j]);
        g = nb::lsx_round(g, nb::lsx_splice<PC>(kwp, w[j], p));
        kwp = w[j];
    }
    if (PC) g = nb::lsx_tail(g, nb::lsx_splice<PC>(kwp, 0, p) & ((1ull << (8 * p)) - 1));
    *h1 = nb::lsx_final(h);
    *h2 = nb::lsx_final(g);
}

template <int FLAVOR>
__device__ __forceinline__ void hash32(const FilterConsts &c, const ulonglong2 &a,
                                       const ulonglong2 &b, uint64_t *h1, uint64_t *h2) {
    const uint64_t w[4] = {a.x, a.y, b.x, b.y};
    if (FLAVOR == NB_FLAVOR_MURMUR3_X64_128) {
        nb::mm3_x64_128([&](uint32_t j) { return j == 0 ? w[0] : j == 1 ? w[1] : j == 2 ? w[2] : w[3]; },
                        32, c.mm3_seed, h1, h2);
    } else if (FLAVOR == NB_FLAVOR_MSVC_FNV1A) {
        uint64_t f1 = nb::kFnvBasis, f2 = c.fnv_pre;
#pragma unroll
        for (int j = 0; j < 4; ++j) nb::fnv_consume(f1, f2, w[j], 8);
        *h1 = f1;
        *h2 = f2;
    } else if (c.prem == 0) {  // kernel-uniform
        lsx32<0>(c, w, h1, h2);
    } else if (c.prem <= 4) {
        lsx32<1>(c, w, h1, h2);
    } else {
        lsx32<2>(c, w, h1, h2);
    }
}

// A block's KPT keys per lane: all loads issued before any hashing, so a lane
// has KPT key loads (fixed 16-byte keys) or offset pairs (variable keys) in
// flight at once instead of one exposed latency per key.
template <int FLAVOR, int LAYOUT, int KPT>
struct KeyBatch {
    ulonglong2 kv[KPT], kv2[LAYOUT == kFixed32 ? KPT : 1];
    uint64_t b[KPT], e[KPT];
    __device__ __forceinline__ void load_one(int p, const uint8_t *keys, const uint64_t *offsets,
                                             uint64_t i, uint64_t n) {
        if (i < n) {
            const ulonglong2 *kq = reinterpret_cast<const ulonglong2 *>(keys);
            if (LAYOUT == kFixed16) kv[p] = kq[i];
            else if (LAYOUT == kFixed32) { kv[p] = kq[2 * i]; kv2[LAYOUT == kFixed32 ? p : 0] = kq[2 * i + 1]; }
            else if (LAYOUT == kOffsets) { b[p] = offsets[i]; e[p] = offsets[i + 1]; }
        }
    }
    __device__ __forceinline__ void load(const uint8_t *keys, const uint64_t *offsets,
                                         uint64_t base, uint64_t stride, uint64_t n) {
#pragma unroll
        for (int p = 0; p < KPT; ++p) load_one(p, keys, offsets, base + p * stride, n);
    }
    __device__ __forceinline__ void hash(const FilterConsts &c, const uint8_t *keys,
                                         uint32_t key_len, uint64_t i, int p, uint64_t *h1,
                                         uint64_t *h2) const {
        if (LAYOUT == kFixed16) hash16<FLAVOR>(c, kv[p], h1, h2);
        else if (LAYOUT == kFixed32) hash32<FLAVOR>(c, kv[p], kv2[LAYOUT == kFixed32 ? p : 0], h1, h2);
        else if (LAYOUT == kFixedStride)
            key_hashes_ptr<FLAVOR, true>(c, keys + i * key_len, key_len, h1, h2);
        else key_hashes_ptr<FLAVOR, false>(c, keys + b[p], (uint32_t)(e[p] - b[p]), h1, h2);
    }
};

template <int FLAVOR, int LAYOUT>
__device__ __forceinline__ void hashes_of(const FilterConsts &c, const uint8_t *keys,
                                          const uint64_t *offsets, uint32_t key_len,
                                          uint64_t i, uint64_t *h1, uint64_t *h2) {
    if (LAYOUT == kFixed16) {
        key_hashes_16<FLAVOR>(c, keys, i, h1, h2);
    } else if (LAYOUT == kFixed32) {
        const ulonglong2 *kq = reinterpret_cast<const ulonglong2 *>(keys);
        hash32<FLAVOR>(c, kq[2 * i], kq[2 * i + 1], h1, h2);
    } else if (LAYOUT == kFixedStride) {
        key_hashes_ptr<FLAVOR, true>(c, keys + i * key_len, key_len, h1, h2);
    } else {
        uint64_t b = offsets[i], e = offsets[i + 1];
        key_hashes_ptr<FLAVOR, false>(c, keys + b, (uint32_t)(e - b), h1, h2);
    }
}

// ------------------------------------------------------------- kernels ----

// Index stream of one key: r_0 = h1 mod m, then r_{j+1} = r_j + (h2 mod m) with a
// -(2^64 mod m) correction whenever the 64-bit x_j = h1 + j*h2 wraps.
using nb::IndexGen;

// Path A ("atomic"): one lane per key, k no-return agent-scope atomic ORs.
// Bounded by the chip's atomic request rate (~27 G/s measured, tools/ubench.hip),
// used for k > 32, for filters too large for the tiled path, and for tiny batches.
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

// The probe's auto mode (launch_probe_tiled): the lane kernel probes a sample of
// the batch first and counts its positives; every later kernel reads that count and
// runs only if its path is the one chosen (a block-uniform early exit), so the
// choice needs no host synchronisation and the launch sequence stays
// graph-capturable.
struct ProbeGate {
    uint32_t *hits;          // sample launch: its blocks' positive counts, one word per block
    const uint32_t *decide;  // nullptr: always run; else the sample's counts: run iff the
                             // choice they make == want
    uint32_t blocks;         // sample blocks (words of decide)
    uint32_t sample;         // keys in the sample
    uint32_t want;           // 1 the lane path, 2 the tiled path, 3 the split tiled path
    uint32_t pct = 30;       // the tiled path from this percentage of the sample present
    uint32_t split_pct = 101;  // the split path from this percentage (> 100: never) up
                               // to pct, where the tiled path takes over
};
// Auto's thresholds with the split path, per shape (the crossings of
// profiles/r05_probe_split_final_{c4,c5shape}.txt and r05_probe_split_c3.txt): lane ->
// split at ~6 % present on C4's filter (16-byte keys, k = 7), ~18 % on C5's shape
// (32-byte keys, k = 10: the lane kernel's absent keys are cheap there) and on C3's
// variable-length keys -- NB_PROBE_SPLIT_PCT 0, the policy -- and split -> tiled at
// ~67 % / ~55 % / ~40 % (the second round hashes a listed variable-length key straight
// from HBM, without the stage).
constexpr uint32_t split_pct_policy(uint32_t k, bool vec) { return vec && k <= 8 ? 7u : 18u; }
constexpr uint32_t split_tiled_pct(uint32_t k, bool vec) { return !vec ? 40u : k <= 8 ? 65u : 55u; }
// Auto's choice from the sample's hit count h of s keys: 1 lane, 2 tiled, 3 split.
// Without the split path: tiled when at least pct % were present (a present key costs
// the lane kernel ~k gathers, an absent one ~2, and the tiled path a fixed pass plus
// ~k/2 miss stores per absent key; on C3 / C4's filter and on C5's shape the two break
// even at ~30 % present).  With it: lane below split_pct %, split below pct %, tiled
// from there.
__host__ __device__ inline uint32_t probe_pick(uint64_t h, uint64_t s, uint32_t pct, uint32_t split_pct) {
    if (100 * h >= (uint64_t)pct * s) return 2u;
    if (split_pct <= 100 && 100 * h >= (uint64_t)split_pct * s) return 3u;
    return 1u;
}
// The counts are read with device-scope atomic loads: coherent with the sample
// kernel's stores whatever a CU's caches hold from an earlier call.  (Round 6: plain
// loads became scalar loads, and in replays of a captured graph some kernels of one
// call decided on the previous replay's counts -- a tiled bin kernel open behind a
// closed tile kernel left its cursors for the split path's buckets, whose tile kernel
// then read another layout's words as key ids: a memory fault,
// tools/diag_graph_auto.py.)
__device__ __forceinline__ uint32_t coherent_load(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool gate_open(const ProbeGate &g) {
    if (!g.decide) return true;
    uint32_t h = 0;
    for (uint32_t b = 0; b < g.blocks; ++b) h += coherent_load(g.decide + b);
    return probe_pick(h, g.sample, g.pct, g.split_pct) == g.want;
}

// One lane per key, k gathers with an early exit at the first zero bit.
template <int FLAVOR, int LAYOUT>
__global__ __launch_bounds__(kBlock) void bloom_probe_kernel(
    const uint8_t *__restrict__ keys, const uint64_t *__restrict__ offsets, uint32_t key_len,
    uint64_t n, FilterConsts c, const uint32_t *__restrict__ words32, uint8_t *__restrict__ out,
    ProbeGate gate) {
    if (!gate_open(gate)) return;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    uint32_t hits = 0;
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
        hits += hit;
    }
    if (gate.hits) {  // the block's count (plain stores: nothing to zero beforehand)
        __shared__ uint32_t wsum[kBlock / 64];
        for (int o = 32; o; o >>= 1) hits += __shfl_xor(hits, o);
        if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = hits;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t t = 0;
            for (int w = 0; w < kBlock / 64; ++w) t += wsum[w];
            // system scope: the slot may be host-mapped memory
            __hip_atomic_store(gate.hits + blockIdx.x, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}


// Path B ("tiled"): the filter is cut into T tiles of 2^ts bits.
//   bin kernel : hash KPB keys per block, count every index per tile in LDS,
//                reserve one run per tile in that tile's bucket (contiguous-lane
//                atomicAdds on cursors sharded G ways by block -- blocks b and b+8
//                share an XCD, so a shard's runs are written through one L2),
//                counting-sort the block's indices in LDS and write the runs out.
//   tile kernel: one block per tile: OR the tile's G bucket shards into a zeroed
//                LDS copy (ds_or), then store the tile into the filter words
//                (overwrite) or OR it in (accumulate).
// Bucket entries are the in-tile bit offset: 16-bit when ts <= 16 (half the
// traffic), else the full 32-bit index.  A shard that would exceed its capacity
// (pathological inputs only, e.g. massively duplicated keys) spills the extra
// indices into a zero-kept spill bitmap that the tile kernel folds in and clears,
// so results never depend on capacity.
//
// The tile of index r is __umulhi(r, mul).  Power-of-two tiles: mul = 2^(32 - ts),
// i.e. r >> ts.  Counted tiles (round 4, the single-level packed path): any T, with
// mul = floor(2^32 T / m); tile t is then the bits [start(t), start(t + 1)),
// start(t) = ceil(t 2^32 / mul), all within a bit of m / T long -- so T can be a
// whole number of tile-kernel rounds on the chip's 256 CUs (C4: 768 tiles of ~1.25M
// bits, three rounds, instead of 915 of 2^20 bits, 3.57 rounds).  Tile boundaries
// then fall inside filter words: the tile kernel ORs its two boundary words in with
// 64-bit atomics (the bin kernel zeroes them first when the build overwrites).
// Every single-level kernel finds a tile through `mul` (bin kernel, all its tails)
// or tile_start (tile kernel), so any TileCfg -- counted or power-of-two -- is valid
// on any single-level path (round 5: round 4's tails shifted by ts, and a counted
// TileCfg that reached one needed a run-time refusal).  The two-level build and the
// tiled probe construct power-of-two tilings of their own (choose_tiles /
// super_tiles, probe_tiles): their re-bin and probe kernels shift.
struct TileCfg {
    uint32_t ts;     // log2 bits per tile (counted tiles: the in-tile offset bits, 21)
    uint32_t T;      // number of tiles
    uint32_t G;      // cursor/bucket shards per tile
    uint32_t cap;    // capacity (entries) of one (tile, shard) bucket, multiple of 8
    uint32_t fts;    // log2 bits of the tiles the spill flags index: ts, except in
                     // pass 1 of the two-level build (super tiles), where it is the
                     // fine tiles' ts
    uint32_t mul;    // tile of r = __umulhi(r, mul)
    uint32_t fmul;   // spill-flag tile of r = __umulhi(r, fmul) (the fts tiling)
    uint32_t w64;    // LDS words (u64) of one tile in the tile kernel, boundary words incl.
};

// First entry (in units of cap) of the bucket of tile t, shard g: buckets are laid
// out shard-major, [G][T][cap].  Shard g's runs come from the bin blocks with
// blockIdx % G == g, which -- blocks go round-robin over the 8 XCDs -- run on one
// XCD, so each XCD's scattered run writes stay inside its own 1/G of the bucket
// array (round 4: C4 1.46-1.50 -> 1.40-1.42 ms against the tile-major [T][G] layout,
// profiles/r04_ab_gmajor_c4.txt; the tile-major layout was removed in round 5).
__host__ __device__ inline uint32_t bucket_region(const TileCfg &tc, uint32_t t, uint32_t g) {
    return g * tc.T + t;
}

__host__ __device__ inline uint64_t tile_start(uint32_t t, uint32_t mul) {
    return (((uint64_t)t << 32) + mul - 1) / mul;
}
__host__ __device__ inline uint32_t pow2_mul(uint32_t ts) { return 1u << (32 - ts); }

// Bucket unit of pass 1 of the two-level build: five 25-bit in-super-tile offsets
// per 16 bytes (3.2 B per entry instead of a 32-bit index).
struct alignas(16) Pack5 {
    uint32_t x, y, z, w;
};
// entries per bucket unit of an entry type: u64 = three 21-bit offsets, Pack5 = five
// 25-bit ones, else one
template <typename ENTRY>
__host__ __device__ constexpr uint32_t pack_of() {
    return sizeof(ENTRY) == 16 ? 5u : sizeof(ENTRY) == 8 ? 3u : 1u;
}

// placement handles (BinPhase1): A_t << kHandleShift | 4 rank
constexpr uint32_t kHandleShift = 18, kHandleMask = (1u << kHandleShift) - 1;
constexpr int kBinThreads = 1024;
constexpr int kBinThreadsWide = 896;    // 32-byte keys at k = 10: 2 x 896 keys per block
constexpr int kBinThreads16Wide = 768;  // 16-byte keys at k = 7: 3 x 768 keys per block
constexpr int kBinThreads3 = 512;       // 16-byte keys at k = 7, few tiles: 2 x 512, 3 blocks/CU
constexpr int kBinThreads3Wide = 576;   // 32-byte keys at k = 10, few tiles: 2 x 576, 3 blocks/CU
constexpr uint32_t kThreeBlockTiles = 384;
constexpr int kBinKPT = 2;       // keys per thread when k <= 8 (1 for larger k)
constexpr int kTileThreads = 1024;
constexpr int kTileUnroll = 4;   // 16-byte bucket loads in flight per lane
constexpr int kShards = 8;
constexpr uint32_t kStageBytes = 48 * 1024;  // LDS staging window for variable-length keys
constexpr uint32_t kLenClasses = 16;         // word-count classes of the staged keys' order
// the stage is followed by the length permutation: key info [NT] | order [NT] | classes
constexpr uint32_t kInitLens = 72;           // per-length hash start states tabulated (0..71 B)
constexpr size_t stage_lds_bytes(int nt) {
    return kStageBytes + (2 * (size_t)nt + kLenClasses) * 4 + 2 * kInitLens * 8;
}
constexpr uint32_t kMaxTiles = 4096;
constexpr uint32_t kMaxCurTiles = 8192;  // cursor / spill-flag slots (two-level fine tiles)

// Diagnostic builds (tools/ubench_tiled.hip) stop a kernel after a phase to price
// it; in the product this is compiled out.
#ifndef NB_DIAG_STOP
#define NB_DIAG_STOP(phase) false
#endif
#ifndef NB_DIAG_PROLOGUE
#define NB_DIAG_PROLOGUE()
#endif
#ifndef NB_DIAG_WO  // diagnostic write-out variants: 1 = LDS reads only, 2 = no run lookup
#define NB_DIAG_WO 0
#endif
#ifndef NB_TWO_TILE  // diagnostic builds may switch the two-tiles-per-thread tail off
#define NB_TWO_TILE 1
#endif
#ifndef NB_DIAG_NOCOUNT
#define NB_DIAG_NOCOUNT false
#endif
// Cache policy of the bucket round trip (A/B knobs): non-temporal bucket-word
// stores in the bin kernel's write-out (2x slower: runs are partial lines that the
// L2 otherwise merges), non-temporal bucket loads in the tile and re-bin kernels
// (read once; on by default).  Non-temporal key loads in the bin kernel measured
// 0.5-1 % slower (C3/C4/C5) and are not used.
#ifndef NB_WO_UNROLL  // packed write-out: words per lane per step (A/B)
#define NB_WO_UNROLL 2
#endif
#ifndef NB_PLACE_BATCH  // bin placement: a key's run-start reads before its stores (A/B: 0)
#define NB_PLACE_BATCH 1
#endif
#ifndef NB_PACK_HALVES  // packed bucket words built in 32-bit halves (A/B: 0 = 64-bit shifts)
#define NB_PACK_HALVES 1
#endif
#ifndef NB_NT_STORE
#define NB_NT_STORE 0
#endif
#ifndef NB_NT_LOAD
#define NB_NT_LOAD 1  // C4 1.538-1.564 -> 1.527-1.535 ms, C2 0.148 -> 0.144 (same-box A/Bs)
#endif
__device__ __forceinline__ void bucket_store(uint64_t *p, uint64_t v) {
    if (NB_NT_STORE) __builtin_nontemporal_store(v, p);
    else *p = v;
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 bucket_load(const uint4 *p) {
    if (NB_NT_LOAD) {
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    return *p;
}

// Inclusive prefix sum across a wave64 with DPP row shifts and the GFX9 row
// broadcasts (6 VALU ops, no LDS round trips): Hillis-Steele inside each 16-lane
// row, then row 15 -> rows 1,3 and lane 31 -> rows 2,3.  Lanes whose DPP source
// is outside the row (or whose row is masked off) add `old` = 0.
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

// An LDS word by its absolute byte address (the address space 3 pointer as an
// integer): the placement handles below carry absolute addresses, so a placement
// is one shift, one read, one SDWA add and one store.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ lds_u32 &lds_at(uint32_t a) { return *(lds_u32 *)(size_t)a; }
__device__ __forceinline__ uint32_t lds_addr(const uint32_t *p) {
    return (uint32_t)(size_t)(const lds_u32 *)p;
}

// __syncthreads_or without the runtime's helper, whose static LDS (256 B) would
// offset every dynamic-LDS address and cost an add per placement store: `flag` is
// an LDS word zeroed before an earlier barrier.
__device__ __forceinline__ bool block_any(int pred, uint32_t *flag) {
    if (pred) *flag = 1u;
    __syncthreads();
    return *flag != 0u;
}

// A workgroup barrier that waits only for the wave's own LDS operations: its global
// memory operations (e.g. reservation atomics) stay in flight across it.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Exclusive scan of hist[0..T) into S[0..T); returns the total.  blockDim = NT.
template <int NT>
__device__ uint32_t block_exclusive_scan(const uint32_t *hist, uint32_t *S, uint32_t T,
                                         uint32_t *wave_sums) {
    constexpr uint32_t kWaves = NT / 64;
    static_assert(kWaves <= 64, "one wave scans the wave totals");
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t per = (T + NT - 1) / NT;
    const uint32_t b = min(tid * per, T), e = min(b + per, T);
    uint32_t local = 0;
    for (uint32_t t = b; t < e; ++t) local += hist[t];
    const uint32_t incl = wave_inclusive_scan(local);
    if (lane == 63) wave_sums[wid] = incl;
    __syncthreads();
    if (wid == 0) {
        const uint32_t w = lane < kWaves ? wave_sums[lane] : 0;
        const uint32_t wi = wave_inclusive_scan(w);
        if (lane < kWaves) wave_sums[lane] = wi - w;  // exclusive wave offsets
        if (lane == kWaves - 1) wave_sums[kWaves] = wi;  // total
    }
    __syncthreads();
    uint32_t run = wave_sums[wid] + incl - local;
    const uint32_t total = wave_sums[kWaves];
    for (uint32_t t = b; t < e; ++t) {
        S[t] = run;
        run += hist[t];
    }
    // Threads own contiguous runs of tiles here but callers walk tiles strided by
    // NT (and may overwrite hist): the barrier orders the two when T > NT.
    __syncthreads();
    return total;
}

// LDS carve of the bin kernel: cnt | S | G | wave_sums[32] | sort/stage area,
// the last one 16-byte aligned (Guideline 17: misaligned b64/b128 LDS accesses
// replay at 64 cycles per wave-instruction).
__host__ __device__ constexpr uint32_t bin_sort_offset_words(uint32_t T) {
    return (2 * T + 32 + 3) & ~3u;
}

struct TileScratch {
    uint32_t *gcur;       // [G][T] bucket cursors (zero between builds)
    uint32_t *spill_flag; // [T]    (zero between builds)
    uint32_t *spill32;    // [2*ceil(m/64)] spill bitmap (zero between builds)
    uint64_t *zero_words = nullptr;  // counted tiles, overwrite: the filter, whose words
                                     // holding a tile boundary the bin kernel zeroes
    uint32_t *vbctr = nullptr;  // tiled probe: [G] bin-block counters of the grid-stride
                                // bin kernels (zero between launches: the tile kernel
                                // after each bin kernel resets them)
    uint32_t *nlive = nullptr;  // split probe: the survivor count, zeroed by the tile
                                // kernels ahead of the compaction (no memset node)
};

// Phases 2-4 of the bin kernel in rank mode when T <= 2 NT: thread tid owns the
// two tiles 2 tid, 2 tid + 1 from the scan to the run table, so the scan is one
// wave-scan round (no per-thread loops) and the reservations use the counts it
// already holds; waves that own no tile skip the scan arithmetic.  The count
// atomics of phase 1 returned placement handles pk = (4 t) << 18 | 4 rank (see
// the kernel), so the run starts go over the counters themselves -- as byte
// offsets of the sort area from `lds` -- and placement is one LDS read of
// cnt[t] and one add (plus the store).  The run table goes over S: byte offsets
// into the buckets (write-out = one add and one 32-bit-offset store per word)
// while the buckets stay under 4 GiB.
template <int NT, int KPT, int KR, typename ENTRY, int KX = 0>
__device__ __forceinline__ void bin_tail_two_tiles(uint32_t *lds, uint32_t sort_off_words,
                                                   const TileCfg &tc, const TileScratch &sc,
                                                   ENTRY *__restrict__ buckets, uint64_t base,
                                                   uint64_t n, uint32_t k,
                                                   const uint32_t (&ridx)[KPT][KR],
                                                   const uint32_t (&pk)[KPT][KR]) {
    constexpr uint32_t kWaves = NT / 64;
    const uint32_t T = tc.T, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    uint32_t *cnt = lds;                  // [T] packed counters; run starts; limits
    uint32_t *GX = lds + T;               // [T] run table
    uint32_t *wave_sums = lds + 2 * T;    // [kWaves + 1]
    const uint32_t lds0 = lds_addr(lds);
    const uint32_t sort_b = lds0 + sort_off_words * 4;  // absolute LDS byte address
    // packed entries (ENTRY = u64, 3 in-tile offsets per word; Pack5, 5 per 16
    // bytes): every run takes a whole number of units, its 1..PK-1 pad slots hold
    // copies of its first entry
    constexpr uint32_t PK = pack_of<ENTRY>();
    constexpr bool PACK = PK > 1;
    auto slots = [](uint32_t c) { return PACK ? (c + PK - 1) / PK * PK : c; };
    auto count_of = [&](uint32_t t) { return (cnt[t] - ((lds0 + 4 * t) << kHandleShift)) >> 2; };
    // ---- phase 2: scan (one round), reservations
    const uint32_t t0 = 2 * tid;
    const bool scan_wave = wid * 128 < T;  // wave-uniform: the wave owns a tile
    uint32_t h0 = 0, h1 = 0, incl = 0, local = 0;
    if (scan_wave) {
        if (t0 < T) h0 = count_of(t0);
        if (t0 + 1 < T) h1 = count_of(t0 + 1);
        local = slots(h0) + slots(h1);
        incl = wave_inclusive_scan(local);
    }
    if (lane == 63) wave_sums[wid] = incl;
    // reservations on tiles tid and tid + NT: a wave's atomics then hit 64
    // consecutive cursors (4 lines) instead of 128 at stride 2 -- each device-scope
    // atomic line is a memory-side request (WRITE_SIZE measured 57 vs 30 MB/build)
    const uint32_t ta = tid, tb = tid + NT;
    uint32_t ha = 0, hb = 0;
    if (wid * 64 < T) {  // wave-uniform
        if (ta < T) ha = count_of(ta);
        if (tb < T) hb = count_of(tb);
    }
    __syncthreads();
    if (wid == 0) {
        const uint32_t w = lane < kWaves ? wave_sums[lane] : 0;
        const uint32_t wi = wave_inclusive_scan(w);
        if (lane < kWaves) wave_sums[lane] = wi - w;
        if (lane == kWaves - 1) wave_sums[kWaves] = wi;
    }
    const uint32_t shard = blockIdx.x & (tc.G - 1);  // G is a power of two
    uint32_t *cur = sc.gcur + (size_t)shard * T;
    const uint32_t ua = (ha + PK - 1) / PK, ub = (hb + PK - 1) / PK;  // bucket units
    uint32_t ga = 0, gb = 0;
    if (wid * 64 < T) {  // wave-uniform
        if (ua) ga = atomicAdd(&cur[ta], ua);
        if (ub) gb = atomicAdd(&cur[tb], ub);
    }
    __syncthreads();  // wave offsets ready; every count has been read
    const uint32_t total = wave_sums[kWaves];
    if (scan_wave) {
        const uint32_t st0 = wave_sums[wid] + incl - local, st1 = st0 + slots(h0);
        // the run start less the counter's handle base (mod 2^32): a placement handle
        // pk = A_t << 18 | 4 rank plus cnt[t] is the slot's LDS address -- one add
        if (t0 < T) cnt[t0] = sort_b + 4 * st0 - ((lds0 + 4 * t0) << kHandleShift);
        if (t0 + 1 < T) cnt[t0 + 1] = sort_b + 4 * st1 - ((lds0 + 4 * t0 + 4) << kHandleShift);
    }
    __syncthreads();
    if (NB_DIAG_STOP(2)) return;
    // ---- phase 3: placement (the reservations' round trips overlap it).  A key's
    // run-start reads are all issued before its stores: the compiler cannot tell a
    // store into the sort area from a later counter read, so read, store, read,
    // store ... waited out one LDS round trip per index (NB_PLACE_BATCH=0).
    if (NB_PLACE_BATCH == 2) {  // every key's reads before any store
        uint32_t st[KPT][KR];
#pragma unroll
        for (int p = 0; p < KPT; ++p)
#pragma unroll
            for (int j = 0; j < KR; ++j)
                if (KX ? j < KX : j < (int)k)
                    st[p][j] = base + (uint64_t)p * NT + tid < n ? lds_at(pk[p][j] >> kHandleShift) : 0u;
#pragma unroll
        for (int p = 0; p < KPT; ++p)
            if (base + (uint64_t)p * NT + tid < n) {
#pragma unroll
                for (int j = 0; j < KR; ++j)
                    if (KX ? j < KX : j < (int)k) lds_at(st[p][j] + pk[p][j]) = ridx[p][j];
            }
    } else
#pragma unroll
    for (int p = 0; p < KPT; ++p) {
        if (base + (uint64_t)p * NT + tid < n) {
            if (NB_PLACE_BATCH) {
                uint32_t st[KR];
#pragma unroll
                for (int j = 0; j < KR; ++j)
                    if (KX ? j < KX : j < (int)k) st[j] = lds_at(pk[p][j] >> kHandleShift);
#pragma unroll
                for (int j = 0; j < KR; ++j)
                    if (KX ? j < KX : j < (int)k) lds_at(st[j] + pk[p][j]) = ridx[p][j];
            } else {
#pragma unroll
                for (int j = 0; j < KR; ++j)
                    if (KX ? j < KX : j < (int)k) {
                        const uint32_t h = pk[p][j];
                        lds_at(lds_at(h >> kHandleShift) + h) = ridx[p][j];
                    }
            }
        }
    }
    const int ovf = ((uint64_t)ga + ua > tc.cap) | ((uint64_t)gb + ub > tc.cap);
    const bool any_ovf = block_any(ovf, wave_sums + kWaves + 1);
    // run table: first-entry index minus the run's local start (wrapping u32), in
    // bytes when the buckets fit 32-bit offsets; limits over the run starts on
    // overflow.  (packed: st and the table in words; the pad slots are filled here
    // -- the placement is complete, and nothing else touches the sort area until
    // phase 4)
    // (Pack5 units are always addressed by unit index: esz 1)
    const bool b32 = PK < 5 && (uint64_t)T * tc.G * tc.cap * sizeof(ENTRY) <= 0xFFFFFFFFull;
    const uint32_t esz = (b32 && !any_ovf) ? (uint32_t)sizeof(ENTRY) : 1u;
    auto run_entry = [&](uint32_t t, uint32_t g, uint32_t h) {
        uint32_t st = (cnt[t] + ((lds0 + 4 * t) << kHandleShift) - sort_b) / 4;
        if (PACK) {  // 0..PK-1 pad slots (straight-line: the compiler would emit a memset loop)
            uint32_t *run = lds + sort_off_words + st;
            const uint32_t np = slots(h) - h;
            if (np) {
                const uint32_t v0 = run[0];
                run[h] = v0;
                if (np > 1) run[h + 1] = v0;
                if (PK > 3 && np > 2) run[h + 2] = v0;
                if (PK > 3 && np > 3) run[h + 3] = v0;
            }
            st /= PK;
        }
        GX[t] = (bucket_region(tc, t, shard) * tc.cap + g - st) * esz;
        return st;
    };
    uint32_t sa = 0, sbb = 0;
    if (ta < T) sa = run_entry(ta, ga, ha);
    if (tb < T) sbb = run_entry(tb, gb, hb);
    if (any_ovf) {
        __syncthreads();  // every thread has read the run starts before limits go over them
        if (ta < T) cnt[ta] = sa + (ga < tc.cap ? tc.cap - ga : 0u);
        if (tb < T) cnt[tb] = sbb + (gb < tc.cap ? tc.cap - gb : 0u);
    }
    __syncthreads();
    if (NB_DIAG_STOP(3)) return;
    // ---- phase 4: coalesced write-out, four independent entries per lane per step
    const uint32_t *sorted = lds + sort_off_words;
    const uint32_t *S4 = cnt;  // limits (overflow only)
    if constexpr (PK == 5) {
        // unit q of the block = slots 5q..5q+4 (one run, super tile of the first
        // slot): 25-bit fields at bits 0, 25, 50, 75, 100 of the 16 bytes
        const uint32_t units = total / 5, msk = (1u << tc.ts) - 1;
        Pack5 *bu = reinterpret_cast<Pack5 *>(buckets);
        for (uint32_t q = tid; q < units; q += NT) {
            const uint32_t *s5 = sorted + 5 * q;  // stride 5: conflict-free
            const uint32_t a = s5[0], t = __umulhi(a, tc.mul);
            if (!any_ovf || q < S4[t]) {
                const uint32_t f0 = a & msk, f1 = s5[1] & msk, f2 = s5[2] & msk,
                               f3 = s5[3] & msk, f4 = s5[4] & msk;
                Pack5 u;
                u.x = f0 | (f1 << 25);
                u.y = (f1 >> 7) | (f2 << 18);
                u.z = (f2 >> 14) | (f3 << 11);
                u.w = (f3 >> 21) | (f4 << 4);
                bu[(uint32_t)(GX[t] + q)] = u;
            } else {  // past the bucket's capacity: the five entries to the spill bitmap
                for (uint32_t r = 0; r < 5; ++r) {
                    const uint32_t v = s5[r];
                    __hip_atomic_fetch_or(sc.spill32 + (v >> 5), 1u << (v & 31),
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    sc.spill_flag[__umulhi(v, tc.fmul)] = 1u;
                }
            }
        }
        return;
    } else if constexpr (PACK) {
        // word q of the block = slots 3q..3q+2 (one run, tile of the first slot)
        const uint32_t words = total / 3, msk = (1u << tc.ts) - 1, hb = tc.ts - 11;
        // a | b << 21 | c << 42 (21-bit fields, offsets masked to ts bits), built in
        // 32-bit halves: lo = a | b[0,11) << 21 (b << 21 drops b's high bits), hi =
        // b[11,ts) | c << 10 -- 5 VALU instead of the 64-bit shifts' 7-8 (17 <= ts <= 20)
        auto word_at = [&](uint32_t q, uint32_t *t) {
            const uint32_t a = sorted[3 * q], b = sorted[3 * q + 1], c = sorted[3 * q + 2];
            *t = __umulhi(a, tc.mul);
            if (!NB_PACK_HALVES)
                return (uint64_t)(a & msk) | ((uint64_t)(b & msk) << 21) | ((uint64_t)(c & msk) << 42);
            const uint32_t lo = (a & msk) | (b << 21);
            const uint32_t hi = __builtin_amdgcn_ubfe(b, 11, hb) | ((c & msk) << 10);
            return (uint64_t)hi << 32 | lo;
        };
        if (!any_ovf && b32) {
            char *bb = reinterpret_cast<char *>(buckets);
            uint32_t q = tid;
            constexpr int WU = NB_WO_UNROLL;  // words per lane in flight (their LDS reads overlap)
            for (; q + (WU - 1) * NT < words; q += WU * NT) {
                uint32_t t[WU];
                uint64_t w[WU];
#pragma unroll
                for (int u = 0; u < WU; ++u) w[u] = word_at(q + u * NT, &t[u]);
#pragma unroll
                for (int u = 0; u < WU; ++u)
                    bucket_store(reinterpret_cast<uint64_t *>(bb + (GX[t[u]] + (q + u * NT) * 8u)),
                                 w[u]);
            }
            for (; q < words; q += NT) {
                uint32_t t;
                const uint64_t w = word_at(q, &t);
                bucket_store(reinterpret_cast<uint64_t *>(bb + (GX[t] + q * 8u)), w);
            }
        } else {
            uint64_t *bw = reinterpret_cast<uint64_t *>(buckets);
            for (uint32_t q = tid; q < words; q += NT) {
                uint32_t t;
                const uint64_t w = word_at(q, &t);
                if (!any_ovf || q < S4[t]) {
                    bw[(uint32_t)(GX[t] + q)] = w;
                } else {  // past the bucket's capacity: the three entries to the spill bitmap
                    for (uint32_t r = 0; r < 3; ++r) {
                        const uint32_t v = sorted[3 * q + r];
                        __hip_atomic_fetch_or(sc.spill32 + (v >> 5), 1u << (v & 31),
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        sc.spill_flag[__umulhi(v, tc.fmul)] = 1u;
                    }
                }
            }
        }
        return;
    } else {
        if (!any_ovf && b32) {
            char *bb = reinterpret_cast<char *>(buckets);
            uint32_t j = tid;
            for (; j + 3 * NT < total; j += 4 * NT) {
                uint32_t v[4], g[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = sorted[j + u * NT];
#pragma unroll
                for (int u = 0; u < 4; ++u) g[u] = NB_DIAG_WO == 2 ? 0u : GX[__umulhi(v[u], tc.mul)];
                if (NB_DIAG_WO == 1) {  // diagnostic: LDS reads only
                    if ((v[0] ^ v[1] ^ v[2] ^ v[3] ^ g[0] ^ g[1] ^ g[2] ^ g[3]) == 0xFFFFFFFFu) bb[0] = 1;
                    continue;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    *reinterpret_cast<ENTRY *>(bb + (g[u] + (j + u * NT) * (uint32_t)sizeof(ENTRY))) =
                        (ENTRY)v[u];
            }
            for (; j < total; j += NT) {
                const uint32_t v = sorted[j];
                *reinterpret_cast<ENTRY *>(bb + (GX[__umulhi(v, tc.mul)] + j * (uint32_t)sizeof(ENTRY))) = (ENTRY)v;
            }
        } else if (!any_ovf) {  // buckets past 4 GiB: entry indices, 64-bit addresses
            uint32_t j = tid;
            for (; j + 3 * NT < total; j += 4 * NT) {
                uint32_t v[4], g[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = sorted[j + u * NT];
#pragma unroll
                for (int u = 0; u < 4; ++u) g[u] = GX[__umulhi(v[u], tc.mul)];
#pragma unroll
                for (int u = 0; u < 4; ++u) buckets[(uint32_t)(g[u] + j + u * NT)] = (ENTRY)v[u];
            }
            for (; j < total; j += NT) {
                const uint32_t v = sorted[j];
                buckets[(uint32_t)(GX[__umulhi(v, tc.mul)] + j)] = (ENTRY)v;
            }
        } else {
            // overflow: entries past a bucket's capacity go to the spill bitmap
            for (uint32_t j = tid; j < total; j += NT) {
                const uint32_t v = sorted[j], t = __umulhi(v, tc.mul);
                if (j < S4[t]) {
                    buckets[(uint32_t)(GX[t] + j)] = (ENTRY)v;
                } else {
                    __hip_atomic_fetch_or(sc.spill32 + (v >> 5), 1u << (v & 31), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
                    sc.spill_flag[__umulhi(v, tc.fmul)] = 1u;
                }
            }
        }
    }
}

// Phase 1 of the bin kernels (the build's bloom_bin_kernel and the tiled probe's
// probe_bin_kernel): initialise the block's tile counters, hash its KPT * NT keys
// once and count every index per tile with an LDS atomic.  In rank mode (KR > 0,
// k <= KR) the count atomic's return value is the index's placement handle, and
// index + handle stay in registers for the placement; otherwise only the index
// generator's start state (6 registers per key) is kept and the placement
// regenerates the indices.  kid[p]: the key (index in the launch) slot p of this
// lane hashed -- staged variable-length keys are hashed in a permuted order.
// The split tiled probe (round 5) counts a range of each key's indices: J0 is the
// first one counted (the earlier ones only advance the generator; KX, when set, is
// the end), and with GATE a key is counted only while gate[kid] != 0 (its answer
// after the first round); live[p] says whether slot p was counted.  With IDS the
// launch's keys are ids[0, n): the second round over the compacted list of the keys
// the first left at 1 (probe_compact_kernel); keys of a staged layout are then hashed
// straight from HBM (a block's listed keys are not one contiguous byte range).
template <int FLAVOR, int LAYOUT, int KPT, int NT, bool STAGE, int KR, int KX = 0, int J0 = 0,
          bool GATE = false, bool IDS = false>
struct BinPhase1 {
    static constexpr int kR = KR > 0 ? KR : 1;
    static_assert(KR == 0 || (uint64_t)KPT * NT * (KX ? KX - J0 : KR) < (1u << (kHandleShift - 2)),
                  "a block's ranks must fit the placement handle's low bits");
    static_assert(J0 == 0 || KR > 0, "an index range needs the rank registers");
    IndexGen gen[KPT];
    uint32_t ridx[KPT][kR], rank[KPT][kR];
    uint32_t kid[KPT];  // (mod 2^32: the probe launches chunks of < 2^32 keys)
    bool live[KPT];
    const uint8_t *gate = nullptr;
    const uint32_t *ids = nullptr;  // IDS: the keys of the launch

    __device__ __forceinline__ void run(const uint8_t *__restrict__ keys,
                                        const uint64_t *__restrict__ offsets, uint32_t key_len,
                                        uint64_t n, const FilterConsts &c, uint32_t tmul, uint32_t T,
                                        uint32_t *cnt, uint32_t *sorted, uint32_t *any_flag,
                                        uint64_t base) {
        const uint32_t tid = threadIdx.x;
        KeyBatch<FLAVOR, LAYOUT, KPT> kb;
        if (IDS) {
#pragma unroll
            for (int p = 0; p < KPT; ++p) {
                const uint64_t j = base + (uint64_t)p * NT + tid;
                live[p] = j < n;
                kid[p] = live[p] ? ids[(uint32_t)j] : 0u;
                kb.load_one(p, keys, offsets, kid[p], live[p] ? ~0ull : 0ull);
            }
        } else if (!STAGE) {
            kb.load(keys, offsets, base + tid, NT, n);
            // (issued with the key loads: the gate bytes are read before the hash)
#pragma unroll
            for (int p = 0; p < KPT; ++p) {
                const uint64_t i = base + (uint64_t)p * NT + tid;
                live[p] = i < n && (!GATE || gate[(uint32_t)i] != 0);
            }
        } else {
#pragma unroll
            for (int p = 0; p < KPT; ++p) live[p] = false;
        }
        for (uint32_t t = tid; t < T; t += NT) cnt[t] = KR > 0 ? lds_addr(cnt + t) << kHandleShift : 0u;
        if (tid == 0) *any_flag = 0u;  // block_any's flag
        if (STAGE && tid < kLenClasses)  // the staged keys' length-class counters (see below)
            sorted[(kStageBytes / 4) + 2 * NT + tid] = 0u;
        __syncthreads();

        // phase 1: hash each key once; count its k indices per tile.  With KR > 0
        // (k <= KR) the count atomic's return value is the index's rank in its tile's
        // block-local run, and index + rank stay in registers for phase 3; otherwise
        // only the index generator's start state (6 registers per key) is kept and
        // phase 3 regenerates the indices.
        auto count_key = [&](int p, uint64_t h1, uint64_t h2) {
            gen[p].start(h1, h2, c);
            IndexGen g = gen[p];
            if (KR > 0) {
#pragma unroll
                for (int j = 0; j < kR; ++j) {
                    if (KX ? j < KX : j < (int)c.k) {
                        if (j) g.next(c);
                        if (j >= J0) {
                            ridx[p][j] = g.r;
                            rank[p][j] = NB_DIAG_NOCOUNT ? g.r : atomicAdd(&cnt[__umulhi(g.r, tmul)], 4u);
                        }
                    }
                }
            } else {
                for (uint32_t j = 0; j < c.k; ++j) {
                    if (j) g.next(c);
                    atomicAdd(&cnt[__umulhi(g.r, tmul)], 1u);
                }
            }
        };
        if (!STAGE || IDS) {
            // every key of the lane hashed before any count atomic is issued: the
            // compiler otherwise drains key p's LDS atomics (s_waitcnt lgkmcnt(0) at the
            // join of the i < n branch) before it hashes key p + 1
            uint64_t h1[KPT], h2[KPT];
#pragma unroll
            for (int p = 0; p < KPT; ++p) {  // (a lane past n hashes its stale registers --
                // key words in registers only; a pointer layout's dead lane reads nothing)
                if (vec_layout(LAYOUT) || live[p])
                    kb.hash(c, keys, key_len, IDS ? (uint64_t)kid[p] : base + (uint64_t)p * NT + tid, p,
                            &h1[p], &h2[p]);
            }
#pragma unroll
            for (int p = 0; p < KPT; ++p)
                if (live[p]) count_key(p, h1[p], h2[p]);
            if (!IDS)
#pragma unroll
                for (int p = 0; p < KPT; ++p) kid[p] = (uint32_t)(base + (uint64_t)p * NT + tid);
        } else {
            // Variable-length (or odd fixed-length) keys, one sub-batch of NT keys at a
            // time: its keys are one contiguous byte range.  When that fits the stage
            // (the not-yet-used sort array) it is loaded into LDS with coalesced 16-byte
            // loads and every key is hashed from LDS; otherwise (very long keys) the
            // lanes read HBM.
            uint8_t *stage = reinterpret_cast<uint8_t *>(sorted);
            auto koff = [&](uint64_t i) -> uint64_t {
                return LAYOUT == kOffsets ? offsets[i] : i * (uint64_t)key_len;
            };
            // libstdc++ start states per key length (h1: lsx_init, h2: after the seed's
            // whole prefix words), tabulated once per block after the stage's key-info,
            // permutation and class arrays; the first sub-batch's barrier publishes them
            uint64_t *init_tab = reinterpret_cast<uint64_t *>(
                stage + kStageBytes + (2 * (size_t)NT + kLenClasses) * 4);  // [2][kInitLens]
            if (FLAVOR == NB_FLAVOR_LIBSTDCXX && tid < kInitLens) {
                init_tab[tid] = nb::lsx_init(tid);
                init_tab[kInitLens + tid] =
                    LAYOUT == kFixedStride ? c.h2_init_fixed : nb::lsx_h2_start(c, tid);
            }
#pragma unroll
            for (int p = 0; p < KPT; ++p) {
                const uint64_t pb = base + (uint64_t)p * NT;  // first key of the sub-batch
                if (pb >= n) break;                           // block-uniform
                const uint64_t pe = min(pb + NT, n);
                const uint64_t i = pb + tid;
                uint64_t b = 0, e = 0;
                if (i < n) {
                    b = koff(i);
                    e = koff(i + 1);
                }
                // the stage copy starts at the 16-byte-aligned address at or below the
                // sub-batch's first key byte: every vector it loads then holds a byte of
                // the caller's key range (or shares its 16-byte granule), so no load
                // crosses into an unmapped page, however the key buffer is aligned
                const uint64_t kb0 = koff(pb);
                const uint32_t a0 = (uint32_t)((reinterpret_cast<uintptr_t>(keys) + kb0) & 15u);
                const uint64_t span = koff(pe) - kb0 + a0;
                const bool staged = span <= (uint64_t)kStageBytes;  // block-uniform
                // staged variable-length keys are hashed in order of their word count: a
                // wave's lanes then loop over like lengths instead of its longest key
                constexpr bool kPermute = LAYOUT == kOffsets;
                uint32_t *kinfo = reinterpret_cast<uint32_t *>(stage + kStageBytes);  // [NT]
                uint32_t *perm = kinfo + NT;                                         // [NT]
                uint32_t *lhist = perm + NT;                                         // [kLenClasses]
                if (p) __syncthreads();  // the previous sub-batch is hashed: the stage is free
                if (staged) {
                    const uint4 *src = reinterpret_cast<const uint4 *>(keys + kb0 - a0);
                    uint4 *dst = reinterpret_cast<uint4 *>(stage);
                    const uint32_t nvec = (uint32_t)((span + 15) / 16);
                    for (uint32_t q = tid; q < nvec; q += NT) dst[q] = src[q];
                }
                uint32_t klo = (uint32_t)(b - kb0 + a0), klen = (uint32_t)(e - b);
                kid[p] = (uint32_t)i;
                bool kvalid = i < n;
                // counting sort of the sub-batch by word count (absent keys last): whole
                // words for the libstdc++ dword path (its loop runs over whole words, then
                // one tail), all words touched for the byte-wise FNV-1a loop.  The class
                // counts need only the offsets, so they are taken while the stage copy is
                // in flight (lhist is zero here: zeroed before the block's first barrier
                // and again after each permutation is read)
                uint32_t cls = 0, r = 0;
                if (kPermute && staged) {
                    const uint32_t nw = FLAVOR == NB_FLAVOR_LIBSTDCXX ? klen >> 3 : (klen + 7) >> 3;
                    cls = kvalid ? min(nw, kLenClasses - 2) : kLenClasses - 1;
                    kinfo[tid] = klo | (klen << 16);  // both < 2^16 inside the stage
                    r = atomicAdd(&lhist[cls], 1u);
                }
                __syncthreads();
                if (kPermute && staged) {
                    if (tid < 64) {
                        const uint32_t cnt = tid < kLenClasses ? lhist[tid] : 0u;
                        const uint32_t st = wave_inclusive_scan(cnt) - cnt;
                        if (tid < kLenClasses) lhist[tid] = st;
                    }
                    __syncthreads();
                    perm[lhist[cls] + r] = tid;
                    __syncthreads();
                    const uint32_t src = perm[tid];  // a key of this sub-batch; valid ones first
                    const uint32_t info = kinfo[src];
                    klo = info & 0xffffu;
                    klen = info >> 16;
                    kvalid = pb + src < n;  // == (i < n): the valid keys fill the first slots
                    kid[p] = (uint32_t)(pb + src);
                    if (tid < kLenClasses) lhist[tid] = 0u;  // read by all before the barrier above
                }
                if (GATE && kvalid) kvalid = gate[kid[p]] != 0;
                live[p] = kvalid;
                if (kvalid) {
                    uint64_t h1, h2;
                    const uint32_t len = klen;
                    if (staged && FLAVOR == NB_FLAVOR_LIBSTDCXX) {
                        // dword stream from LDS (bloom_math.h lsx_hash_dwords); its reads run
                        // <= 12 bytes past the key, inside the stage's allocation
                        const uint32_t *dw = reinterpret_cast<const uint32_t *>(stage) + (klo >> 2);
                        auto D = [dw](uint32_t j) { return dw[j]; };
                        const uint32_t sh = 8 * (klo & 3u);
                        uint64_t h0, g0;
                        if (len < kInitLens) {
                            h0 = init_tab[len];
                            g0 = init_tab[kInitLens + len];
                        } else {
                            h0 = nb::lsx_init(len);
                            g0 = LAYOUT == kFixedStride ? c.h2_init_fixed : nb::lsx_h2_start(c, len);
                        }
                        if (c.prem == 0) nb::lsx_hash_dwords<0>(c, D, sh, len, h0, g0, &h1, &h2);
                        else if (c.prem <= 4) nb::lsx_hash_dwords<1>(c, D, sh, len, h0, g0, &h1, &h2);
                        else nb::lsx_hash_dwords<2>(c, D, sh, len, h0, g0, &h1, &h2);
                    } else if (staged) {
                        const uint32_t lo = klo, a = lo & 7u;
                        const uint64_t *q = reinterpret_cast<const uint64_t *>(stage + (lo - a));
                        auto load = [q](uint32_t j) { return q[j]; };
                        nb::hash_aligned_words<FLAVOR, decltype(load), LAYOUT == kFixedStride>(
                            c, load, a, len, &h1, &h2);
                    } else {
                        key_hashes_ptr<FLAVOR, LAYOUT == kFixedStride>(c, keys + b, len, &h1, &h2);
                    }
                    count_key(p, h1, h2);
                }
            }
        }
        __syncthreads();
    }
};

// Two resident blocks per CU (8 waves per SIMD at NT = 1024): <= 64 VGPRs.
#ifndef NB_BIN_MIN_WAVES
#define NB_BIN_MIN_WAVES(NT) (2 * (NT) / 256)
#endif
template <int FLAVOR, int LAYOUT, int KPT, typename ENTRY, int NT = kBinThreads,
          bool STAGE = !vec_layout(LAYOUT), int KR = 0, int KX = 0>
__global__ __launch_bounds__(NT, NB_BIN_MIN_WAVES(NT)) void bloom_bin_kernel(
    const uint8_t *__restrict__ keys, const uint64_t *__restrict__ offsets, uint32_t key_len,
    uint64_t n, FilterConsts c, TileCfg tc, TileScratch sc, ENTRY *__restrict__ buckets) {
    extern __shared__ uint32_t lds[];
    const uint32_t T = tc.T;
    uint32_t *cnt = lds;               // [T] per-tile counts (then placement cursors)
    uint32_t *S = cnt + T;             // [T] block-local run starts
    uint2 *GL = reinterpret_cast<uint2 *>(lds);  // [T] over cnt|S once both are dead:
                                       // {global entry index of the run - S[t], limit}
    uint32_t *wave_sums = S + T;       // [NT/64 + 1]
    uint32_t *sorted = lds + bin_sort_offset_words(T);  // [KPB * k], 16-byte aligned
    const uint32_t tid = threadIdx.x;
    NB_DIAG_PROLOGUE();
    if (sc.zero_words && tid == 0)  // counted tiles, overwrite: see TileCfg
        for (uint32_t t = blockIdx.x + 1; t < T; t += gridDim.x) {
            const uint64_t b = tile_start(t, tc.mul);
            if (b & 63) sc.zero_words[b >> 6] = 0;
        }
    // rank mode (KR > 0): cnt[t] starts at A_t << 18, A_t = the LDS byte address of
    // cnt[t] (< 2^14: the counters lead the LDS, T <= 4 096), and each index adds 4,
    // so the count atomic returns its index's placement handle pk = A_t << 18 |
    // 4 rank: where the run start will be (the scan writes it over cnt[t], as an
    // absolute address) and the index's byte offset within the run.  A block has
    // fewer than 2^16 indices (static_assert in BinPhase1), so 4 rank stays in the
    // low 18 bits and the decode (cnt[t] - (A_t << 18)) >> 2 is exact.
    // register-loaded keys: their loads are issued first, in flight across the LDS
    // initialisation and its barrier
    const uint64_t base = (uint64_t)blockIdx.x * (KPT * NT);
    constexpr int kR = KR > 0 ? KR : 1;
    BinPhase1<FLAVOR, LAYOUT, KPT, NT, STAGE, KR, KX> ph;
    ph.run(keys, offsets, key_len, n, c, tc.mul, T, cnt, sorted, wave_sums + NT / 64 + 1, base);
    IndexGen (&gen)[KPT] = ph.gen;
    const uint32_t (&ridx)[KPT][kR] = ph.ridx;
    const uint32_t (&rank)[KPT][kR] = ph.rank;
    if (NB_DIAG_STOP(1)) return;
    if constexpr (pack_of<ENTRY>() > 1) {  // packed entries (host-checked T <= 2 NT, KR > 0)
        bin_tail_two_tiles<NT, KPT, kR, ENTRY, KX>(lds, bin_sort_offset_words(T), tc, sc, buckets, base, n,
                                        c.k, ridx, rank);
    } else {
        if (NB_TWO_TILE && KR > 0 && T <= 2 * NT) {  // block-uniform: the common case (C2)
            bin_tail_two_tiles<NT, KPT, kR, ENTRY, KX>(lds, bin_sort_offset_words(T), tc, sc, buckets, base,
                                            n, c.k, ridx, rank);
            return;
        }

        // phase 2: block-local run starts; reserve a run in every touched tile's
        // bucket shard (cursor shard = blockIdx % G, laid out [shard][tile]).  Per tile
        // the write-out needs only two words afterwards: G[t] := global entry index of
        // the block's run minus S[t] (u32 wrap-around arithmetic), S[t] := first local
        // position past the bucket's capacity.
        if (KR > 0) {  // packed counters (see phase 1) back to counts
            for (uint32_t t = tid; t < T; t += NT) cnt[t] = (cnt[t] - (lds_addr(cnt + t) << kHandleShift)) >> 2;
            __syncthreads();
        }
        const uint32_t total = block_exclusive_scan<NT>(cnt, S, T, wave_sums);
        const uint32_t shard = blockIdx.x & (tc.G - 1);
        uint32_t *cur = sc.gcur + (size_t)shard * T;
        // tiles owned by this thread in phase 2: t = tid + u*NT
        constexpr int kTPT = (kMaxTiles + NT - 1) / NT;
        uint32_t gres[kTPT], hcnt[kTPT], gl_g[kTPT], gl_l[kTPT];
#pragma unroll
        for (int u = 0; u < kTPT; ++u) {
            const uint32_t t = tid + u * NT;
            hcnt[u] = t < T ? cnt[t] : 0u;
            gres[u] = hcnt[u] ? atomicAdd(&cur[t], hcnt[u]) : 0u;
        }
        if (NB_DIAG_STOP(2)) return;
        // The {G, limit} pair of a tile: G = global entry index of the block's run
        // minus its local start (u32 wrap-around), limit = first local position past
        // the bucket's capacity.  `ovf` notes a run that does not fit its bucket.
        int ovf = 0;
        auto run_pair = [&](int u, uint32_t t) {
            const uint32_t st = S[t], g = gres[u];
            gl_g[u] = bucket_region(tc, t, shard) * tc.cap + g - st;
            gl_l[u] = st + (g < tc.cap ? tc.cap - g : 0u);
            ovf |= (uint64_t)g + hcnt[u] > tc.cap;
        };
        if (KR > 0) {
            // phase 3, rank mode: each index goes to its tile's run start + rank; the
            // reservations' round trips overlap this LDS placement
#pragma unroll
            for (int p = 0; p < KPT; ++p) {
                const uint64_t i = base + (uint64_t)p * NT + tid;
                if (i < n) {
#pragma unroll
                    for (int j = 0; j < kR; ++j)
                        if (KX ? j < KX : j < (int)c.k)
                            sorted[S[__umulhi(ridx[p][j], tc.mul)] + ((rank[p][j] & kHandleMask) >> 2)] = ridx[p][j];
                }
            }
#pragma unroll
            for (int u = 0; u < kTPT; ++u) {
                const uint32_t t = tid + u * NT;
                if (t < T) run_pair(u, t);
            }
        } else {
            // phase 3, k > 16: regenerate the indices and counting-sort them with
            // cursor atomics (all k of a key issued before their results are consumed)
#pragma unroll
            for (int u = 0; u < kTPT; ++u) {
                const uint32_t t = tid + u * NT;
                if (t < T) {
                    run_pair(u, t);
                    cnt[t] = S[t];  // placement cursor
                }
            }
            __syncthreads();
#pragma unroll
            for (int p = 0; p < KPT; ++p) {
                const uint64_t i = base + (uint64_t)p * NT + tid;
                if (i < n) {
                    IndexGen g = gen[p];
                    uint32_t j = 0;
                    for (; j + 4 <= c.k; j += 4) {
                        uint32_t r[4], q[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            if (j + u) g.next(c);
                            r[u] = g.r;
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u) q[u] = atomicAdd(&cnt[__umulhi(r[u], tc.mul)], 1u);
#pragma unroll
                        for (int u = 0; u < 4; ++u) sorted[q[u]] = r[u];
                    }
                    for (; j < c.k; ++j) {
                        if (j) g.next(c);
                        sorted[atomicAdd(&cnt[__umulhi(g.r, tc.mul)], 1u)] = g.r;
                    }
                }
            }
        }
        // cnt and S are dead: the run table goes over them.  Every run fits its bucket
        // unless the input is pathological (massively duplicated keys): then the
        // table holds {G, limit} pairs and the write-out checks each entry.
        const bool any_ovf = block_any(ovf, wave_sums + NT / 64 + 1);  // block-uniform
        uint32_t *GX = lds;  // [T] G only, when nothing overflows
#pragma unroll
        for (int u = 0; u < kTPT; ++u) {
            const uint32_t t = tid + u * NT;
            if (t < T) {
                if (any_ovf) GL[t] = make_uint2(gl_g[u], gl_l[u]);
                else GX[t] = gl_g[u];
            }
        }
        __syncthreads();
        if (NB_DIAG_STOP(3)) return;

        // phase 4: coalesced write-out of the runs, four independent entries per
        // lane per step so the LDS lookups overlap.  Entries are stored unmasked (a
        // u16 store keeps the low bits; the tile kernel masks).
        if (!any_ovf) {
            uint32_t j = tid;
            for (; j + 3 * NT < total; j += 4 * NT) {
                uint32_t v[4], g[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = sorted[j + u * NT];
#pragma unroll
                for (int u = 0; u < 4; ++u) g[u] = GX[__umulhi(v[u], tc.mul)];
#pragma unroll
                for (int u = 0; u < 4; ++u) buckets[g[u] + j + u * NT] = (ENTRY)v[u];
            }
            for (; j < total; j += NT) {
                const uint32_t v = sorted[j];
                buckets[GX[__umulhi(v, tc.mul)] + j] = (ENTRY)v;
            }
            return;
        }
        // slow path: entries past a bucket's capacity go to the spill bitmap
        auto emit = [&](uint32_t j, uint32_t v, uint2 gl) {
            if (j < gl.y) {
                buckets[gl.x + j] = (ENTRY)v;
            } else {
                __hip_atomic_fetch_or(sc.spill32 + (v >> 5), 1u << (v & 31), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
                sc.spill_flag[__umulhi(v, tc.fmul)] = 1u;
            }
        };
        uint32_t j = tid;
        for (; j + 3 * NT < total; j += 4 * NT) {
            uint32_t v[4];
            uint2 gl[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = sorted[j + u * NT];
#pragma unroll
            for (int u = 0; u < 4; ++u) gl[u] = GL[__umulhi(v[u], tc.mul)];
#pragma unroll
            for (int u = 0; u < 4; ++u) emit(j + u * NT, v[u], gl[u]);
        }
        for (; j < total; j += NT) {
            const uint32_t v = sorted[j];
            emit(j, v, GL[__umulhi(v, tc.mul)]);
        }
    }
}

// Two-level build for very large filters (T > 2 NT fine tiles, e.g. C5's 4 096
// tiles of 2^20 bits): binned straight into fine tiles, a block's 1 024 keys x k
// indices spread over T tiles make runs of ~2.5 entries -- every run a separate
// reservation atomic and L2 write request.  Pass 1 (the bin kernel on super tiles
// of 2^(ts+5) bits, entries packed five 25-bit in-super-tile offsets per 16 bytes
// (Pack5); or, with NB_PACK5=0 / k > 16, 2^(ts+6)-bit super tiles and full 32-bit
// indices) makes runs of ~k x 1 024 / T1; pass 2 (this kernel) re-bins each super
// tile's entries into its 32 (64) fine tiles by an LDS counting sort over ~16k
// entries per block (runs of ~500 (256)); pass 3 is the tile kernel on the fine
// tiles.  One extra read + write of the entries buys runs two orders of magnitude
// longer.  grid = (blocks per super tile, super tiles).
constexpr uint32_t kSuperFine = 64;  // fine tiles per super tile (at most)
constexpr uint32_t kMaxSuper = 128;  // super tiles (m < 2^32 with 2^25-bit super tiles)
constexpr int kRebinThreads = 1024;
// entries per thread: 16 32-bit entries, or three Pack5 units (15 entries)
template <bool IN5>
__host__ __device__ constexpr uint32_t rebin_ept() { return IN5 ? 15u : 16u; }
template <bool IN5>
__host__ __device__ constexpr uint32_t rebin_span() { return kRebinThreads * rebin_ept<IN5>(); }

// PACK: fine entries three per 64-bit word (runs padded to a multiple of 3 slots
// with copies of their first entry, as in bin_tail_two_tiles); capacities,
// cursors and the run table in words.  IN5: pass-1 buckets of Pack5 units
// (cursors, capacities in units; their pad slots are copies of real entries,
// re-binned like any other).
template <bool PACK, bool IN5>
__global__ __launch_bounds__(kRebinThreads) void bloom_rebin_kernel(
    TileCfg t1, TileCfg t2, TileScratch sc1, TileScratch sc2, const void *__restrict__ b1v,
    void *__restrict__ b2v) {
    constexpr uint32_t EPT = rebin_ept<IN5>(), UPT = IN5 ? EPT / 5 : EPT;  // units per thread
    constexpr uint32_t kSpanUnits = kRebinThreads * UPT;
    __shared__ uint32_t v0[kShards + 1];
    __shared__ uint32_t fcnt[kSuperFine], fS[kSuperFine], fGX[kSuperFine], flim[kSuperFine];
    __shared__ uint32_t slot_total;
    __shared__ int any_ovf;
    uint32_t *b2 = reinterpret_cast<uint32_t *>(b2v);
    extern __shared__ uint32_t sorted[];  // [rebin_span + pads]
    const uint32_t tid = threadIdx.x, s = blockIdx.y;
    const uint32_t nfine = 1u << (t1.ts - t2.ts);  // fine tiles per super tile (<= 64)
    if (tid == 0) {
        uint32_t acc = 0;
        for (uint32_t g = 0; g < t1.G; ++g) {
            v0[g] = acc;
            acc += min(sc1.gcur[(size_t)g * t1.T + s], t1.cap);
        }
        v0[t1.G] = acc;
        any_ovf = 0;
    }
    if (tid < kSuperFine) fcnt[tid] = 0;
    __syncthreads();
    const uint32_t total = v0[t1.G];  // units
    const uint32_t first = blockIdx.x * kSpanUnits;
    if (first >= total) return;  // block-uniform
    const uint32_t cntu = min(kSpanUnits, total - first);
    const uint32_t fbase = s * nfine;  // first fine tile of super tile s
    // load this block's entries (the G shards as one flat range), count per fine tile.
    // All UPT loads are issued before any is consumed: a lane past the block's
    // range reloads its last unit (clamped index, never used), so the loads are
    // unconditional -- under a per-unit `if` the compiler waited for each load
    // inside its branch, three exposed HBM latencies per lane.
    uint32_t v[EPT], r[EPT];
    uint4 p[IN5 ? UPT : 1];
    uint32_t g = 0;
#pragma unroll
    for (uint32_t u = 0; u < UPT; ++u) {
        const uint32_t q = min(first + tid + u * kRebinThreads, first + cntu - 1);
        while (g + 1 < t1.G && q >= v0[g + 1]) ++g;
        const size_t at = (size_t)bucket_region(t1, s, g) * t1.cap + (q - v0[g]);
        if constexpr (IN5) p[u] = bucket_load(reinterpret_cast<const uint4 *>(b1v) + at);
        else v[u] = reinterpret_cast<const uint32_t *>(b1v)[at];
    }
    if constexpr (IN5) {
        const uint32_t msk = (1u << 25) - 1, sb = s << t1.ts;
#pragma unroll
        for (uint32_t u = 0; u < UPT; ++u) {
            v[5 * u + 0] = sb | (p[u].x & msk);
            v[5 * u + 1] = sb | (((p[u].x >> 25) | (p[u].y << 7)) & msk);
            v[5 * u + 2] = sb | (((p[u].y >> 18) | (p[u].z << 14)) & msk);
            v[5 * u + 3] = sb | (((p[u].z >> 11) | (p[u].w << 21)) & msk);
            v[5 * u + 4] = sb | (p[u].w >> 4);
        }
    }
    // entry e of the thread is valid while its unit is
    auto valid = [&](uint32_t e) { return tid + (IN5 ? e / 5 : e) * kRebinThreads < cntu; };
#pragma unroll
    for (uint32_t e = 0; e < EPT; ++e)
        if (valid(e)) r[e] = atomicAdd(&fcnt[(v[e] >> t2.ts) - fbase], 1u);
    __syncthreads();
    // wave 0: scan the fine tiles' counts and reserve their runs.  The reservation
    // atomics stay in flight through the placement (an LDS-only barrier publishes
    // the run starts); the run table is written after it.
    uint32_t gr = 0, fu = 0, fstu = 0, fshard = 0;
    if (tid < kSuperFine) {
        const uint32_t c = tid < nfine ? fcnt[tid] : 0u;
        const uint32_t sl = PACK ? (c + 2) / 3 * 3 : c;
        fu = PACK ? sl / 3 : c;
        const uint32_t incl = wave_inclusive_scan(sl), st = incl - sl;
        if (tid == kSuperFine - 1) slot_total = incl;
        fshard = (blockIdx.y * gridDim.x + blockIdx.x) & (t2.G - 1);
        gr = fu ? atomicAdd(&sc2.gcur[(size_t)fshard * t2.T + fbase + tid], fu) : 0u;
        fstu = PACK ? st / 3 : st;
        fS[tid] = st;
    }
    lds_barrier();
    // placement; the entry of rank 0 in its fine tile also fills the run's pad
    // slots (PACK: up to a multiple of 3) with copies of itself
#pragma unroll
    for (uint32_t e = 0; e < EPT; ++e) {
        if (valid(e)) {
            const uint32_t f = (v[e] >> t2.ts) - fbase, st = fS[f];
            sorted[st + r[e]] = v[e];
            if (PACK && r[e] == 0) {
                const uint32_t c = fcnt[f];
                for (uint32_t q = c; q < (c + 2) / 3 * 3; ++q) sorted[st + q] = v[e];
            }
        }
    }
    if (tid < kSuperFine) {
        const uint32_t t = fbase + tid;
        fGX[tid] = bucket_region(t2, t, fshard) * t2.cap + gr - fstu;
        flim[tid] = fstu + (gr < t2.cap ? t2.cap - gr : 0u);
        if ((uint64_t)gr + fu > t2.cap) any_ovf = 1;
    }
    __syncthreads();
    const bool ovf = any_ovf != 0;
    if constexpr (PACK) {
        uint64_t *bw = reinterpret_cast<uint64_t *>(b2v);
        const uint32_t words = slot_total / 3, msk = (1u << t2.ts) - 1;
        for (uint32_t q = tid; q < words; q += kRebinThreads) {
            const uint32_t a = sorted[3 * q], b = sorted[3 * q + 1], c = sorted[3 * q + 2];
            const uint32_t f = (a >> t2.ts) - fbase;
            if (!ovf || q < flim[f]) {  // a | b << 21 | c << 42 in 32-bit halves (as in bin_tail_two_tiles)
                const uint32_t lo = (a & msk) | (b << 21);
                const uint32_t hi = __builtin_amdgcn_ubfe(b, 11, t2.ts - 11) | ((c & msk) << 10);
                bw[fGX[f] + q] = (uint64_t)hi << 32 | lo;
            } else {
                for (uint32_t rr = 0; rr < 3; ++rr) {
                    const uint32_t x = sorted[3 * q + rr];
                    __hip_atomic_fetch_or(sc2.spill32 + (x >> 5), 1u << (x & 31), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
                    sc2.spill_flag[x >> t2.ts] = 1u;
                }
            }
        }
        return;
    }
    for (uint32_t j = tid; j < slot_total; j += kRebinThreads) {
        const uint32_t x = sorted[j], f = (x >> t2.ts) - fbase;
        if (!ovf || j < flim[f]) {
            b2[fGX[f] + j] = x;
        } else {  // past the fine bucket's capacity: the spill bitmap
            __hip_atomic_fetch_or(sc2.spill32 + (x >> 5), 1u << (x & 31), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
            sc2.spill_flag[x >> t2.ts] = 1u;
        }
    }
}

template <typename ENTRY, bool OVERWRITE, int NT = kTileThreads, int UNROLL = kTileUnroll>
__global__ __launch_bounds__(NT) void bloom_tile_or_kernel(
    TileCfg tc, TileScratch sc, const ENTRY *__restrict__ buckets, uint64_t *__restrict__ words,
    uint64_t nwords) {
    extern __shared__ uint32_t tile[];  // [2 w64] tile words, then 2*kShards+1 words
    constexpr uint32_t kPerVec = 16 / sizeof(ENTRY);  // entries per 16-byte load
    const uint32_t t = blockIdx.x, tid = threadIdx.x;
    // the tile's bits [b0, b1) (power-of-two tiles: [t << ts, (t + 1) << ts)), held in
    // LDS from the filter word holding b0 on: LDS bit i is filter bit a0 + i
    const uint64_t b0 = tile_start(t, tc.mul), b1 = tile_start(t + 1, tc.mul);
    const uint64_t w0 = b0 >> 6, we = min((b1 + 63) >> 6, nwords);  // filter words [w0, we)
    const uint32_t nw64 = (uint32_t)(we - w0), a0 = (uint32_t)(w0 << 6);
    // an entry holds the low ts bits of its index: its LDS bit is (entry - a0) mod 2^ts
    // (power-of-two tiles: a0's low ts bits are zero)
    const uint32_t mask = (1u << tc.ts) - 1, abase = a0 & mask;
    uint32_t *shard_cnt = tile + 2 * tc.w64;    // [kShards]
    uint32_t *shard_v0 = shard_cnt + kShards;   // [kShards + 1] first flat vector of each shard
    for (uint32_t w = tid; w < 2 * nw64; w += NT) tile[w] = 0;
    if (tid < tc.G) {
        uint32_t *cp = sc.gcur + (size_t)tid * tc.T + t;
        shard_cnt[tid] = min(coherent_load(cp), tc.cap);  // (written by another kernel's atomics)
        *cp = 0;  // workspace invariant: cursors are zero between builds
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t v0 = 0;
        for (uint32_t g = 0; g < tc.G; ++g) {
            shard_v0[g] = v0;
            v0 += shard_cnt[g] / kPerVec;
        }
        shard_v0[tc.G] = v0;
    }
    __syncthreads();
    auto orv = [&](uint32_t v) {
        v = (v - abase) & mask;
        atomicOr(&tile[v >> 5], 1u << (v & 31));
    };
    auto or_vec = [&](const uint4 &q) {
        if (sizeof(ENTRY) == 2) {
            orv(q.x & 0xffff); orv(q.x >> 16); orv(q.y & 0xffff); orv(q.y >> 16);
            orv(q.z & 0xffff); orv(q.z >> 16); orv(q.w & 0xffff); orv(q.w >> 16);
        } else if (sizeof(ENTRY) == 8) {  // two words of three 21-bit offsets
            orv(q.x); orv((q.x >> 21) | (q.y << 11)); orv(q.y >> 10);
            orv(q.z); orv((q.z >> 21) | (q.w << 11)); orv(q.w >> 10);
        } else {
            orv(q.x); orv(q.y); orv(q.z); orv(q.w);
        }
    };
    // the G shards as one flat range of 16-byte vectors
    const uint32_t nvec = shard_v0[tc.G];
    // a lane's vector indices only grow, so its shard index is advanced, never searched
    uint32_t g = 0;
    auto vec_at = [&](uint32_t v) {
        while (g + 1 < tc.G && v >= shard_v0[g + 1]) ++g;
        const uint4 *ev = reinterpret_cast<const uint4 *>(buckets + (size_t)bucket_region(tc, t, g) * tc.cap);
        return bucket_load(ev + (v - shard_v0[g]));
    };
    uint32_t q = tid;
    for (; q + (UNROLL - 1) * NT < nvec; q += UNROLL * NT) {
        uint4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = vec_at(q + u * NT);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) or_vec(v[u]);
    }
    for (; q < nvec; q += NT) or_vec(vec_at(q));
    if (tid < tc.G) {  // each shard's tail (< kPerVec entries)
        const uint32_t cnt = shard_cnt[tid];
        const ENTRY *e = buckets + (size_t)bucket_region(tc, t, tid) * tc.cap;
        for (uint32_t r = cnt / kPerVec * kPerVec; r < cnt; ++r) {
            const uint64_t x = (uint64_t)e[r];
            orv((uint32_t)x);
            if (sizeof(ENTRY) == 8) {
                orv((uint32_t)(x >> 21));
                orv((uint32_t)(x >> 42));
            }
        }
    }
    if (sc.spill_flag[t]) {  // fold in (and clear) this tile's spilled bits
        __syncthreads();
        uint32_t *sp = sc.spill32 + 2 * w0;
        for (uint32_t w = tid; w < 2 * nw64; w += NT) {
            uint32_t v = sp[w];
            // only the bits of [b0, b1): a boundary word's others are the neighbour's
            const uint64_t bit0 = (uint64_t)a0 + 32 * w;
            const uint64_t lo = max(b0, bit0), hi = min(b1, bit0 + 32);
            v = lo < hi ? v & (uint32_t)((((hi - bit0) == 32 ? 0x100000000ull : 1ull << (hi - bit0)) - 1) &
                                         ~((1ull << (lo - bit0)) - 1))
                        : 0u;
            if (v) {
                atomicOr(&tile[w], v);
                atomicAnd(&sp[w], ~v);
            }
        }
        if (tid == 0) sc.spill_flag[t] = 0;
    }
    __syncthreads();
    // a word holding a tile boundary (counted tiles only) is shared with the
    // neighbour tile's block: ORed in atomically (zeroed by the bin kernel when the
    // build overwrites); every other word is this block's alone
    const bool lo_shared = (b0 & 63) != 0, hi_shared = t + 1 < tc.T && (b1 & 63) != 0;
    const uint64_t *tile64 = reinterpret_cast<const uint64_t *>(tile);
    for (uint32_t w = tid; w < nw64; w += NT) {
        const uint64_t gw = w0 + w, v = tile64[w];
        if ((w == 0 && lo_shared) || (w == nw64 - 1 && hi_shared)) {
            if (v) __hip_atomic_fetch_or(words + gw, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (OVERWRITE) {
            words[gw] = v;
        } else if (v) {
            words[gw] |= v;
        }
    }
}

// ------------------------------------------------------------ tiled probe ----
// The batch form of possiblyContains (BloomFilter.cpp:67-80) for large, mostly
// present batches.  One lane per key gathers k random words of the filter (~56 G
// gathers/s chip-wide for a 114 MiB filter: 12.5 ms for C4's 100M present keys);
// binned like the build, the same lookups become streaming traffic:
//   probe_bin_kernel : phase 1 of the build's bin kernel (hash, count per tile),
//                      then every index is written to its tile's bucket as a 64-bit
//                      entry (key << 32 | in-tile offset) -- no packing, no pads;
//                      each key's answer starts at 1;
//   probe_tile_kernel: one block per tile: the tile's filter words into LDS, then
//                      every entry tests its bit there; a zero bit stores 0 into the
//                      key's answer byte (plain byte stores: every writer writes the
//                      same value).
// Present keys cost no stores at all; an absent key costs one store per zero bit
// (~k/2), which is why absent-heavy batches keep the lane path (ProbeGate).
constexpr int kProbeThreads = 1024;

__host__ __device__ constexpr uint32_t probe_sort_offset_words(uint32_t T) {
    return (4 * T + 32 + 3) & ~3u;  // cnt | S | GX | L | wave_sums, 16-byte aligned
}

// The E32 probe bin kernel's phases 2-4 (see probe_bin_kernel): cnt[t] already holds
// each touched tile's run length including its header slot.  Scan, one reservation
// per run, the run's header slot (by the thread reserving it) and every index placed
// behind it as its 32-bit entry.  In LDS a header slot holds 0x80000000 | t: the
// write-out (each wave one contiguous range of slots, 64 at a time) finds a slot's
// tile as a wave-wide running maximum (the tiles ascend along the slots), so the sort
// area is 4 B per slot -- two blocks of 2 048 keys fit a CU -- and stores the bin
// block's header word 0x80000000 | vb in its place.  An entry past its bucket's capacity
// (duplicated keys only) is tested right here.
__device__ __forceinline__ uint32_t wave_inclusive_max(uint32_t v);
template <int NT, int PKPT, int KR, int J0, int J1, bool IDS, class PH>
__device__ __forceinline__ void probe_bin_tail_e32(uint32_t vb, const PH &ph, const TileCfg &tc, const TileScratch &sc,
                                                   uint32_t *cnt, uint32_t *S, uint32_t *GX, uint32_t *L,
                                                   uint32_t *wave_sums, uint32_t *sword,
                                                   uint32_t *__restrict__ buckets,
                                                   const uint64_t *__restrict__ words,
                                                   uint8_t *__restrict__ out,
                                                   const uint32_t *__restrict__ ids, uint64_t base,
                                                   uint32_t k) {
    const uint32_t T = tc.T, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t total = block_exclusive_scan<NT>(cnt, S, T, wave_sums);
    const uint32_t shard = vb & (tc.G - 1);
    uint32_t *cur = sc.gcur + (size_t)shard * T;
    uint2 *GXL = reinterpret_cast<uint2 *>(GX);  // [T] {run table, capacity limit} (GX | L, 2T words)
    for (uint32_t t = tid; t < T; t += NT) {
        const uint32_t h = cnt[t], g = h ? atomicAdd(&cur[t], h) : 0u;
        GXL[t] = make_uint2(bucket_region(tc, t, shard) * tc.cap + g - S[t],
                            S[t] + (g < tc.cap ? tc.cap - g : 0u));
        if (h) sword[S[t]] = 0x80000000u | t;
    }
    (void)L;
    // placement behind the header slot (the reservations' round trips overlap it)
    const uint32_t msk = (1u << tc.ts) - 1, b32 = (uint32_t)base;
#pragma unroll
    for (int p = 0; p < PKPT; ++p) {
        if (ph.live[p]) {
            // the key's position in the block (staged keys: kid is base + its slot)
            const uint32_t kib = IDS ? (uint32_t)(p * NT) + tid : ph.kid[p] - b32;
#pragma unroll
            for (int j = J0; j < KR; ++j)
                if (J1 ? j < J1 : j < (int)k) {
                    const uint32_t r = ph.ridx[p][j], t = r >> tc.ts;
                    sword[S[t] + 1 + ((ph.rank[p][j] & kHandleMask) >> 2)] = (kib << tc.ts) | (r & msk);
                }
        }
    }
    __syncthreads();
    // write-out: each wave one contiguous range of slots, 64 at a time (one slot per
    // lane: a store instruction covers ~7 runs.  Four slots per lane -- one 16-byte LDS
    // read and one tile scan per 256 slots -- measured slower, 0.87 -> 1.02 ms per 50M
    // keys: each store instruction then spans ~28 runs, profiles/r06r_probe_trace.txt).
    // The tiles ascend along the slots and a header slot holds 0x80000000 | t, above
    // every entry word, so the header in force at a slot is the running maximum of the
    // raw words: one DPP max per step (a select-based "last header" scan cost 4 VALU a
    // step, and the loop ~45 VALU per 64 slots).
    constexpr uint32_t kW = NT / 64;
    const uint32_t per = (total + kW - 1) / kW;
    const uint32_t s0 = min(wid * per, total), s1 = min(s0 + per, total);
    if (s0 >= s1) return;  // wave-uniform; no barrier follows
    // the header in force at s0 (slot 0 is a header)
    uint32_t carry = 0x80000000u;
    for (uint32_t b = s0; b > 0; b = b > 64 ? b - 64 : 0) {
        const bool in = lane < b;
        const uint32_t w = in ? sword[b - 1 - lane] : 0u;
        const uint64_t hm = __ballot(in && (w >> 31));
        if (hm) {
            carry = __shfl(w, (int)__builtin_ctzll(hm));
            break;
        }
    }
    const uint32_t hdr = 0x80000000u | vb;
    for (uint32_t q0 = s0; q0 < s1; q0 += 64) {
        const uint32_t q = q0 + lane;
        const bool valid = q < s1;
        const uint32_t w = valid ? sword[q] : 0u;
        const uint32_t X = max(wave_inclusive_max(w), carry);
        carry = __builtin_amdgcn_readlane(X, 63);
        const uint32_t t = X & 0x7fffffffu;
        const uint2 gl = GXL[t];
        const bool is_hdr = w >> 31;
        if (valid && q < gl.y) {
            buckets[(uint32_t)(gl.x + q)] = is_hdr ? hdr : w;
        } else if (valid && !is_hdr) {
            const uint32_t v = (t << tc.ts) | (w & msk);
            if (!((words[v >> 6] >> (v & 63)) & 1u)) {
                const uint32_t j = b32 + (w >> tc.ts);
                out[IDS ? ids[j] : j] = 0;
            }
        }
    }
}

// Inclusive maximum across a wave64 (the wave_inclusive_scan pattern with max for add;
// 0 is max's identity, so lanes whose DPP source is out of range are unaffected).
__device__ __forceinline__ uint32_t wave_inclusive_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false));  // row_shr:8
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return v;
}

// Inclusive "last nonzero" scan across a wave64 (the wave_inclusive_scan pattern with
// a select for the add): lane i gets the value of the highest lane <= i whose input
// is nonzero, or 0.
__device__ __forceinline__ uint32_t wave_last_nonzero(uint32_t v) {
    uint32_t s;
    s = __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false); v = v ? v : s;  // row_shr:1
    s = __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false); v = v ? v : s;  // row_shr:2
    s = __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false); v = v ? v : s;  // row_shr:4
    s = __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false); v = v ? v : s;  // row_shr:8
    s = __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false); v = v ? v : s;  // row_bcast:15
    s = __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false); v = v ? v : s;  // row_bcast:31
    return v;
}

// Split probe (round 5): J0..J1 (J1 = 0: k) is the range of each key's indices this
// launch bins; R2 marks the second round, which bins only the keys whose answer the
// first round left at 1 and leaves the answers' initialisation to the first.  PKPT
// keys per thread: the first round bins two indices per key, so it takes four keys
// per thread (runs four times as long, a quarter of the reservations) in the LDS the
// one-round kernel's k indices of one key take.  IDS (the second round, register-loaded
// keys): the keys are the compacted list ids[0, *nlive) of the first round's survivors
// (probe_compact_kernel), so the hash and the runs go to live keys only; the grid is
// sized for every key of the pass and the blocks past the list return at once.
// E32 (round 6, NB_PROBE_ENTRY=32): 32-bit bucket entries.  Every run a block writes
// into a (tile, shard) bucket starts with a header word, bit 31 set, holding the
// block's index in the launch; the run's entries are kib << ts | in-tile offset, kib
// the key's position in the block (< NT * PKPT <= 2^(31 - ts)), so the tile kernel
// (probe_tile32_kernel) recovers the key as header * NT * PKPT + kib (IDS: the
// list entry ids[header * NT + kib]).  4 B per lookup plus a header per run (~1 per
// 8 lookups at C4's shape) instead of 8 B: the bucket round trip drops from 16 to
// ~9 B per lookup.
// One (virtual) bin block vb of the probe: keys [vb * NT * PKPT, +NT * PKPT) of the
// launch (IDS: of its list).  The kernel below loops over them.
template <int FLAVOR, int LAYOUT, bool STAGE, int KR, int J0, int J1, bool R2, int PKPT, bool IDS, bool E32>
__device__ __forceinline__ void probe_bin_block(
    uint32_t vb, const uint8_t *__restrict__ keys, const uint64_t *__restrict__ offsets, uint32_t key_len,
    uint64_t n, const FilterConsts &c, const TileCfg &tc, const TileScratch &sc, uint64_t *__restrict__ buckets,
    const uint64_t *__restrict__ words, uint8_t *__restrict__ out, const uint32_t *__restrict__ ids) {
    constexpr int NT = kProbeThreads;
    extern __shared__ uint32_t lds[];
    const uint32_t T = tc.T, tid = threadIdx.x, k = c.k;
    uint32_t *cnt = lds, *S = lds + T, *GX = lds + 2 * T, *L = lds + 3 * T;
    uint32_t *wave_sums = lds + 4 * T;  // [NT/64 + 2]
    const uint32_t keff = PKPT * ((J1 ? (uint32_t)J1 : k) - J0);  // (probe_keff on the host)
    uint32_t *sidx = lds + probe_sort_offset_words(T);  // [NT * keff] indices, sorted by tile
    uint32_t *skid = sidx + NT * keff;                  // [NT * keff] their keys
    const uint64_t base = (uint64_t)vb * (NT * PKPT);
    BinPhase1<FLAVOR, LAYOUT, PKPT, NT, STAGE, KR, J1, J0, R2, IDS> ph;
    if (R2) ph.gate = out;
    ph.ids = ids;
    ph.run(keys, offsets, key_len, n, c, tc.mul, T, cnt, sidx, wave_sums + NT / 64 + 1, base);
    if (!R2) {
#pragma unroll
        for (int p = 0; p < PKPT; ++p)  // (staged keys: the valid ones fill the first slots)
            if (base + (uint64_t)p * NT + tid < n) out[ph.kid[p]] = 1;
    }
    // counts from the placement handles (A_t << kHandleShift | 4 rank, see BinPhase1)
    if constexpr (E32) {
        // a touched tile's run is its header word, then its entries
        for (uint32_t t = tid; t < T; t += NT) {
            const uint32_t h = (cnt[t] - (lds_addr(cnt + t) << kHandleShift)) >> 2;
            cnt[t] = h ? h + 1 : 0u;
        }
        __syncthreads();
        probe_bin_tail_e32<NT, PKPT, KR, J0, J1, IDS>(vb, ph, tc, sc, cnt, S, GX, L, wave_sums, sidx,
                                                      reinterpret_cast<uint32_t *>(buckets), words, out,
                                                      ids, base, k);
        return;
    }
    for (uint32_t t = tid; t < T; t += NT) cnt[t] = (cnt[t] - (lds_addr(cnt + t) << kHandleShift)) >> 2;
    __syncthreads();
    const uint32_t total = block_exclusive_scan<NT>(cnt, S, T, wave_sums);
    // reserve a run in every touched tile's bucket shard; GX[t] = its first entry
    // minus the run's local start, L[t] = the first local position past capacity
    const uint32_t shard = vb & (tc.G - 1);
    uint32_t *cur = sc.gcur + (size_t)shard * T;
    for (uint32_t t = tid; t < T; t += NT) {
        const uint32_t h = cnt[t], g = h ? atomicAdd(&cur[t], h) : 0u;
        GX[t] = bucket_region(tc, t, shard) * tc.cap + g - S[t];
        L[t] = S[t] + (g < tc.cap ? tc.cap - g : 0u);
    }
    // placement (the reservations' round trips overlap it)
#pragma unroll
    for (int p = 0; p < PKPT; ++p) {
        if (ph.live[p]) {
#pragma unroll
            for (int j = J0; j < KR; ++j)
                if (J1 ? j < J1 : j < (int)k) {
                    const uint32_t pos = S[ph.ridx[p][j] >> tc.ts] + ((ph.rank[p][j] & kHandleMask) >> 2);
                    sidx[pos] = ph.ridx[p][j];
                    skid[pos] = ph.kid[p];
                }
        }
    }
    __syncthreads();
    // write-out: one 64-bit entry per index, runs contiguous; an entry past its
    // bucket's capacity (pathological duplicates only) is tested right here
    const uint32_t msk = (1u << tc.ts) - 1;
    for (uint32_t q = tid; q < total; q += NT) {
        const uint32_t v = sidx[q], t = v >> tc.ts, kq = skid[q];
        if (q < L[t]) {
            buckets[(uint32_t)(GX[t] + q)] = ((uint64_t)kq << 32) | (v & msk);
        } else if (!((words[v >> 6] >> (v & 63)) & 1u)) {
            out[kq] = 0;
        }
    }
}

// A value the compiler must treat as changed here (an empty asm rewrites each 32-bit
// word in its SGPR): what is computed from it cannot be hoisted out of a loop.
template <class V>
__device__ __forceinline__ V launder(const V &v) {
    static_assert(sizeof(V) % 4 == 0, "whole dwords");
    uint32_t w[sizeof(V) / 4];
    __builtin_memcpy(w, (const void *)&v, sizeof(V));
#pragma unroll
    for (size_t i = 0; i < sizeof(V) / 4; ++i) asm volatile("" : "+s"(w[i]));
    V r;
    __builtin_memcpy((void *)&r, w, sizeof(V));
    return r;
}
constexpr uint32_t kVbClasses = 64;  // bin-block counter classes of the probe's bin kernels
// The probe's bin kernel: one bin block (NT x PKPT keys) per workgroup.
template <int FLAVOR, int LAYOUT, bool STAGE, int KR, int J0 = 0, int J1 = 0, bool R2 = false, int PKPT = 1,
          bool IDS = false, bool E32 = false>
__global__ __launch_bounds__(kProbeThreads, NB_BIN_MIN_WAVES(kProbeThreads)) void probe_bin_kernel(
    const uint8_t *__restrict__ keys, const uint64_t *__restrict__ offsets, uint32_t key_len,
    uint64_t n, FilterConsts c, TileCfg tc, TileScratch sc, uint64_t *__restrict__ buckets,
    const uint64_t *__restrict__ words, uint8_t *__restrict__ out, ProbeGate gate,
    const uint32_t *__restrict__ ids, const uint32_t *__restrict__ nlive) {
    constexpr uint64_t kpb = (uint64_t)kProbeThreads * PKPT;
    static_assert(!E32 || kpb <= (1 << 11), "E32: kib << ts must stay below bit 31 (ts <= 20)");
    if (!gate_open(gate)) return;
    if (IDS) n = min<uint64_t>(__builtin_amdgcn_readfirstlane(coherent_load(nlive)), n);  // <= the list's capacity
    if (blockIdx.x < (n + kpb - 1) / kpb)
        probe_bin_block<FLAVOR, LAYOUT, STAGE, KR, J0, J1, R2, PKPT, IDS, E32>(
            blockIdx.x, keys, offsets, key_len, n, c, tc, sc, buckets, words, out, ids);
}

// The same kernel looping over the bin blocks (round 6, auto's gated launches, which
// may be closed): a grid of kProbeBinBlocksPerCU per CU, so a closed launch dispatches
// a few thousand workgroups instead of one per bin block.  Its only argument is this
// struct, and every iteration reads it afresh from the kernel-argument segment
// through a laundered pointer: a loop over the plain kernel's arguments kept them and
// what is derived from them live across iterations (~70 SGPRs spilled to VGPR lanes,
// the open kernel ~15 % slower than one workgroup per bin block).
struct ProbeBinArgs {
    const uint8_t *keys;
    const uint64_t *offsets;
    uint64_t n;
    uint8_t *out;
    uint64_t *buckets;
    const uint64_t *words;
    const uint32_t *ids;
    const uint32_t *nlive;
    uint32_t key_len;
    uint32_t pad_;
    FilterConsts c;
    TileCfg tc;
    TileScratch sc;
    ProbeGate gate;
};
// A kernel's single struct argument, read afresh from the kernel-argument segment
// through a laundered pointer (scalar loads; nothing of it stays live across a loop).
template <class A>
__device__ __forceinline__ A reload_kernel_args() {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) A *KArgs;
    const KArgs ap = launder((KArgs)__builtin_amdgcn_kernarg_segment_ptr());
    return *ap;
#else
    return A{};  // (host pass only; never runs)
#endif
}
template <int FLAVOR, int LAYOUT, bool STAGE, int KR, int J0 = 0, int J1 = 0, bool R2 = false, int PKPT = 1,
          bool IDS = false, bool E32 = false>
__global__ __launch_bounds__(kProbeThreads, NB_BIN_MIN_WAVES(kProbeThreads)) void probe_bin_loop_kernel(
    ProbeBinArgs a) {
    constexpr uint64_t kpb = (uint64_t)kProbeThreads * PKPT;
    static_assert(!E32 || kpb <= (1 << 11), "E32: kib << ts must stay below bit 31 (ts <= 20)");
    if (!gate_open(a.gate)) return;
    uint64_t n = a.n;
    if (IDS) n = min<uint64_t>(__builtin_amdgcn_readfirstlane(coherent_load(a.nlive)), n);  // <= the list's capacity
    const uint64_t nvb = (n + kpb - 1) / kpb;
    // Blocks take their first bin block by index.  A grid that covers every bin block
    // stops there; a capped one takes the next ones from kVbClasses counters, class
    // c = blockIdx % kVbClasses handing out bin blocks c, c + kVbClasses, ... (a
    // multiple of the G shards: a bin block's shard stays on its workgroup's XCD; 64
    // classes keep the counters' atomics from queueing on a few addresses), so a short
    // grid finishes together instead of in generations.
    const uint32_t c_ = blockIdx.x & (kVbClasses - 1), per = gridDim.x / kVbClasses;
    uint32_t *const vbctr = a.sc.vbctr;
    extern __shared__ uint32_t lds_next[];
    uint32_t *next = lds_next + probe_sort_offset_words(a.tc.T) - 1;  // (a free word before the sort area)
    const bool fetch = gridDim.x < nvb;  // uniform
    for (uint64_t vb = blockIdx.x; vb < nvb;) {
        // the next bin block's counter fetch goes out before this one's work (its round
        // trip is hidden behind it)
        uint32_t pre = 0;
        if (fetch && threadIdx.x == 0) pre = atomicAdd(&vbctr[c_], 1u);
        {
            const ProbeBinArgs b = reload_kernel_args<ProbeBinArgs>();
            probe_bin_block<FLAVOR, LAYOUT, STAGE, KR, J0, J1, R2, PKPT, IDS, E32>(
                (uint32_t)vb, b.keys, b.offsets, b.key_len, n, b.c, b.tc, b.sc, b.buckets, b.words, b.out, b.ids);
        }
        if (!fetch) break;
        if (threadIdx.x == 0) *next = per + pre;
        __syncthreads();  // (also: the block's LDS reads are done before the next one)
        vb = c_ + (uint64_t)kVbClasses * *next;
        __syncthreads();  // everyone has read *next
    }
}

// The split probe's survivors of its first round: ids (in the pass) of the keys whose
// answer is still 1, appended to ids[] (block order arbitrary, in key order within a
// block) and counted in *nlive (zeroed before the launch).  16 answers per thread (four
// 4-byte loads when the answers are 4-byte aligned), one reservation atomic per block
// of 16 384 keys: the blocks' atomics all hit *nlive, which serialises them (~10 ns
// each; four answers per thread took 0.15 ms per 50M-key pass on them alone).  The
// block's ids are staged in LDS (dynamic, kCompactLds) and copied out coalesced: a
// lane's own 16 stores would each hit a different line.
constexpr int kCompactThreads = 1024, kCompactPer = 16;
constexpr size_t kCompactLds = ((size_t)kCompactThreads * kCompactPer + kCompactThreads / 64 + 2) * 4;
// (a grid-stride loop over the 16 384-answer chunks: auto's gated launches, which may
// be closed, take a short grid)
__global__ __launch_bounds__(kCompactThreads) void probe_compact_kernel(const uint8_t *__restrict__ ans,
                                                                         uint32_t n, uint32_t *__restrict__ ids,
                                                                         uint32_t *__restrict__ nlive,
                                                                         ProbeGate gate) {
    if (!gate_open(gate)) return;
    extern __shared__ uint32_t stage[];  // [NT * 16] the block's ids, then the wave sums
    uint32_t *wsum = stage + kCompactThreads * kCompactPer;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    constexpr uint32_t kChunk = kCompactThreads * kCompactPer;
    const uint32_t nchunks = (n + kChunk - 1) / kChunk;
    for (uint32_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
        if (ch != blockIdx.x) __syncthreads();  // the previous chunk's ids are out
        const uint32_t i0 = ch * kChunk + tid * kCompactPer;
        uint32_t live = 0;
        if ((reinterpret_cast<uintptr_t>(ans) & 3) == 0 && i0 + kCompactPer <= n) {  // (kernel-uniform alignment)
            const uint32_t *a4 = reinterpret_cast<const uint32_t *>(ans + i0);
#pragma unroll
            for (int w = 0; w < kCompactPer / 4; ++w) {
                const uint32_t v = a4[w];
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if ((v >> (8 * b)) & 0xffu) live |= 1u << (4 * w + b);
            }
        } else {
#pragma unroll
            for (int q = 0; q < kCompactPer; ++q)
                if (i0 + q < n && ans[i0 + q]) live |= 1u << q;
        }
        const uint32_t cnt = __popc(live), incl = wave_inclusive_scan(cnt);
        if (lane == 63) wsum[wid] = incl;
        __syncthreads();
        if (wid == 0) {
            constexpr uint32_t kW = kCompactThreads / 64;
            const uint32_t w = lane < kW ? wsum[lane] : 0u, wi = wave_inclusive_scan(w);
            if (lane < kW) wsum[lane] = wi - w;
            if (lane == kW - 1) {
                wsum[kW] = wi;
                wsum[kW + 1] = wi ? atomicAdd(nlive, wi) : 0u;
            }
        }
        __syncthreads();
        uint32_t o = wsum[wid] + incl - cnt;  // in the block
        while (live) {
            const uint32_t q = __builtin_ctz(live);
            live &= live - 1;
            stage[o++] = i0 + q;
        }
        __syncthreads();
        const uint32_t total = wsum[kCompactThreads / 64], gb = wsum[kCompactThreads / 64 + 1];
        for (uint32_t j = tid; j < total; j += kCompactThreads)
            if (gb + j < n) ids[gb + j] = stage[j];  // (the list holds n ids: a guard, never taken)
    }
}

// (n: the pass's keys -- an entry's key is checked against it before its answer is
// stored, so no bucket content can address memory outside the answers)
template <int NT = kTileThreads>
__global__ __launch_bounds__(NT) void probe_tile_kernel(TileCfg tc, TileScratch sc,
                                                        const uint64_t *__restrict__ buckets,
                                                        const uint64_t *__restrict__ words,
                                                        uint64_t nwords, uint8_t *__restrict__ out,
                                                        ProbeGate gate, uint32_t n) {
    if (!gate_open(gate)) return;
    extern __shared__ uint32_t tile[];  // [2^ts / 32] filter words, then 2*kShards+1 words
    const uint32_t t = blockIdx.x, tid = threadIdx.x;
    const uint32_t tile_words32 = 1u << (tc.ts - 5), mask = (1u << tc.ts) - 1;
    if (t == 0 && tid < kVbClasses && sc.vbctr) sc.vbctr[tid] = 0;  // the bin kernel's counters
    if (t == 0 && tid == 0 && sc.nlive) *sc.nlive = 0;        // the next compaction's count
    uint32_t *shard_cnt = tile + tile_words32;  // [kShards]
    uint32_t *shard_v0 = shard_cnt + kShards;   // [kShards + 1]
    // the tile's filter words (past the filter's end: zero, never tested)
    const uint64_t w0 = (uint64_t)t << (tc.ts - 6);
    uint64_t *tile64 = reinterpret_cast<uint64_t *>(tile);
    for (uint32_t w = tid; w < tile_words32 / 2; w += NT)
        tile64[w] = w0 + w < nwords ? words[w0 + w] : 0ull;
    if (tid < tc.G) {
        uint32_t *cp = sc.gcur + (size_t)tid * tc.T + t;
        shard_cnt[tid] = min(coherent_load(cp), tc.cap);  // (written by another kernel's atomics)
        *cp = 0;  // workspace invariant: cursors are zero between launches
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t v0 = 0;
        for (uint32_t g = 0; g < tc.G; ++g) {
            shard_v0[g] = v0;
            v0 += shard_cnt[g];
        }
        shard_v0[tc.G] = v0;
    }
    __syncthreads();
    const uint32_t ne = shard_v0[tc.G];
    auto test = [&](uint64_t e) {
        const uint32_t off = (uint32_t)e & mask, kid = (uint32_t)(e >> 32);
        if (!((tile[off >> 5] >> (off & 31)) & 1u) && kid < n) out[kid] = 0;
    };
    // the G shards as one flat range of entries; a lane's entry indices only grow,
    // so its shard index is advanced, never searched
    uint32_t g = 0;
    auto entry_at = [&](uint32_t q) {
        while (g + 1 < tc.G && q >= shard_v0[g + 1]) ++g;
        return buckets[(size_t)bucket_region(tc, t, g) * tc.cap + (q - shard_v0[g])];
    };
    uint32_t q = tid;
    for (; q + 3 * NT < ne; q += 4 * NT) {
        uint64_t e[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) e[u] = entry_at(q + u * NT);
#pragma unroll
        for (int u = 0; u < 4; ++u) test(e[u]);
    }
    for (; q < ne; q += NT) test(entry_at(q));
}

// The tile kernel of E32 buckets (probe_bin_tail_e32): an entry's key comes from the
// header word that opens its run, so a bucket is read in order.  Each (tile, shard)
// bucket is one contiguous range: its NT/64/G waves take a contiguous segment each
// (split at 16-byte boundaries) and stream it in 256-word steps, one 16-byte load per
// lane; a wave-wide "last header" scan hands every lane the header in force at its
// first word, and the last header of a step carries into the next.  A segment that
// starts inside a run finds its header by one backward look (a run is ~9 words at
// C4's shape; word 0 of every bucket is a header).  kpb = keys per bin block of the
// launch; IDS: keys are list entries ids[header * kpb + kib] (the split path's second
// round, with NB_PROBE_ENTRY=32 only).
// (Measured, not kept: one 4-byte load per lane, so that a miss-store instruction
// covers 64 consecutive entries instead of 256 -- round one of the split path at 30 %
// present 597 -> 725 us per 50M-key pass, tools/trace_rounds.py, r06c / r06e; and, in
// this kernel and probe_tile_kernel, the next step's loads issued before this step's
// tests and miss stores -- split absent 4.50 -> 4.73 ms, 30 % present 3.68 -> 3.98,
// profiles/r06f_probe_prefetch_ab.txt.)
constexpr int kProbeTileUnroll = 4;  // 16-byte loads in flight per lane
template <int NT = kTileThreads, bool IDS = false>
__global__ __launch_bounds__(NT) void probe_tile32_kernel(TileCfg tc, TileScratch sc,
                                                          const uint32_t *__restrict__ buckets,
                                                          const uint64_t *__restrict__ words,
                                                          uint64_t nwords, uint8_t *__restrict__ out,
                                                          ProbeGate gate, uint32_t kpb,
                                                          const uint32_t *__restrict__ ids, uint32_t n) {
    if (!gate_open(gate)) return;
    extern __shared__ uint32_t tile[];  // [2^ts / 32] filter words, then kShards counts
    const uint32_t t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (t == 0 && tid < kVbClasses && sc.vbctr) sc.vbctr[tid] = 0;  // the bin kernel's counters
    if (t == 0 && tid == 0 && sc.nlive) *sc.nlive = 0;        // the next compaction's count
    const uint32_t tile_words32 = 1u << (tc.ts - 5), mask = (1u << tc.ts) - 1;
    uint32_t *shard_cnt = tile + tile_words32;  // [kShards]
    const uint64_t w0 = (uint64_t)t << (tc.ts - 6);
    uint64_t *tile64 = reinterpret_cast<uint64_t *>(tile);
    for (uint32_t w = tid; w < tile_words32 / 2; w += NT)
        tile64[w] = w0 + w < nwords ? words[w0 + w] : 0ull;
    if (tid < tc.G) {
        uint32_t *cp = sc.gcur + (size_t)tid * tc.T + t;
        shard_cnt[tid] = min(coherent_load(cp), tc.cap);  // (written by another kernel's atomics)
        *cp = 0;  // workspace invariant: cursors are zero between launches
    }
    __syncthreads();
    // (no barrier below: a wave leaves when its segment is done)
    const uint32_t wps = max(1u, (uint32_t)(NT / 64) / tc.G);  // waves per shard
    const uint32_t g = wid / wps, part = wid % wps;
    if (g >= tc.G) return;
    const uint32_t c = shard_cnt[g];
    const uint32_t per = ((c + wps - 1) / wps + 3) & ~3u;
    const uint32_t s0 = min(part * per, c), s1 = min(s0 + per, c);
    if (s0 >= s1) return;  // wave-uniform
    const uint32_t *e = buckets + (size_t)bucket_region(tc, t, g) * tc.cap;
    // header + 1 in force at the current position (0: none seen yet)
    uint32_t carry = 0;
    for (uint32_t b = s0; b > 0 && carry == 0; b = b > 64 ? b - 64 : 0) {
        const bool in = lane < b;
        const uint32_t w = in ? e[b - 1 - lane] : 0u;
        const uint64_t hm = __ballot(in && (w >> 31));
        if (hm) carry = (__shfl(w, (int)__builtin_ctzll(hm)) & 0x7fffffffu) + 1;
    }
    auto test = [&](uint32_t w, uint32_t hv) {
        const uint32_t off = w & mask;
        if (!((tile[off >> 5] >> (off & 31)) & 1u)) {
            const uint32_t j = (hv - 1) * kpb + (w >> tc.ts);  // (n: a guard, as probe_tile_kernel)
            if (j < n) {
                const uint32_t kid = IDS ? ids[j] : j;
                if (kid < n) out[kid] = 0;
            }
        }
    };
    // one step: the lane's 4 words (the first `valid` of them real), wave-uniform call
    auto step = [&](const uint4 &v, uint32_t valid) {
        const uint32_t ws[4] = {v.x, v.y, v.z, v.w};
        uint32_t last = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if ((uint32_t)i < valid && (ws[i] >> 31)) last = (ws[i] & 0x7fffffffu) + 1;
        const uint32_t X = wave_last_nonzero(last);
        const uint32_t prev = __shfl_up(X, 1);
        uint32_t cur = lane && prev ? prev : carry;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if ((uint32_t)i < valid) {
                if (ws[i] >> 31) cur = (ws[i] & 0x7fffffffu) + 1;
                else if (cur) test(ws[i], cur);
            }
        }
        const uint32_t tail = __builtin_amdgcn_readlane(X, 63);
        if (tail) carry = tail;
    };
    constexpr uint32_t kStep = 256, U = kProbeTileUnroll;
    uint32_t q = s0;
    for (; q + U * kStep <= s1; q += U * kStep) {
        uint4 v[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) v[u] = bucket_load(reinterpret_cast<const uint4 *>(e + q + u * kStep) + lane);
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) step(v[u], 4);
    }
    for (; q < s1; q += kStep) {
        const uint32_t p = q + 4 * lane, valid = p < s1 ? min(4u, s1 - p) : 0u;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (valid == 4) {
            v = bucket_load(reinterpret_cast<const uint4 *>(e + p));
        } else if (valid) {
            v.x = e[p];
            if (valid > 1) v.y = e[p + 1];
            if (valid > 2) v.z = e[p + 2];
        }
        step(v, valid);
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

// dst[w] |= src_0[w] | ... | src_{n-1}[w], the sources read in place: other
// allocations on this device, or peer devices' memory over xGMI once peer access
// is enabled (nb_build_sharded's slice merge).  Up to kGatherSrcs per launch.
constexpr int kGatherSrcs = 16;
struct GatherSrcs {
    const uint64_t *p[kGatherSrcs];
};
__global__ __launch_bounds__(kBlock) void or_gather_kernel(uint64_t *__restrict__ dst, GatherSrcs s,
                                                           uint32_t nsrc, uint64_t nwords) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x; w < nwords; w += stride) {
        uint64_t v = dst[w];
        for (uint32_t i = 0; i < nsrc; ++i) v |= s.p[i][w];
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
    if (flavor != NB_FLAVOR_LIBSTDCXX && flavor != NB_FLAVOR_MSVC_FNV1A &&
        flavor != NB_FLAVOR_MURMUR3_X64_128)
        return fail(NB_ERR_ARG, "unknown flavor");
    if (n && m == 0) return fail(NB_ERR_ARG, "m == 0 with keys (reference divides by zero)");
    if (n && (!keys || !words)) return fail(NB_ERR_ARG, "NULL keys or words");
    return NB_OK;
}

// Per-(device, stream) scratch of the tiled path: bucket cursors, spill flags and
// the spill bitmap (all kept zero between builds by the tile kernel), and the
// bucket array.  `mu` is held from the reservation through the last launch of a
// build, so two host threads building on the same stream enqueue whole builds
// (bin A, tile A, bin B, tile B), never interleaved kernels over one workspace.
struct Workspace {
    std::mutex mu;
    int dev = -1;
    hipStream_t st = nullptr;
    uint32_t *zeroed = nullptr;   // gcur [kShards*kMaxTiles] | spill_flag [kMaxTiles] |
                                  // super-tile cursors [kShards*kMaxSuper] | spill32
    size_t zeroed_bytes = 0;
    void *buckets = nullptr;
    size_t bucket_bytes = 0;
    void *buckets2 = nullptr;     // fine buckets of the two-level build
    size_t bucket2_bytes = 0;
    uint32_t *probe_hits = nullptr;       // the auto probe's sample counts (ProbeGate)
    uint32_t *probe_hits_host = nullptr;  // host-mapped coherent words the sample writes
    uint32_t *probe_hits_map = nullptr;   // ... their device address
    hipEvent_t ev_probe = nullptr;        // recorded after the sample
    // pipelined two-level passes (NB_OVERLAP): a second stream for the re-bin + tile
    // kernels, the odd passes' pass-1 buckets, super-tile cursors and spill scratch
    hipStream_t aux = nullptr;
    int aux_prio = 0;
    hipEvent_t ev_bin[2] = {nullptr, nullptr}, ev_done[2] = {nullptr, nullptr};
    hipEvent_t ev_tile[2] = {nullptr, nullptr}, ev_start = nullptr;
    uint32_t *zeroed_alt = nullptr;
    size_t zeroed_alt_bytes = 0;
    void *buckets_alt = nullptr;
    size_t bucket_alt_bytes = 0;
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

constexpr size_t kCurWords = (size_t)kShards * kMaxCurTiles;
constexpr size_t kFlagWords = kMaxCurTiles;

// Grows the workspace (synchronising the stream before freeing old buffers).
// Not graph-capturable when it has to grow: call once with the largest shape first.
int grow(Workspace &w, void **buf, size_t *have, size_t want_bytes) {
    if (want_bytes <= *have) return NB_OK;
    if (*buf) NB_HIP(hipFree(*buf));
    *buf = nullptr;
    *have = 0;
    const size_t want = want_bytes + want_bytes / 8;
    NB_HIP(hipMalloc(buf, want));
    *have = want;
    return NB_OK;
}

constexpr size_t kSuperCurWords = (size_t)kShards * kMaxSuper;

// Grows the workspace (synchronising the stream before freeing old buffers).
// Not graph-capturable when it has to grow: call once with the largest shape first.
int ws_reserve(Workspace &w, uint32_t m, size_t bucket_bytes, TileScratch *sc,
               size_t bucket2_bytes = 0) {
    const size_t spill_words32 = 2 * (((size_t)m + 63) / 64);
    const size_t zb = (kCurWords + kFlagWords + kSuperCurWords + spill_words32) * 4;
    if (zb > w.zeroed_bytes || bucket_bytes > w.bucket_bytes || bucket2_bytes > w.bucket2_bytes)
        NB_HIP(hipStreamSynchronize(w.st));
    if (zb > w.zeroed_bytes) {
        if (w.zeroed) NB_HIP(hipFree(w.zeroed));
        w.zeroed = nullptr;
        w.zeroed_bytes = 0;
        NB_HIP(hipMalloc(&w.zeroed, zb));
        // on the workspace's stream: a blocking hipMemset runs on the null stream,
        // which non-blocking streams do not wait for (same hazard as the sharded
        // merge's staging copy)
        NB_HIP(hipMemsetAsync(w.zeroed, 0, zb, w.st));
        w.zeroed_bytes = zb;
    }
    int rc;
    if ((rc = grow(w, &w.buckets, &w.bucket_bytes, bucket_bytes)) ||
        (rc = grow(w, &w.buckets2, &w.bucket2_bytes, bucket2_bytes)))
        return rc;
    sc->gcur = w.zeroed;
    sc->spill_flag = w.zeroed + kCurWords;
    sc->spill32 = w.zeroed + kCurWords + kFlagWords + kSuperCurWords;
    return NB_OK;
}

// the super-tile cursors of the two-level build (zero between builds)
uint32_t *super_cursors(Workspace &w) { return w.zeroed + kCurWords + kFlagWords; }

// The pipelined two-level build's extras: the aux stream (priority: 0 normal, 1
// high) and its events, and a second zeroed block (spill flags, super cursors and
// spill bitmap of the odd passes; its fine cursors are unused) plus second pass-1
// buckets.  Zeroed on the workspace's stream, as ws_reserve does.
int ws_reserve_alt(Workspace &w, uint32_t m, size_t bucket_bytes, int prio) {
    const size_t spill_words32 = 2 * (((size_t)m + 63) / 64);
    const size_t zb = (kCurWords + kFlagWords + kSuperCurWords + spill_words32) * 4;
    if (w.aux && w.aux_prio != prio) {
        NB_HIP(hipStreamSynchronize(w.aux));
        NB_HIP(hipStreamDestroy(w.aux));
        w.aux = nullptr;
    }
    if (!w.aux) {
        int lo = 0, hi = 0;
        NB_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
        NB_HIP(hipStreamCreateWithPriority(&w.aux, hipStreamNonBlocking, prio ? hi : lo));
        w.aux_prio = prio;
        for (hipEvent_t *e : {&w.ev_bin[0], &w.ev_bin[1], &w.ev_done[0], &w.ev_done[1],
                              &w.ev_tile[0], &w.ev_tile[1], &w.ev_start})
            if (!*e) NB_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
    if (zb > w.zeroed_alt_bytes || bucket_bytes > w.bucket_alt_bytes) NB_HIP(hipStreamSynchronize(w.st));
    if (zb > w.zeroed_alt_bytes) {
        if (w.zeroed_alt) NB_HIP(hipFree(w.zeroed_alt));
        w.zeroed_alt = nullptr;
        w.zeroed_alt_bytes = 0;
        NB_HIP(hipMalloc(&w.zeroed_alt, zb));
        NB_HIP(hipMemsetAsync(w.zeroed_alt, 0, zb, w.st));
        w.zeroed_alt_bytes = zb;
    }
    return grow(w, &w.buckets_alt, &w.bucket_alt_bytes, bucket_bytes);
}

using nb::knob;  // the A/B switches (nb_knobs.h): read once, atomics

// Tile size policy (measured, tools/ubench_tiled.hip): 2^16-bit tiles with 16-bit
// bucket entries while that needs <= 2048 tiles (m <= 2^27, e.g. C2); smaller
// tiles for small m (>= ~1024 tiles, 2^12 bits minimum); above 2^27 bits the
// entries are 32-bit whatever the tile size, so the largest tiles (up to 2^20
// bits) that still leave >= 512 tile blocks: fewer tiles make a block's runs
// longer (fewer reservation atomics and L2 write requests).  C3/C4: ts = 20,
// T = 915 (C4 2.31 -> 1.99 ms, C3 3.68 -> 3.35 ms vs ts = 19, T = 1 829);
// C5: ts = 20, 4 096 fine tiles.
TileCfg choose_tiles(uint32_t m, uint64_t n_chunk, uint32_t k) {
    TileCfg tc;
    uint32_t ts = 12;
    while (ts < 16 && ((uint64_t)m >> (ts + 1)) >= 1024) ++ts;
    while (ts < 20 && (((uint64_t)m + (1ull << ts) - 1) >> ts) > 2048) ++ts;
    auto tiles = [m](uint32_t s) { return ((uint64_t)m + (1ull << s) - 1) >> s; };
    if (m >= (1u << 24) && k <= 16 && knob(nb::kKnobPack) != 0) {
        // packed 21-bit entries (k <= 16: the rank-mode tail): larger tiles, down
        // to ~160 of them -- C2 at 2^19-bit tiles (T = 183) 0.162-0.167 ms vs
        // 0.171-0.176 with u16 entries at 2^16 bits (3 interleaved repeats,
        // tools/sweep_c2.sh): a third more entry bytes, runs 8x longer
        ts = std::max<uint32_t>(ts, 17);
        while (ts < 20 && tiles(ts + 1) >= 160) ++ts;
    } else if (ts > 16) {
        while (ts < 20 && tiles(ts + 1) >= 512) ++ts;
    }
    ts = std::min<uint32_t>(std::max<uint32_t>(knob(nb::kKnobTileBits) ? (uint32_t)knob(nb::kKnobTileBits) : ts, 12), 20);
    tc.ts = ts;
    tc.T = (uint32_t)(((uint64_t)m + (1ull << ts) - 1) >> ts);
    // cursor shards: a power of two (the kernels pick a block's shard with a mask)
    tc.G = std::min<uint32_t>(std::max<uint32_t>((uint32_t)std::min<uint64_t>(knob(nb::kKnobShards), kShards), 1), kShards);
    while (tc.G & (tc.G - 1)) tc.G &= tc.G - 1;
    const double e = (double)n_chunk * k / ((double)tc.T * tc.G);
    uint64_t cap = (uint64_t)(e + 8.0 * std::sqrt(e) + 64.0);
    cap = (cap + 7) & ~7ull;
    tc.cap = (uint32_t)std::min<uint64_t>(cap, 0xFFFFFFC0ull);
    tc.fts = ts;
    tc.mul = tc.fmul = pow2_mul(ts);
    tc.w64 = 1u << (ts - 6);
    return tc;
}

// Counted tiles for the single-level packed path (TileCfg): the fewest tiles that
// fill whole tile-kernel rounds -- a multiple of the device's CU count -- and still
// fit one tile block's LDS (160 KiB less the shard counters: <= 1 310 048 bits with
// the two boundary words), while the power-of-two tiling (`p2`) leaves a partial
// last round.  NB_TILE_COUNT: 0 this policy, 1 off, N > 1 exactly N tiles.  Entries
// then hold 21-bit in-tile offsets (ts = 21: tiles < 2^21 bits with their boundary
// words).  C4 / C3 (m = 958 505 838): 768 tiles, three rounds, instead of 915.
// The CU count of the calling thread's current device, cached per device ID (a
// process may build on devices of different sizes).
uint32_t device_cus() {
    constexpr int kMaxDev = 64;
    static std::atomic<int> cus[kMaxDev];  // 0: not yet asked (static storage is zeroed)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    std::atomic<int> *slot = dev >= 0 && dev < kMaxDev ? &cus[dev] : nullptr;
    int v = slot ? slot->load(std::memory_order_relaxed) : 0;
    if (!v) {
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
            v = 256;
        if (slot) slot->store(v, std::memory_order_relaxed);
    }
    return (uint32_t)v;
}

uint32_t cap_for(uint32_t T, uint32_t G, uint64_t n, uint32_t k);

bool counted_tiles(uint32_t m, uint64_t n_chunk, uint32_t k, const TileCfg &p2, TileCfg *out) {
    const uint64_t kv = knob(nb::kKnobTileCount);
    if (kv == 1 || m < (1u << 24)) return false;
    if (kv == 0 && knob(nb::kKnobTileBits)) return false;  // an explicit tile size wins
    constexpr uint64_t kMaxBits = (160 * 1024 - (2 * kShards + 1) * 4) * 8ull - 128;
    const uint64_t tmin = ((uint64_t)m + kMaxBits - 1) / kMaxBits;
    uint64_t T = kv;
    if (kv == 0) {
        const uint32_t cus = device_cus();
        if (p2.T <= cus || p2.T % cus == 0) return false;  // already whole rounds
        T = (tmin + cus - 1) / cus * cus;
        if (T >= p2.T) return false;
    }
    if (T < tmin || T > kMaxTiles || T >= m) return false;
    TileCfg tc = p2;
    tc.mul = (uint32_t)((T << 32) / m);  // floor(2^32 T / m) < 2^32
    tc.T = (uint32_t)(((uint64_t)(m - 1) * tc.mul >> 32) + 1);
    const uint64_t maxlen = ((1ull << 32) + tc.mul - 1) / tc.mul + 1;
    tc.w64 = (uint32_t)((maxlen + 63) / 64 + 1);
    tc.ts = tc.fts = 21;
    tc.fmul = tc.mul;
    if ((uint64_t)tc.w64 * 64 >= (1ull << 21) || (uint64_t)tc.w64 * 8 + (2 * kShards + 1) * 4 > 160 * 1024)
        return false;
    tc.cap = cap_for(tc.T, tc.G, n_chunk, k);
    *out = tc;
    return true;
}

// Pass 1 of the two-level build: super tiles of kSuperFine fine tiles each.
TileCfg super_tiles(const TileCfg &fine, uint32_t m, uint64_t n_chunk, uint32_t k,
                    uint32_t fine_log2) {
    TileCfg tc = fine;
    tc.ts = fine.ts + fine_log2;  // 2^fine_log2 fine tiles per super tile
    tc.T = (uint32_t)(((uint64_t)m + (1ull << tc.ts) - 1) >> tc.ts);
    const double e = (double)n_chunk * k / ((double)tc.T * tc.G);
    uint64_t cap = (uint64_t)(e + 8.0 * std::sqrt(e) + 64.0);
    cap = (cap + 7) & ~7ull;
    tc.cap = (uint32_t)std::min<uint64_t>(cap, 0xFFFFFFC0ull);
    tc.fts = fine.ts;
    tc.mul = pow2_mul(tc.ts);
    tc.fmul = pow2_mul(fine.ts);
    tc.w64 = 0;  // (super tiles never reach the tile kernel)
    return tc;
}

enum class BuildPath { kAuto, kAtomic, kTiled };

BuildPath path_override() {
    const uint64_t v = knob(nb::kKnobBuildPath);
    return v == 1 ? BuildPath::kAtomic : v == 2 ? BuildPath::kTiled : BuildPath::kAuto;
}

// Keys per bin/tile pass: the whole batch while its buckets stay under ~8 GB of
// HBM (one pass over the filter), else equal chunks under that budget.
uint64_t chunk_keys(uint64_t n, uint32_t k) {
    if (const uint64_t v = knob(nb::kKnobChunkKeys)) return v;
    const uint64_t budget = (8ull << 30) / (4ull * std::max<uint32_t>(k, 1));  // keys
    const uint64_t passes = (n + budget - 1) / budget;
    return std::max<uint64_t>(1, (n + passes - 1) / std::max<uint64_t>(passes, 1));
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
                  const FilterConsts &c, uint64_t *words, bool overwrite, hipStream_t st) {
    if (overwrite) NB_HIP(hipMemsetAsync(words, 0, (((size_t)c.fm.m + 63) / 64) * 8, st));
    hipLaunchKernelGGL((bloom_build_atomic_kernel<FLAVOR, LAYOUT>), dim3(grid_for(n)),
                       dim3(kBlock), 0, st, keys, offsets, key_len, n, c,
                       reinterpret_cast<uint32_t *>(words));
    NB_HIP(hipGetLastError());
    return NB_OK;
}

template <int FLAVOR, int LAYOUT, int KPT, typename ENTRY, int NT, bool STAGE, int KR, int KX>
int launch_tiled_e(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                   const FilterConsts &c, uint64_t *words, bool overwrite, hipStream_t st,
                   uint64_t chunk, const TileCfg &tc) {
    constexpr uint64_t kpb = (uint64_t)KPT * NT;
    Workspace *ws;
    TileScratch sc;
    int rc;
    if ((rc = get_ws(st, &ws))) return rc;
    std::lock_guard<std::mutex> lk(ws->mu);
    if ((rc = ws_reserve(*ws, c.fm.m, (size_t)tc.T * tc.G * tc.cap * sizeof(ENTRY), &sc)))
        return rc;
    size_t sort_bytes = kpb * c.k * 4;
    if (sizeof(ENTRY) == 8) sort_bytes += (size_t)tc.T * 8;  // <= 2 pad slots per run
    if (STAGE) sort_bytes = std::max<size_t>(sort_bytes, stage_lds_bytes(NT));
    const size_t bin_lds = (size_t)bin_sort_offset_words(tc.T) * 4 + sort_bytes;
    const size_t tile_lds = (size_t)tc.w64 * 8 + (2 * kShards + 1) * 4;
    auto bin = bloom_bin_kernel<FLAVOR, LAYOUT, KPT, ENTRY, NT, STAGE, KR, KX>;
    auto tile_ow = bloom_tile_or_kernel<ENTRY, true>;
    auto tile_or = bloom_tile_or_kernel<ENTRY, false>;
    if ((rc = allow_lds(bin, bin_lds)) || (rc = allow_lds(tile_ow, tile_lds)) ||
        (rc = allow_lds(tile_or, tile_lds)))
        return rc;
    const uint64_t nwords = ((uint64_t)c.fm.m + 63) / 64;
    ENTRY *bk = reinterpret_cast<ENTRY *>(ws->buckets);
    for (uint64_t done = 0; done < n; done += chunk) {
        const uint64_t cn = std::min(chunk, n - done);
        const uint8_t *ck = offsets ? keys : keys + done * key_len;
        const uint64_t *co = offsets ? offsets + done : nullptr;
        TileScratch scb = sc;  // counted tiles, overwrite: the bin kernel zeroes the
                               // boundary words the tile kernel ORs into
        scb.zero_words = overwrite && done == 0 && tc.mul != pow2_mul(tc.ts) ? words : nullptr;
        hipLaunchKernelGGL(bin, dim3((uint32_t)((cn + kpb - 1) / kpb)), dim3(NT), bin_lds, st, ck, co,
                           key_len, cn, c, tc, scb, bk);
        NB_HIP(hipGetLastError());
        hipLaunchKernelGGL((overwrite && done == 0) ? tile_ow : tile_or, dim3(tc.T),
                           dim3(kTileThreads), tile_lds, st, tc, sc, bk, words, nwords);
        NB_HIP(hipGetLastError());
    }
    return NB_OK;
}

// The tile kernel for an entry type, as a type-erased launch target.
template <typename ENTRY, bool OVERWRITE>
void (*tile_kernel_of())(TileCfg, TileScratch, const void *, uint64_t *, uint64_t) {
    return reinterpret_cast<void (*)(TileCfg, TileScratch, const void *, uint64_t *, uint64_t)>(
        bloom_tile_or_kernel<ENTRY, OVERWRITE>);
}

// Pass-1 entry type of the two-level build: Pack5 units (k <= 16, the rank-mode
// tail; NB_PACK5=0 for the A/B) or 32-bit indices.
bool two_level_pack5() { return knob(nb::kKnobPack5) != 0; }

// Bucket capacity (entries) of one (tile, shard) for n keys: mean + 8 sigma + 64.
uint32_t cap_for(uint32_t T, uint32_t G, uint64_t n, uint32_t k) {
    const double e = (double)n * k / ((double)T * G);
    uint64_t cap = (uint64_t)(e + 8.0 * std::sqrt(e) + 64.0);
    cap = (cap + 7) & ~7ull;
    return (uint32_t)std::min<uint64_t>(cap, 0xFFFFFFC0ull);
}

// The two-level build (see bloom_rebin_kernel): per pass (`chunk` keys), the bin
// kernel into super tiles and the re-bin into fine tiles for each of its
// NB_SUBPASSES sub-passes (the fine buckets accumulate), then the tile kernel on the
// fine tiles.  E1: pass-1 entry type (Pack5 or uint32_t); t2 comes with its capacity
// in entries for `chunk` keys.
//
// NB_OVERLAP: the sub-passes pipelined over two streams -- every bin kernel
// (VALU-bound) on the build stream, every re-bin and tile kernel (HBM-bound) on the
// workspace's aux stream, so that sub-pass s's re-bin runs beside sub-pass s+1's
// bin kernel (a re-bin block fits a CU beside a bin block; a 128 KB tile block does
// not, so a pass's first bin kernel waits for the previous pass's tile kernel unless
// NB_OVERLAP & 4).  Sub-pass parity selects the pass-1 buckets and super-tile
// cursors, pass parity the spill scratch; the fine buckets and cursors are used on
// the aux stream only, in order.  NB_OVERLAP & 3 == 2: the aux stream at high priority.
template <int FLAVOR, int LAYOUT, int KPT, int NT, bool STAGE, int KR, int KX, typename E1>
int launch_two_level(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                     const FilterConsts &c, uint64_t *words, bool overwrite, hipStream_t st,
                     uint64_t chunk, const TileCfg &t1e, const TileCfg &t2) {
    constexpr uint64_t kpb = (uint64_t)KPT * NT;
    constexpr bool IN5 = pack_of<E1>() == 5;
    Workspace *ws;
    TileScratch sc;
    int rc;
    if ((rc = get_ws(st, &ws))) return rc;
    std::lock_guard<std::mutex> lk(ws->mu);
    // sub-passes: NB_SUBPASSES, or by policy 2 when the build takes several passes (the
    // C5 step at N = 1: 34.6 -> 33.6 ms pipelined, profiles/r03_ab_c5_subpasses.txt)
    // and 1 for a single pass (one rank's share at N = 8: 4.38-4.43 vs 4.48-4.51 ms,
    // profiles/r04_ab_c5r_subpasses.txt)
    const uint64_t kn = knob(nb::kKnobSubpasses);
    const uint64_t nsub = kn ? std::min<uint64_t>(kn, 64) : (n > chunk ? 2 : 1);
    const uint64_t sub = std::min<uint64_t>(chunk, ((chunk + nsub - 1) / nsub + kpb - 1) / kpb * kpb);
    const uint64_t spp = (chunk + sub - 1) / sub;  // sub-passes per pass
    // pass-1 capacity in units: the entries' plus <= 4 pad slots per bin block of
    // the shard, / 5
    const uint64_t nblk = (sub + kpb - 1) / kpb;
    TileCfg t1 = t1e;
    t1.cap = cap_for(t1.T, t1.G, sub, c.k);
    if (IN5) {
        const uint64_t bps = (nblk + t1.G - 1) / t1.G;
        const uint64_t capu = ((uint64_t)t1.cap + 4 * bps + 4) / 5;
        t1.cap = (uint32_t)std::min<uint64_t>((capu + 7) & ~7ull, 0xFFFFFFC0ull);
    }
    const uint32_t span_units = kRebinThreads * (IN5 ? rebin_ept<true>() / 5 : rebin_ept<false>());
    const uint32_t rebin_x = (uint32_t)(((uint64_t)t1.cap * t1.G + span_units - 1) / span_units);
    // fine entries packed three per word (2^ts2 <= 2^21): capacity in words, the
    // entries' plus <= 2 pad slots per re-bin block of the shard (every sub-pass's)
    const bool pack = t2.ts <= 20 && knob(nb::kKnobPack) != 0;
    TileCfg t2p = t2;
    if (pack) {
        const uint64_t bps = ((uint64_t)rebin_x * spp + t2.G - 1) / t2.G;
        const uint64_t capw = ((uint64_t)t2.cap + 2 * bps + 2) / 3;
        t2p.cap = (uint32_t)std::min<uint64_t>((capw + 7) & ~7ull, 0xFFFFFFC0ull);
    }
    const size_t e2 = pack ? 8 : 4;
    const size_t b1_bytes = (size_t)t1.T * t1.G * t1.cap * sizeof(E1);
    if ((rc = ws_reserve(*ws, c.fm.m, b1_bytes, &sc, (size_t)t2p.T * t2p.G * t2p.cap * e2)))
        return rc;
    const uint64_t ov = n > sub ? knob(nb::kKnobOverlap) : 0;
    if (ov && (rc = ws_reserve_alt(*ws, c.fm.m, b1_bytes, (ov & 3) >= 2 ? 1 : 0))) return rc;
    size_t sort_bytes = kpb * c.k * 4;
    if (IN5) sort_bytes += (size_t)t1.T * 16;  // <= 4 pad slots per run
    if (STAGE) sort_bytes = std::max<size_t>(sort_bytes, stage_lds_bytes(NT));
    const size_t bin_lds = (size_t)bin_sort_offset_words(t1.T) * 4 + sort_bytes;
    const size_t rebin_lds = ((size_t)rebin_span<IN5>() + 2 * kSuperFine) * 4;
    const size_t tile_lds = (size_t)t2.w64 * 8 + (2 * kShards + 1) * 4;
    auto bin = bloom_bin_kernel<FLAVOR, LAYOUT, KPT, E1, NT, STAGE, KR, KX>;
    auto rebin = pack ? bloom_rebin_kernel<true, IN5> : bloom_rebin_kernel<false, IN5>;
    auto tile_ow = pack ? tile_kernel_of<uint64_t, true>() : tile_kernel_of<uint32_t, true>();
    auto tile_or = pack ? tile_kernel_of<uint64_t, false>() : tile_kernel_of<uint32_t, false>();
    if ((rc = allow_lds(bin, bin_lds)) || (rc = allow_lds(tile_ow, tile_lds)) ||
        (rc = allow_lds(tile_or, tile_lds)))
        return rc;
    NB_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(rebin),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)rebin_lds));
    const uint64_t nwords = ((uint64_t)c.fm.m + 63) / 64;
    // scratch by parity: [0] the workspace's, [1] the alt block's (NB_OVERLAP only)
    TileScratch fine[2] = {sc, sc}, super[2] = {sc, sc};
    super[0].gcur = super[1].gcur = super_cursors(*ws);
    E1 *b1q[2] = {reinterpret_cast<E1 *>(ws->buckets), reinterpret_cast<E1 *>(ws->buckets)};
    if (ov) {
        fine[1].spill_flag = super[1].spill_flag = ws->zeroed_alt + kCurWords;
        fine[1].spill32 = super[1].spill32 = ws->zeroed_alt + kCurWords + kFlagWords + kSuperCurWords;
        super[1].gcur = ws->zeroed_alt + kCurWords + kFlagWords;
        b1q[1] = reinterpret_cast<E1 *>(ws->buckets_alt);
        // the aux stream starts after everything enqueued on the build stream so far
        NB_HIP(hipEventRecord(ws->ev_start, st));
        NB_HIP(hipStreamWaitEvent(ws->aux, ws->ev_start, 0));
    }
    hipStream_t sa = ov ? ws->aux : st;  // re-bin + tile stream
    void *b2 = ws->buckets2;
    uint64_t s_i = 0, pass = 0;
    for (uint64_t pdone = 0; pdone < n; pdone += chunk, ++pass) {
        const uint64_t pend = std::min(n, pdone + chunk);
        const uint32_t r = ov ? pass & 1 : 0;  // spill scratch of this pass
        for (uint64_t done = pdone; done < pend; done += sub, ++s_i) {
            const uint32_t q = ov ? s_i & 1 : 0;  // pass-1 buckets + super cursors
            const uint64_t cn = std::min(sub, pend - done);
            const uint8_t *ck = offsets ? keys : keys + done * key_len;
            const uint64_t *co = offsets ? offsets + done : nullptr;
            TileScratch s1 = super[q];
            s1.spill_flag = fine[r].spill_flag;
            s1.spill32 = fine[r].spill32;
            if (ov) {
                // b1q[q] and super[q] are free once sub-pass s_i - 2's re-bin (and the
                // cursor reset behind it) is done; the spill scratch r once pass - 2's
                // tile kernel is; and the tile kernel enqueued last is waited for
                if (s_i >= 2) NB_HIP(hipStreamWaitEvent(st, ws->ev_done[q], 0));
                if (pass >= 2 && done == pdone) NB_HIP(hipStreamWaitEvent(st, ws->ev_tile[r], 0));
                if (pass >= 1 && done == pdone && !(ov & 4))  // (NB_OVERLAP & 4: no wait)
                    NB_HIP(hipStreamWaitEvent(st, ws->ev_tile[r ^ 1], 0));
            }
            hipLaunchKernelGGL(bin, dim3((uint32_t)((cn + kpb - 1) / kpb)), dim3(NT), bin_lds, st,
                               ck, co, key_len, cn, c, t1, s1, b1q[q]);
            NB_HIP(hipGetLastError());
            if (ov) {
                NB_HIP(hipEventRecord(ws->ev_bin[q], st));
                NB_HIP(hipStreamWaitEvent(sa, ws->ev_bin[q], 0));
            }
            hipLaunchKernelGGL(rebin, dim3(rebin_x, t1.T), dim3(kRebinThreads), rebin_lds, sa, t1,
                               t2p, s1, fine[r], (const void *)b1q[q], b2);
            NB_HIP(hipGetLastError());
            NB_HIP(hipMemsetAsync(s1.gcur, 0, (size_t)t1.G * t1.T * 4, sa));  // keep them zero
            if (ov) NB_HIP(hipEventRecord(ws->ev_done[q], sa));
        }
        hipLaunchKernelGGL((overwrite && pdone == 0) ? tile_ow : tile_or, dim3(t2.T),
                           dim3(kTileThreads), tile_lds, sa, t2p, fine[r], b2, words, nwords);
        NB_HIP(hipGetLastError());
        if (ov) NB_HIP(hipEventRecord(ws->ev_tile[r], sa));
    }
    // the build stream joins: the filter is complete when its next work runs
    if (ov) NB_HIP(hipStreamWaitEvent(st, ws->ev_tile[(pass - 1) & 1], 0));
    return NB_OK;
}

template <int FLAVOR, int LAYOUT, int KPT, int NT, bool STAGE, int KR, int KX = 0>
int launch_tiled(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                 const FilterConsts &c, uint64_t *words, bool overwrite, hipStream_t st) {
    constexpr uint64_t kpb = (uint64_t)KPT * NT;
    uint64_t chunk = std::min<uint64_t>(n, std::max<uint64_t>(kpb, chunk_keys(n, c.k)));
    TileCfg tc = choose_tiles(c.fm.m, chunk, c.k);
    if (tc.T > 2 * (uint32_t)NT && knob(nb::kKnobTwoLevel) != 0) {
        // passes of <= 5 Gi indices / 4 (C5: 8 passes of 125M keys; measured 35.97-36.19
        // ms vs 36.50-36.86 with 5 passes of 200M, 36.2-36.5 with 10, 37.4 with 16 and
        // 36.9-38.2 with 2-3, profiles/r02_ab_c5_passes.txt); u32 entry indices stay in range
        const uint64_t budget = std::max<uint64_t>(kpb, (5ull << 30) / (4ull * c.k));
        const uint64_t passes = (n + budget - 1) / budget;
        chunk = std::min<uint64_t>(n, std::max<uint64_t>(kpb, (n + passes - 1) / passes));
        if (const uint64_t v = knob(nb::kKnobChunkKeys)) chunk = std::min<uint64_t>(n, v);
        tc = choose_tiles(c.fm.m, chunk, c.k);
        if constexpr (KR > 0) {
            if (two_level_pack5())  // 2^(ts+5)-bit super tiles: 25-bit offsets
                return launch_two_level<FLAVOR, LAYOUT, KPT, NT, STAGE, KR, KX, Pack5>(
                    keys, offsets, key_len, n, c, words, overwrite, st, chunk,
                    super_tiles(tc, c.fm.m, chunk, c.k, 5), tc);
        }
        return launch_two_level<FLAVOR, LAYOUT, KPT, NT, STAGE, KR, KX, uint32_t>(
            keys, offsets, key_len, n, c, words, overwrite, st, chunk,
            super_tiles(tc, c.fm.m, chunk, c.k, 6), tc);
    }
    if (tc.ts <= 16 && knob(nb::kKnobEntry32) == 0)
        return launch_tiled_e<FLAVOR, LAYOUT, KPT, uint16_t, NT, STAGE, KR, KX>(
            keys, offsets, key_len, n, c, words, overwrite, st, chunk, tc);
    if constexpr (KR > 0) {
        // 17-20-bit in-tile offsets: three per 64-bit bucket word (the two-tile
        // tail pads each block-local run to a multiple of 3 with copies of its
        // first entry).  Capacity in words: the entries' plus <= 2 pads per run,
        // i.e. per block of the shard.
        // ... only while two bin blocks still fit a CU's LDS with the pad slots (up to
        // T ~ 1 100: packed C4 at 2^19-bit tiles, T = 1 829, ran 2.47 vs 2.30 ms with
        // one block per CU)
        auto pk_lds_of = [&](uint32_t T) {
            size_t b = (size_t)kpb * c.k * 4 + (size_t)T * 8;
            if (STAGE) b = std::max<size_t>(b, stage_lds_bytes(NT));
            return b + (size_t)bin_sort_offset_words(T) * 4;
        };
        // counted tiles only where the packed tail will take them: every other path
        // finds a tile by shifting (power-of-two tiles)
        const bool can_pack = tc.ts <= 20 && NB_TWO_TILE && knob(nb::kKnobPack) != 0;
        TileCfg ct;
        if (can_pack && counted_tiles(c.fm.m, chunk, c.k, tc, &ct) && ct.T <= 2u * NT &&
            pk_lds_of(ct.T) <= 80 * 1024)
            tc = ct;
        if (can_pack && tc.T <= 2u * NT && pk_lds_of(tc.T) <= 80 * 1024) {
            TileCfg tp = tc;
            const uint64_t nblk = (chunk + kpb - 1) / kpb;
            const uint64_t bps = (nblk + tc.G - 1) / tc.G;
            const uint64_t capw = ((uint64_t)tc.cap + 2 * bps + 2) / 3;
            tp.cap = (uint32_t)std::min<uint64_t>((capw + 7) & ~7ull, 0xFFFFFFC0ull);
            return launch_tiled_e<FLAVOR, LAYOUT, KPT, uint64_t, NT, STAGE, KR, KX>(
                keys, offsets, key_len, n, c, words, overwrite, st, chunk, tp);
        }
    }
    // 32-bit entries: power-of-two tiles by policy; an explicit tile count
    // (NB_TILE_COUNT > 1) applies here too -- every single-level tail finds tiles
    // through the TileCfg's multiplier (tests/test_gpu_buckets.py)
    if (knob(nb::kKnobTileCount) > 1) {
        TileCfg ct;
        if (counted_tiles(c.fm.m, chunk, c.k, tc, &ct)) tc = ct;
    }
    return launch_tiled_e<FLAVOR, LAYOUT, KPT, uint32_t, NT, STAGE, KR, KX>(
        keys, offsets, key_len, n, c, words, overwrite, st, chunk, tc);
}

template <int FLAVOR, int LAYOUT>
int launch_build_l(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                   const FilterConsts &c, uint64_t *words, bool overwrite, hipStream_t st) {
    BuildPath p = path_override();
    const bool tiled_ok = c.k <= 32 && choose_tiles(c.fm.m, 1, c.k).T <= kMaxTiles;
    if (p == BuildPath::kAuto) p = (tiled_ok && n >= 4096) ? BuildPath::kTiled : BuildPath::kAtomic;
    if (p == BuildPath::kTiled && tiled_ok) {
        // keys per block sized so the block's sorted indices fit in LDS; indices
        // and their in-tile ranks kept in registers while k <= 16 (NB_RANK=0: the
        // regenerate-and-recount variant, kept for A/B)
        const bool rank = knob(nb::kKnobRank) != 0;
        // the parity flavours' common k (7 = the reference's k at p = 0.01; 10 = C5's)
        // as a compile-time constant: index loops without per-index k checks, and
        // exactly k rank registers per key (NB_KEXACT=0: the k <= 8 / 16 kernels)
        constexpr bool kParity = FLAVOR != NB_FLAVOR_MURMUR3_X64_128;
        const bool exact = kParity && rank && knob(nb::kKnobKExact) != 0;
        if constexpr (kParity && LAYOUT == kFixed16) {
            // (NB_BIN_WIDE: 768 threads x 3 keys, 2 304 keys per block -- two blocks
            // still fit a CU's LDS at C4's 915 tiles -- at 6 waves per SIMD)
            // Filters of few tiles (C2: 183) run 512 threads x 2 keys, three blocks per
            // CU: the blocks' runs stay long (~39 entries at T = 183) and three resident
            // blocks overlap one block's LDS-bound sort with another's VALU-bound hash
            // (C2 0.137-0.143 -> 0.132-0.136 ms); at C4's 915 tiles the short runs' pads
            // and reservations cost more (1.68 vs 1.44 ms), so larger filters keep the
            // 2 304-key blocks.  NB_BIN_WIDE: 1 this policy, 2 / 3 force either.
            const uint64_t bw = knob(nb::kKnobBinWide);
            if (exact && c.k == 7 && bw != 0) {
                const bool three = bw == 2 || (bw == 1 && choose_tiles(c.fm.m, n, c.k).T <= kThreeBlockTiles);
                if (three)
                    return launch_tiled<FLAVOR, LAYOUT, 2, kBinThreads3, false, 7, 7>(
                        keys, offsets, key_len, n, c, words, overwrite, st);
                return launch_tiled<FLAVOR, LAYOUT, 3, kBinThreads16Wide, false, 7, 7>(
                    keys, offsets, key_len, n, c, words, overwrite, st);
            }
        }
        if constexpr (kParity && (LAYOUT == kFixed16 || LAYOUT == kOffsets)) {
            if (exact && c.k == 7)
                return launch_tiled<FLAVOR, LAYOUT, kBinKPT, kBinThreads, !vec_layout(LAYOUT), 7, 7>(
                    keys, offsets, key_len, n, c, words, overwrite, st);
        }
        if constexpr (kParity && LAYOUT == kFixed32) {
            // (NB_BIN_WIDE: 896 threads x 2 keys, 1 792 keys per block -- two blocks of
            // 10 indices per key still fit a CU's LDS -- amortising the per-block scan,
            // reservations and pads over 1.75x the keys)
            // the same shape policy: 576 threads x 2 keys, three blocks per CU, when the
            // bin kernel's tiles are few -- <= 384 tiles, or the two-level build's 64-128
            // super tiles (C5 33.64-33.82 -> 33.18-33.43 ms, per-rank share 4.57-4.60 ->
            // 4.49-4.51 ms); NB_BIN_WIDE 4 / 3 force either
            const uint64_t bw = knob(nb::kKnobBinWide);
            if (exact && c.k == 10 && bw != 0) {
                const uint32_t T = choose_tiles(c.fm.m, n, c.k).T;
                const bool three = bw == 4 || (bw == 1 && (T <= kThreeBlockTiles ||
                                                           (T > 2u * kBinThreadsWide &&
                                                            knob(nb::kKnobTwoLevel) != 0)));
                if (three)
                    return launch_tiled<FLAVOR, LAYOUT, 2, kBinThreads3Wide, false, 10, 10>(
                        keys, offsets, key_len, n, c, words, overwrite, st);
                return launch_tiled<FLAVOR, LAYOUT, 2, kBinThreadsWide, false, 10, 10>(
                    keys, offsets, key_len, n, c, words, overwrite, st);
            }
            if (exact && c.k == 10)
                return launch_tiled<FLAVOR, LAYOUT, 1, kBinThreads, false, 10, 10>(
                    keys, offsets, key_len, n, c, words, overwrite, st);
        }
        if constexpr (vec_layout(LAYOUT)) {
            if (c.k <= 8)
                return rank ? launch_tiled<FLAVOR, LAYOUT, kBinKPT, kBinThreads, false, 8>(
                                  keys, offsets, key_len, n, c, words, overwrite, st)
                            : launch_tiled<FLAVOR, LAYOUT, kBinKPT, kBinThreads, false, 0>(
                                  keys, offsets, key_len, n, c, words, overwrite, st);
            if (c.k <= 16 && rank)
                return launch_tiled<FLAVOR, LAYOUT, 1, kBinThreads, false, 16>(
                    keys, offsets, key_len, n, c, words, overwrite, st);
            return launch_tiled<FLAVOR, LAYOUT, 1, kBinThreads, false, 0>(
                keys, offsets, key_len, n, c, words, overwrite, st);
        } else {  // variable-length / odd-stride keys: LDS-staged reads, NT keys at a time
            if (c.k <= 8 && rank)
                return launch_tiled<FLAVOR, LAYOUT, kBinKPT, kBinThreads, true, 8>(
                    keys, offsets, key_len, n, c, words, overwrite, st);
            if (c.k <= 16 && rank)
                return launch_tiled<FLAVOR, LAYOUT, 1, kBinThreads, true, 16>(
                    keys, offsets, key_len, n, c, words, overwrite, st);
            return launch_tiled<FLAVOR, LAYOUT, 1, kBinThreads, true, 0>(
                keys, offsets, key_len, n, c, words, overwrite, st);
        }
    }
    return launch_atomic<FLAVOR, LAYOUT>(keys, offsets, key_len, n, c, words, overwrite, st);
}

template <int FLAVOR>
int launch_build_f(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                   const FilterConsts &c, uint64_t *words, bool overwrite, hipStream_t st) {
    if (!offsets && key_len == 16 && (reinterpret_cast<uintptr_t>(keys) & 15) == 0)
        return launch_build_l<FLAVOR, kFixed16>(keys, offsets, key_len, n, c, words, overwrite, st);
    if (!offsets && key_len == 32 && (reinterpret_cast<uintptr_t>(keys) & 15) == 0 &&
        knob(nb::kKnobFixed32) != 0)
        return launch_build_l<FLAVOR, kFixed32>(keys, offsets, key_len, n, c, words, overwrite, st);
    if (!offsets)
        return launch_build_l<FLAVOR, kFixedStride>(keys, offsets, key_len, n, c, words,
                                                    overwrite, st);
    return launch_build_l<FLAVOR, kOffsets>(keys, offsets, key_len, n, c, words, overwrite, st);
}

// Probe tiles: the largest 2^ts <= 2^20 (the tile kernel's LDS copy) that still
// leaves >= 256 tiles; cap per (tile, shard) as the build's.
// E32 buckets also hold one header per run: at most one per bin block and tile.
TileCfg probe_tiles(uint32_t m, uint64_t n_chunk, uint32_t k, bool e32 = false) {
    TileCfg tc;
    uint32_t ts = 12;
    while (ts < 20 && (((uint64_t)m + (1ull << (ts + 1)) - 1) >> (ts + 1)) >= 256) ++ts;
    tc.ts = ts;
    tc.T = (uint32_t)(((uint64_t)m + (1ull << ts) - 1) >> ts);
    tc.G = kShards;
    const double e = (double)n_chunk * k / ((double)tc.T * tc.G);
    const uint64_t hdrs = e32 ? ((n_chunk + kProbeThreads - 1) / kProbeThreads + tc.G - 1) / tc.G : 0;
    uint64_t cap = (uint64_t)(e + 8.0 * std::sqrt(e) + 64.0) + hdrs;
    tc.cap = (uint32_t)std::min<uint64_t>((cap + 7) & ~7ull, 0xFFFFFFC0ull);
    tc.fts = ts;
    tc.mul = tc.fmul = pow2_mul(ts);
    tc.w64 = 1u << (ts - 6);
    return tc;
}

// LDS of the tiled probe's bin kernel: counters, scan and run tables, then the
// block's indices sorted by tile and their keys (or the staged key bytes).  Must fit
// one workgroup's 160 KiB: 32-byte keys at k = 12..16 over 4 096 tiles do not
// (163 968 B at k = 12), and those batches take the lane path.
constexpr size_t kMaxBlockLds = 160 * 1024;
// keff = entries a thread bins: k for the one-round kernel (probe_keff for a round)
// (E32: a 32-bit word per sort slot, plus a header slot per tile)
size_t probe_bin_lds_bytes(uint32_t T, uint32_t keff, bool stage, bool e32 = false) {
    size_t sort_bytes = e32 ? (((size_t)kProbeThreads * keff + T) * 4 + 15) & ~(size_t)15
                            : (size_t)2 * kProbeThreads * keff * 4;
    if (stage) sort_bytes = std::max<size_t>(sort_bytes, stage_lds_bytes(kProbeThreads));
    return (size_t)probe_sort_offset_words(T) * 4 + sort_bytes;
}

// Auto mode's sample (the first kProbeSample keys, probed by the lane kernel) and
// the smallest batch the tiled path is considered for.
constexpr uint32_t kProbeSampleBlocks = 16;                 // one key per lane
constexpr uint64_t kProbeSample = kProbeSampleBlocks * kBlock;  // 4 096 keys
constexpr uint64_t kProbeTiledMin = 1 << 22;
// Auto's choice settled by shape (round 6, measured on shapes the sample thresholds
// were not fitted to, profiles/r06sh_auto_shapes.txt): a filter of at most
// kProbeL2Bits bits fits each XCD's 4 MB L2, and the lane kernel's gathers hit there;
// below kProbeSplitMin keys, or at k = 3 (the first round's two indices leave one),
// the split path stays out -- its five gated launches cost more than it saves -- and
// lane / tiled split at kProbeTwoWayPct present.
constexpr uint64_t kProbeL2Bits = 1ull << 25;
constexpr uint64_t kProbeSplitMin = 1 << 24;
constexpr uint32_t kProbeTwoWayPct = 10;

template <int FLAVOR, int LAYOUT>
int launch_probe_lane(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                      const FilterConsts &c, const uint64_t *words, uint8_t *out, hipStream_t st,
                      const ProbeGate &gate) {
    // (a gated launch, which may be closed, takes a grid of 8 blocks per CU -- full
    // occupancy for its grid-stride loop -- so that a closed one dispatches little)
    const uint32_t grid = gate.decide ? std::min<uint32_t>(grid_for(n), 8 * device_cus()) : grid_for(n);
    hipLaunchKernelGGL((bloom_probe_kernel<FLAVOR, LAYOUT>), dim3(grid), dim3(kBlock), 0, st,
                       keys, offsets, key_len, n, c, reinterpret_cast<const uint32_t *>(words), out,
                       gate);
    NB_HIP(hipGetLastError());
    return NB_OK;
}

// The split tiled probe's first round: each key's first kSplitJ indices.
constexpr int kSplitJ = 2;
constexpr int kSplitKPT = 4;  // keys per thread of the split path's first round
constexpr int kSplitKPT32 = 2;  // the same with E32 entries (a block's keys < 2^11)
constexpr uint32_t kProbeBinBlocksPerCU = 2;  // grid of the probe's looping bin kernels (two resident)
// entries per thread of a probe_bin_kernel launch (its keff)
constexpr uint32_t probe_keff(uint32_t k, int j0, int j1, int pkpt) {
    return (uint32_t)pkpt * ((j1 ? (uint32_t)j1 : k) - (uint32_t)j0);
}

// split: two rounds per pass -- the first bins every key's first kSplitJ indices and
// answers the keys with a zero among them, the second bins the other k - kSplitJ
// indices of the keys still at 1.  An absent key costs ~1 miss store
// in the first round and, one time in four (filter half full), ~(k - 2) / 2 in the
// second, instead of ~k/2; a present key costs the same k entries and two hashes.
template <int FLAVOR, int LAYOUT, int KR>
int launch_probe_tiled(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                       const FilterConsts &c, const uint64_t *words, uint8_t *out, hipStream_t st,
                       const ProbeGate &gate, bool split = false) {
    constexpr bool STAGE = !vec_layout(LAYOUT);
    constexpr int NT = kProbeThreads;
    Workspace *ws;
    TileScratch sc;
    int rc;
    if ((rc = get_ws(st, &ws))) return rc;
    std::lock_guard<std::mutex> lk(ws->mu);
    // E32 (NB_PROBE_ENTRY=32, default): 32-bit entries behind run headers; 64: key << 32 |
    // offset.  E32 keeps a block's keys below 2^(31 - ts): the split path's first round
    // then bins two keys per thread instead of four.
    // E32 entries for the one-round path; the split path keeps 64-bit ones (its first
    // round at two keys per thread and its second round's list lookups per miss cost
    // more than the bytes save: 30 % present 3.93 vs 4.82 ms, absent 4.95 vs 5.32 ms,
    // same box, profiles/r06e_probe_c4.txt).  NB_PROBE_ENTRY: 0 this policy, 32 / 64
    // either format everywhere.
    const uint64_t ek = knob(nb::kKnobProbeEntry);
    const bool e32 = ek == 32 || (ek == 0 && !split);
    const int kpt1 = e32 ? kSplitKPT32 : kSplitKPT;
    const uint32_t ebytes = e32 ? 4u : 8u;
    // chunks whose buckets stay under ~6 GB (entries, headers, answers, with margin:
    // 10 B per index for 64-bit entries, 6 B for 32-bit ones; the split path's rounds
    // bin max(2, k - 2) indices of a key -- C4's 100M keys in one pass either way) --
    // key ids < 2^32
    const uint64_t kc = knob(nb::kKnobProbeChunk);
    const uint64_t kidx = split && c.k > (uint32_t)kSplitJ ? std::max<uint32_t>(kSplitJ, c.k - kSplitJ) : c.k;
    const uint64_t cap_keys = (6ull << 30) / ((e32 ? 6ull : 10ull) * kidx);
    const uint64_t budget = std::max<uint64_t>(NT, kc ? std::min<uint64_t>(kc, cap_keys) : cap_keys);
    const uint64_t passes = (n + budget - 1) / budget;
    const uint64_t chunk = std::max<uint64_t>(1, (n + passes - 1) / passes);
    const TileCfg tc = probe_tiles(c.fm.m, chunk, (uint32_t)kidx, e32);  // (capacity: a round's indices)
    // the split path's second round runs over the compacted list of the first round's
    // survivors -- a count word, then the ids -- kept in the workspace's second bucket
    // array (the two-level build's; unused by the probe) and reserved on every tiled
    // probe with k > 2, so that a warm-up on the one-round path sizes it for a later
    // capture of auto's gated paths
    const bool compact = c.k > (uint32_t)kSplitJ;
    const size_t ids_bytes = compact ? (chunk + 16) * 4 : 0;
    if ((rc = ws_reserve(*ws, c.fm.m, (size_t)tc.T * tc.G * tc.cap * ebytes, &sc, ids_bytes))) return rc;
    sc.vbctr = super_cursors(*ws);  // (the two-level build's; unused by the probe)
    uint32_t *nlive = compact ? reinterpret_cast<uint32_t *>(ws->buckets2) : nullptr;
    sc.nlive = nlive;
    uint32_t *ids = compact ? nlive + 16 : nullptr;
    split = split && c.k > (uint32_t)kSplitJ;
    // the one-round E32 bin kernel takes two keys per thread for 16- / 32-byte keys at
    // k = 7 (2 048 per block: half the blocks' reservations and fixed costs per key) when
    // two such blocks fit a CU
    const uint64_t kptk = knob(nb::kKnobProbeKPT);
    const bool kpt2 = e32 && !split && c.k == 7 && !STAGE && kptk != 1 &&
                      (kptk == 2 || probe_bin_lds_bytes(tc.T, probe_keff(c.k, 0, 0, 2), STAGE, true) <= kMaxBlockLds / 2);
    const size_t bin_lds = probe_bin_lds_bytes(tc.T, probe_keff(c.k, 0, 0, kpt2 ? 2 : 1), STAGE, e32);
    const size_t lds1 = probe_bin_lds_bytes(tc.T, probe_keff(c.k, 0, kSplitJ, kpt1), STAGE, e32);
    const size_t lds2 = probe_bin_lds_bytes(tc.T, probe_keff(c.k, kSplitJ, 0, 1), STAGE, e32);
    if (bin_lds > kMaxBlockLds || (split && lds1 > kMaxBlockLds))
        return fail(NB_ERR_UNSUPPORTED, "tiled probe: LDS of the shape");
    const size_t tile_lds = ((size_t)1 << (tc.ts - 3)) + (2 * kShards + 1) * 4;
    using BinFn = void (*)(const uint8_t *, const uint64_t *, uint32_t, uint64_t, FilterConsts, TileCfg,
                           TileScratch, uint64_t *, const uint64_t *, uint8_t *, ProbeGate, const uint32_t *,
                           const uint32_t *);
    // gated launches (auto; possibly closed) take the looping bin kernels on a capped
    // grid; the forced-format variants (NB_PROBE_ENTRY=32 split, =64 one-round) exist
    // without the loop only
    const bool loop = gate.decide != nullptr;
    using LoopFn = void (*)(ProbeBinArgs);
    BinFn bin, bin1, bin2;
    LoopFn lbin = nullptr, lbin1 = nullptr, lbin2 = nullptr;
    if (e32) {
        if (kpt2 && KR == 8 && !STAGE) {  // (k = 7 exactly: index loops without k checks, 7 rank registers)
            bin = probe_bin_kernel<FLAVOR, LAYOUT, false, 7, 0, 7, false, 2, false, true>;
            lbin = probe_bin_loop_kernel<FLAVOR, LAYOUT, false, 7, 0, 7, false, 2, false, true>;
        } else {
            bin = probe_bin_kernel<FLAVOR, LAYOUT, STAGE, KR, 0, 0, false, 1, false, true>;
            lbin = probe_bin_loop_kernel<FLAVOR, LAYOUT, STAGE, KR, 0, 0, false, 1, false, true>;
        }
        bin1 = probe_bin_kernel<FLAVOR, LAYOUT, STAGE, KR, 0, kSplitJ, false, kSplitKPT32, false, true>;
        bin2 = probe_bin_kernel<FLAVOR, LAYOUT, STAGE, KR, kSplitJ, 0, true, 1, true, true>;
    } else {
        bin = probe_bin_kernel<FLAVOR, LAYOUT, STAGE, KR>;
        bin1 = probe_bin_kernel<FLAVOR, LAYOUT, STAGE, KR, 0, kSplitJ, false, kSplitKPT>;
        bin2 = probe_bin_kernel<FLAVOR, LAYOUT, STAGE, KR, kSplitJ, 0, true, 1, true>;
        lbin1 = probe_bin_loop_kernel<FLAVOR, LAYOUT, STAGE, KR, 0, kSplitJ, false, kSplitKPT>;
        lbin2 = probe_bin_loop_kernel<FLAVOR, LAYOUT, STAGE, KR, kSplitJ, 0, true, 1, true>;
    }
    const bool looping = loop && (split ? lbin1 != nullptr : lbin != nullptr);
    auto tile = probe_tile_kernel<kTileThreads>;
    auto tile32 = probe_tile32_kernel<kTileThreads, false>;
    auto tile32i = probe_tile32_kernel<kTileThreads, true>;
    if ((rc = allow_lds(bin, bin_lds)) || (split && (rc = allow_lds(bin1, lds1))) ||
        (split && (rc = allow_lds(bin2, lds2))) || (lbin && (rc = allow_lds(lbin, bin_lds))) ||
        (split && lbin1 && (rc = allow_lds(lbin1, lds1))) || (split && lbin2 && (rc = allow_lds(lbin2, lds2))) ||
        (rc = e32 ? allow_lds(tile32, tile_lds) : allow_lds(tile, tile_lds)) ||
        (e32 && split && (rc = allow_lds(tile32i, tile_lds))) ||
        (split && compact && (rc = allow_lds(probe_compact_kernel, kCompactLds))))
        return rc;
    const uint64_t nwords = ((uint64_t)c.fm.m + 63) / 64;
    uint64_t *bk = reinterpret_cast<uint64_t *>(ws->buckets);
    // the looping bin kernels (gated launches) run a grid of kProbeBinBlocksPerCU per CU
    // (NB_PROBE_BIN_GRID: that many instead), a multiple of their kVbClasses counter
    // classes; every other launch one workgroup per bin block
    const uint64_t gk = knob(nb::kKnobProbeBinGrid);
    const uint64_t bin_grid_cap =
        looping ? std::max<uint64_t>(kVbClasses, (uint64_t)device_cus() * (gk ? gk : kProbeBinBlocksPerCU) /
                                                     kVbClasses * kVbClasses)
                : ~0ull;
    for (uint64_t done = 0; done < n; done += chunk) {
        const uint64_t cn = std::min(chunk, n - done);
        const uint8_t *ck = offsets ? keys : keys + done * key_len;
        const uint64_t *co = offsets ? offsets + done : nullptr;
        for (int round = 0; round < (split ? 2 : 1); ++round) {
            auto b = !split ? bin : round == 0 ? bin1 : bin2;
            const uint64_t kpb = split && round == 0 ? (uint64_t)NT * kpt1 : kpt2 ? 2ull * NT : NT;
            if (round == 1 && compact) {  // the survivors of round one (*nlive zeroed by
                                          // round one's tile kernel)
                const uint64_t per = (uint64_t)kCompactThreads * kCompactPer;
                const uint64_t cgrid = std::min<uint64_t>((cn + per - 1) / per, loop ? device_cus() : ~0ull);
                hipLaunchKernelGGL(probe_compact_kernel, dim3((uint32_t)cgrid),
                                   dim3(kCompactThreads), kCompactLds, st, out + done, (uint32_t)cn, ids, nlive,
                                   gate);
                NB_HIP(hipGetLastError());
            }
            // (a capped grid is a multiple of kVbClasses: its counter classes are equal)
            const uint64_t bgrid = std::min<uint64_t>((cn + kpb - 1) / kpb, bin_grid_cap);
            const size_t blds = !split ? bin_lds : round == 0 ? lds1 : lds2;
            if (looping) {
                ProbeBinArgs pa{ck, co, cn, out + done, bk, words, ids, nlive, key_len, 0, c, tc, sc, gate};
                hipLaunchKernelGGL((!split ? lbin : round == 0 ? lbin1 : lbin2), dim3((uint32_t)bgrid), dim3(NT),
                                   blds, st, pa);
            } else {
                hipLaunchKernelGGL(b, dim3((uint32_t)bgrid), dim3(NT), blds, st, ck, co, key_len, cn, c, tc, sc, bk,
                                   words, out + done, gate, ids, nlive);
            }
            NB_HIP(hipGetLastError());
            if (!e32)
                hipLaunchKernelGGL(tile, dim3(tc.T), dim3(kTileThreads), tile_lds, st, tc, sc,
                                   (const uint64_t *)bk, words, nwords, out + done, gate, (uint32_t)cn);
            else
                hipLaunchKernelGGL(round == 1 ? tile32i : tile32, dim3(tc.T), dim3(kTileThreads), tile_lds, st,
                                   tc, sc, (const uint32_t *)bk, words, nwords, out + done, gate, (uint32_t)kpb,
                                   (const uint32_t *)ids, (uint32_t)cn);
            NB_HIP(hipGetLastError());
        }
    }
    return NB_OK;
}

// The path of a batch probe (NB_PROBE_PATH: 0 auto, 1 lane, 2 tiled, 3 split): lane
// for small batches, k > 8 (k > 16 for 32-byte keys) and the non-parity MurmurHash3
// flavour; auto probes a sample with the lane kernel first and lets its hit rate pick
// one of the three paths for the rest (ProbeGate), without a host round trip.
template <int FLAVOR, int LAYOUT>
int launch_probe_l(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                   const FilterConsts &c, const uint64_t *words, uint8_t *out, hipStream_t st) {
    const uint64_t path = knob(nb::kKnobProbePath);
    constexpr bool kTiledLayout = LAYOUT != kFixedStride && FLAVOR != NB_FLAVOR_MURMUR3_X64_128;
    const uint32_t kmax = LAYOUT == kFixed32 ? 16u : 8u;
    // (the bin kernels' LDS in both entry formats: auto may launch either)
    const uint32_t pT = probe_tiles(c.fm.m, n, c.k).T;
    const bool tiled_ok = kTiledLayout && c.k <= kmax && pT <= kMaxTiles &&
                          probe_bin_lds_bytes(pT, c.k, !vec_layout(LAYOUT), false) <= kMaxBlockLds &&
                          probe_bin_lds_bytes(pT, c.k, !vec_layout(LAYOUT), true) <= kMaxBlockLds;
    const ProbeGate none{nullptr, nullptr, 0, 0, 0};
    // the split path takes part in auto's choice where the tiled path does (k > 2), on
    // batches of kProbeSplitMin keys or more and k > 3 -- or wherever NB_PROBE_SPLIT_PCT
    // is set.  NB_PROBE_TILED_PCT set (non-zero) is honoured as the threshold of the
    // tiled path; at 0 it is the policy: split_tiled_pct when the split path takes part,
    // kProbeTwoWayPct where it is left out (by the policy or NB_PROBE_SPLIT_PCT > 100),
    // 30 at k <= 2 (not measured since round 4).  A split threshold at or above the tiled one leaves the two-way choice
    // (ADVICE r05).
    constexpr bool kVec = vec_layout(LAYOUT);
    const uint64_t tpk = knob(nb::kKnobProbeTiledPct), spk = knob(nb::kKnobProbeSplitPct);
    const bool split_out = c.k <= (uint32_t)kSplitJ || (!spk && (c.k <= 3 || n < kProbeSplitMin));
    uint32_t pct = tpk ? (uint32_t)std::min<uint64_t>(tpk, 101) : c.k <= (uint32_t)kSplitJ ? 30u : kProbeTwoWayPct;
    uint32_t split_pct = split_out ? 101u
                         : spk ? (uint32_t)std::min<uint64_t>(spk, 101) : split_pct_policy(c.k, kVec);
    if (split_pct <= 100) {
        const uint32_t to_tiled = tpk ? pct : split_tiled_pct(c.k, kVec);
        if (split_pct < to_tiled) pct = to_tiled;
        else split_pct = 101;
    }
    if (path == 1 || !tiled_ok || (path == 0 && (n < kProbeTiledMin || c.fm.m <= kProbeL2Bits)))
        return launch_probe_lane<FLAVOR, LAYOUT>(keys, offsets, key_len, n, c, words, out, st, none);
    auto tiled = [&](const uint8_t *k_, const uint64_t *o_, uint64_t n_, uint8_t *out_,
                     const ProbeGate &g, bool split = false) -> int {
        if constexpr (kTiledLayout) {
            if (c.k <= 8)
                return launch_probe_tiled<FLAVOR, LAYOUT, 8>(k_, o_, key_len, n_, c, words, out_, st, g, split);
            if constexpr (LAYOUT == kFixed32)
                return launch_probe_tiled<FLAVOR, LAYOUT, 16>(k_, o_, key_len, n_, c, words, out_, st, g,
                                                              split);
        }
        return fail(NB_ERR_UNSUPPORTED, "tiled probe: unsupported shape");
    };
    if (path == 2 || path == 3) return tiled(keys, offsets, n, out, none, path == 3);
    // auto: the sample (one key per lane, one count per block), then every path
    // launched behind it, each gated on the sample's counts on the device (ProbeGate):
    // the closed paths' blocks return at once, and no host wait (round 6, VERDICT r05
    // item 6; the bin kernels' capped grids keep a closed launch to a few thousand
    // blocks).  NB_PROBE_HOST_PICK=1 (outside stream capture only): rounds 3-5's host
    // read-back instead -- the counts land in host-mapped memory, the host waits for
    // the sample and launches only the chosen path.
    Workspace *ws;
    int rc;
    if ((rc = get_ws(st, &ws))) return rc;
    {
        std::lock_guard<std::mutex> lk(ws->mu);
        if (!ws->probe_hits) NB_HIP(hipMalloc(&ws->probe_hits, kProbeSampleBlocks * 4));
        if (!ws->probe_hits_host) {
            NB_HIP(hipHostMalloc(&ws->probe_hits_host, kProbeSampleBlocks * 4,
                                 hipHostMallocMapped | hipHostMallocCoherent));
            NB_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&ws->probe_hits_map),
                                           ws->probe_hits_host, 0));
        }
        if (!ws->ev_probe) NB_HIP(hipEventCreateWithFlags(&ws->ev_probe, hipEventDisableTiming));
    }
    const uint64_t S = kProbeSample;
    const uint8_t *rk = offsets ? keys : keys + S * key_len;
    const uint64_t *ro = offsets ? offsets + S : nullptr;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    NB_HIP(hipStreamIsCapturing(st, &cs));
    const bool host_pick = cs == hipStreamCaptureStatusNone && knob(nb::kKnobProbeHostPick) != 0;
    // with the host pick the sample's blocks write their counts straight into
    // host-mapped memory (no copy launch); else into device words the gated launches read
    const ProbeGate sample{host_pick ? ws->probe_hits_map : ws->probe_hits, nullptr, kProbeSampleBlocks,
                           (uint32_t)S, 1};
    hipLaunchKernelGGL((bloom_probe_kernel<FLAVOR, LAYOUT>), dim3(kProbeSampleBlocks), dim3(kBlock), 0,
                       st, keys, offsets, key_len, S, c, reinterpret_cast<const uint32_t *>(words),
                       out, sample);
    NB_HIP(hipGetLastError());
    if (host_pick) {
        NB_HIP(hipEventRecord(ws->ev_probe, st));
        NB_HIP(hipEventSynchronize(ws->ev_probe));
        volatile uint32_t *hs = ws->probe_hits_host;
        uint64_t h = 0;
        for (uint32_t b = 0; b < kProbeSampleBlocks; ++b) h += hs[b];
        const uint32_t pick = probe_pick(h, S, pct, split_pct);  // as gate_open decides
        if (pick != 1) return tiled(rk, ro, n - S, out + S, none, pick == 3);
        return launch_probe_lane<FLAVOR, LAYOUT>(rk, ro, key_len, n - S, c, words, out + S, st, none);
    }
    const ProbeGate lane{nullptr, ws->probe_hits, kProbeSampleBlocks, (uint32_t)S, 1, pct, split_pct};
    const ProbeGate tile{nullptr, ws->probe_hits, kProbeSampleBlocks, (uint32_t)S, 2, pct, split_pct};
    const ProbeGate splt{nullptr, ws->probe_hits, kProbeSampleBlocks, (uint32_t)S, 3, pct, split_pct};
    if ((rc = launch_probe_lane<FLAVOR, LAYOUT>(rk, ro, key_len, n - S, c, words, out + S, st, lane)))
        return rc;
    if ((rc = tiled(rk, ro, n - S, out + S, tile))) return rc;
    if (split_pct <= 100) return tiled(rk, ro, n - S, out + S, splt, true);
    return NB_OK;
}

template <int FLAVOR>
int launch_probe_f(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                   const FilterConsts &c, const uint64_t *words, uint8_t *out, hipStream_t st) {
    if (!offsets && key_len == 16 && (reinterpret_cast<uintptr_t>(keys) & 15) == 0)
        return launch_probe_l<FLAVOR, kFixed16>(keys, offsets, key_len, n, c, words, out, st);
    if (!offsets && key_len == 32 && (reinterpret_cast<uintptr_t>(keys) & 15) == 0)
        return launch_probe_l<FLAVOR, kFixed32>(keys, offsets, key_len, n, c, words, out, st);
    if (!offsets)
        return launch_probe_l<FLAVOR, kFixedStride>(keys, offsets, key_len, n, c, words, out, st);
    return launch_probe_l<FLAVOR, kOffsets>(keys, offsets, key_len, n, c, words, out, st);
}

std::atomic<uint64_t> g_device_builds{0};  // nb_device_build_count()

int launch_build(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                 uint32_t m, uint32_t k, uint64_t seed, int flavor, uint64_t *words,
                 bool overwrite, hipStream_t st) {
    if (n == 0 || k == 0) {
        if (overwrite && m) NB_HIP(hipMemsetAsync(words, 0, (((size_t)m + 63) / 64) * 8, st));
        return NB_OK;
    }
    if (nb::knob_take(nb::kKnobFailBuilds))  // fault injection (drop-in fallback tests)
        return fail(NB_ERR_HIP, "injected device build failure (NB_FAIL_BUILDS)");
    FilterConsts c = nb::make_consts(m, k, seed, (uint32_t)flavor);
    if (!offsets) nb::set_fixed_len(c, key_len);
    if (knob(nb::kKnobFpMod) == 0) c.fm.fp = 0;  // A/B: integer remainders only
    g_device_builds.fetch_add(1, std::memory_order_relaxed);
    if (flavor == NB_FLAVOR_MURMUR3_X64_128)
        return launch_build_f<NB_FLAVOR_MURMUR3_X64_128>(keys, offsets, key_len, n, c, words,
                                                         overwrite, st);
    return flavor == NB_FLAVOR_MSVC_FNV1A
               ? launch_build_f<NB_FLAVOR_MSVC_FNV1A>(keys, offsets, key_len, n, c, words,
                                                      overwrite, st)
               : launch_build_f<NB_FLAVOR_LIBSTDCXX>(keys, offsets, key_len, n, c, words,
                                                     overwrite, st);
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
    if (!offsets) nb::set_fixed_len(c, key_len);
    if (knob(nb::kKnobFpMod) == 0) c.fm.fp = 0;
    if (flavor == NB_FLAVOR_MURMUR3_X64_128)
        return launch_probe_f<NB_FLAVOR_MURMUR3_X64_128>(keys, offsets, key_len, n, c, words, out, st);
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
    {
        std::lock_guard<std::mutex> lk(d.mu);  // the first callers on a device race here
        if (!d.init) {
            NB_HIP(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
            d.init = true;
        }
    }
    *out = &d;
    return NB_OK;
}

inline size_t nwords_of(uint32_t m) { return ((size_t)m + 63) / 64; }

size_t keys_bytes(const uint64_t *offsets, uint32_t key_len, uint64_t n) {
    return offsets ? (size_t)offsets[n] : (size_t)n * key_len;
}

}  // namespace

// Internal entry points for the other translation units of the library
// (bloom_stream.cpp): the device build on a caller's stream, and the error slot.
int nb_internal_build(const uint8_t *d_keys, const uint64_t *d_offsets, uint32_t key_len,
                      uint64_t n, uint32_t m, uint32_t k, uint64_t seed, int flavor,
                      uint64_t *d_words, bool overwrite, hipStream_t st) {
    return launch_build(d_keys, d_offsets, key_len, n, m, k, seed, flavor, d_words, overwrite, st);
}
int nb_internal_fail(int code, const char *msg) { return fail(code, msg); }

// Launches or_gather_kernel over the sources in groups (stream-ordered).
int nb_internal_or_gather(uint64_t *dst, const uint64_t *const *srcs, uint32_t nsrc, uint64_t nwords,
                          hipStream_t st) {
    for (uint32_t b = 0; b < nsrc && nwords; b += kGatherSrcs) {
        GatherSrcs g{};
        const uint32_t cnt = std::min<uint32_t>(kGatherSrcs, nsrc - b);
        for (uint32_t i = 0; i < cnt; ++i) g.p[i] = srcs[b + i];
        hipLaunchKernelGGL(or_gather_kernel, dim3(grid_for(nwords)), dim3(kBlock), 0, st, dst, g,
                           cnt, nwords);
        NB_HIP(hipGetLastError());
    }
    return NB_OK;
}
void nb_internal_stream_shutdown();  // bloom_stream.cpp: releases the builders' slot pool

// =================================================================== C ABI ==

extern "C" {

int nb_abi_version(void) { return NB_ABI_VERSION; }

int nb_device_count(void) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) return 0;
    return c;
}

const char *nb_last_error(void) { return g_last_error.c_str(); }

uint64_t nb_device_build_count(void) { return g_device_builds.load(std::memory_order_relaxed); }

int nb_shutdown(void) {
    {
        std::lock_guard<std::mutex> lk(g_ws_mu);
        for (Workspace *w : g_ws) {
            (void)hipSetDevice(w->dev);
            (void)hipStreamSynchronize(w->st);
            if (w->zeroed) (void)hipFree(w->zeroed);
            if (w->buckets) (void)hipFree(w->buckets);
            if (w->buckets2) (void)hipFree(w->buckets2);
            if (w->aux) {
                (void)hipStreamSynchronize(w->aux);
                (void)hipStreamDestroy(w->aux);
            }
            for (hipEvent_t e : {w->ev_bin[0], w->ev_bin[1], w->ev_done[0], w->ev_done[1],
                                 w->ev_tile[0], w->ev_tile[1], w->ev_start})
                if (e) (void)hipEventDestroy(e);
            if (w->zeroed_alt) (void)hipFree(w->zeroed_alt);
            if (w->buckets_alt) (void)hipFree(w->buckets_alt);
            if (w->probe_hits) (void)hipFree(w->probe_hits);
            if (w->probe_hits_host) (void)hipHostFree(w->probe_hits_host);
            if (w->ev_probe) (void)hipEventDestroy(w->ev_probe);
            delete w;
        }
        g_ws.clear();
    }
    nb_internal_stream_shutdown();
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
    // the streaming builder (bloom_stream.cpp): the current words go up once,
    // the keys chunk by chunk with every chunk's build overlapping the next upload
    int rc = check_common(n, m, flavor, keys, words);
    if (rc || n == 0 || k == 0) return rc;
    nb_builder *b = nullptr;
    if ((rc = nb_builder_create(m, k, h2_seed, flavor, words, device, &b))) return rc;
    if (!(rc = nb_builder_add_batch(b, keys, offsets, key_len, n))) rc = nb_builder_finish(b, words);
    const int rd = nb_builder_destroy(b);
    return rc ? rc : rd;
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
    return launch_build(d_keys, d_offsets, key_len, n, m, k, h2_seed, flavor, d_words, false,
                        (hipStream_t)stream);
}

int nb_build_device_ex(const uint8_t *d_keys, const uint64_t *d_offsets, uint32_t key_len,
                       uint64_t n, uint32_t m, uint32_t k, uint64_t h2_seed, int flavor,
                       uint64_t *d_words, uint32_t flags, void *stream) {
    if (flags & ~(uint32_t)NB_BUILD_OVERWRITE) return fail(NB_ERR_ARG, "unknown flags");
    const bool overwrite = (flags & NB_BUILD_OVERWRITE) != 0;
    if (overwrite && m && !d_words) return fail(NB_ERR_ARG, "NULL words");
    int rc = check_common(n, m, flavor, d_keys, d_words);
    if (rc) return rc;
    return launch_build(d_keys, d_offsets, key_len, n, m, k, h2_seed, flavor, d_words, overwrite,
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

int nb_frame_filter_device(uint32_t m, uint32_t k, double p, uint32_t time_const,
                           uint64_t h2_seed, const uint64_t *d_words, int framing,
                           uint32_t block_size, uint8_t *out, void *stream) {
    if (!out || (m && !d_words)) return fail(NB_ERR_ARG, "NULL buffer");
    if (framing != NB_FRAME_RAW && framing != NB_FRAME_COMP) return fail(NB_ERR_ARG, "framing");
    const size_t body = nb_internal_frame_header(m, k, p, time_const, h2_seed, framing, out);
    const size_t nbytes = (uint32_t)(m + 7u) / 8u;  // the reference's 32-bit (m+7)/8
    hipStream_t st = (hipStream_t)stream;
    if (nbytes) NB_HIP(hipMemcpyAsync(out + body, d_words, nbytes, hipMemcpyDeviceToHost, st));
    const size_t total = nb_framed_filter_size(m, framing, block_size);
    std::memset(out + body + nbytes, '0', total - body - nbytes);
    NB_HIP(hipStreamSynchronize(st));
    return NB_OK;
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
