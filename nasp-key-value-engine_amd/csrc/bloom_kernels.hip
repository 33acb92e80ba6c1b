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

template <int FLAVOR, int LAYOUT>
__global__ __launch_bounds__(kBlock) void bloom_build_kernel(
    const uint8_t *__restrict__ keys, const uint64_t *__restrict__ offsets, uint32_t key_len,
    uint64_t n, FilterConsts c, uint32_t *__restrict__ words32) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        uint64_t h1, h2;
        hashes_of<FLAVOR, LAYOUT>(c, keys, offsets, key_len, i, &h1, &h2);
        const uint32_t m = c.fm.m;
        uint32_t r = nb::mod64(h1, c.fm);
        const uint32_t s2 = nb::mod64(h2, c.fm);
        uint64_t x = h1;
        for (uint32_t j = 0; j < c.k; ++j) {
            if (j) {
                const uint64_t nx = x + h2;
                r = nb::addmod(r, s2, m);
                if (nx < x) r = nb::submod(r, c.c64, m);
                x = nx;
            }
            __hip_atomic_fetch_or(words32 + (r >> 5), 1u << (r & 31), __ATOMIC_RELAXED,
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
        const uint32_t m = c.fm.m;
        uint32_t r = nb::mod64(h1, c.fm);
        const uint32_t s2 = nb::mod64(h2, c.fm);
        uint64_t x = h1;
        uint8_t hit = 1;
        for (uint32_t j = 0; j < c.k; ++j) {
            if (j) {
                const uint64_t nx = x + h2;
                r = nb::addmod(r, s2, m);
                if (nx < x) r = nb::submod(r, c.c64, m);
                x = nx;
            }
            if (!((words32[r >> 5] >> (r & 31)) & 1u)) { hit = 0; break; }
        }
        out[i] = hit;
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

template <int FLAVOR>
int launch_build_f(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                   const FilterConsts &c, uint64_t *words, hipStream_t st) {
    dim3 grid(grid_for(n)), block(kBlock);
    uint32_t *w32 = reinterpret_cast<uint32_t *>(words);
    if (!offsets && key_len == 16 && (reinterpret_cast<uintptr_t>(keys) & 15) == 0)
        hipLaunchKernelGGL((bloom_build_kernel<FLAVOR, kFixed16>), grid, block, 0, st, keys,
                           offsets, key_len, n, c, w32);
    else if (!offsets)
        hipLaunchKernelGGL((bloom_build_kernel<FLAVOR, kFixedStride>), grid, block, 0, st, keys,
                           offsets, key_len, n, c, w32);
    else
        hipLaunchKernelGGL((bloom_build_kernel<FLAVOR, kOffsets>), grid, block, 0, st, keys,
                           offsets, key_len, n, c, w32);
    NB_HIP(hipGetLastError());
    return NB_OK;
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
