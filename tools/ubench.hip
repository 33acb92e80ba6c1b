// ubench.hip -- microbenchmarks that size the design of the build kernel on
// gfx950 (not product code).  Prints one line per experiment:
//   name  ms  rate
// Experiments: streaming read, hash-only, global atomic OR (agent / workgroup
// scope, 32/64-bit), plain scattered stores, LDS ds_or throughput.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../nasp-key-value-engine_amd/csrc/bloom_math.h"

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e = (x);                                                   \
        if (e != hipSuccess) {                                                \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);   \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

__device__ __forceinline__ uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void k_fill(uint64_t *p, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) p[i] = sm64(i);
}

__global__ void k_read(const ulonglong2 *p, uint64_t n, uint64_t *sink) {
    uint64_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        ulonglong2 v = p[i];
        acc ^= v.x ^ v.y;
    }
    if (acc == 0x12345) sink[0] = acc;
}

// hash-only: the real fixed-16 hashing + k indices, XOR-folded
__global__ void k_hash(const ulonglong2 *keys, uint64_t n, nb::FilterConsts c, uint64_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        ulonglong2 kv = keys[i];
        nb::LsxState s;
        nb::lsx_begin(c, s, 16);
        nb::lsx_consume(c, s, 0, kv.x, 16);
        nb::lsx_consume(c, s, 1, kv.y, 16);
        uint64_t h1, h2;
        nb::lsx_end(c, s, 16, &h1, &h2);
        uint32_t r = nb::mod64(h1, c.fm), s2 = nb::mod64(h2, c.fm);
        uint64_t x = h1;
        for (uint32_t j = 0; j < c.k; ++j) {
            if (j) {
                uint64_t nx = x + h2;
                r = nb::addmod(r, s2, c.fm.m);
                if (nx < x) r = nb::submod(r, c.c64, c.fm.m);
                x = nx;
            }
            acc ^= r;
        }
    }
    if (acc == 0x12345) sink[0] = acc;
}

template <int SCOPE, int W64>
__global__ void k_atomic(uint32_t *words, uint64_t nops, uint32_t m) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nops; i += gridDim.x * 256ull) {
        uint32_t r = (uint32_t)(sm64(i) % m);
        if (W64)
            __hip_atomic_fetch_or(reinterpret_cast<unsigned long long *>(words) + (r >> 6),
                                  1ull << (r & 63), __ATOMIC_RELAXED, SCOPE);
        else
            __hip_atomic_fetch_or(words + (r >> 5), 1u << (r & 31), __ATOMIC_RELAXED, SCOPE);
    }
}

__global__ void k_store(uint32_t *words, uint64_t nops, uint32_t m) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nops; i += gridDim.x * 256ull) {
        uint32_t r = (uint32_t)(sm64(i) % m);
        words[r >> 5] = r;
    }
}

// sequential-ish 4B stores of nops values (coalesced): write bandwidth reference
__global__ void k_seqstore(uint32_t *out, uint64_t nops) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nops; i += gridDim.x * 256ull)
        out[i] = (uint32_t)i;
}

// LDS OR throughput: each block ORs ops random bits into a TILE-byte LDS tile
template <int TILE>
__global__ __launch_bounds__(1024) void k_lds(uint64_t ops_per_block, uint32_t *out) {
    extern __shared__ uint32_t tile[];
    for (int w = threadIdx.x; w < TILE / 4; w += blockDim.x) tile[w] = 0;
    __syncthreads();
    uint64_t base = (uint64_t)blockIdx.x * ops_per_block;
    for (uint64_t i = threadIdx.x; i < ops_per_block; i += blockDim.x) {
        uint32_t r = (uint32_t)sm64(base + i) & (TILE * 8 - 1);
        atomicOr(&tile[r >> 5], 1u << (r & 31));
    }
    __syncthreads();
    for (int w = threadIdx.x; w < TILE / 4; w += blockDim.x) out[blockIdx.x * (TILE / 4) + w] = tile[w];
}

struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    void start() { CK(hipEventRecord(a)); }
    float stop() {
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms;
    }
};

template <class F>
float best_of(int reps, F f) {
    Timer t;
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        t.start();
        f();
        float ms = t.stop();
        if (ms < best) best = ms;
    }
    return best;
}

int main() {
    const uint64_t n = 10000000;  // C2 keys
    const uint32_t m = 95850584;  // C2 bits
    uint64_t *keys, *sink;
    uint32_t *words, *big;
    CK(hipMalloc(&keys, n * 16 + 64));
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&words, (m / 8) + 64));
    const uint64_t bigops = 70000000;
    CK(hipMalloc(&big, bigops * 4 + 64));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, keys, 2 * n);
    CK(hipDeviceSynchronize());
    dim3 g(256 * 16), b(256);

    float ms = best_of(5, [&] { hipLaunchKernelGGL(k_read, g, b, 0, 0, (const ulonglong2 *)keys, n, sink); });
    printf("read_keys_160MB        %8.4f ms  %8.1f GB/s\n", ms, n * 16 / ms / 1e6);

    nb::FilterConsts c = nb::make_consts(m, 7, 17027509906831645879ull, 0);
    ms = best_of(5, [&] { hipLaunchKernelGGL(k_hash, g, b, 0, 0, (const ulonglong2 *)keys, n, c, sink); });
    printf("hash_only_c2           %8.4f ms  %8.1f Gkeys/s\n", ms, n / ms / 1e6);
    hipLaunchKernelGGL(k_hash, dim3(256 * 64), b, 0, 0, (const ulonglong2 *)keys, n, c, sink);
    ms = best_of(5, [&] { hipLaunchKernelGGL(k_hash, dim3(256 * 64), b, 0, 0, (const ulonglong2 *)keys, n, c, sink); });
    printf("hash_only_c2_g16k      %8.4f ms  %8.1f Gkeys/s\n", ms, n / ms / 1e6);

    const uint64_t nops = 7 * n;
    uint32_t ms_list[] = {m, 1u << 20, 1u << 24, 958505838u};
    for (uint32_t mm : ms_list) {
        uint32_t *w2;
        CK(hipMalloc(&w2, mm / 8 + 64));
        CK(hipMemset(w2, 0, mm / 8 + 64));
        ms = best_of(3, [&] { hipLaunchKernelGGL((k_atomic<__HIP_MEMORY_SCOPE_AGENT, 0>), g, b, 0, 0, w2, nops, mm); });
        printf("atomic32_agent m=%-10u %8.4f ms  %8.2f Gops/s\n", mm, ms, nops / ms / 1e6);
        ms = best_of(3, [&] { hipLaunchKernelGGL((k_atomic<__HIP_MEMORY_SCOPE_WORKGROUP, 0>), g, b, 0, 0, w2, nops, mm); });
        printf("atomic32_wg    m=%-10u %8.4f ms  %8.2f Gops/s\n", mm, ms, nops / ms / 1e6);
        ms = best_of(3, [&] { hipLaunchKernelGGL((k_atomic<__HIP_MEMORY_SCOPE_AGENT, 1>), g, b, 0, 0, w2, nops, mm); });
        printf("atomic64_agent m=%-10u %8.4f ms  %8.2f Gops/s\n", mm, ms, nops / ms / 1e6);
        ms = best_of(3, [&] { hipLaunchKernelGGL(k_store, g, b, 0, 0, w2, nops, mm); });
        printf("store32_rand   m=%-10u %8.4f ms  %8.2f Gops/s\n", mm, ms, nops / ms / 1e6);
        CK(hipFree(w2));
    }
    ms = best_of(3, [&] { hipLaunchKernelGGL(k_seqstore, g, b, 0, 0, big, bigops); });
    printf("store32_seq_280MB      %8.4f ms  %8.1f GB/s\n", ms, bigops * 4 / ms / 1e6);

    uint32_t *lout;
    CK(hipMalloc(&lout, 4096ull * 65536));
    const uint64_t opb = 1 << 20;
    ms = best_of(3, [&] { hipLaunchKernelGGL((k_lds<65536>), dim3(1024), dim3(1024), 65536, 0, opb, lout); });
    printf("lds_or_64KB 1024x1M    %8.4f ms  %8.1f Gops/s\n", ms, 1024.0 * opb / ms / 1e6);
    ms = best_of(3, [&] { hipLaunchKernelGGL((k_lds<131072>), dim3(512), dim3(1024), 131072, 0, opb, lout); });
    printf("lds_or_128KB 512x1M    %8.4f ms  %8.1f Gops/s\n", ms, 512.0 * opb / ms / 1e6);
    ms = best_of(3, [&] { hipLaunchKernelGGL((k_lds<32768>), dim3(2048), dim3(1024), 32768, 0, opb, lout); });
    printf("lds_or_32KB 2048x1M    %8.4f ms  %8.1f Gops/s\n", ms, 2048.0 * opb / ms / 1e6);
    CK(hipDeviceSynchronize());
    return 0;
}
