// ubench_alu.hip -- diagnostic (not product code): issue rate of the VALU
// instructions the reference hash compiles to on gfx950 (64-bit multiplies by
// a constant = v_mad_u64_u32 + 2 v_mul_lo_u32; shifts; xor; adds).
// Each lane runs 8 independent chains so latency never limits; 8 waves/SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e = (x);                                                 \
        if (e != hipSuccess) {                                              \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                        \
        }                                                                   \
    } while (0)

constexpr int kIters = 2048;
constexpr int kChains = 8;

#define BODY(INSN)                                                                   \
    uint32_t x[kChains];                                                             \
    for (int c = 0; c < kChains; ++c) x[c] = threadIdx.x * 977u + c * 131u + seed;  \
    const uint32_t y = seed | 1u;                                                    \
    for (int i = 0; i < kIters; ++i) {                                               \
        _Pragma("unroll") for (int c = 0; c < kChains; ++c) INSN;                    \
    }                                                                                \
    uint32_t acc = 0;                                                                \
    for (int c = 0; c < kChains; ++c) acc ^= x[c];                                   \
    if (acc == 0x12345678u) out[blockIdx.x] = acc;

__global__ __launch_bounds__(256) void k_mul_lo(uint32_t *out, uint32_t seed) {
    BODY(asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[c]) : "v"(y)))
}
__global__ __launch_bounds__(256) void k_mul_hi(uint32_t *out, uint32_t seed) {
    BODY(asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[c]) : "v"(y)))
}
__global__ __launch_bounds__(256) void k_mul_u24(uint32_t *out, uint32_t seed) {
    BODY(asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[c]) : "v"(y)))
}
__global__ __launch_bounds__(256) void k_xor(uint32_t *out, uint32_t seed) {
    BODY(asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y)))
}
__global__ __launch_bounds__(256) void k_add3(uint32_t *out, uint32_t seed) {
    BODY(asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x[c]) : "v"(y)))
}
// 64-bit ops on register pairs
#define BODY64(INSN)                                                                 \
    uint64_t x[kChains];                                                             \
    for (int c = 0; c < kChains; ++c) x[c] = threadIdx.x * 977ull + c * 131u + seed; \
    const uint32_t y = seed | 1u;                                                    \
    const uint64_t y64 = 0xc6a4a7935bd1e995ull ^ seed;                              \
    for (int i = 0; i < kIters; ++i) {                                               \
        _Pragma("unroll") for (int c = 0; c < kChains; ++c) INSN;                    \
    }                                                                                \
    uint64_t acc = 0;                                                                \
    for (int c = 0; c < kChains; ++c) acc ^= x[c];                                   \
    if (acc == 0x12345678ull) out[blockIdx.x] = (uint32_t)acc;

__global__ __launch_bounds__(256) void k_mad64(uint32_t *out, uint32_t seed) {
    BODY64(asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(x[c]) : "v"(y) : "vcc"))
}
__global__ __launch_bounds__(256) void k_lshr64(uint32_t *out, uint32_t seed) {
    BODY64(asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(x[c])))
}
__global__ __launch_bounds__(256) void k_mul64_c(uint32_t *out, uint32_t seed) {
    BODY64(x[c] = x[c] * y64)
}
__global__ __launch_bounds__(256) void k_lsx_round(uint32_t *out, uint32_t seed) {
    // h = (h ^ shift_mix(w*M)*M) * M with w = h (a dependent chain of hash rounds)
    BODY64(({ uint64_t d = x[c] * 0xc6a4a7935bd1e995ull; d ^= d >> 47; d *= 0xc6a4a7935bd1e995ull;
              x[c] = (x[c] ^ d) * 0xc6a4a7935bd1e995ull; }))
}

// f64 path of a 64-by-32 remainder (bloom_math.h mod64_f64): conversions and FMAs
__global__ __launch_bounds__(256) void k_cvt_f64(uint32_t *out, uint32_t seed) {
    double d[kChains];
    const uint32_t y = seed | 1u;
    for (int i = 0; i < kIters; ++i) {
        _Pragma("unroll") for (int c = 0; c < kChains; ++c)
            asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(d[c]) : "v"(y + c));
    }
    double acc = 0;
    for (int c = 0; c < kChains; ++c) acc += d[c];
    if (acc == 1.5) out[blockIdx.x] = 1;
}
__global__ __launch_bounds__(256) void k_fma64(uint32_t *out, uint32_t seed) {
    double d[kChains];
    for (int c = 0; c < kChains; ++c) d[c] = threadIdx.x * 0.5 + c + seed;
    const double y = 1.0000001, z = 0.25;
    for (int i = 0; i < kIters; ++i) {
        _Pragma("unroll") for (int c = 0; c < kChains; ++c)
            asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[c]) : "v"(y), "v"(z));
    }
    double acc = 0;
    for (int c = 0; c < kChains; ++c) acc += d[c];
    if (acc == 1.5) out[blockIdx.x] = 1;
}
// 64-bit multiply by a constant as three v_mad_u64_u32 (low product, then the two
// cross products accumulated into the high half)
__device__ __forceinline__ uint64_t mul64_mad3(uint64_t x, uint64_t k) {
    uint64_t p, q, r;
    asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p) : "v"((uint32_t)x), "v"((uint32_t)k) : "vcc");
    asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(q) : "v"((uint32_t)(x >> 32)), "v"((uint32_t)k), "v"(p >> 32) : "vcc");
    asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(r) : "v"((uint32_t)x), "v"((uint32_t)(k >> 32)), "v"(q) : "vcc");
    return (p & 0xffffffffull) | (r << 32);
}
__global__ __launch_bounds__(256) void k_mul64_mad3(uint32_t *out, uint32_t seed) {
    BODY64(x[c] = mul64_mad3(x[c], y64))
}

template <class K>
static void run(const char *name, K kern, double ops_per_iter_chain) {
    uint32_t *out;
    CK(hipMalloc(&out, 1 << 20));
    const int blocks = 256 * 8;  // 8 blocks of 256 threads per CU = 8 waves/SIMD
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 3u);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 3u);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    const double lanes = (double)blocks * 256;
    const double ops = lanes * kIters * kChains * ops_per_iter_chain;
    // wave-instructions per SIMD per cycle at 2.4 GHz: 1.0 = one wave64 op per 4 cycles? report raw
    const double wave_insts = ops / 64.0;
    const double per_simd_cycles = best * 1e-3 * 2.4e9;
    printf("%-12s %.4f ms  %.1f Tops/s  %.2f cycles per wave-instruction per SIMD (at 2.4 GHz)\n",
           name, best, ops / (best * 1e-3) / 1e12, per_simd_cycles / (wave_insts / 1024.0));
    CK(hipFree(out));
}

int main() {
    run("xor", k_xor, 1);
    run("add3", k_add3, 1);
    run("mul_u24", k_mul_u24, 1);
    run("mul_lo", k_mul_lo, 1);
    run("mul_hi", k_mul_hi, 1);
    run("mad_u64", k_mad64, 1);
    run("lshr64", k_lshr64, 1);
    run("mul64xC", k_mul64_c, 1);    // ops = 64-bit multiplies
    run("lsx_round", k_lsx_round, 1);  // ops = hash rounds
    run("cvt_f64_u32", k_cvt_f64, 1);
    run("fma_f64", k_fma64, 1);
    run("mul64_mad3", k_mul64_mad3, 1);  // ops = 64-bit multiplies
    return 0;
}
