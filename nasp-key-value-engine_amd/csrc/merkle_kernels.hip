// merkle_kernels.hip -- gfx950 kernels of the SSTable Merkle tree built beside the
// filter on the same flush (reference SSTable/SSTable.cpp:29-40,
// SSTableRaw.cpp:238,392-397; MerkleTree/merkle.cpp:7-55), and their C ABI
// (include/nasp_bloom.h, nb_merkle*).
//
//   leaves : one lane per record, H(record) with the filter's word-stream hash
//            (bloom_math.h hash1_aligned_words), into tree[0..n)
//   levels : one 256-thread block per 512 nodes, up to 3 levels per launch in
//            LDS: parent i = H(to_string(node 2i) ++ to_string(node 2i+1)), the
//            last node of an odd level paired with itself (merkle.cpp:44-48);
//            every level is stored into the tree (generateProof's treeLevels)
// Integer/byte work; HBM-bound at the leaves (record bytes read once), VALU-bound
// in the levels (decimal conversion + hash of <= 40 bytes per parent).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <string>

#include "../../include/nasp_bloom.h"
#include "bloom_math.h"
#include "nb_knobs.h"

int nb_internal_fail(int code, const char *msg);  // bloom_kernels.hip

namespace {

// Level-kernel geometry (tools/ubench_merkle.hip, C2's 10M records): a block
// halves its busy threads every level, so long in-LDS chains idle most lanes --
// 1 024 threads x 11 levels took 0.356 ms, 256 threads x 3 levels 0.224 ms.
#ifndef NB_MERKLE_THREADS
#define NB_MERKLE_THREADS 256
#endif
#ifndef NB_MERKLE_SUBLEVELS
#define NB_MERKLE_SUBLEVELS 3
#endif
constexpr int kLeafBlock = 256;
constexpr int kLevelThreads = NB_MERKLE_THREADS;
constexpr int kLevelSpan = 2 * kLevelThreads;  // nodes read per block
constexpr int kMaxSub = NB_MERKLE_SUBLEVELS;   // levels per launch (<= log2(kLevelSpan))

template <int FLAVOR, bool OFFSETS>
__global__ __launch_bounds__(kLeafBlock) void merkle_leaf_kernel(
    const uint8_t *__restrict__ data, const uint64_t *__restrict__ offsets, uint32_t rec_len,
    uint64_t n, uint64_t *__restrict__ leaves) {
    const uint64_t stride = (uint64_t)gridDim.x * kLeafBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kLeafBlock + threadIdx.x; i < n; i += stride) {
        const uint64_t b = OFFSETS ? offsets[i] : i * (uint64_t)rec_len;
        const uint32_t len = OFFSETS ? (uint32_t)(offsets[i + 1] - b) : rec_len;
        const uintptr_t addr = reinterpret_cast<uintptr_t>(data + b);
        const uint32_t a = (uint32_t)(addr & 7);
        const uint64_t *q = reinterpret_cast<const uint64_t *>(addr - a);
        auto load = [q](uint32_t j) { return q[j]; };
        leaves[i] = nb::hash1_aligned_words<FLAVOR>(load, a, len);
    }
}

struct LevelPlan {
    uint32_t levels;               // sub-levels this launch computes (1..kMaxSub)
    uint64_t out_off[kMaxSub];     // tree index of each sub-level's first node
};

template <int FLAVOR>
__global__ __launch_bounds__(kLevelThreads) void merkle_level_kernel(
    const uint64_t *__restrict__ in, uint64_t n_in, uint64_t *__restrict__ tree, LevelPlan plan) {
    __shared__ uint64_t node[kLevelSpan];
    const uint32_t tid = threadIdx.x;
    const uint64_t first = (uint64_t)blockIdx.x * kLevelSpan;
    uint32_t cnt = (uint32_t)min<uint64_t>(kLevelSpan, n_in - first);  // block-uniform
    for (uint32_t i = tid; i < cnt; i += kLevelThreads) node[i] = in[first + i];
    __syncthreads();
    for (uint32_t s = 0; s < plan.levels; ++s) {
        // only the grid's last block can hold an odd count: its last node is the
        // level's last one, paired with itself as merkle.cpp:46 does
        const uint32_t next = (cnt + 1) / 2;
        uint64_t parent = 0;
        if (tid < next) {
            const uint64_t l = node[2 * tid];
            const uint64_t r = 2 * tid + 1 < cnt ? node[2 * tid + 1] : l;
            parent = nb::hash_dec_pair<FLAVOR>(l, r);
            tree[plan.out_off[s] + (first >> (s + 1)) + tid] = parent;
        }
        __syncthreads();
        if (tid < next) node[tid] = parent;
        __syncthreads();
        cnt = next;
    }
}

#define MK_HIP(expr)                                                                         \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return nb_internal_fail(NB_ERR_HIP, (std::string(#expr ": ") + hipGetErrorString(e_)).c_str()); \
    } while (0)

template <int FLAVOR>
int launch_merkle(const uint8_t *d_data, const uint64_t *d_offsets, uint32_t rec_len, uint64_t n,
                  uint64_t *d_tree, hipStream_t st) {
    const uint32_t lgrid = (uint32_t)std::min<uint64_t>((n + kLeafBlock - 1) / kLeafBlock, 256ull * 64);
    if (d_offsets)
        hipLaunchKernelGGL((merkle_leaf_kernel<FLAVOR, true>), dim3(lgrid), dim3(kLeafBlock), 0, st,
                           d_data, d_offsets, rec_len, n, d_tree);
    else
        hipLaunchKernelGGL((merkle_leaf_kernel<FLAVOR, false>), dim3(lgrid), dim3(kLeafBlock), 0,
                           st, d_data, d_offsets, rec_len, n, d_tree);
    MK_HIP(hipGetLastError());
    uint64_t cnt = n, in_off = 0, out_off = n;
    while (cnt > 1) {  // merkle.cpp:41: until one node is left
        LevelPlan plan{};
        uint64_t c = cnt, o = out_off;
        while (c > 1 && plan.levels < (uint32_t)kMaxSub) {
            plan.out_off[plan.levels++] = o;
            c = (c + 1) / 2;
            o += c;
        }
        const uint64_t grid = (cnt + kLevelSpan - 1) / kLevelSpan;
        hipLaunchKernelGGL((merkle_level_kernel<FLAVOR>), dim3((uint32_t)grid), dim3(kLevelThreads),
                           0, st, d_tree + in_off, cnt, d_tree, plan);
        MK_HIP(hipGetLastError());
        in_off = plan.out_off[plan.levels - 1];
        cnt = c;
        out_off = o;
    }
    return NB_OK;
}

std::atomic<uint64_t> g_device_merkles{0};  // nb_device_merkle_count()

}  // namespace

extern "C" {

uint64_t nb_device_merkle_count(void) { return g_device_merkles.load(std::memory_order_relaxed); }

uint64_t nb_merkle_tree_size(uint64_t n) {
    uint64_t total = n;
    while (n > 1) {
        n = (n + 1) / 2;
        total += n;
    }
    return total;
}

int nb_merkle_device(const uint8_t *d_data, const uint64_t *d_offsets, uint32_t rec_len,
                     uint64_t n, int flavor, uint64_t *d_tree, void *stream) {
    if (n == 0) return nb_internal_fail(NB_ERR_ARG, "MerkleTree of no records (merkle.cpp:8-10 throws)");
    if (!d_data || !d_tree) return nb_internal_fail(NB_ERR_ARG, "NULL buffer");
    if (flavor != NB_FLAVOR_LIBSTDCXX && flavor != NB_FLAVOR_MSVC_FNV1A)
        return nb_internal_fail(NB_ERR_ARG, "unknown flavor");
    if (nb::knob_take(nb::kKnobFailMerkles))  // fault injection (drop-in fallback tests)
        return nb_internal_fail(NB_ERR_HIP, "injected device Merkle failure (NB_FAIL_MERKLES)");
    g_device_merkles.fetch_add(1, std::memory_order_relaxed);
    hipStream_t st = (hipStream_t)stream;
    return flavor == NB_FLAVOR_MSVC_FNV1A
               ? launch_merkle<NB_FLAVOR_MSVC_FNV1A>(d_data, d_offsets, rec_len, n, d_tree, st)
               : launch_merkle<NB_FLAVOR_LIBSTDCXX>(d_data, d_offsets, rec_len, n, d_tree, st);
}

int nb_merkle(const uint8_t *data, const uint64_t *offsets, uint32_t rec_len, uint64_t n,
              int flavor, uint64_t *tree, uint64_t *leaves, uint64_t *root, int device) {
    if (n == 0) return nb_internal_fail(NB_ERR_ARG, "MerkleTree of no records (merkle.cpp:8-10 throws)");
    if (!data || !root) return nb_internal_fail(NB_ERR_ARG, "NULL buffer");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        return nb_internal_fail(NB_ERR_NODEV, "no HIP device visible");
    if (device < 0 || device >= count) return nb_internal_fail(NB_ERR_ARG, "device index out of range");
    MK_HIP(hipSetDevice(device));
    const uint64_t bytes = offsets ? offsets[n] : n * (uint64_t)rec_len;
    const uint64_t tsize = nb_merkle_tree_size(n);
    hipStream_t st;
    MK_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    uint8_t *d_data = nullptr;
    uint64_t *d_offs = nullptr, *d_tree = nullptr;
    int rc = NB_OK;
    auto cleanup = [&]() {
        (void)hipStreamSynchronize(st);
        if (d_data) (void)hipFree(d_data);
        if (d_offs) (void)hipFree(d_offs);
        if (d_tree) (void)hipFree(d_tree);
        (void)hipStreamDestroy(st);
    };
#define MK_TRY(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) {                                                               \
            rc = nb_internal_fail(NB_ERR_HIP, (std::string(#expr ": ") + hipGetErrorString(e_)).c_str()); \
            cleanup();                                                                        \
            return rc;                                                                        \
        }                                                                                     \
    } while (0)
    MK_TRY(hipMalloc(&d_data, bytes + 16));
    MK_TRY(hipMalloc(&d_tree, tsize * 8));
    MK_TRY(hipMemcpyAsync(d_data, data, bytes, hipMemcpyHostToDevice, st));
    if (offsets) {
        MK_TRY(hipMalloc(&d_offs, (n + 1) * 8));
        MK_TRY(hipMemcpyAsync(d_offs, offsets, (n + 1) * 8, hipMemcpyHostToDevice, st));
    }
    rc = nb_merkle_device(d_data, d_offs, rec_len, n, flavor, d_tree, st);
    if (rc) {
        cleanup();
        return rc;
    }
    if (tree) MK_TRY(hipMemcpyAsync(tree, d_tree, tsize * 8, hipMemcpyDeviceToHost, st));
    if (leaves) MK_TRY(hipMemcpyAsync(leaves, d_tree, n * 8, hipMemcpyDeviceToHost, st));
    MK_TRY(hipMemcpyAsync(root, d_tree + tsize - 1, 8, hipMemcpyDeviceToHost, st));
    MK_TRY(hipStreamSynchronize(st));
#undef MK_TRY
    cleanup();
    return NB_OK;
}

}  // extern "C"
