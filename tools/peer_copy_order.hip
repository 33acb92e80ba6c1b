// peer_copy_order.hip -- root-cause probe for the nb_build_sharded staging branch
// (DESIGN.md §7).  The merge staged a source slice with the blocking
// hipMemcpyPeer (issued on the device's null stream) and then launched the OR
// kernel on the owner's stream, which the slot sets create with
// hipStreamNonBlocking.  This program checks, for the copy variants the merge
// could use, whether a kernel enqueued on such a stream right after the copy
// always sees the copied bytes:
//   peer      hipMemcpyPeer(tmp, src)                  then kernel on the stream
//   memcpy    hipMemcpy(tmp, src, DeviceToDevice)      then kernel on the stream
//   peerasync hipMemcpyPeerAsync(tmp, src, stream)     then kernel on the stream
// with 1 or 3 host threads (the failing test ran 3 owner threads on one device).
// Each trial zeroes tmp, copies a pattern slice, and the kernel counts words of
// tmp that do not hold the pattern.  Prints one line per variant.
//   hipcc -O2 --offload-arch=gfx950 -o tools/peer_copy_order tools/peer_copy_order.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

__global__ void count_bad(const unsigned long long *tmp, size_t nwords, unsigned long long pat,
                          unsigned long long *bad) {
    unsigned long long c = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nwords;
         i += (size_t)gridDim.x * blockDim.x)
        c += tmp[i] != pat;
    if (c) atomicAdd(bad, c);
}

__global__ void fill(unsigned long long *p, size_t nwords, unsigned long long v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nwords;
         i += (size_t)gridDim.x * blockDim.x)
        p[i] = v;
}

enum Variant { kPeer = 0, kMemcpy = 1, kPeerAsync = 2 };
const char *kNames[] = {"peer", "memcpy", "peerasync"};

// One owner thread: `trials` stage+check rounds on its own non-blocking stream.
void owner(int variant, int trials, size_t nwords, const unsigned long long *src,
           unsigned long long pat, unsigned long long *bad_total, int *bad_trials) {
    CK(hipSetDevice(0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    unsigned long long *bad;
    CK(hipMalloc(&bad, 8));
    for (int t = 0; t < trials; ++t) {
        unsigned long long *tmp;
        CK(hipMalloc(&tmp, nwords * 8));
        hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, st, tmp, nwords, 0ull);
        CK(hipMemsetAsync(bad, 0, 8, st));
        CK(hipStreamSynchronize(st));
        if (variant == kPeer) CK(hipMemcpyPeer(tmp, 0, src, 0, nwords * 8));
        else if (variant == kMemcpy) CK(hipMemcpy(tmp, src, nwords * 8, hipMemcpyDeviceToDevice));
        else CK(hipMemcpyPeerAsync(tmp, 0, src, 0, nwords * 8, st));
        hipLaunchKernelGGL(count_bad, dim3(1024), dim3(256), 0, st, tmp, nwords, pat, bad);
        unsigned long long h = 0;
        CK(hipMemcpyAsync(&h, bad, 8, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        CK(hipFree(tmp));
        if (h) {
            __atomic_add_fetch(bad_total, h, __ATOMIC_RELAXED);
            __atomic_add_fetch(bad_trials, 1, __ATOMIC_RELAXED);
        }
    }
    CK(hipFree(bad));
    CK(hipStreamDestroy(st));
}

int main(int argc, char **argv) {
    const size_t nwords = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 128) << 7;  // KiB
    const int trials = argc > 2 ? std::atoi(argv[2]) : 20;
    CK(hipSetDevice(0));
    const unsigned long long pat = 0x5a5a00ff00ff5a5aull;
    unsigned long long *src;
    CK(hipMalloc(&src, nwords * 8));
    hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, src, nwords, pat);
    CK(hipDeviceSynchronize());
    for (int threads : {1, 3}) {
        for (int v : {kPeer, kMemcpy, kPeerAsync}) {
            unsigned long long bad_total = 0;
            int bad_trials = 0;
            std::vector<std::thread> th;
            for (int i = 0; i < threads; ++i)
                th.emplace_back(owner, v, trials, nwords, src, pat, &bad_total, &bad_trials);
            for (auto &t : th) t.join();
            std::printf("variant=%-9s threads=%d trials=%d slice=%zu KiB  stale_trials=%d stale_words=%llu\n",
                        kNames[v], threads, trials * threads, nwords * 8 >> 10, bad_trials, bad_total);
            std::fflush(stdout);
        }
    }
    CK(hipFree(src));
    return 0;
}
