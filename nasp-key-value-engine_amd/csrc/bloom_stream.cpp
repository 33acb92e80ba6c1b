// bloom_stream.cpp -- the streaming host builder of the C ABI (nb_builder_*,
// include/nasp_bloom.h): the host side of SSTable::build's filter block
// (reference SSTable/SSTable.cpp:28-35, BloomFilter::add BloomFilter.cpp:82-86).
//
// Keys are packed into a ring of pinned host chunks.  A full chunk is uploaded
// on the copy stream and built on the compute stream (OR-accumulated into the
// device-resident filter) while the caller packs the next chunk, so key packing,
// PCIe and the device build overlap; nothing waits until a slot comes round
// again.  Chunks whose keys share one length travel without offsets (16-byte
// keys then take the kernels' dwordx4 path).  add_batch uploads straight from
// the caller's buffer, chunk by chunk, each build overlapping the next upload.
// Slot sets (pinned + device chunk buffers, two streams) are pooled per device:
// pinned allocations cost milliseconds and a flush builds one filter per table.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/nasp_bloom.h"
#include "nb_knobs.h"

int nb_internal_build(const uint8_t *d_keys, const uint64_t *d_offsets, uint32_t key_len,
                      uint64_t n, uint32_t m, uint32_t k, uint64_t seed, int flavor,
                      uint64_t *d_words, bool overwrite, hipStream_t st);  // bloom_kernels.hip
int nb_internal_fail(int code, const char *msg);
int nb_internal_or_gather(uint64_t *dst, const uint64_t *const *srcs, uint32_t nsrc, uint64_t nwords,
                          hipStream_t st);  // bloom_kernels.hip

namespace {

constexpr size_t kChunkBytes = size_t(16) << 20;  // key bytes per chunk
constexpr size_t kChunkKeys = size_t(1) << 20;    // keys per chunk
constexpr size_t kSlack = 32;                     // aligned-read slack past a chunk
constexpr int kSlots = 3;
constexpr int kMaxShards = 64;  // nb_build_sharded: shards (= host threads) used at most

#define SB_HIP(expr)                                                                     \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return nb_internal_fail(NB_ERR_HIP,                                          \
                                    (std::string(#expr ": ") + hipGetErrorString(e_)).c_str()); \
    } while (0)

struct Slot {
    uint8_t *h_keys = nullptr;   // pinned [kChunkBytes + kSlack]
    uint64_t *h_offs = nullptr;  // pinned [kChunkKeys + 1]
    uint8_t *d_keys = nullptr;   // device [kChunkBytes + kSlack]
    uint64_t *d_offs = nullptr;  // device [kChunkKeys + 1]
    hipEvent_t uploaded = nullptr, built = nullptr;
    bool busy = false;           // submitted, not yet known to be built
};

struct SlotSet {
    int dev = 0;
    hipStream_t copy = nullptr, comp = nullptr;
    Slot s[kSlots];
    uint64_t *d_words = nullptr;
    size_t words_cap = 0;  // bytes
};

std::mutex g_pool_mu;
std::vector<SlotSet *> g_pool;

int slotset_alloc(int dev, SlotSet **out) {
    SlotSet *ss = new SlotSet;
    ss->dev = dev;
    *out = ss;
    SB_HIP(hipStreamCreateWithFlags(&ss->copy, hipStreamNonBlocking));
    SB_HIP(hipStreamCreateWithFlags(&ss->comp, hipStreamNonBlocking));
    for (Slot &sl : ss->s) {
        SB_HIP(hipHostMalloc(reinterpret_cast<void **>(&sl.h_keys), kChunkBytes + kSlack,
                             hipHostMallocDefault));
        SB_HIP(hipHostMalloc(reinterpret_cast<void **>(&sl.h_offs), (kChunkKeys + 1) * 8,
                             hipHostMallocDefault));
        SB_HIP(hipMalloc(&sl.d_keys, kChunkBytes + kSlack));
        SB_HIP(hipMalloc(&sl.d_offs, (kChunkKeys + 1) * 8));
        SB_HIP(hipEventCreateWithFlags(&sl.uploaded, hipEventDisableTiming));
        SB_HIP(hipEventCreateWithFlags(&sl.built, hipEventDisableTiming));
    }
    return NB_OK;
}

void slotset_free(SlotSet *ss) {
    (void)hipSetDevice(ss->dev);
    for (Slot &sl : ss->s) {
        if (sl.h_keys) (void)hipHostFree(sl.h_keys);
        if (sl.h_offs) (void)hipHostFree(sl.h_offs);
        if (sl.d_keys) (void)hipFree(sl.d_keys);
        if (sl.d_offs) (void)hipFree(sl.d_offs);
        if (sl.uploaded) (void)hipEventDestroy(sl.uploaded);
        if (sl.built) (void)hipEventDestroy(sl.built);
    }
    if (ss->d_words) (void)hipFree(ss->d_words);
    if (ss->copy) (void)hipStreamDestroy(ss->copy);
    if (ss->comp) (void)hipStreamDestroy(ss->comp);
    delete ss;
}

}  // namespace

struct nb_builder {
    SlotSet *ss = nullptr;
    uint32_t m = 0, k = 0;
    uint64_t seed = 0;
    int flavor = 0;
    size_t nwords = 0;
    int cur = 0;             // slot being packed
    uint64_t nkeys = 0, nbytes = 0;
    int64_t fixed = -1;      // common key length of the chunk (-1: none yet, -2: mixed)

    Slot &slot(int i) { return ss->s[i]; }

    // Wait until slot i's previous chunk is built (its buffers are then free).
    int reclaim(int i) {
        Slot &sl = slot(i);
        if (sl.busy) {
            SB_HIP(hipEventSynchronize(sl.built));
            sl.busy = false;
        }
        return NB_OK;
    }

    // Build the chunk in slot i: keys at d_keys (offsets d_offs, or fixed length).
    int launch(int i, const uint8_t *d_keys, const uint64_t *d_offs, uint32_t key_len,
               uint64_t n) {
        Slot &sl = slot(i);
        SB_HIP(hipEventRecord(sl.uploaded, ss->copy));
        SB_HIP(hipStreamWaitEvent(ss->comp, sl.uploaded, 0));
        const int rc = nb_internal_build(d_keys, d_offs, key_len, n, m, k, seed, flavor,
                                         ss->d_words, false, ss->comp);
        if (rc) return rc;
        SB_HIP(hipEventRecord(sl.built, ss->comp));
        sl.busy = true;
        return NB_OK;
    }

    // Upload and build the pinned chunk being packed; move to the next slot.
    int submit() {
        if (nkeys == 0) return NB_OK;
        if (m == 0 && k) return nb_internal_fail(NB_ERR_ARG, "add() on a filter with m == 0");
        Slot &sl = slot(cur);
        const bool fixed_len = fixed > 0;
        SB_HIP(hipMemcpyAsync(sl.d_keys, sl.h_keys, nbytes, hipMemcpyHostToDevice, ss->copy));
        if (!fixed_len)
            SB_HIP(hipMemcpyAsync(sl.d_offs, sl.h_offs, (nkeys + 1) * 8, hipMemcpyHostToDevice,
                                  ss->copy));
        int rc = launch(cur, sl.d_keys, fixed_len ? nullptr : sl.d_offs,
                        fixed_len ? (uint32_t)fixed : 0u, nkeys);
        if (rc) return rc;
        cur = (cur + 1) % kSlots;
        nkeys = nbytes = 0;
        fixed = -1;
        if ((rc = reclaim(cur))) return rc;
        slot(cur).h_offs[0] = 0;
        return NB_OK;
    }
};

extern "C" {

int nb_host_alloc(size_t bytes, void **out) {
    if (!out) return nb_internal_fail(NB_ERR_ARG, "NULL out");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        return nb_internal_fail(NB_ERR_NODEV, "no HIP device visible");
    SB_HIP(hipHostMalloc(out, std::max<size_t>(bytes, 1), hipHostMallocDefault));
    return NB_OK;
}

int nb_host_free(void *p) {
    if (p) SB_HIP(hipHostFree(p));
    return NB_OK;
}

int nb_builder_create(uint32_t m, uint32_t k, uint64_t h2_seed, int flavor,
                      const uint64_t *init_words, int device, nb_builder **out) {
    if (!out) return nb_internal_fail(NB_ERR_ARG, "NULL out");
    *out = nullptr;
    if (flavor != NB_FLAVOR_LIBSTDCXX && flavor != NB_FLAVOR_MSVC_FNV1A &&
        flavor != NB_FLAVOR_MURMUR3_X64_128)
        return nb_internal_fail(NB_ERR_ARG, "unknown flavor");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        return nb_internal_fail(NB_ERR_NODEV, "no HIP device visible");
    if (device < 0 || device >= count) return nb_internal_fail(NB_ERR_ARG, "device index out of range");
    SB_HIP(hipSetDevice(device));
    SlotSet *ss = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (size_t i = 0; i < g_pool.size(); ++i)
            if (g_pool[i]->dev == device) {
                ss = g_pool[i];
                g_pool.erase(g_pool.begin() + i);
                break;
            }
    }
    if (!ss) {
        const int rc = slotset_alloc(device, &ss);
        if (rc) {
            slotset_free(ss);
            return rc;
        }
    }
    nb_builder *b = new nb_builder;
    b->ss = ss;
    b->m = m;
    b->k = k;
    b->seed = h2_seed;
    b->flavor = flavor;
    b->nwords = ((size_t)m + 63) / 64;
    *out = b;
    const size_t wb = std::max<size_t>(b->nwords, 1) * 8;
    if (wb > ss->words_cap) {
        if (ss->d_words) SB_HIP(hipFree(ss->d_words));
        ss->d_words = nullptr;
        ss->words_cap = 0;
        SB_HIP(hipMalloc(&ss->d_words, wb));
        ss->words_cap = wb;
    }
    if (init_words && b->nwords)
        SB_HIP(hipMemcpyAsync(ss->d_words, init_words, b->nwords * 8, hipMemcpyHostToDevice,
                              ss->comp));
    else
        SB_HIP(hipMemsetAsync(ss->d_words, 0, wb, ss->comp));
    ss->s[0].h_offs[0] = 0;
    return NB_OK;
}

int nb_builder_add(nb_builder *b, const uint8_t *key, uint64_t len) {
    if (!b || (len && !key)) return nb_internal_fail(NB_ERR_ARG, "NULL builder or key");
    if (b->m == 0 && b->k) return nb_internal_fail(NB_ERR_ARG, "add() on a filter with m == 0");
    if (len > kChunkBytes) {  // one oversized key: its own chunk, synchronously
        int rc = b->submit();
        if (rc) return rc;
        SB_HIP(hipSetDevice(b->ss->dev));
        uint8_t *d = nullptr;
        uint64_t *o = nullptr;
        const uint64_t offs[2] = {0, len};
        SB_HIP(hipMalloc(&d, len + kSlack));
        SB_HIP(hipMalloc(&o, 16));
        SB_HIP(hipMemcpyAsync(d, key, len, hipMemcpyHostToDevice, b->ss->comp));
        SB_HIP(hipMemcpyAsync(o, offs, 16, hipMemcpyHostToDevice, b->ss->comp));
        rc = nb_internal_build(d, o, 0, 1, b->m, b->k, b->seed, b->flavor, b->ss->d_words, false,
                               b->ss->comp);
        SB_HIP(hipStreamSynchronize(b->ss->comp));
        (void)hipFree(d);
        (void)hipFree(o);
        return rc;
    }
    if (b->nkeys == kChunkKeys || b->nbytes + len > kChunkBytes) {
        SB_HIP(hipSetDevice(b->ss->dev));
        const int rc = b->submit();
        if (rc) return rc;
    }
    Slot &sl = b->slot(b->cur);
    if (len) std::memcpy(sl.h_keys + b->nbytes, key, len);
    b->nbytes += len;
    sl.h_offs[++b->nkeys] = b->nbytes;
    if (b->fixed == -1) b->fixed = (int64_t)len;
    else if (b->fixed != (int64_t)len) b->fixed = -2;
    return NB_OK;
}

static int add_batch(nb_builder *b, const uint8_t *keys, const uint64_t *offsets, uint32_t key_len,
                     uint64_t n, bool wait_uploads);

int nb_builder_add_batch(nb_builder *b, const uint8_t *keys, const uint64_t *offsets,
                         uint32_t key_len, uint64_t n) {
    return add_batch(b, keys, offsets, key_len, n, true);
}

int nb_builder_add_batch_async(nb_builder *b, const uint8_t *keys, const uint64_t *offsets,
                               uint32_t key_len, uint64_t n) {
    return add_batch(b, keys, offsets, key_len, n, false);
}

int nb_builder_sync_uploads(nb_builder *b) {
    if (!b) return nb_internal_fail(NB_ERR_ARG, "NULL builder");
    SB_HIP(hipSetDevice(b->ss->dev));
    SB_HIP(hipStreamSynchronize(b->ss->copy));
    return NB_OK;
}

static int add_batch(nb_builder *b, const uint8_t *keys, const uint64_t *offsets, uint32_t key_len,
                     uint64_t n, bool wait_uploads) {
    if (!b) return nb_internal_fail(NB_ERR_ARG, "NULL builder");
    if (n == 0) return NB_OK;
    if (!keys) return nb_internal_fail(NB_ERR_ARG, "NULL keys");
    if (b->m == 0 && b->k) return nb_internal_fail(NB_ERR_ARG, "add() on a filter with m == 0");
    SB_HIP(hipSetDevice(b->ss->dev));
    int rc = b->submit();  // the partly packed chunk first
    if (rc) return rc;
    if (!offsets && key_len > kChunkBytes) {
        // fixed-length keys longer than a chunk: each one through the oversized-key
        // path (its own device buffer), as variable-length keys of that size go
        for (uint64_t i = 0; i < n; ++i)
            if ((rc = nb_builder_add(b, keys + i * (uint64_t)key_len, key_len))) return rc;
        b->slot(b->cur).h_offs[0] = 0;
        return NB_OK;
    }
    SlotSet *ss = b->ss;
    uint64_t i = 0;
    while (i < n) {
        // next chunk [i, e): <= kChunkKeys keys and (variable-length) <= kChunkBytes bytes
        uint64_t e = std::min<uint64_t>(n, i + kChunkKeys);
        if (offsets) {
            const uint64_t lim = offsets[i] + kChunkBytes - 16;
            e = (uint64_t)(std::upper_bound(offsets + i + 1, offsets + e + 1, lim) - offsets) - 1;
            if (e == i) {  // one key longer than a chunk
                if ((rc = nb_builder_add(b, keys + offsets[i], offsets[i + 1] - offsets[i])) ||
                    (rc = b->submit()))
                    return rc;
                ++i;
                continue;
            }
        } else {
            e = std::min<uint64_t>(e, i + std::max<uint64_t>(1, kChunkBytes / std::max(key_len, 1u)));
        }
        const int s = b->cur;
        Slot &sl = b->slot(s);
        if (offsets) {
            // bytes [A, offsets[e]) with A = offsets[i] rounded down to 16: the kernel's
            // aligned staging reads stay inside the copy (keys base = d_keys - A)
            const uint64_t A = offsets[i] & ~15ull;
            SB_HIP(hipMemcpyAsync(sl.d_keys, keys + A, offsets[e] - A, hipMemcpyHostToDevice,
                                  ss->copy));
            SB_HIP(hipMemcpyAsync(sl.d_offs, offsets + i, (e - i + 1) * 8, hipMemcpyHostToDevice,
                                  ss->copy));
            rc = b->launch(s, sl.d_keys - A, sl.d_offs, 0, e - i);
        } else {
            SB_HIP(hipMemcpyAsync(sl.d_keys, keys + i * key_len, (e - i) * key_len,
                                  hipMemcpyHostToDevice, ss->copy));
            rc = b->launch(s, sl.d_keys, nullptr, key_len, e - i);
        }
        if (rc) return rc;
        b->cur = (s + 1) % kSlots;
        if ((rc = b->reclaim(b->cur))) return rc;
        i = e;
    }
    b->slot(b->cur).h_offs[0] = 0;
    // every upload from the caller's buffers has landed: they may be reused (the
    // builds stay in flight).  The async form leaves that to nb_builder_sync_uploads /
    // finish / destroy.
    if (wait_uploads) SB_HIP(hipStreamSynchronize(ss->copy));
    return NB_OK;
}

int nb_builder_finish(nb_builder *b, uint64_t *words) {
    if (!b) return nb_internal_fail(NB_ERR_ARG, "NULL builder");
    if (b->nwords && !words) return nb_internal_fail(NB_ERR_ARG, "NULL words");
    SB_HIP(hipSetDevice(b->ss->dev));
    int rc = b->submit();
    if (rc) return rc;
    if (b->nwords)
        SB_HIP(hipMemcpyAsync(words, b->ss->d_words, b->nwords * 8, hipMemcpyDeviceToHost,
                              b->ss->comp));
    SB_HIP(hipStreamSynchronize(b->ss->comp));
    SB_HIP(hipStreamSynchronize(b->ss->copy));  // (async batches: their uploads too)
    for (Slot &sl : b->ss->s) sl.busy = false;
    return NB_OK;
}

int nb_builder_destroy(nb_builder *b) {
    if (!b) return NB_OK;
    SlotSet *ss = b->ss;
    delete b;
    if (!ss) return NB_OK;
    (void)hipSetDevice(ss->dev);
    const bool ok = hipStreamSynchronize(ss->comp) == hipSuccess &&
                    hipStreamSynchronize(ss->copy) == hipSuccess;
    for (Slot &sl : ss->s) sl.busy = false;
    if (!ok) {
        slotset_free(ss);
        return nb_internal_fail(NB_ERR_HIP, "stream synchronisation failed in nb_builder_destroy");
    }
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_pool.push_back(ss);
    return NB_OK;
}

}  // extern "C"

namespace {

// Everything added so far is built: the partial chunk submitted, the stream drained.
int drain(nb_builder *b) {
    SB_HIP(hipSetDevice(b->ss->dev));
    const int rc = b->submit();
    if (rc) return rc;
    SB_HIP(hipStreamSynchronize(b->ss->comp));
    SB_HIP(hipStreamSynchronize(b->ss->copy));  // (async batches: their uploads too)
    for (Slot &sl : b->ss->s) sl.busy = false;
    return NB_OK;
}

// Download device words [0, nwords) into host `dst` through the slot set's pinned
// key chunks (two at a time: chunk i+1's DMA overlaps chunk i's host copy), so the
// concurrent per-owner downloads of the merge are plain DMA into memory the
// library owns -- none of them relies on the runtime's staging of pageable copies.
int download_pinned(SlotSet *ss, const uint64_t *d, uint64_t nwords, uint64_t *dst) {
    const uint64_t per = kChunkBytes / 8;  // words per chunk
    const uint64_t pieces = (nwords + per - 1) / per;
    for (uint64_t i = 0; i < pieces + 1; ++i) {
        if (i < pieces) {
            Slot &sl = ss->s[i % 2];
            const uint64_t w = std::min(per, nwords - i * per);
            SB_HIP(hipMemcpyAsync(sl.h_keys, d + i * per, w * 8, hipMemcpyDeviceToHost, ss->comp));
            SB_HIP(hipEventRecord(sl.built, ss->comp));
        }
        if (i > 0) {
            Slot &sl = ss->s[(i - 1) % 2];
            SB_HIP(hipEventSynchronize(sl.built));
            const uint64_t w = std::min(per, nwords - (i - 1) * per);
            std::memcpy(dst + (i - 1) * per, sl.h_keys, w * 8);
        }
    }
    return NB_OK;
}

// Owner o's step of the merge: OR word slice [lo, lo + len) of every other
// partial into its own, reading the sources in place (same device, or a peer over
// xGMI with peer access enabled) in one stream-ordered kernel, then download the
// merged slice into the caller's words.  A source the owner cannot address
// directly is first brought over with a peer copy on the owner's stream (ordered
// before the OR kernel); NB_SHARDED_STAGE=1 forces that staging branch for every
// source, so a one-GPU box can test it.
int merge_slice(std::vector<nb_builder *> &bs, int o, uint64_t lo, uint64_t len, uint64_t *words,
                const std::vector<char> &peer, int ndev) {
    nb_builder *own = bs[o];
    const int dev = own->ss->dev;
    hipStream_t st = own->ss->comp;
    SB_HIP(hipSetDevice(dev));
    const bool stage_all = nb::knob(nb::kKnobShardedStage) != 0;
    std::vector<const uint64_t *> srcs;
    uint64_t *tmp = nullptr;
    size_t staged = 0;
    int rc = NB_OK;
    for (size_t s = 0; s < bs.size() && !rc; ++s) {
        if ((int)s == o) continue;
        const int sdev = bs[s]->ss->dev;
        if (!stage_all && (sdev == dev || peer[(size_t)dev * ndev + sdev])) {
            srcs.push_back(bs[s]->ss->d_words + lo);
            continue;
        }
        if (!tmp && hipMalloc(&tmp, (bs.size() - 1) * len * 8) != hipSuccess) {
            rc = nb_internal_fail(NB_ERR_HIP, "hipMalloc of the merge staging buffer failed");
            break;
        }
        // on the owner's stream, so the OR kernel below is ordered after it.  The
        // blocking hipMemcpyPeer is NOT: a device-to-device copy returns before it
        // lands and runs on the null stream, which the slot sets' non-blocking
        // streams do not wait for (tools/peer_copy_order.hip: stale slices in 32 of
        // 240 trials vs 0 of 240 on the stream)
        const hipError_t e = hipMemcpyPeerAsync(tmp + staged * len, dev, bs[s]->ss->d_words + lo,
                                                sdev, len * 8, st);
        if (e != hipSuccess)
            rc = nb_internal_fail(NB_ERR_HIP, (std::string("hipMemcpyPeerAsync: ") + hipGetErrorString(e)).c_str());
        else
            srcs.push_back(tmp + (staged++) * len);
    }
    if (!rc) rc = nb_internal_or_gather(own->ss->d_words + lo, srcs.data(), (uint32_t)srcs.size(), len, st);
    if (!rc) rc = download_pinned(own->ss, own->ss->d_words + lo, len, words + lo);
    const hipError_t e2 = hipStreamSynchronize(st);  // tmp is read by the OR kernel
    if (tmp) (void)hipFree(tmp);
    if (rc) return rc;
    SB_HIP(e2);
    return NB_OK;
}

}  // namespace

extern "C" int nb_build_sharded(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len,
                                uint64_t n, uint32_t m, uint32_t k, uint64_t h2_seed, int flavor,
                                uint64_t *words, int nshards) {
    if (flavor != NB_FLAVOR_LIBSTDCXX && flavor != NB_FLAVOR_MSVC_FNV1A &&
        flavor != NB_FLAVOR_MURMUR3_X64_128)
        return nb_internal_fail(NB_ERR_ARG, "unknown flavor");
    if (n && m == 0) return nb_internal_fail(NB_ERR_ARG, "m == 0 with keys (reference divides by zero)");
    if (n && (!keys || !words)) return nb_internal_fail(NB_ERR_ARG, "NULL keys or words");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        return nb_internal_fail(NB_ERR_NODEV, "no HIP device visible");
    if (nshards <= 0) nshards = count;
    // the filter does not depend on the split: more shards than this only cost
    // threads and pinned chunk rings
    nshards = std::min(nshards, kMaxShards);
    if (n == 0 || k == 0) return NB_OK;
    if (nshards == 1) return nb_build(keys, offsets, key_len, n, m, k, h2_seed, flavor, words, 0);
    // peer access for the merge's in-place reads over xGMI; peer[a * ndev + b] = 1
    // once device a may read device b's memory (an already-enabled pair reports an
    // error that is not one; the sticky error is cleared so no later check sees it)
    const int ndev = std::min(nshards, count);
    std::vector<char> peer((size_t)ndev * ndev, 0);
    for (int a = 0; a < ndev; ++a) {
        (void)hipSetDevice(a);
        for (int b = 0; b < ndev; ++b) {
            int can = 0;
            if (a == b || hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) continue;
            const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
            peer[(size_t)a * ndev + b] = e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled;
        }
        (void)hipGetLastError();
    }
    // phase 1: shard s = keys [n s / S, n (s+1) / S) on device s % count, one host
    // thread each; shard 0's filter starts from the caller's bits
    std::vector<nb_builder *> bs(nshards, nullptr);
    std::vector<int> rcs(nshards, NB_OK);
    std::vector<std::string> msgs(nshards);
    auto run_shard = [&](int s) {
        const uint64_t b = n * (uint64_t)s / nshards, e = n * (uint64_t)(s + 1) / nshards;
        int rc = nb_builder_create(m, k, h2_seed, flavor, s == 0 ? words : nullptr, s % count, &bs[s]);
        if (!rc && e > b)
            rc = offsets ? nb_builder_add_batch(bs[s], keys, offsets + b, 0, e - b)
                         : nb_builder_add_batch(bs[s], keys + b * key_len, nullptr, key_len, e - b);
        if (!rc) rc = drain(bs[s]);
        if (rc) msgs[s] = nb_last_error();
        rcs[s] = rc;
    };
    auto run_all = [&](auto &&fn) {
        std::vector<std::thread> th;
        for (int s = 0; s < nshards; ++s) th.emplace_back(fn, s);
        for (auto &t : th) t.join();
        for (int s = 0; s < nshards; ++s)
            if (rcs[s]) return nb_internal_fail(rcs[s], msgs[s].c_str());
        return (int)NB_OK;
    };
    int rc = run_all(run_shard);
    // phase 2: owner o merges and downloads word slice o
    if (!rc) {
        const uint64_t nw = ((uint64_t)m + 63) / 64;
        rc = run_all([&](int o) {
            const uint64_t lo = nw * (uint64_t)o / nshards, hi = nw * (uint64_t)(o + 1) / nshards;
            rcs[o] = hi > lo ? merge_slice(bs, o, lo, hi - lo, words, peer, ndev) : NB_OK;
            if (rcs[o]) msgs[o] = nb_last_error();
        });
    }
    for (nb_builder *b : bs) (void)nb_builder_destroy(b);
    return rc;
}

// Release the pooled slot sets (called by nb_shutdown).
void nb_internal_stream_shutdown() {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (SlotSet *ss : g_pool) slotset_free(ss);
    g_pool.clear();
}
