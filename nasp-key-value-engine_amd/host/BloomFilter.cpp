// BloomFilter.cpp -- the drop-in class over the C ABI (include/nasp_bloom.h).
// See BloomFilter.h for the contract; reference behaviour cited per method.
#include "BloomFilter.h"

#include <atomic>
#include <cstring>
#include <ctime>
#include <iostream>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>

#include "../../include/nasp_bloom.h"
#include "../csrc/bloom_math.h"

namespace {
int g_default_flavor = NB_FLAVOR_LIBSTDCXX;
std::atomic<uint64_t> g_host_batch_limit{4096};
std::atomic<uint64_t> g_retain_bytes{uint64_t(256) << 20};
std::once_flag g_nodev_note;

constexpr uint64_t kChunkBytes = uint64_t(16) << 20;  // key bytes per chunk
constexpr uint64_t kChunkKeys = uint64_t(1) << 20;    // keys per chunk
constexpr uint64_t kSlack = 16;

// Process-wide pools of chunk buffers: a flush that streams 10M keys reuses the
// buffers (pinned by nb_host_alloc, so their uploads are asynchronous DMA; plain
// memory on a host without a device) of the previous flush.  Key buffers and
// offset buffers (needed only once a chunk's key lengths differ) pool separately.
struct Buf {
    void *p;
    bool pinned;
};
std::mutex g_pool_mu;
std::vector<Buf> g_pool[2];  // [0] key bytes, [1] offsets
constexpr size_t kPoolMax = 20;
constexpr size_t kBufBytes[2] = {kChunkBytes + kSlack, (kChunkKeys + 1) * 8};

Buf pool_get(int which) {
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        if (!g_pool[which].empty()) {
            const Buf b = g_pool[which].back();
            g_pool[which].pop_back();
            return b;
        }
    }
    void *p = nullptr;
    if (nb_host_alloc(kBufBytes[which], &p) == NB_OK) return {p, true};
    return {::operator new(kBufBytes[which]), false};
}

void pool_put(int which, void *p, bool pinned) {
    if (!p) return;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        if (g_pool[which].size() < kPoolMax) {
            g_pool[which].push_back({p, pinned});
            return;
        }
    }
    if (pinned) (void)nb_host_free(p);
    else ::operator delete(p);
}
}  // namespace

void BloomFilter::setDefaultFlavor(int f) { g_default_flavor = f; }
void BloomFilter::setHostBatchLimit(uint64_t keys) { g_host_batch_limit = keys; }
uint64_t BloomFilter::hostBatchLimit() { return g_host_batch_limit; }
void BloomFilter::setRetainBytes(uint64_t bytes) { g_retain_bytes = bytes; }
uint64_t BloomFilter::retainBytes() { return g_retain_bytes; }

// BloomFilter.cpp:26 -- no hash closures: every probe answers true.
BloomFilter::BloomFilter() : flavor(g_default_flavor) {}

// BloomFilter.cpp:28-65 (the bit set starts all zero: `bits` stays null until set)
BloomFilter::BloomFilter(unsigned int n, double falsePositiveRate) : flavor(g_default_flavor) {
    m = calculateSizeOfBitSet(n, falsePositiveRate);
    k = calculateNumberOfHashFunctions(n, m);
    p = falsePositiveRate;
    timeConst = static_cast<unsigned int>(time(nullptr));
    h2_seed = nb_seed_from_time(timeConst);
    closures = true;
}

unsigned int BloomFilter::calculateSizeOfBitSet(unsigned int expectedElements, double falsePositiveRate) {
    return nb_size_of_bitset(expectedElements, falsePositiveRate);
}

unsigned int BloomFilter::calculateNumberOfHashFunctions(unsigned int expectedElements, unsigned int mm) {
    return nb_num_hashes(expectedElements, mm);
}

BloomFilter::BloomFilter(const BloomFilter &o)
    : m(o.m), k(o.k), p(o.p), timeConst(o.timeConst), h2_seed(o.h2_seed), closures(o.closures),
      flavor(o.flavor), device(o.device) {
    o.flush();
    bits = o.bits;  // shared until either side changes it
    last_on_device = o.last_on_device;
}

BloomFilter &BloomFilter::operator=(const BloomFilter &o) {
    if (this == &o) return *this;
    o.flush();
    release_chunks();
    m = o.m; k = o.k; p = o.p; timeConst = o.timeConst; h2_seed = o.h2_seed;
    closures = o.closures; flavor = o.flavor; device = o.device;
    bits = o.bits;
    last_on_device = o.last_on_device;
    return *this;
}

BloomFilter::BloomFilter(BloomFilter &&o) noexcept
    : m(o.m), k(o.k), p(o.p), bits(std::move(o.bits)), timeConst(o.timeConst), h2_seed(o.h2_seed),
      closures(o.closures), flavor(o.flavor), device(o.device), pending(std::move(o.pending)),
      retained(std::move(o.retained)), pending_n(o.pending_n), mode(o.mode), stream(o.stream),
      retained_all(o.retained_all), bits_before(std::move(o.bits_before)),
      last_on_device(o.last_on_device) {
    o.stream = nullptr;
    o.reset_moved();
}

BloomFilter &BloomFilter::operator=(BloomFilter &&o) noexcept {
    if (this == &o) return *this;
    release_chunks();
    m = o.m; k = o.k; p = o.p; timeConst = o.timeConst; h2_seed = o.h2_seed;
    closures = o.closures; flavor = o.flavor; device = o.device;
    bits = std::move(o.bits);
    pending = std::move(o.pending);
    retained = std::move(o.retained);
    pending_n = o.pending_n;
    mode = o.mode;
    stream = o.stream;
    o.stream = nullptr;
    retained_all = o.retained_all;
    bits_before = std::move(o.bits_before);
    last_on_device = o.last_on_device;
    o.reset_moved();
    return *this;
}

BloomFilter::~BloomFilter() { release_chunks(); }

// The moved-from state: a default-constructed filter (answers true, holds nothing).
void BloomFilter::reset_moved() noexcept {
    m = 0; k = 0; p = 0.0; timeConst = 0; h2_seed = 0; closures = false;
    bits.reset();
    bits_before.reset();
    pending.clear();
    retained.clear();
    pending_n = 0;
    mode = Mode::kPending;
    stream = nullptr;
    retained_all = true;
    last_on_device = false;
}

// Drop every pending / retained key and an open builder (the filter's bits stay).
void BloomFilter::release_chunks() const {
    if (stream) {
        (void)nb_builder_destroy(stream);
        stream = nullptr;
    }
    for (Chunk &c : pending) free_chunk(c);
    for (Chunk &c : retained) free_chunk(c);
    pending.clear();
    retained.clear();
    pending_n = 0;
    mode = Mode::kPending;
    retained_all = true;
    bits_before.reset();
}

void BloomFilter::free_chunk(Chunk &c) {
    if (c.key_cap == kChunkKeys) {
        pool_put(0, c.bytes, c.pinned);
        pool_put(1, c.offs, c.offs_pinned);
    } else {  // an oversized key's own chunk
        delete[] c.bytes;
        delete[] c.offs;
    }
    c.bytes = nullptr;
    c.offs = nullptr;
}

// The chunk's offsets array (n + 1 entries), allocated on first need.
void BloomFilter::need_offsets(Chunk &c) {
    if (c.offs) return;
    const Buf b = pool_get(1);
    c.offs = static_cast<uint64_t *>(b.p);
    c.offs_pinned = b.pinned;
}

// The words, allocated and owned by this filter alone (copy on write).
std::vector<uint64_t> &BloomFilter::own_bits() const {
    if (!bits) bits = std::make_shared<std::vector<uint64_t>>(((size_t)m + 63) / 64, 0);
    else if (bits.use_count() > 1) bits = std::make_shared<std::vector<uint64_t>>(*bits);
    return *bits;
}

// BloomFilter.cpp:82-86: the key joins the packed batch (see BloomFilter.h).
void BloomFilter::add(const std::string &elem) {
    if (!closures || k == 0) return;  // no hash closures: nothing to set
    // the reference divides by m in every closure: m == 0 is undefined there
    if (m == 0) throw std::runtime_error("nasp_bloom: add() on a filter with m == 0");
    const uint64_t len = elem.size();
    if (pending.empty() || pending.back().n == pending.back().key_cap ||
        pending.back().used + len > pending.back().byte_cap) {
        if (!pending.empty()) hand_off();
        Chunk c;
        if (len <= kChunkBytes) {
            const Buf b = pool_get(0);
            c.bytes = static_cast<uint8_t *>(b.p);
            c.pinned = b.pinned;
            c.byte_cap = kChunkBytes;
            c.key_cap = kChunkKeys;
        } else {  // one oversized key: a chunk of its own
            c.bytes = new uint8_t[len + kSlack];
            c.offs = new uint64_t[2];
            c.byte_cap = len;
            c.key_cap = 1;
        }
        pending.push_back(c);
    }
    Chunk &c = pending.back();
    if (c.fixed == -1) {
        c.fixed = (int64_t)len;
    } else if (c.fixed >= 0 && c.fixed != (int64_t)len) {  // lengths differ from here on
        need_offsets(c);
        for (uint64_t i = 0; i <= c.n; ++i) c.offs[i] = i * (uint64_t)c.fixed;
        c.fixed = -2;
    }
    if (len) std::memcpy(c.bytes + c.used, elem.data(), len);
    c.used += len;
    ++c.n;
    if (c.fixed == -2) c.offs[c.n] = c.used;
    ++pending_n;
}

void BloomFilter::addBatch(const std::vector<std::string> &elems) {
    for (const std::string &e : elems) add(e);
}

// kPending -> kDevice (a builder from the current bits), or kHost when none opens.
void BloomFilter::open_device() const {
    bits_before = bits;  // shared: host writes copy it, so it stays the builder's start
    const int rc = nb_builder_create(m, k, h2_seed, flavor, bits ? bits->data() : nullptr, device,
                                     &stream);
    if (rc == NB_OK) {
        mode = Mode::kDevice;
        retained_all = true;
        return;
    }
    if (rc == NB_ERR_NODEV) {
        std::call_once(g_nodev_note, [] {
            std::cerr << "[BloomFilter] GPU build failed (no HIP device visible); building "
                         "filters on the host\n";
        });
    } else {
        std::cerr << "[BloomFilter] GPU build failed (" << nb_last_error() << "); building "
                  << pending_n << " keys on the host\n";
    }
    stream = nullptr;
    bits_before.reset();
    mode = Mode::kHost;
}

// The chunk's upload is only enqueued: its buffers stay untouched until the builder
// syncs its uploads (a chunk let go past retainBytes(), finish, destroy).
bool BloomFilter::stream_chunk(Chunk &c) const {
    if (c.fixed > 0)
        return nb_builder_add_batch_async(stream, c.bytes, nullptr, (uint32_t)c.fixed, c.n) == NB_OK;
    if (c.fixed == 0) {  // all keys empty
        need_offsets(c);
        for (uint64_t i = 0; i <= c.n; ++i) c.offs[i] = 0;
    }
    return nb_builder_add_batch_async(stream, c.bytes, c.offs, 0, c.n) == NB_OK;
}

// The pending batch through nb_build_cpu (the kernels' index arithmetic) into the
// filter's own words.
void BloomFilter::build_chunk_on_host(Chunk &c) const {
    std::vector<uint64_t> &w = own_bits();
    if (c.fixed == 0) {
        need_offsets(c);
        for (uint64_t i = 0; i <= c.n; ++i) c.offs[i] = 0;
    }
    const int rc = c.fixed > 0 ? nb_build_cpu(c.bytes, nullptr, (uint32_t)c.fixed, c.n, m, k, h2_seed,
                                              flavor, w.data())
                               : nb_build_cpu(c.bytes, c.offs, 0, c.n, m, k, h2_seed, flavor, w.data());
    if (rc != NB_OK)  // only argument errors reach here (m, k, flavor checked on entry)
        throw std::runtime_error(std::string("nasp_bloom: nb_build_cpu failed: ") + nb_last_error());
}

// A device error while keys are streaming: rebuild every streamed key on the host
// from the bits the builder started with, or -- when streamed keys were let go past
// retainBytes() -- report it.
void BloomFilter::device_failed(const char *what) const {
    const std::string err = nb_last_error();
    if (stream) (void)nb_builder_destroy(stream);
    stream = nullptr;
    bits = bits_before;
    bits_before.reset();
    mode = Mode::kHost;
    if (!retained_all) {
        const uint64_t lost = pending_n;
        release_chunks();
        throw std::runtime_error(std::string("nasp_bloom: device build failed during ") + what + " (" +
                                 err + ") after more streamed keys than retainBytes() keeps; " +
                                 std::to_string(lost) + " keys are not in the filter");
    }
    std::cerr << "[BloomFilter] GPU build failed (" << err << "); building " << pending_n
              << " keys on the host\n";
    std::vector<Chunk> redo;
    redo.swap(retained);
    for (size_t i = 0; i < redo.size(); ++i) {
        try {
            build_chunk_on_host(redo[i]);
        } catch (...) {
            for (size_t j = i; j < redo.size(); ++j) free_chunk(redo[j]);
            throw;
        }
        free_chunk(redo[i]);
    }
}

// The chunks in `pending` leave it (the last one is full, or the filter is being
// read): streamed to the device builder (and kept for a host rebuild while the
// retention budget lasts), built on the host, or -- while the batch is still too
// small to decide -- kept.
void BloomFilter::hand_off() const {
    if (mode == Mode::kPending) {
        if (pending_n < g_host_batch_limit) return;  // undecided: keep packing
        open_device();
    }
    std::vector<Chunk> todo;
    todo.swap(pending);
    uint64_t kept = 0;
    for (const Chunk &c : retained) kept += c.used;
    size_t i = 0;
    bool moved = false;  // todo[i] belongs to `retained`
    try {
        for (; i < todo.size(); ++i) {
            Chunk &c = todo[i];
            moved = false;
            if (mode == Mode::kDevice) {
                if (stream_chunk(c)) {
                    if (retained_all && kept + c.used <= g_retain_bytes) {
                        retained.push_back(c);
                        kept += c.used;
                    } else {  // let go: its upload must land before the buffer is reused
                        if (nb_builder_sync_uploads(stream) != NB_OK) {
                            retained.push_back(c);  // nothing lost yet: rebuild on the host
                            moved = true;
                            device_failed("a chunk upload");
                            continue;
                        }
                        retained_all = false;
                        free_chunk(c);
                    }
                    continue;
                }
                retained.push_back(c);  // the failed chunk joins the host rebuild
                moved = true;
                device_failed("a chunk upload / build");  // -> kHost, or throws
                continue;
            }
            build_chunk_on_host(c);
            free_chunk(c);
        }
    } catch (...) {
        for (size_t j = moved ? i + 1 : i; j < todo.size(); ++j) free_chunk(todo[j]);
        throw;
    }
}

// Materialise: every key added since the last read is in `bits`.
void BloomFilter::flush() const {
    if (pending_n == 0) return;
    if (mode == Mode::kPending && pending_n < g_host_batch_limit) mode = Mode::kHost;
    hand_off();
    last_on_device = false;
    if (mode == Mode::kDevice) {
        auto out = std::make_shared<std::vector<uint64_t>>(((size_t)m + 63) / 64);
        if (nb_builder_finish(stream, out->data()) == NB_OK) {
            (void)nb_builder_destroy(stream);
            stream = nullptr;
            bits = std::move(out);
            bits_before.reset();
            for (Chunk &c : retained) free_chunk(c);
            retained.clear();
            last_on_device = true;
        } else {
            device_failed("the filter download");
        }
    }
    pending_n = 0;
    mode = Mode::kPending;
    retained_all = true;
}

// BloomFilter.cpp:67-80 for one key, on the host against the same bits.
bool BloomFilter::possiblyContains(const std::string &elem) const {
    if (!closures || k == 0) return true;
    if (m == 0) throw std::runtime_error("nasp_bloom: possiblyContains() on a filter with m == 0");
    flush();
    if (!bits) return false;  // every bit zero
    const nb::FilterConsts c = nb::make_consts(m, k, h2_seed, (uint32_t)flavor);
    uint64_t h1, h2;
    nb::key_hashes_host(c, reinterpret_cast<const uint8_t *>(elem.data()), elem.size(), &h1, &h2);
    nb::IndexGen g;
    g.start(h1, h2, c);
    const uint64_t *w = bits->data();
    for (uint32_t i = 0; i < k; ++i) {
        if (i) g.next(c);
        if (!((w[g.r >> 6] >> (g.r & 63)) & 1u)) return false;
    }
    return true;
}

// BloomFilter.cpp:88-129
std::vector<std::byte> BloomFilter::serialize() const {
    flush();
    std::vector<std::byte> out(nb_serialized_size(m));
    if (bits) {
        nb_serialize(m, k, p, timeConst, h2_seed, bits->data(), reinterpret_cast<uint8_t *>(out.data()));
    } else {  // all zero: the header over an empty payload (`out` is zero-filled)
        static const uint64_t zero = 0;
        nb_serialize(0, k, p, timeConst, h2_seed, &zero, reinterpret_cast<uint8_t *>(out.data()));
        std::memcpy(out.data(), &m, 4);
    }
    return out;
}

// BloomFilter.cpp:131-190 (hash closures exist whenever the header's k > 0).
// The reference reads past a short image; here a short one throws.
BloomFilter BloomFilter::deserialize(const std::vector<std::byte> &data) {
    BloomFilter bf;
    uint32_t mm = 0, kk = 0, tc = 0;
    double pp = 0;
    uint64_t seed = 0;
    const uint8_t *img = reinterpret_cast<const uint8_t *>(data.data());
    if (nb_deserialize(img, data.size(), &mm, &kk, &pp, &tc, &seed, nullptr) != NB_OK)
        throw std::runtime_error(std::string("nasp_bloom: deserialize: ") + nb_last_error());
    bf.m = mm;
    bf.k = kk;
    bf.p = pp;
    bf.timeConst = tc;
    bf.h2_seed = seed;
    auto w = std::make_shared<std::vector<uint64_t>>(((size_t)mm + 63) / 64, 0);
    if (!w->empty() &&
        nb_deserialize(img, data.size(), nullptr, nullptr, nullptr, nullptr, nullptr, w->data()) != NB_OK)
        throw std::runtime_error(std::string("nasp_bloom: deserialize: ") + nb_last_error());
    bf.bits = std::move(w);
    bf.closures = true;
    return bf;
}
