// BloomFilter.cpp -- the drop-in class over the C ABI (include/nasp_bloom.h).
// See BloomFilter.h for the contract; reference behaviour cited per method.
#include "BloomFilter.h"

#include <atomic>
#include <cstring>
#include <ctime>
#include <iostream>
#include <stdexcept>
#include <string>

#include "../../include/nasp_bloom.h"
#include "../csrc/bloom_math.h"

namespace {
int g_default_flavor = NB_FLAVOR_LIBSTDCXX;
std::atomic<uint64_t> g_host_batch_limit{4096};

constexpr size_t kChunkBytes = size_t(16) << 20;  // the streaming builder's chunk
constexpr uint64_t kChunkKeys = uint64_t(1) << 20;
}  // namespace

void BloomFilter::setDefaultFlavor(int f) { g_default_flavor = f; }
void BloomFilter::setHostBatchLimit(uint64_t keys) { g_host_batch_limit = keys; }
uint64_t BloomFilter::hostBatchLimit() { return g_host_batch_limit; }

// BloomFilter.cpp:26 -- no hash closures: every probe answers true.
BloomFilter::BloomFilter() : flavor(g_default_flavor) {}

// BloomFilter.cpp:28-65
BloomFilter::BloomFilter(unsigned int n, double falsePositiveRate) : flavor(g_default_flavor) {
    m = calculateSizeOfBitSet(n, falsePositiveRate);
    k = calculateNumberOfHashFunctions(n, m);
    p = falsePositiveRate;
    bits.assign(((size_t)m + 63) / 64, 0);
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
    bits = o.bits;
    bits_zero = o.bits_zero;
    last_on_device = o.last_on_device;
}

BloomFilter &BloomFilter::operator=(const BloomFilter &o) {
    if (this == &o) return *this;
    o.flush();
    m = o.m; k = o.k; p = o.p; timeConst = o.timeConst; h2_seed = o.h2_seed;
    closures = o.closures; flavor = o.flavor; device = o.device;
    bits = o.bits;
    bits_zero = o.bits_zero;
    last_on_device = o.last_on_device;
    pending.clear();
    pending_n = 0;
    return *this;
}

// BloomFilter.cpp:82-86: the key joins the packed batch; it is built (on the GPU,
// or on the host for small batches) when the filter is next read.
void BloomFilter::add(const std::string &elem) {
    if (!closures || k == 0) return;  // no hash closures: nothing to set
    // the reference divides by m in every closure: m == 0 is undefined there
    if (m == 0) throw std::runtime_error("nasp_bloom: add() on a filter with m == 0");
    const uint64_t len = elem.size();
    if (pending.empty() || pending.back().n == kChunkKeys ||
        (pending.back().n && pending.back().bytes.size() + len > kChunkBytes))
        pending.emplace_back();
    Chunk &c = pending.back();
    if (c.fixed == -1) {
        c.fixed = (int64_t)len;
    } else if (c.fixed >= 0 && c.fixed != (int64_t)len) {  // lengths differ from here on
        c.offs.resize(c.n + 1);
        for (uint64_t i = 0; i <= c.n; ++i) c.offs[i] = i * (uint64_t)c.fixed;
        c.fixed = -2;
    }
    c.bytes.insert(c.bytes.end(), elem.begin(), elem.end());
    if (c.fixed == -2) c.offs.push_back(c.bytes.size());
    ++c.n;
    ++pending_n;
}

void BloomFilter::addBatch(const std::vector<std::string> &elems) {
    for (const std::string &e : elems) add(e);
}

// The pending batch through the streaming builder on `device`, into a fresh
// buffer that replaces `bits` only if every step succeeded.
bool BloomFilter::build_on_device() const {
    nb_builder *b = nullptr;
    int rc = nb_builder_create(m, k, h2_seed, flavor, bits_zero ? nullptr : bits.data(), device, &b);
    for (size_t i = 0; i < pending.size() && rc == NB_OK; ++i) {
        Chunk &c = pending[i];
        if (c.fixed > 0) {
            rc = nb_builder_add_batch(b, c.bytes.data(), nullptr, (uint32_t)c.fixed, c.n);
        } else {
            if (c.fixed == 0) c.offs.assign(c.n + 1, 0);  // all keys empty
            rc = nb_builder_add_batch(b, c.bytes.data(), c.offs.data(), 0, c.n);
        }
    }
    std::vector<uint64_t> out;
    if (rc == NB_OK) {
        out.resize(bits.size());
        rc = nb_builder_finish(b, out.data());
    }
    std::string err = rc == NB_OK ? std::string() : std::string(nb_last_error());
    if (b) (void)nb_builder_destroy(b);
    if (rc != NB_OK) {
        std::cerr << "[BloomFilter] GPU build failed (" << err << "); building " << pending_n
                  << " keys on the host\n";
        return false;
    }
    bits.swap(out);
    return true;
}

// The pending batch on the host (nb_build_cpu: the kernels' index arithmetic).
void BloomFilter::build_on_host() const {
    for (Chunk &c : pending) {
        if (c.fixed == 0) c.offs.assign(c.n + 1, 0);
        // nb_build_cpu reads whole aligned 8-byte words that hold key bytes (as the
        // kernels do): pad the chunk so its last word is inside the allocation
        c.bytes.resize(c.bytes.size() + 8);
        const int rc = c.fixed > 0
                           ? nb_build_cpu(c.bytes.data(), nullptr, (uint32_t)c.fixed, c.n, m, k,
                                          h2_seed, flavor, bits.data())
                           : nb_build_cpu(c.bytes.data(), c.offs.data(), 0, c.n, m, k, h2_seed,
                                          flavor, bits.data());
        if (rc != NB_OK)  // only argument errors reach here (m, k, flavor checked on entry)
            throw std::runtime_error(std::string("nasp_bloom: nb_build_cpu failed: ") + nb_last_error());
    }
}

// Materialise: build the pending batch into `bits`.
void BloomFilter::flush() const {
    if (pending_n == 0) return;
    last_on_device = pending_n >= g_host_batch_limit && build_on_device();
    if (!last_on_device) build_on_host();
    pending.clear();
    pending_n = 0;
    bits_zero = false;
}

// BloomFilter.cpp:67-80 for one key, on the host against the same bits.
bool BloomFilter::possiblyContains(const std::string &elem) const {
    if (!closures || k == 0) return true;
    if (m == 0) throw std::runtime_error("nasp_bloom: possiblyContains() on a filter with m == 0");
    flush();
    const nb::FilterConsts c = nb::make_consts(m, k, h2_seed, (uint32_t)flavor);
    uint64_t h1, h2;
    nb::key_hashes_host(c, reinterpret_cast<const uint8_t *>(elem.data()), elem.size(), &h1, &h2);
    nb::IndexGen g;
    g.start(h1, h2, c);
    for (uint32_t i = 0; i < k; ++i) {
        if (i) g.next(c);
        if (!((bits[g.r >> 6] >> (g.r & 63)) & 1u)) return false;
    }
    return true;
}

// BloomFilter.cpp:88-129
std::vector<std::byte> BloomFilter::serialize() const {
    flush();
    std::vector<std::byte> out(nb_serialized_size(m));
    static const uint64_t zero = 0;
    nb_serialize(m, k, p, timeConst, h2_seed, bits.empty() ? &zero : bits.data(),
                 reinterpret_cast<uint8_t *>(out.data()));
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
    bf.bits.assign(((size_t)mm + 63) / 64, 0);
    bf.bits_zero = false;
    if (!bf.bits.empty() &&
        nb_deserialize(img, data.size(), nullptr, nullptr, nullptr, nullptr, nullptr,
                       bf.bits.data()) != NB_OK)
        throw std::runtime_error(std::string("nasp_bloom: deserialize: ") + nb_last_error());
    bf.closures = true;
    return bf;
}
