// BloomFilter.cpp -- the drop-in class over the C ABI (include/nasp_bloom.h).
// See BloomFilter.h for the contract; reference behaviour cited per method.
#include "BloomFilter.h"

#include <cstring>
#include <ctime>
#include <stdexcept>
#include <string>

#include "../../include/nasp_bloom.h"
#include "../csrc/bloom_math.h"

namespace {
int g_default_flavor = NB_FLAVOR_LIBSTDCXX;

void check(int rc, const char *what) {
    if (rc != NB_OK)
        throw std::runtime_error(std::string("nasp_bloom: ") + what + " failed: " + nb_last_error());
}
}  // namespace

void BloomFilter::setDefaultFlavor(int f) { g_default_flavor = f; }

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
}

BloomFilter &BloomFilter::operator=(const BloomFilter &o) {
    if (this == &o) return *this;
    o.flush();
    release();
    m = o.m; k = o.k; p = o.p; timeConst = o.timeConst; h2_seed = o.h2_seed;
    closures = o.closures; flavor = o.flavor; device = o.device;
    bits = o.bits;
    bits_zero = o.bits_zero;
    return *this;
}

BloomFilter::BloomFilter(BloomFilter &&o) noexcept
    : m(o.m), k(o.k), p(o.p), bits(std::move(o.bits)), timeConst(o.timeConst),
      h2_seed(o.h2_seed), closures(o.closures), flavor(o.flavor), device(o.device),
      builder(o.builder), bits_zero(o.bits_zero) {
    o.builder = nullptr;
}

BloomFilter &BloomFilter::operator=(BloomFilter &&o) noexcept {
    if (this == &o) return *this;
    release();
    m = o.m; k = o.k; p = o.p; timeConst = o.timeConst; h2_seed = o.h2_seed;
    closures = o.closures; flavor = o.flavor; device = o.device;
    bits = std::move(o.bits);
    bits_zero = o.bits_zero;
    builder = o.builder;
    o.builder = nullptr;
    return *this;
}

BloomFilter::~BloomFilter() { release(); }

void BloomFilter::release() noexcept {
    if (builder) (void)nb_builder_destroy(builder);  // pending keys are dropped with the object
    builder = nullptr;
}

// BloomFilter.cpp:82-86: the key is packed into the streaming builder; its chunk
// is uploaded and built on the GPU while later keys are packed.
void BloomFilter::add(const std::string &elem) {
    if (!closures || k == 0) return;  // no hash closures: nothing to set
    if (m == 0) throw std::runtime_error("nasp_bloom: add() on a filter with m == 0");
    if (!builder)
        check(nb_builder_create(m, k, h2_seed, flavor, bits_zero ? nullptr : bits.data(), device,
                                &builder),
              "nb_builder_create");
    check(nb_builder_add(builder, reinterpret_cast<const uint8_t *>(elem.data()), elem.size()),
          "nb_builder_add");
}

void BloomFilter::addBatch(const std::vector<std::string> &elems) {
    for (const std::string &e : elems) add(e);
}

// Materialise: download the filter the builder holds, return its buffers.
void BloomFilter::flush() const {
    if (!builder) return;
    nb_builder *b = builder;
    builder = nullptr;
    const int rc = nb_builder_finish(b, bits.data());
    (void)nb_builder_destroy(b);
    check(rc, "nb_builder_finish");
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
    for (uint32_t i = 0; i < k; ++i) {
        const uint32_t b = (uint32_t)((h1 + (uint64_t)i * h2) % m);
        if (!((bits[b >> 6] >> (b & 63)) & 1u)) return false;
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

// BloomFilter.cpp:131-190 (hash closures exist whenever the header's k > 0)
BloomFilter BloomFilter::deserialize(const std::vector<std::byte> &data) {
    BloomFilter bf;
    uint32_t mm = 0, kk = 0, tc = 0;
    double pp = 0;
    uint64_t seed = 0;
    const uint8_t *img = reinterpret_cast<const uint8_t *>(data.data());
    check(nb_deserialize(img, data.size(), &mm, &kk, &pp, &tc, &seed, nullptr), "nb_deserialize");
    bf.m = mm;
    bf.k = kk;
    bf.p = pp;
    bf.timeConst = tc;
    bf.h2_seed = seed;
    bf.bits.assign(((size_t)mm + 63) / 64, 0);
    bf.bits_zero = false;
    if (!bf.bits.empty())
        check(nb_deserialize(img, data.size(), nullptr, nullptr, nullptr, nullptr, nullptr,
                             bf.bits.data()),
              "nb_deserialize");
    bf.closures = true;
    return bf;
}
