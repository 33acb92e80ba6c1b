// ref_harness.cpp -- extern "C" shim around the REAL reference BloomFilter,
// compiled from /root/reference/BloomFilter/BloomFilter.cpp where it lies
// (recipe: oracle/Makefile target `ref`; output only into oracle/_ref/).
//
// TEST INFRASTRUCTURE ONLY: used to pin the oracle restatement, to generate the
// golden vectors (tests/golden/gen_golden.py) and as bench.py's cpu_baseline
// (kind "reference").  This file is our own code; no reference source is copied.
//
// (m, k, seed) are injected through the reference's own deserialize()
// (BloomFilter.cpp:131-190), then keys go through the reference add()
// (BloomFilter.cpp:82-86) one std::string at a time, exactly as SSTable::build
// does (SSTable/SSTable.cpp:28-35).
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "BloomFilter.h"

namespace {

std::vector<std::byte> header_only(uint32_t m, uint32_t k, double p, uint32_t tc,
                                   uint64_t seed) {
    size_t nbytes = static_cast<uint32_t>(m + 7u) / 8u;
    std::vector<std::byte> img(28 + nbytes, std::byte{0});
    std::memcpy(img.data() + 0, &m, 4);
    std::memcpy(img.data() + 4, &k, 4);
    std::memcpy(img.data() + 8, &p, 8);
    std::memcpy(img.data() + 16, &tc, 4);
    std::memcpy(img.data() + 20, &seed, 8);
    return img;
}

inline void key_at(const uint8_t* keys, const uint64_t* offs, uint32_t key_len,
                   uint64_t i, std::string& s) {
    if (offs)
        s.assign(reinterpret_cast<const char*>(keys + offs[i]), offs[i + 1] - offs[i]);
    else
        s.assign(reinterpret_cast<const char*>(keys + i * key_len), key_len);
}

}  // namespace

extern "C" {

uint64_t ref_std_hash(const uint8_t* p, uint64_t len) {
    return std::hash<std::string>()(std::string(reinterpret_cast<const char*>(p), len));
}

// Constructor path: BloomFilter(n, p) then serialize; returns header fields.
int ref_ctor_params(uint32_t n, double p, uint32_t* m, uint32_t* k,
                    uint32_t* time_const, uint64_t* seed) {
    BloomFilter bf(n, p);
    std::vector<std::byte> img = bf.serialize();
    std::memcpy(m, img.data() + 0, 4);
    std::memcpy(k, img.data() + 4, 4);
    std::memcpy(time_const, img.data() + 16, 4);
    std::memcpy(seed, img.data() + 20, 8);
    return 0;
}

uint32_t ref_size_of_bitset(uint32_t n, double p) {
    return BloomFilter::calculateSizeOfBitSet(n, p);
}
uint32_t ref_num_hashes(uint32_t n, uint32_t m) {
    return BloomFilter::calculateNumberOfHashFunctions(n, m);
}

// Build with explicit (m, k, seed); if `initial` is non-null it is a full
// serialized image to start from (accumulate semantics, TypesManager.cpp:84-86).
// Writes the serialized image to `out` (28 + (uint32)(m+7)/8 bytes).
int ref_build(const uint8_t* keys, const uint64_t* offs, uint32_t key_len, uint64_t n,
              uint32_t m, uint32_t k, double p, uint32_t tc, uint64_t seed,
              const uint8_t* initial, uint8_t* out) {
    std::vector<std::byte> img = header_only(m, k, p, tc, seed);
    if (initial) std::memcpy(img.data(), initial, img.size());
    BloomFilter bf = BloomFilter::deserialize(img);
    std::string s;
    for (uint64_t i = 0; i < n; ++i) {
        key_at(keys, offs, key_len, i, s);
        bf.add(s);
    }
    std::vector<std::byte> res = bf.serialize();
    std::memcpy(out, res.data(), res.size());
    return 0;
}

// Timed form for bench.py's cpu_baseline: the same add() loop, with only the
// loop itself inside the clock (deserialize/serialize are O(m) setup).
double ref_build_timed(const uint8_t* keys, const uint64_t* offs, uint32_t key_len, uint64_t n,
                       uint32_t m, uint32_t k, uint64_t seed, uint8_t* out_first_bytes,
                       uint64_t nout) {
    std::vector<std::byte> img = header_only(m, k, 0.01, 0, seed);
    BloomFilter bf = BloomFilter::deserialize(img);
    std::string s;
    auto t0 = std::chrono::steady_clock::now();
    for (uint64_t i = 0; i < n; ++i) {
        key_at(keys, offs, key_len, i, s);
        bf.add(s);
    }
    auto t1 = std::chrono::steady_clock::now();
    if (out_first_bytes && nout) {
        std::vector<std::byte> res = bf.serialize();
        std::memcpy(out_first_bytes, res.data(), std::min<uint64_t>(nout, res.size()));
    }
    return std::chrono::duration<double>(t1 - t0).count();
}

// Probe `n` keys against a serialized image.
int ref_probe(const uint8_t* image, uint64_t image_len, const uint8_t* keys,
              const uint64_t* offs, uint32_t key_len, uint64_t n, uint8_t* out) {
    std::vector<std::byte> img(image_len);
    std::memcpy(img.data(), image, image_len);
    BloomFilter bf = BloomFilter::deserialize(img);
    std::string s;
    for (uint64_t i = 0; i < n; ++i) {
        key_at(keys, offs, key_len, i, s);
        out[i] = bf.possiblyContains(s) ? 1 : 0;
    }
    return 0;
}

// Default-constructed filter probe (BloomFilter.cpp:26 + :67-80): no closures.
int ref_default_contains(const uint8_t* key, uint64_t len) {
    BloomFilter bf;
    return bf.possiblyContains(std::string(reinterpret_cast<const char*>(key), len)) ? 1 : 0;
}

}  // extern "C"
