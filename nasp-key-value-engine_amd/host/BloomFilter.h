// BloomFilter.h -- drop-in replacement for the reference class
// (reference BloomFilter/BloomFilter.h:12-42), backed by the MI355X build path.
//
// Same public surface, argument meaning and semantics, so the reference callers
// compile unchanged: SSTable::build (SSTable/SSTable.cpp:28-35), the Raw/Comp
// filter writers and readers (SSTableRaw.cpp:539,620; SSTableComp.cpp:476,555),
// TypesManager (System/TypesManager.cpp:58-107).
//
// What changes inside (SURVEY.md §8(b) batching strategy):
//   - the bit set is a std::vector<uint64_t> (little-endian words == the
//     serialized LSB-first byte image) instead of vector<bool>;
//   - add() appends the key to a packed host batch (16 MB chunks: bytes, and
//     offsets only once the chunk's key lengths differ); the batch is built when
//     the filter is next read (possiblyContains / serialize / copy);
//   - a batch of at least hostBatchLimit() keys (default 4 096, the same cut-over
//     the library's `auto` path uses) is built on the GPU through the streaming
//     builder (nb_builder_*), chunk by chunk; a smaller one -- e.g. the
//     TypesManager deserialize -> add(one value) -> serialize round trip
//     (TypesManager.cpp:74-92) -- is built on the host by nb_build_cpu with the
//     kernels' own index arithmetic (csrc/bloom_math.h): no device round trip;
//   - if the device build fails (no GPU, device error) the batch is built on the
//     host instead and one line goes to std::cerr, in the reference's error style
//     (SSTableComp.cpp:543): add() and serialize() never throw for it;
//   - possiblyContains() of one key is evaluated on the host against the same
//     bits (the latency-bound lookup path, SSTManager.cpp:203,224).
// Semantics kept: default-constructed filter answers true for every key
// (BloomFilter.cpp:26,67-80); add() after deserialize() ORs into the loaded bits
// (TypesManager.cpp:84-86); serialize() is byte-identical (BloomFilter.cpp:88-129).
#pragma once

// The reference header's includes are kept: its callers rely on them
// transitively (e.g. SSTable.cpp uses std::memcpy via <cstring>).
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <ctime>
#include <functional>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

class BloomFilter {
private:
    unsigned int m = 0;         // Size of the bit set/array
    unsigned int k = 0;         // Number of hash functions
    double p = 0.0;             // False-positive probability
    mutable std::vector<uint64_t> bits;  // Bit set: ceil(m/64) little-endian words
                                         // (mutable: const readers build pending keys)
    unsigned int timeConst = 0; // Seed for generating hash functions
    size_t h2_seed = 0;         // Seed for the second hash function
    bool closures = false;      // the reference's hashFunctions is non-empty

    int flavor;                 // std::hash flavour (NB_FLAVOR_*)
    int device = 0;
    // Keys added since the last read, packed (mutable: const readers build them).
    struct Chunk {
        std::vector<uint8_t> bytes;
        std::vector<uint64_t> offs;  // n + 1 entries once lengths differ (fixed < 0)
        int64_t fixed = -1;          // common key length (-1: no key yet, -2: mixed)
        uint64_t n = 0;
    };
    mutable std::vector<Chunk> pending;
    mutable uint64_t pending_n = 0;
    mutable bool bits_zero = true;   // `bits` is still all zero
    mutable bool last_on_device = false;

    void flush() const;
    bool build_on_device() const;
    void build_on_host() const;

public:
    // Constructor
    BloomFilter();
    BloomFilter(unsigned int n, double falsePositiveRate);
    // Copyable and assignable like the reference class (SSTable.cpp:35 assigns
    // the built filter): a copy materialises the source's pending keys first.
    BloomFilter(const BloomFilter &o);
    BloomFilter &operator=(const BloomFilter &o);
    BloomFilter(BloomFilter &&o) noexcept = default;
    BloomFilter &operator=(BloomFilter &&o) noexcept = default;
    ~BloomFilter() = default;

    // Add an element to the Bloom Filter
    void add(const std::string& elem);

    // Check if an element is present
    bool possiblyContains(const std::string& elem) const;

    // Serialize Bloom Filter to a vector of bytes
    std::vector<std::byte> serialize() const;

    // Deserialize Bloom Filter from a vector of bytes
    static BloomFilter deserialize(const std::vector<std::byte>& data);

    // Helper functions
    static unsigned int calculateSizeOfBitSet(unsigned int expectedElements, double falsePositiveRate);
    static unsigned int calculateNumberOfHashFunctions(unsigned int expectedElements, unsigned int m);

    // ---- extensions (not in the reference) ----
    // Which std::hash the filter's indices follow: NB_FLAVOR_LIBSTDCXX (default,
    // a Linux build of the reference) or NB_FLAVOR_MSVC_FNV1A (files written by
    // the authors' Windows build, e.g. the reference's committed *.sst filters).
    static void setDefaultFlavor(int flavor);
    // Batches of fewer keys than this are built on the host (default 4 096).
    static void setHostBatchLimit(uint64_t keys);
    static uint64_t hostBatchLimit();
    void setFlavor(int f) { flush(); flavor = f; }
    void setDevice(int d) { device = d; }
    // Add many keys at once (same result as add() on each).
    void addBatch(const std::vector<std::string>& elems);
    // Build every pending key now (no-op if none).
    void materialize() const { flush(); }
    // Whether the last materialised batch was built on the GPU.
    bool lastBuildOnDevice() const { return last_on_device; }
    unsigned int bitCount() const { return m; }
    unsigned int hashCount() const { return k; }
};
