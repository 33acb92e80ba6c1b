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
//     serialized LSB-first byte image) instead of vector<bool>, shared between
//     copies until one of them changes (`bloom_ = bf`, SSTable.cpp:35, copies no
//     bits);
//   - add() packs the key into a host chunk (16 MB of key bytes / 1M keys; offsets
//     only once the chunk's key lengths differ; page-locked via nb_host_alloc and
//     pooled across filters, so a chunk's upload is an asynchronous DMA).  Once the keys added since the
//     last read reach hostBatchLimit() (4 096, the library's own host/device
//     cut-over) a streaming device builder (nb_builder_*) is opened, and from then
//     on every chunk that fills is handed to it at once: its upload and device
//     build overlap the packing of the next keys.  The filter is downloaded when
//     it is next read (possiblyContains / serialize / copy);
//   - a read with fewer pending keys -- e.g. the TypesManager deserialize ->
//     add(one value) -> serialize round trip (TypesManager.cpp:74-92) -- builds
//     them on the host with nb_build_cpu, the kernels' own index arithmetic
//     (csrc/bloom_math.h): no device round trip;
//   - device failure (§8(b) errors): with no usable GPU (NB_ERR_NODEV) every batch
//     is built on the host, chunk by chunk as it fills, after one std::cerr line per
//     process.  A device error once keys are streaming: the streamed chunks are
//     kept on the host up to retainBytes() (default 256 MiB of key bytes, i.e.
//     SSTables of up to ~16M 16-byte keys), so the batch is rebuilt on the host
//     after one std::cerr line, in the reference's error style (SSTableComp.cpp:543);
//     past that budget the keys are gone and add()/serialize() throw
//     std::runtime_error carrying the device error -- a faulted GPU is reported,
//     not hidden behind slow host builds;
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
#include <memory>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

struct nb_builder;  // include/nasp_bloom.h

class BloomFilter {
private:
    unsigned int m = 0;         // Size of the bit set/array
    unsigned int k = 0;         // Number of hash functions
    double p = 0.0;             // False-positive probability
    // Bit set: ceil(m/64) little-endian words, shared by copies (copy on write);
    // null while every bit is zero (mutable: const readers build pending keys).
    mutable std::shared_ptr<std::vector<uint64_t>> bits;
    unsigned int timeConst = 0; // Seed for generating hash functions
    size_t h2_seed = 0;         // Seed for the second hash function
    bool closures = false;      // the reference's hashFunctions is non-empty

    int flavor;                 // std::hash flavour (NB_FLAVOR_*)
    int device = 0;

    // A host chunk of packed keys (buffers come from a process-wide pool).
    struct Chunk {
        uint8_t *bytes = nullptr;    // kChunkBytes capacity (pinned when a device is visible)
        uint64_t *offs = nullptr;    // kChunkKeys + 1 entries, allocated once lengths differ
        bool pinned = false, offs_pinned = false;
        uint64_t used = 0, n = 0;    // key bytes, keys
        uint64_t byte_cap = 0, key_cap = 0;  // kChunkBytes / kChunkKeys (pooled), or
                                             // one oversized key's exact size
        int64_t fixed = -1;          // common key length (-1: no key yet, -2: mixed)
    };
    enum class Mode { kPending, kHost, kDevice };
    // Keys added since the last read (mutable: const readers build them).
    mutable std::vector<Chunk> pending;   // not yet built or streamed (last = filling)
    mutable std::vector<Chunk> retained;  // streamed, kept for a host rebuild
    mutable uint64_t pending_n = 0;       // keys added since the last read
    mutable Mode mode = Mode::kPending;
    mutable nb_builder *stream = nullptr; // open device builder (kDevice)
    mutable bool retained_all = true;     // every streamed chunk is in `retained`
    mutable std::shared_ptr<std::vector<uint64_t>> bits_before;  // bits the builder started from
    mutable bool last_on_device = false;

    void flush() const;
    void hand_off() const;                   // the chunks in `pending` leave it
    void open_device() const;                // kPending -> kDevice (or kHost)
    bool stream_chunk(Chunk &c) const;       // false: the device failed
    void device_failed(const char *what) const;
    void build_chunk_on_host(Chunk &c) const;
    std::vector<uint64_t> &own_bits() const; // unshared, allocated words
    void release_chunks() const;
    static void free_chunk(Chunk &c);
    static void need_offsets(Chunk &c);
    void reset_moved() noexcept;

public:
    // Constructor
    BloomFilter();
    BloomFilter(unsigned int n, double falsePositiveRate);
    // Copyable and assignable like the reference class (SSTable.cpp:35 assigns
    // the built filter): a copy materialises the source's pending keys first and
    // then shares its words until either side changes them.
    BloomFilter(const BloomFilter &o);
    BloomFilter &operator=(const BloomFilter &o);
    // A moved-from filter is left default-constructed (answers true, no bits).
    BloomFilter(BloomFilter &&o) noexcept;
    BloomFilter &operator=(BloomFilter &&o) noexcept;
    ~BloomFilter();

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
    // Reads with fewer pending keys than this build them on the host (default 4 096).
    static void setHostBatchLimit(uint64_t keys);
    static uint64_t hostBatchLimit();
    // Streamed key bytes kept on the host for a rebuild after a device error.
    static void setRetainBytes(uint64_t bytes);
    static uint64_t retainBytes();
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
