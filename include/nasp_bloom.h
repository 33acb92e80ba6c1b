/*
 * nasp_bloom.h -- C ABI of the MI355X-native SSTable Bloom-filter build/probe path.
 *
 * This is the drop-in boundary.  The reference has no FFI of its
 * own: its callers use the C++ class `BloomFilter` (reference
 * BloomFilter/BloomFilter.h:12-42) directly.  The replacement class in
 * nasp-key-value-engine_amd/host/BloomFilter.h keeps that surface and calls the
 * entry points below; any other language binds them the way INTEGRATION.md shows.
 *
 * Conventions
 *   - Plain pointers and sizes only; nothing here throws.  Every function returns
 *     NB_OK (0) or a negative NB_ERR_* code; nb_last_error() describes the last
 *     failure of the calling thread.
 *   - Keys are arbitrary bytes (embedded NUL and empty keys allowed), packed:
 *       offsets != NULL : key i = keys[offsets[i] .. offsets[i+1]),  offsets has n+1 entries
 *       offsets == NULL : key i = keys[i*key_len .. (i+1)*key_len)   (fixed-length keys)
 *   - The filter is `words`: ceil(m/64) little-endian uint64 words; bit j of the
 *     reference bitSet (BloomFilter.h:17) is bit (j % 64) of words[j / 64].  This
 *     is byte-for-byte the bit payload of BloomFilter::serialize()
 *     (BloomFilter.cpp:117-126).  Builds OR into `words` (never clear it), which
 *     is the reference's add-after-deserialize semantics (TypesManager.cpp:84-86).
 *   - The caller owns every buffer.  The library owns only cached device scratch
 *     (per device) and releases it in nb_shutdown().
 *   - Re-entrant per (device, stream).  Host-buffer entry points serialize on a
 *     per-device lock around their cached scratch.
 *   - Index function (BloomFilter.cpp:57-62):  idx_i = (h1 + i*h2) mod m in 64-bit
 *     wrapping arithmetic, h1 = H(key), h2 = H(to_string(h2_seed) + key), where H is
 *     std::hash<std::string> of the selected flavor.
 */
#ifndef NASP_BLOOM_H
#define NASP_BLOOM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NB_ABI_VERSION 1

enum nb_status {
    NB_OK = 0,
    NB_ERR_ARG = -1,      /* invalid argument (e.g. m == 0 with keys, k == 0, NULL buffer) */
    NB_ERR_HIP = -2,      /* HIP runtime error (allocation, copy, launch) */
    NB_ERR_NODEV = -3,    /* no usable gfx950 device */
    NB_ERR_UNSUPPORTED = -4
};

/* Which std::hash<std::string> the reference binary was built with. */
enum nb_flavor {
    NB_FLAVOR_LIBSTDCXX = 0,  /* GCC libstdc++ std::_Hash_bytes(p, len, 0xc70f6907) (Linux build) */
    NB_FLAVOR_MSVC_FNV1A = 1, /* MSVC STL FNV-1a-64 (the authors' Windows build) */
    /* NOT the reference filter (no parity with any reference file): h1, h2 = the two
     * halves of MurmurHash3_x64_128(key, len, (uint32_t)h2_seed) -- the reference's
     * MurmurHash3/MurmurHash3.cpp:255-332 -- with the same (h1 + i*h2) % m closure.
     * The north star's "k MurmurHash3_x64_128 hashes" wording; filter builds and
     * probes only (nb_std_hash / Merkle stay std::hash flavours). */
    NB_FLAVOR_MURMUR3_X64_128 = 2
};

/* ---------------------------------------------------------------- info --- */
int nb_abi_version(void);
/* Number of visible HIP devices (0 when none). */
int nb_device_count(void);
/* Last error message of the calling thread ("" if none). */
const char *nb_last_error(void);
/* Release cached device scratch and streams on every device. */
int nb_shutdown(void);
/* Device builds enqueued by this process so far (every build entry point, any
 * device): lets a caller check whether a path reached the GPU. */
uint64_t nb_device_build_count(void);
/* The same for device Merkle trees (nb_merkle / nb_merkle_device). */
uint64_t nb_device_merkle_count(void);

/* Library switches (not part of the filter contract; no switch changes a filter's
 * bits): the A/B selections between equivalent build paths and the fault
 * injection the drop-in classes' fallback tests use.  Each is read from the
 * environment variable of the same name once, on first use; nb_set_knob changes
 * it for the whole process afterwards (thread-safe).  Names: NB_BUILD_PATH
 * (0 auto, 1 atomic, 2 tiled), NB_PROBE_PATH (0 auto, 1 one lane per key, 2 tiled,
 * 3 split: the tiled probe in two rounds), NB_PROBE_SPLIT_PCT (auto, k > 2: the split
 * path from this percentage of present keys in its sample up to 65 for 16- / 32-byte
 * keys at k <= 8, 55 above, 40 for variable-length keys; default 0, the policy: 7 for
 * 16- / 32-byte keys at k <= 8, 18 otherwise, on batches of 2^24 keys or more at k > 3,
 * never on smaller batches or at k = 3; > 100: never),
 * NB_PROBE_CHUNK (keys per tiled-probe pass; 0: the policy), NB_PROBE_TILED_PCT (auto's
 * tiled path from this percentage of present keys in its sample; default 0, the policy:
 * the split policy's upper bound above, 10 where the policy leaves the split path out,
 * 30 at k <= 2; a split threshold at or above it leaves the two-way choice), NB_PROBE_ENTRY (tiled-probe bucket entries:
 * 32 or 64 bits everywhere; default 0: 32 for the one-round tiled path, 64 for the
 * split path), NB_PROBE_BIN_GRID (blocks per CU of auto's gated, looping tiled-probe bin
 * kernels; 0: 2), NB_PROBE_KPT (keys per bin thread of the one-round 32-bit path; 0:
 * the policy, 2 at k = 7 for 16- / 32-byte keys), NB_PROBE_HOST_PICK (1: auto reads its sample back
 * on the host outside graph capture; 0, default: gated on the device),
 * NB_PACK, NB_TILE_BITS, NB_SHARDS, NB_CHUNK_KEYS, NB_TWO_LEVEL, NB_PACK5,
 * NB_ENTRY32, NB_RANK, NB_FIXED32, NB_FPMOD, NB_KEXACT, NB_BIN_WIDE, NB_OVERLAP (two-level
 * sub-passes pipelined over a second stream of the workspace: 0 off, 1/2 normal/high
 * priority, +4 tile kernels beside the next pass's bin kernel; default 6),
 * NB_SUBPASSES (bin + re-bin sub-passes per tile pass; default 0: 2 for builds of
 * several passes, 1 for one -- 0 is the policy, not one sub-pass),
 * NB_TILE_COUNT (0 counted-tile policy, 1 power-of-two tiles only, else that many),
 * NB_SHARDED_STAGE, NB_FAIL_BUILDS / NB_FAIL_MERKLES (the next N device builds /
 * trees fail with NB_ERR_HIP).  Round 5 removed the switches of variants measured
 * slower (NB_BIN_PIPE, NB_BIN_MIX, NB_BUCKET_GMAJOR = 0, NB_FINE_BITS = 19).
 * Unknown names: NB_ERR_ARG. */
int nb_set_knob(const char *name, uint64_t value);
int nb_get_knob(const char *name, uint64_t *value);

/* ------------------------------------------------- parameter formulas --- */
/* BloomFilter::calculateSizeOfBitSet (BloomFilter.cpp:192-194), including the
 * reference's wrap modulo 2^32 of an out-of-range double->unsigned conversion. */
uint32_t nb_size_of_bitset(uint32_t n, double p);
/* BloomFilter::calculateNumberOfHashFunctions (BloomFilter.cpp:196-199). */
uint32_t nb_num_hashes(uint32_t n, uint32_t m);
/* std::hash<std::string> of `len` bytes in the selected flavour (host only): the
 * reference's h1 (BloomFilter.cpp:59) and MerkleTree::hash (merkle.cpp:26-32).
 * NB_FLAVOR_MURMUR3_X64_128 gives the first half of MurmurHash3_x64_128(p, len, 0);
 * an unknown flavor returns 0 and sets nb_last_error(). */
uint64_t nb_std_hash(const uint8_t *p, uint64_t len, int flavor);
/* h2_seed from timeConst: mt19937(timeConst) + uniform_int_distribution<uint64_t>
 * (BloomFilter.cpp:37,44-46). */
uint64_t nb_seed_from_time(uint32_t time_const);

/* --------------------------------------------- host-buffer entry points --- */
/* Replaces the add() loop of SSTable::build (SSTable/SSTable.cpp:31-34) and
 * BloomFilter::add (BloomFilter.cpp:82-86) for a whole batch: uploads the keys,
 * builds on `device`, ORs the result into the host `words`. */
int nb_build(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
             uint32_t m, uint32_t k, uint64_t h2_seed, int flavor,
             uint64_t *words, int device);

/* Single-process multi-GPU nb_build (the C++ host's form of the cooperative C5
 * build, §8(e)): keys split into `nshards` contiguous ranges (<= 0: one per visible
 * device), shard s built on device s % device_count by its own streaming builder
 * and host thread; the partial filters are OR-merged slice-wise -- owner o ORs
 * word slice o of every other partial into its own, read in place (over xGMI
 * with peer access), and downloads its slice into `words`.  Same result and
 * OR-accumulate semantics as nb_build; at most 64 shards are used. */
int nb_build_sharded(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                     uint32_t m, uint32_t k, uint64_t h2_seed, int flavor, uint64_t *words,
                     int nshards);

/* The same build on the calling CPU thread: the drop-in class's path for small
 * batches and for hosts without a usable GPU, e.g. the
 * TypesManager deserialize -> add(one value) -> serialize round trip
 * (System/TypesManager.cpp:74-92).  Same index arithmetic as the kernels
 * (csrc/bloom_math.h); OR-accumulates into host `words`.  Reads the key bytes only
 * (no slack or alignment needed). */
int nb_build_cpu(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                 uint32_t m, uint32_t k, uint64_t h2_seed, int flavor, uint64_t *words);
/* nb_probe on the calling CPU thread (reads the key bytes only). */
int nb_probe_cpu(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                 uint32_t m, uint32_t k, uint64_t h2_seed, int flavor, const uint64_t *words,
                 uint8_t *out);

/* Batch form of BloomFilter::possiblyContains (BloomFilter.cpp:67-80):
 * out[i] = 1 if all k bits of key i are set, else 0.  k == 0 answers 1
 * (the default-constructed filter, BloomFilter.cpp:26). */
int nb_probe(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
             uint32_t m, uint32_t k, uint64_t h2_seed, int flavor,
             const uint64_t *words, uint8_t *out, int device);

/* ---------------------------------------------- streaming host builder --- */
/* The host side of SSTable::build's filter block (SSTable/SSTable.cpp:28-35):
 * keys arrive one at a time from the flushing memtable / compaction merge
 * (MemtableManager.cpp:109-130, LSMManager.cpp:42-90) and BloomFilter::add
 * (BloomFilter.cpp:82-86) is called per key.  A builder packs the keys into a
 * ring of pinned host chunks; every full chunk is uploaded asynchronously and
 * built on the device (OR-accumulated into the device-resident filter) while the
 * caller keeps packing the next one, so packing, PCIe and the build overlap.
 * Chunks whose keys all have one length travel without offsets.
 * Not thread-safe (one builder per caller thread, like the reference class). */
typedef struct nb_builder nb_builder;
/* init_words: ceil(m/64) host words the keys are OR-ed into (the add-after-
 * deserialize semantics, TypesManager.cpp:84-86), or NULL for a fresh filter. */
int nb_builder_create(uint32_t m, uint32_t k, uint64_t h2_seed, int flavor,
                      const uint64_t *init_words, int device, nb_builder **out);
/* BloomFilter::add of one key (any bytes, len may be 0). */
int nb_builder_add(nb_builder *b, const uint8_t *key, uint64_t len);
/* Many keys (same packing as nb_build): uploaded chunk by chunk straight from
 * the caller's buffer, each chunk's build overlapping the next chunk's upload.
 * The caller's buffers may be reused as soon as this returns (every upload from
 * them has completed); the builds stay asynchronous. */
int nb_builder_add_batch(nb_builder *b, const uint8_t *keys, const uint64_t *offsets,
                         uint32_t key_len, uint64_t n);
/* The same, returning once the uploads are enqueued: the caller keeps its buffers
 * untouched until nb_builder_sync_uploads, nb_builder_finish or nb_builder_destroy
 * returns (the drop-in class hands it the page-locked chunks it retains anyway, so
 * packing the next chunk overlaps the DMA of this one). */
int nb_builder_add_batch_async(nb_builder *b, const uint8_t *keys, const uint64_t *offsets,
                               uint32_t key_len, uint64_t n);
int nb_builder_sync_uploads(nb_builder *b);
/* Build everything added so far and copy the filter to `words` (ceil(m/64) host
 * words).  The builder stays usable: later adds OR into the same filter. */
int nb_builder_finish(nb_builder *b, uint64_t *words);
int nb_builder_destroy(nb_builder *b);

/* Page-locked host memory for key chunks handed to a builder (their uploads are
 * then true asynchronous DMA): the drop-in class packs keys straight into such
 * chunks.  NB_ERR_NODEV without a device (use ordinary memory then). */
int nb_host_alloc(size_t bytes, void **out);
int nb_host_free(void *p);

/* ------------------------------------------ device-resident entry points --- */
/* Same contracts; every pointer is device memory on the current device and
 * the work is enqueued on `stream` (a hipStream_t; NULL = the null stream).
 * No host synchronisation once the library's per-(device, stream) workspace is
 * large enough; the first call with a larger shape grows it (hipMalloc, stream
 * synchronised), so warm a stream up with its largest shape before capturing it
 * into a hipGraph.  Filters of more than 2 048 tiles (m > ~2^31, e.g. 2^32-1) are
 * built in passes whose re-bin and tile kernels run on a second stream of the
 * workspace (NB_OVERLAP): it waits on `stream` at entry and `stream` waits on it at
 * exit (events), so callers -- and stream capture, as a fork/join -- see one
 * stream.  Key memory is read only in aligned 8- and 16-byte granules
 * that hold key bytes, so a key buffer needs no slack past its last byte and
 * may start at any alignment (16-byte-aligned 16-byte keys take a faster path). */
int nb_build_device(const uint8_t *d_keys, const uint64_t *d_offsets, uint32_t key_len,
                    uint64_t n, uint32_t m, uint32_t k, uint64_t h2_seed, int flavor,
                    uint64_t *d_words, void *stream);

/* Flags of nb_build_device_ex. */
#define NB_BUILD_OVERWRITE 1u /* d_words := filter of this batch (a fresh filter, as
                                 SSTable::build makes; SSTable/SSTable.cpp:28) instead
                                 of OR-accumulating into it */

/* nb_build_device with flags (0 = exactly nb_build_device). */
int nb_build_device_ex(const uint8_t *d_keys, const uint64_t *d_offsets, uint32_t key_len,
                       uint64_t n, uint32_t m, uint32_t k, uint64_t h2_seed, int flavor,
                       uint64_t *d_words, uint32_t flags, void *stream);

/* Batch probe, device-resident.  Large batches (>= 4M keys) of 16-, 32-byte or
 * variable-length keys with k <= 8 (k <= 16 for 32-byte keys) may take the tiled
 * path (lookups binned by filter tile and tested in LDS: ~4x the one-lane-per-key
 * rate for present keys, ~half of it for absent ones) or, for k > 2, the split tiled
 * path (two rounds: every key's first two indices, then the rest for the keys still
 * possibly present); NB_PROBE_PATH=0 (auto) probes the first 4 096 keys one lane per
 * key and picks from the share of them present: the lane path below NB_PROBE_SPLIT_PCT
 * (the policy: 7 % for 16- / 32-byte keys at k <= 8, 18 % otherwise), the split path
 * up to 65 % (55 % for k > 8, 40 % for variable-length keys), the tiled path from
 * there.  The policy leaves the split path out below 2^24 keys and at k = 3 (the lane
 * path below 10 %, the tiled path from there; NB_PROBE_SPLIT_PCT > 100: the same
 * two-way choice everywhere), and a filter of at most 2^25 bits (4 MiB: one XCD's L2 holds it) takes the
 * lane path without a sample.  The choice is made on
 * the device: every path is launched behind the sample and gated on its count, so
 * auto never waits on the host (NB_PROBE_HOST_PICK=1 restores rounds 3-5's host
 * read-back outside graph capture).  The one-round tiled path's bucket entries are
 * 32-bit words behind one header word per run, the split path's key << 32 | offset
 * (NB_PROBE_ENTRY).  Same answers on every path. */
int nb_probe_device(const uint8_t *d_keys, const uint64_t *d_offsets, uint32_t key_len,
                    uint64_t n, uint32_t m, uint32_t k, uint64_t h2_seed, int flavor,
                    const uint64_t *d_words, uint8_t *d_out, void *stream);

/* d_dst[w] |= d_src[s*src_stride + w] for s < nsrc, w < nwords: the local OR step
 * of the cooperative multi-GPU build (RCCL has no bitwise-OR reduction). */
int nb_or_merge_device(uint64_t *d_dst, const uint64_t *d_src, uint64_t nwords,
                       uint32_t nsrc, uint64_t src_stride, void *stream);

/* ------------------------------------------------------------ Merkle tree --- */
/* The Merkle tree SSTable::build makes on the same flush (SSTable/SSTable.cpp:29-40;
 * SSTableRaw.cpp:238,392-397 over key ++ value), replacing MerkleTree(data)
 * (MerkleTree/merkle.cpp:7-55).  Records are packed like keys (offsets, or a fixed
 * rec_len).  The tree holds every level as std::hash values, leaves first, root
 * last: leaves[i] = H(record i); a parent is H(to_string(left) ++ to_string(right)),
 * the last node of an odd level paired with itself; the reference's strings are
 * the decimal forms of these values (getLeaves(), getRootHash(), and the
 * treeLevels generateProof walks).  n == 0 is NB_ERR_ARG (the reference throws). */
uint64_t nb_merkle_tree_size(uint64_t n);  /* n + ceil(n/2) + ... + 1 */
/* d_tree: nb_merkle_tree_size(n) device words; asynchronous on `stream`. */
int nb_merkle_device(const uint8_t *d_data, const uint64_t *d_offsets, uint32_t rec_len,
                     uint64_t n, int flavor, uint64_t *d_tree, void *stream);
/* Host buffers: tree (nb_merkle_tree_size(n) words) and leaves (n words) may be
 * NULL; *root always receives the root hash. */
int nb_merkle(const uint8_t *data, const uint64_t *offsets, uint32_t rec_len, uint64_t n,
              int flavor, uint64_t *tree, uint64_t *leaves, uint64_t *root, int device);
/* The same tree on the calling CPU thread (the drop-in MerkleTree's path for small
 * flushes and hosts without a usable GPU; the kernels' hashing, bloom_math.h).
 * Reads the record bytes only. */
int nb_merkle_cpu(const uint8_t *data, const uint64_t *offsets, uint32_t rec_len, uint64_t n,
                  int flavor, uint64_t *tree, uint64_t *leaves, uint64_t *root);

/* ------------------------------------------------------ serialization --- */
/* Size of BloomFilter::serialize()'s image: 28 + (uint32_t)(m+7)/8 bytes
 * (BloomFilter.cpp:89-90; the (m+7) wraps in 32 bits exactly as the reference). */
size_t nb_serialized_size(uint32_t m);
/* BloomFilter::serialize (BloomFilter.cpp:88-129). Returns bytes written. */
size_t nb_serialize(uint32_t m, uint32_t k, double p, uint32_t time_const, uint64_t h2_seed,
                    const uint64_t *words, uint8_t *out);
/* BloomFilter::deserialize (BloomFilter.cpp:131-190): header fields, and the bit
 * payload into `words` (ceil(m/64) words; may be NULL to read the header only).
 * Unlike the reference it checks `len` and returns NB_ERR_ARG if it is short. */
int nb_deserialize(const uint8_t *img, size_t len, uint32_t *m, uint32_t *k, double *p,
                   uint32_t *time_const, uint64_t *h2_seed, uint64_t *words);

/* -------------------------------------------- SSTable filter write-back --- */
/* The filter region of an SSTable exactly as the reference writes it:
 *   NB_FRAME_RAW : u64 LE image length + image  (SSTableRaw::writeBloomToFile,
 *                  SSTable/SSTableRaw.cpp:534-567)
 *   NB_FRAME_COMP: LEB128 varint image length + image  (SSTableComp::writeBloomToFile,
 *                  SSTable/SSTableComp.cpp:469-504, Utils/VarEncoding.h:13-27)
 * cut into block_size blocks, the last one padded with '0' (0x30) bytes
 * (Block_manager::write_block / fill_in_padding, block-manager/block-manager.cpp:12-44),
 * so one write of nb_framed_filter_size() bytes at the region's block offset
 * reproduces the file.  The image is nb_serialize()'s. */
enum nb_framing { NB_FRAME_RAW = 0, NB_FRAME_COMP = 1 };
size_t nb_framed_filter_size(uint32_t m, int framing, uint32_t block_size);
size_t nb_frame_filter(uint32_t m, uint32_t k, double p, uint32_t time_const, uint64_t h2_seed,
                       const uint64_t *words, int framing, uint32_t block_size, uint8_t *out);
/* Same, with the filter words still in device memory: the header is written on
 * the host and the bit payload is copied D2H straight into its place in `out`
 * (host memory; pinned memory makes the copy asynchronous-capable).  Synchronises
 * `stream` before returning. */
int nb_frame_filter_device(uint32_t m, uint32_t k, double p, uint32_t time_const,
                           uint64_t h2_seed, const uint64_t *d_words, int framing,
                           uint32_t block_size, uint8_t *out, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* NASP_BLOOM_H */
