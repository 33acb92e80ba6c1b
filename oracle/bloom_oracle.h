/*
 * bloom_oracle.h -- CPU restatement of the reference Bloom-filter path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker.
 * The product path (nasp-key-value-engine_amd/) never links or calls it.
 *
 * Parity pinned by: (1) the six MSVC/FNV filters committed in the reference
 * (tests/golden/msvc_filters.json), (2) golden vectors produced by the real
 * reference BloomFilter.cpp compiled here (oracle/_ref, tests/golden/gen_golden.py).
 */
#ifndef NASP_BLOOM_ORACLE_H
#define NASP_BLOOM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_FLAVOR_LIBSTDCXX = 0, ORC_FLAVOR_MSVC_FNV1A = 1,
       /* non-parity: (h1, h2) = MurmurHash3_x64_128(key, len, (uint32_t)seed) */
       ORC_FLAVOR_MURMUR3_X64_128 = 2 };
/* MurmurHash3_x64_128 restated (reference MurmurHash3/MurmurHash3.cpp:255-332). */
void orc_murmur3_x64_128(const uint8_t *p, size_t len, uint32_t seed, uint64_t out[2]);

/* std::hash<std::string> of each platform (reference BloomFilter.cpp:59-60). */
uint64_t orc_hash_libstdcxx(const uint8_t *p, size_t len);
uint64_t orc_hash_fnv1a(const uint8_t *p, size_t len);
uint64_t orc_hash(int flavor, const uint8_t *p, size_t len);

/* BloomFilter.cpp:192-199 */
uint32_t orc_size_of_bitset(uint32_t n, double p);
uint32_t orc_num_hashes(uint32_t n, uint32_t m);
/* BloomFilter.cpp:37,44-46: mt19937(timeConst) -> uniform_int_distribution<size_t>(0, max) */
uint64_t orc_seed_from_time(uint32_t time_const);
/* to_string(seed) (BloomFilter.cpp:60); writes up to 20 digits, returns length */
int orc_seed_digits(uint64_t seed, char out[24]);

/* Index of hash function i (BloomFilter.cpp:57-62) for one key. */
uint32_t orc_index(int flavor, const uint8_t *key, size_t len, uint32_t i,
                   uint32_t m, uint64_t seed);

/*
 * Batch build: OR every key's k bits into `words` (ceil(m/64) little-endian u64
 * words; bit j -> word j/64, bit j%64, which is exactly the LSB-first byte image
 * of BloomFilter.cpp:117-126).  Keys are packed: key i is
 * keys[offsets[i] .. offsets[i+1]) or, if offsets == NULL, keys[i*key_len ..).
 */
int orc_build(int flavor, const uint8_t *keys, const uint64_t *offsets,
              uint32_t key_len, uint64_t n, uint32_t m, uint32_t k,
              uint64_t seed, uint64_t *words);
/* Batch probe (BloomFilter.cpp:67-80): out[i] = 1 if every bit set. */
int orc_probe(int flavor, const uint8_t *keys, const uint64_t *offsets,
              uint32_t key_len, uint64_t n, uint32_t m, uint32_t k,
              uint64_t seed, const uint64_t *words, uint8_t *out);

/*
 * MerkleTree(data) (reference MerkleTree/merkle.cpp:7-55): leaves[i] = H(record i)
 * (its decimal string is leaf i, merkle.cpp:13-15,26-32); each level pairs nodes
 * i, i+1 (the last one with itself when the level is odd) into
 * H(to_string(left) ++ to_string(right)) until one node is left (merkle.cpp:41-52).
 * tree (optional, orc_merkle_tree_size(n) words): every level, leaves first.
 * Returns the root hash (getRootHash() is its decimal string).  n >= 1.
 */
uint64_t orc_merkle(int flavor, const uint8_t *data, const uint64_t *offsets, uint32_t rec_len,
                    uint64_t n, uint64_t *leaves, uint64_t *tree);
uint64_t orc_merkle_tree_size(uint64_t n);

/* Serialized image (BloomFilter.cpp:88-129): 28-byte header + (uint32)(m+7)/8 bytes. */
size_t orc_serialized_size(uint32_t m);
size_t orc_serialize(uint32_t m, uint32_t k, double p, uint32_t time_const,
                     uint64_t seed, const uint64_t *words, uint8_t *out);

#ifdef __cplusplus
}
#endif
#endif
