/*
 * bloom_oracle.c -- clean-room CPU restatement of the reference Bloom filter.
 *
 * TEST INFRASTRUCTURE ONLY (see bloom_oracle.h).  Never linked by the product.
 *
 * Follows, by behaviour (not by text):
 *   reference BloomFilter/BloomFilter.cpp:28-65   constructor (m, k, seed)
 *   reference BloomFilter/BloomFilter.cpp:57-62   hash closure (h1 + i*h2) % m
 *   reference BloomFilter/BloomFilter.cpp:67-86   possiblyContains / add
 *   reference BloomFilter/BloomFilter.cpp:88-129  serialize
 *   reference BloomFilter/BloomFilter.cpp:192-199 m / k formulas
 * and the two third-party std::hash<std::string> implementations the reference
 * is compiled against (neither is vendored under /root/reference):
 *   - libstdc++ (GCC 11.4.0) std::_Hash_bytes(ptr, len, 0xc70f6907)
 *     (libsupc++/hash_bytes.cc, 64-bit size_t branch: a MurmurHash2-64A variant)
 *   - MSVC STL v143 (VS2022) _Fnv1a_append_bytes: FNV-1a 64-bit.
 */
#include "bloom_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- hashes -- */

#define LIBSTDCXX_MUL 0xc6a4a7935bd1e995ULL
#define LIBSTDCXX_SEED 0xc70f6907ULL

static inline uint64_t shift_mix(uint64_t v) { return v ^ (v >> 47); }

static inline uint64_t load_le(const uint8_t *p, size_t n) {
    uint64_t r = 0;
    for (size_t b = 0; b < n; ++b) r |= (uint64_t)p[b] << (8 * b);
    return r;
}

uint64_t orc_hash_libstdcxx(const uint8_t *p, size_t len) {
    const size_t whole = len & ~(size_t)7;
    uint64_t h = LIBSTDCXX_SEED ^ ((uint64_t)len * LIBSTDCXX_MUL);
    for (size_t off = 0; off < whole; off += 8) {
        uint64_t d = shift_mix(load_le(p + off, 8) * LIBSTDCXX_MUL) * LIBSTDCXX_MUL;
        h = (h ^ d) * LIBSTDCXX_MUL;
    }
    if (len & 7) {
        h = (h ^ load_le(p + whole, len & 7)) * LIBSTDCXX_MUL;
    }
    h = shift_mix(h) * LIBSTDCXX_MUL;
    return shift_mix(h);
}

#define FNV_BASIS 14695981039346656037ULL
#define FNV_PRIME 1099511628211ULL

uint64_t orc_hash_fnv1a(const uint8_t *p, size_t len) {
    uint64_t h = FNV_BASIS;
    for (size_t i = 0; i < len; ++i) h = (h ^ p[i]) * FNV_PRIME;
    return h;
}

/* MurmurHash3_x64_128, by behaviour (reference MurmurHash3/MurmurHash3.cpp:255-332):
 * 16-byte blocks as two little-endian 64-bit lanes, the len & 15 tail (the high
 * lane first, as the reference's fall-through switch does), then fmix64. */
#define MM_C1 0x87c37b91114253d5ULL
#define MM_C2 0x4cf5ad432745937fULL
static inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t fmix(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL;
    return k ^ (k >> 33);
}
void orc_murmur3_x64_128(const uint8_t *p, size_t len, uint32_t seed, uint64_t out[2]) {
    uint64_t h1 = seed, h2 = seed;
    const size_t nb = len / 16;
    for (size_t i = 0; i < nb; ++i) {
        uint64_t k1 = load_le(p + 16 * i, 8), k2 = load_le(p + 16 * i + 8, 8);
        k1 *= MM_C1; k1 = rotl(k1, 31); k1 *= MM_C2; h1 ^= k1;
        h1 = rotl(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= MM_C2; k2 = rotl(k2, 33); k2 *= MM_C1; h2 ^= k2;
        h2 = rotl(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }
    const uint8_t *t = p + 16 * nb;
    const size_t rem = len & 15;
    if (rem > 8) {
        uint64_t k2 = load_le(t + 8, rem - 8);
        k2 *= MM_C2; k2 = rotl(k2, 33); k2 *= MM_C1; h2 ^= k2;
    }
    if (rem) {
        uint64_t k1 = load_le(t, rem < 8 ? rem : 8);
        k1 *= MM_C1; k1 = rotl(k1, 31); k1 *= MM_C2; h1 ^= k1;
    }
    h1 ^= (uint64_t)len; h2 ^= (uint64_t)len;
    h1 += h2; h2 += h1;
    h1 = fmix(h1); h2 = fmix(h2);
    h1 += h2; h2 += h1;
    out[0] = h1; out[1] = h2;
}

uint64_t orc_hash(int flavor, const uint8_t *p, size_t len) {
    if (flavor == ORC_FLAVOR_MURMUR3_X64_128) {  /* first half, seed 0 */
        uint64_t o[2];
        orc_murmur3_x64_128(p, len, 0, o);
        return o[0];
    }
    return flavor == ORC_FLAVOR_MSVC_FNV1A ? orc_hash_fnv1a(p, len)
                                            : orc_hash_libstdcxx(p, len);
}

/* ------------------------------------------------------ parameter formulas -- */

/* double -> unsigned int the way x86-64 GCC/MSVC lower it (cvttsd2si to 64 bit,
 * keep the low 32 bits): out-of-range values wrap modulo 2^32 (SURVEY finding 5). */
static uint32_t x86_double_to_u32(double v) { return (uint32_t)(uint64_t)(int64_t)v; }

uint32_t orc_size_of_bitset(uint32_t n, double p) {
    double ln2 = log(2.0);
    return x86_double_to_u32(ceil(-(double)n * log(p) / (ln2 * ln2)));
}

uint32_t orc_num_hashes(uint32_t n, uint32_t m) {
    uint32_t k = x86_double_to_u32(round(((double)m / (double)n) * log(2.0)));
    return k == 0 ? 1 : k;
}

/* MT19937 (32-bit Mersenne twister, standard parameters). */
typedef struct { uint32_t s[624]; int i; } mt_state;

static void mt_seed(mt_state *st, uint32_t seed) {
    st->s[0] = seed;
    for (int i = 1; i < 624; ++i)
        st->s[i] = 1812433253u * (st->s[i - 1] ^ (st->s[i - 1] >> 30)) + (uint32_t)i;
    st->i = 624;
}

static uint32_t mt_next(mt_state *st) {
    if (st->i >= 624) {
        for (int j = 0; j < 624; ++j) {
            uint32_t y = (st->s[j] & 0x80000000u) | (st->s[(j + 1) % 624] & 0x7fffffffu);
            uint32_t v = st->s[(j + 397) % 624] ^ (y >> 1);
            if (y & 1u) v ^= 0x9908b0dfu;
            st->s[j] = v;
        }
        st->i = 0;
    }
    uint32_t y = st->s[st->i++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

/* uniform_int_distribution<uint64_t>(0, 2^64-1) over a 32-bit engine draws two
 * words and composes them high-first; the range check can never reject. */
uint64_t orc_seed_from_time(uint32_t time_const) {
    mt_state st;
    mt_seed(&st, time_const);
    uint64_t hi = mt_next(&st);
    uint64_t lo = mt_next(&st);
    return (hi << 32) + lo;
}

int orc_seed_digits(uint64_t seed, char out[24]) {
    return snprintf(out, 24, "%llu", (unsigned long long)seed);
}

/* ------------------------------------------------------------ index math -- */

/* h2 = H(to_string(seed) + key), hashed over the concatenated bytes. */
static uint64_t hash_with_prefix(int flavor, const char *pre, int plen,
                                 const uint8_t *key, size_t len, uint8_t *scratch) {
    memcpy(scratch, pre, (size_t)plen);
    memcpy(scratch + plen, key, len);
    return orc_hash(flavor, scratch, (size_t)plen + len);
}

typedef struct {
    int flavor;
    uint32_t m;
    char digits[24];
    int ndig;
    uint64_t seed;
} orc_ctx;

static void key_hashes(const orc_ctx *c, const uint8_t *key, size_t len,
                       uint64_t *h1, uint64_t *h2, uint8_t *scratch) {
    if (c->flavor == ORC_FLAVOR_MURMUR3_X64_128) {  /* not the reference filter */
        uint64_t o[2];
        orc_murmur3_x64_128(key, len, (uint32_t)c->seed, o);
        *h1 = o[0];
        *h2 = o[1];
        return;
    }
    *h1 = orc_hash(c->flavor, key, len);
    *h2 = hash_with_prefix(c->flavor, c->digits, c->ndig, key, len, scratch);
}

/* The closure computes (h1 + i*h2) % m in size_t: 64-bit wrapping, m widened. */
static inline uint32_t index_of(uint64_t h1, uint64_t h2, uint32_t i, uint32_t m) {
    return (uint32_t)((h1 + (uint64_t)i * h2) % (uint64_t)m);
}

uint32_t orc_index(int flavor, const uint8_t *key, size_t len, uint32_t i,
                   uint32_t m, uint64_t seed) {
    orc_ctx c = {flavor, m, {0}, 0, seed};
    c.ndig = orc_seed_digits(seed, c.digits);
    uint8_t stackbuf[512];
    uint8_t *scratch = len + 24 <= sizeof stackbuf ? stackbuf : (uint8_t *)malloc(len + 24);
    uint64_t h1, h2;
    key_hashes(&c, key, len, &h1, &h2, scratch);
    if (scratch != stackbuf) free(scratch);
    return index_of(h1, h2, i, m);
}

static size_t max_key_len(const uint64_t *offsets, uint32_t key_len, uint64_t n) {
    if (!offsets) return key_len;
    size_t mx = 0;
    for (uint64_t i = 0; i < n; ++i) {
        size_t l = (size_t)(offsets[i + 1] - offsets[i]);
        if (l > mx) mx = l;
    }
    return mx;
}

int orc_build(int flavor, const uint8_t *keys, const uint64_t *offsets,
              uint32_t key_len, uint64_t n, uint32_t m, uint32_t k,
              uint64_t seed, uint64_t *words) {
    if (n == 0) return 0;
    if (m == 0) return -1; /* the reference divides by zero here */
    orc_ctx c = {flavor, m, {0}, 0, seed};
    c.ndig = orc_seed_digits(seed, c.digits);
    uint8_t *scratch = (uint8_t *)malloc(max_key_len(offsets, key_len, n) + 24);
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t *p = offsets ? keys + offsets[i] : keys + i * (uint64_t)key_len;
        size_t len = offsets ? (size_t)(offsets[i + 1] - offsets[i]) : key_len;
        uint64_t h1, h2;
        key_hashes(&c, p, len, &h1, &h2, scratch);
        for (uint32_t j = 0; j < k; ++j) {
            uint32_t b = index_of(h1, h2, j, m);
            words[b >> 6] |= 1ULL << (b & 63);
        }
    }
    free(scratch);
    return 0;
}

int orc_probe(int flavor, const uint8_t *keys, const uint64_t *offsets,
              uint32_t key_len, uint64_t n, uint32_t m, uint32_t k,
              uint64_t seed, const uint64_t *words, uint8_t *out) {
    if (n == 0) return 0;
    if (m == 0 && k > 0) return -1;
    orc_ctx c = {flavor, m, {0}, 0, seed};
    c.ndig = orc_seed_digits(seed, c.digits);
    uint8_t *scratch = (uint8_t *)malloc(max_key_len(offsets, key_len, n) + 24);
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t *p = offsets ? keys + offsets[i] : keys + i * (uint64_t)key_len;
        size_t len = offsets ? (size_t)(offsets[i + 1] - offsets[i]) : key_len;
        uint64_t h1, h2;
        key_hashes(&c, p, len, &h1, &h2, scratch);
        uint8_t hit = 1;
        for (uint32_t j = 0; j < k && hit; ++j) {
            uint32_t b = index_of(h1, h2, j, m);
            hit = (words[b >> 6] >> (b & 63)) & 1u;
        }
        out[i] = hit;
    }
    free(scratch);
    return 0;
}

/* ----------------------------------------------------------- serialization -- */

/* (m + 7) / 8 is evaluated in unsigned int by the reference (BloomFilter.cpp:90),
 * so it wraps for m > 2^32 - 8. */
size_t orc_serialized_size(uint32_t m) { return 28 + (size_t)((uint32_t)(m + 7u) / 8u); }

size_t orc_serialize(uint32_t m, uint32_t k, double p, uint32_t time_const,
                     uint64_t seed, const uint64_t *words, uint8_t *out) {
    memcpy(out + 0, &m, 4);
    memcpy(out + 4, &k, 4);
    memcpy(out + 8, &p, 8);
    memcpy(out + 16, &time_const, 4);
    memcpy(out + 20, &seed, 8);
    size_t nbytes = (uint32_t)(m + 7u) / 8u;
    /* LE u64 words are the LSB-first byte image; bits >= m are never set. */
    memcpy(out + 28, words, nbytes);
    return 28 + nbytes;
}

/* ---------------------------------------------------------------- Merkle --
 * merkle.cpp:26-32: hash(data) = stringstream << std::hash<std::string>(data),
 * i.e. the decimal digits of the size_t hash.  Restated with snprintf. */
static int dec_of(uint64_t v, char out[24]) {
    return snprintf(out, 24, "%llu", (unsigned long long)v);
}

static uint64_t hash_pair(int flavor, uint64_t l, uint64_t r) {
    char buf[48];
    int a = dec_of(l, buf);
    int b = dec_of(r, buf + a);
    return orc_hash(flavor, (const uint8_t *)buf, (size_t)(a + b));
}

uint64_t orc_merkle_tree_size(uint64_t n) {
    uint64_t total = n;
    while (n > 1) {
        n = (n + 1) / 2;
        total += n;
    }
    return total;
}

uint64_t orc_merkle(int flavor, const uint8_t *data, const uint64_t *offsets, uint32_t rec_len,
                    uint64_t n, uint64_t *leaves, uint64_t *tree) {
    if (n == 0) return 0;  /* the reference throws std::invalid_argument (merkle.cpp:8-10) */
    uint64_t *level = (uint64_t *)malloc(n * sizeof(uint64_t));
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t *p = offsets ? data + offsets[i] : data + i * (uint64_t)rec_len;
        const size_t len = offsets ? (size_t)(offsets[i + 1] - offsets[i]) : rec_len;
        level[i] = orc_hash(flavor, p, len);
    }
    if (leaves) memcpy(leaves, level, n * sizeof(uint64_t));
    uint64_t at = 0;
    if (tree) memcpy(tree, level, n * sizeof(uint64_t));
    at = n;
    uint64_t cnt = n;
    while (cnt > 1) {  /* merkle.cpp:41-52 */
        const uint64_t next = (cnt + 1) / 2;
        for (uint64_t i = 0; i < next; ++i) {
            const uint64_t l = level[2 * i];
            const uint64_t r = (2 * i + 1 < cnt) ? level[2 * i + 1] : l;
            level[i] = hash_pair(flavor, l, r);
        }
        cnt = next;
        if (tree) memcpy(tree + at, level, cnt * sizeof(uint64_t));
        at += cnt;
    }
    const uint64_t root = level[0];
    free(level);
    return root;
}
