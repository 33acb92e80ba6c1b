// bloom_host.cpp -- host-only parts of the C ABI (include/nasp_bloom.h):
// seed derivation and the serialized image.  No device code.
//
//   nb_seed_from_time  <- BloomFilter.cpp:37,44-46 (mt19937 + uniform_int_distribution)
//   nb_serialize       <- BloomFilter.cpp:88-129
//   nb_deserialize     <- BloomFilter.cpp:131-190
//   nb_std_hash        <- std::hash<std::string> (BloomFilter.cpp:59, merkle.cpp:27-28)
//   nb_build_cpu       <- BloomFilter::add (BloomFilter.cpp:82-86) for a small batch on
//                         the host: the drop-in class's small-batch / no-device path
//                         (SURVEY §8(b)), with the kernels' own index arithmetic
//   nb_merkle_cpu      <- MerkleTree(data) (merkle.cpp:7-55) on the host: the drop-in
//                         MerkleTree's small-flush / no-device path
#include <cstdint>
#include <cstring>
#include <limits>
#include <random>
#include <vector>

#include "../../include/nasp_bloom.h"
#include "bloom_math.h"

int nb_internal_fail(int code, const char *msg);  // bloom_kernels.hip: the error slot

extern "C" {

uint64_t nb_seed_from_time(uint32_t time_const) {
    std::mt19937 rng(time_const);
    std::uniform_int_distribution<uint64_t> dist(0, std::numeric_limits<uint64_t>::max());
    return dist(rng);
}

uint64_t nb_std_hash(const uint8_t *p, uint64_t len, int flavor) {
    if (flavor != NB_FLAVOR_LIBSTDCXX && flavor != NB_FLAVOR_MSVC_FNV1A &&
        flavor != NB_FLAVOR_MURMUR3_X64_128) {
        (void)nb_internal_fail(NB_ERR_ARG, "nb_std_hash: unknown flavor");
        return 0;
    }
    // the kernels' word-stream hash over byte-assembled words (never reads past len)
    auto load = [p, len](uint32_t j) {
        uint64_t w = 0;
        for (uint64_t b = 0; b < 8 && 8ull * j + b < len; ++b) w |= (uint64_t)p[8ull * j + b] << (8 * b);
        return w;
    };
    if (flavor == NB_FLAVOR_MURMUR3_X64_128) {  // the first half, seed 0
        uint64_t h1, h2;
        nb::mm3_x64_128(load, (uint32_t)len, 0u, &h1, &h2);
        return h1;
    }
    return flavor == NB_FLAVOR_MSVC_FNV1A
               ? nb::hash1_aligned_words<NB_FLAVOR_MSVC_FNV1A>(load, 0, (uint32_t)len)
               : nb::hash1_aligned_words<NB_FLAVOR_LIBSTDCXX>(load, 0, (uint32_t)len);
}

size_t nb_serialized_size(uint32_t m) {
    // The reference computes (m + 7) / 8 in unsigned int: it wraps for m > 2^32-8.
    return 28 + (size_t)((uint32_t)(m + 7u) / 8u);
}

size_t nb_serialize(uint32_t m, uint32_t k, double p, uint32_t time_const, uint64_t h2_seed,
                    const uint64_t *words, uint8_t *out) {
    std::memcpy(out + 0, &m, 4);
    std::memcpy(out + 4, &k, 4);
    std::memcpy(out + 8, &p, 8);
    std::memcpy(out + 16, &time_const, 4);
    std::memcpy(out + 20, &h2_seed, 8);
    const size_t nbytes = (uint32_t)(m + 7u) / 8u;
    // Little-endian u64 words are the LSB-first byte image (bit j -> byte j/8, bit j%8).
    if (nbytes) std::memcpy(out + 28, words, nbytes);
    return 28 + nbytes;
}

int nb_deserialize(const uint8_t *img, size_t len, uint32_t *m, uint32_t *k, double *p,
                   uint32_t *time_const, uint64_t *h2_seed, uint64_t *words) {
    if (!img || len < 28)
        return nb_internal_fail(NB_ERR_ARG, "serialized filter shorter than its 28-byte header");
    uint32_t mm;
    std::memcpy(&mm, img + 0, 4);
    if (m) *m = mm;
    if (k) std::memcpy(k, img + 4, 4);
    if (p) std::memcpy(p, img + 8, 8);
    if (time_const) std::memcpy(time_const, img + 16, 4);
    if (h2_seed) std::memcpy(h2_seed, img + 20, 8);
    if (!words) return NB_OK;
    const size_t nbytes = (uint32_t)(mm + 7u) / 8u;
    if (len < 28 + nbytes)
        return nb_internal_fail(NB_ERR_ARG, "serialized filter shorter than its bit payload");
    const size_t nwords = ((size_t)mm + 63) / 64;
    if (nwords) words[nwords - 1] = 0;  // clear the partial last word before the copy
    if (nbytes) std::memcpy(words, img + 28, nbytes);
    // Bits at positions >= m are ignored by the reference (BloomFilter.cpp:183).
    if (mm & 63) words[nwords - 1] &= (1ull << (mm & 63)) - 1;
    return NB_OK;
}

}  // extern "C"

namespace {
// Aligned word j of a key whose bytes are [lo, hi) (addresses), counted from the
// aligned word holding byte lo -- the words the kernels' hashes consume -- with
// the bytes outside the key read as zero (the hashes shift or mask them out), so
// the host paths read nothing but the caller's key bytes.
struct KeyWords {
    uintptr_t base, lo, hi;
    KeyWords(const uint8_t *p, uint64_t len)
        : base(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)7),
          lo(reinterpret_cast<uintptr_t>(p)), hi(reinterpret_cast<uintptr_t>(p) + len) {}
    uint32_t a() const { return (uint32_t)(lo - base); }
    uint64_t operator()(uint32_t j) const {
        const uintptr_t w = base + 8ull * j;
        uint64_t r = 0;
        if (w >= lo && w + 8 <= hi) {
            std::memcpy(&r, reinterpret_cast<const void *>(w), 8);
            return r;
        }
        for (uint32_t b = 0; b < 8; ++b)
            if (w + b >= lo && w + b < hi)
                r |= (uint64_t)*reinterpret_cast<const uint8_t *>(w + b) << (8 * b);
        return r;
    }
};

// The kernels' word-stream hashes of key i on the host, then the index
// generator -- csrc/bloom_math.h, the code the kernels run.
template <class F>
void for_each_key_indices(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len,
                          uint64_t n, const nb::FilterConsts &c, int flavor, F &&fn) {
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t b = offsets ? offsets[i] : i * (uint64_t)key_len;
        const uint32_t len = (uint32_t)(offsets ? offsets[i + 1] - b : key_len);
        const KeyWords load(keys + b, len);
        const uint32_t a = load.a();
        uint64_t h1, h2;
        if (flavor == NB_FLAVOR_MURMUR3_X64_128)
            nb::hash_aligned_words<NB_FLAVOR_MURMUR3_X64_128>(c, load, a, len, &h1, &h2);
        else if (flavor == NB_FLAVOR_MSVC_FNV1A)
            nb::hash_aligned_words<NB_FLAVOR_MSVC_FNV1A>(c, load, a, len, &h1, &h2);
        else if (offsets)
            nb::hash_aligned_words<NB_FLAVOR_LIBSTDCXX, KeyWords, false>(c, load, a, len, &h1, &h2);
        else
            nb::hash_aligned_words<NB_FLAVOR_LIBSTDCXX, KeyWords, true>(c, load, a, len, &h1, &h2);
        nb::IndexGen g;
        g.start(h1, h2, c);
        fn(i, g);
    }
}

int cpu_args(uint64_t n, uint32_t m, uint32_t k, int flavor, const void *keys, const void *words) {
    if (flavor != NB_FLAVOR_LIBSTDCXX && flavor != NB_FLAVOR_MSVC_FNV1A &&
        flavor != NB_FLAVOR_MURMUR3_X64_128)
        return nb_internal_fail(NB_ERR_ARG, "unknown flavor");
    if (n && k && m == 0) return nb_internal_fail(NB_ERR_ARG, "m == 0 with keys (reference divides by zero)");
    if (n && k && (!keys || !words)) return nb_internal_fail(NB_ERR_ARG, "NULL keys or words");
    return NB_OK;
}
}  // namespace

extern "C" {

int nb_build_cpu(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                 uint32_t m, uint32_t k, uint64_t h2_seed, int flavor, uint64_t *words) {
    const int rc = cpu_args(n, m, k, flavor, keys, words);
    if (rc || n == 0 || k == 0) return rc;
    nb::FilterConsts c = nb::make_consts(m, k, h2_seed, (uint32_t)flavor);
    if (!offsets) nb::set_fixed_len(c, key_len);
    for_each_key_indices(keys, offsets, key_len, n, c, flavor, [&](uint64_t, nb::IndexGen &g) {
        for (uint32_t j = 0; j < k; ++j) {
            if (j) g.next(c);
            words[g.r >> 6] |= 1ull << (g.r & 63);
        }
    });
    return NB_OK;
}

int nb_probe_cpu(const uint8_t *keys, const uint64_t *offsets, uint32_t key_len, uint64_t n,
                 uint32_t m, uint32_t k, uint64_t h2_seed, int flavor, const uint64_t *words,
                 uint8_t *out) {
    if (n && !out) return nb_internal_fail(NB_ERR_ARG, "NULL out");
    if (n && k == 0) {  // no hash closures: possiblyContains answers true
        std::memset(out, 1, n);
        return NB_OK;
    }
    const int rc = cpu_args(n, m, k, flavor, keys, words);
    if (rc || n == 0) return rc;
    nb::FilterConsts c = nb::make_consts(m, k, h2_seed, (uint32_t)flavor);
    if (!offsets) nb::set_fixed_len(c, key_len);
    for_each_key_indices(keys, offsets, key_len, n, c, flavor, [&](uint64_t i, nb::IndexGen &g) {
        uint8_t hit = 1;
        for (uint32_t j = 0; j < k && hit; ++j) {
            if (j) g.next(c);
            hit = (words[g.r >> 6] >> (g.r & 63)) & 1u;
        }
        out[i] = hit;
    });
    return NB_OK;
}

// MerkleTree(data) (merkle.cpp:7-55) on the calling CPU thread, with the Merkle
// kernels' own hashing (bloom_math.h hash1_aligned_words, hash_dec_pair): the
// drop-in MerkleTree's path for small flushes and hosts without a usable GPU.
int nb_merkle_cpu(const uint8_t *data, const uint64_t *offsets, uint32_t rec_len, uint64_t n,
                  int flavor, uint64_t *tree, uint64_t *leaves, uint64_t *root) {
    if (n == 0) return nb_internal_fail(NB_ERR_ARG, "MerkleTree of no records (merkle.cpp:8-10 throws)");
    if (!data || !root) return nb_internal_fail(NB_ERR_ARG, "NULL buffer");
    if (flavor != NB_FLAVOR_LIBSTDCXX && flavor != NB_FLAVOR_MSVC_FNV1A)
        return nb_internal_fail(NB_ERR_ARG, "unknown flavor");
    std::vector<uint64_t> own;
    uint64_t *t = tree;
    if (!t) {
        own.resize(nb_merkle_tree_size(n));
        t = own.data();
    }
    for (uint64_t i = 0; i < n; ++i) {  // leaves: H(record) (merkle.cpp:13-15)
        const uint64_t b = offsets ? offsets[i] : i * (uint64_t)rec_len;
        const uint32_t len = (uint32_t)(offsets ? offsets[i + 1] - b : rec_len);
        const KeyWords load(data + b, len);
        t[i] = flavor == NB_FLAVOR_MSVC_FNV1A
                   ? nb::hash1_aligned_words<NB_FLAVOR_MSVC_FNV1A>(load, load.a(), len)
                   : nb::hash1_aligned_words<NB_FLAVOR_LIBSTDCXX>(load, load.a(), len);
    }
    // levels (merkle.cpp:34-55): parent = H(to_string(l) ++ to_string(r)), the last
    // node of an odd level paired with itself
    uint64_t in = 0, cnt = n;
    while (cnt > 1) {
        const uint64_t out = in + cnt, next = (cnt + 1) / 2;
        for (uint64_t i = 0; i < next; ++i) {
            const uint64_t l = t[in + 2 * i], r = 2 * i + 1 < cnt ? t[in + 2 * i + 1] : l;
            t[out + i] = flavor == NB_FLAVOR_MSVC_FNV1A ? nb::hash_dec_pair<NB_FLAVOR_MSVC_FNV1A>(l, r)
                                                        : nb::hash_dec_pair<NB_FLAVOR_LIBSTDCXX>(l, r);
        }
        in = out;
        cnt = next;
    }
    if (leaves) std::memcpy(leaves, t, n * 8);
    *root = t[in];
    return NB_OK;
}

}  // extern "C"

extern "C" {

static size_t varint_len(uint64_t v) {
    size_t n = 1;
    while (v >>= 7) ++n;
    return n;
}

static size_t frame_prefix(uint64_t img_len, int framing, uint8_t *out) {
    if (framing == NB_FRAME_RAW) {
        if (out) std::memcpy(out, &img_len, 8);
        return 8;
    }
    size_t n = 0;
    do {
        uint8_t chunk = img_len & 0x7F;
        img_len >>= 7;
        if (img_len) chunk |= 0x80;
        if (out) out[n] = chunk;
        ++n;
    } while (img_len);
    return n;
}

size_t nb_framed_filter_size(uint32_t m, int framing, uint32_t block_size) {
    const size_t img = nb_serialized_size(m);
    const size_t payload = (framing == NB_FRAME_RAW ? 8 : varint_len(img)) + img;
    if (block_size == 0) return payload;
    return (payload + block_size - 1) / block_size * block_size;
}

size_t nb_frame_filter(uint32_t m, uint32_t k, double p, uint32_t time_const, uint64_t h2_seed,
                       const uint64_t *words, int framing, uint32_t block_size, uint8_t *out) {
    const size_t img = nb_serialized_size(m);
    const size_t pre = frame_prefix(img, framing, out);
    nb_serialize(m, k, p, time_const, h2_seed, words, out + pre);
    const size_t total = nb_framed_filter_size(m, framing, block_size);
    std::memset(out + pre + img, '0', total - pre - img);
    return total;
}

}  // extern "C"

// Host-side framing helpers shared with the device variant (bloom_kernels.hip).
size_t nb_internal_frame_header(uint32_t m, uint32_t k, double p, uint32_t time_const,
                                uint64_t h2_seed, int framing, uint8_t *out) {
    const size_t img = nb_serialized_size(m);
    const size_t pre = frame_prefix(img, framing, out);
    std::memcpy(out + pre + 0, &m, 4);
    std::memcpy(out + pre + 4, &k, 4);
    std::memcpy(out + pre + 8, &p, 8);
    std::memcpy(out + pre + 16, &time_const, 4);
    std::memcpy(out + pre + 20, &h2_seed, 8);
    return pre + 28;  // offset of the bit payload
}
