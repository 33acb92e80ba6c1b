// bloom_math.h -- index arithmetic of the reference filter, shared by the gfx950
// kernels (bloom_kernels.hip) and the host-side parameter setup / single-key
// probe of the drop-in class.  Header-only; NB_HD marks functions that are
// compiled for both sides when the including TU is built by hipcc.
//
// What it computes (reference BloomFilter/BloomFilter.cpp:57-62):
//   idx_i = (h1 + i*h2) mod m,   64-bit wrapping add/mul, m < 2^32
//   h1 = H(key), h2 = H(to_string(h2_seed) + key)
// with H = std::hash<std::string> of the selected flavour:
//   libstdc++ _Hash_bytes(p, len, 0xc70f6907)  (MurmurHash2-64A-style, 8-byte words)
//   MSVC FNV-1a-64                              (byte at a time)
//
// Two exact rewrites make this cheap on a GPU (both are proven equal to the
// closure's arithmetic, and the parity tests check them bit for bit):
//   1. mod by a runtime 32-bit m without a divide: normalized-reciprocal
//      2-by-1 remainder (Moller & Granlund, "Improved division by invariant
//      integers", 2011, Alg. 4) applied twice to the 96-bit shifted value.
//   2. incremental indices: x_{i+1} = x_i + h2 (mod 2^64), so
//      r_{i+1} = r_i + (h2 mod m) - [x_{i+1} wrapped] * (2^64 mod m)   (mod m),
//      i.e. 2 true reductions per key instead of k.
//   3. h2's seed prefix: the whole 8-byte words of to_string(seed) are mixed
//      into constants once per filter (pre_d[]); the leftover r = D%8 prefix
//      bytes are spliced in front of the key words with funnel shifts.
#pragma once

#include <stdint.h>

#if defined(__HIP__)  // compiled as HIP (hipcc); plain C++ (g++) otherwise
#include <hip/hip_runtime.h>
#define NB_HD __host__ __device__ __forceinline__
#else
#define NB_HD inline
#endif

namespace nb {

constexpr uint64_t kMul = 0xc6a4a7935bd1e995ULL;   // libstdc++ _Hash_bytes multiplier
constexpr uint64_t kStdSeed = 0xc70f6907ULL;       // seed std::hash<string> passes
constexpr uint64_t kFnvBasis = 14695981039346656037ULL;
constexpr uint64_t kFnvPrime = 1099511628211ULL;   // 2^40 + 0x1b3

NB_HD uint64_t shift_mix(uint64_t v) { return v ^ (v >> 47); }

// One 8-byte word of the libstdc++ main loop.
NB_HD uint64_t lsx_round(uint64_t h, uint64_t w) {
    uint64_t d = shift_mix(w * kMul) * kMul;
    return (h ^ d) * kMul;
}
// The (len & 7) tail: bytes loaded little-endian, no pre-mix.
NB_HD uint64_t lsx_tail(uint64_t h, uint64_t t) { return (h ^ t) * kMul; }
NB_HD uint64_t lsx_final(uint64_t h) { return shift_mix(shift_mix(h) * kMul); }
NB_HD uint64_t lsx_init(uint64_t len) { return kStdSeed ^ (len * kMul); }

NB_HD uint64_t fnv_step(uint64_t h, uint32_t byte) { return (h ^ byte) * kFnvPrime; }

// MurmurHash3_x64_128 (the reference's MurmurHash3/MurmurHash3.cpp:255-332; used by
// the non-parity NB_FLAVOR_MURMUR3_X64_128 only) over little-endian key words K(j),
// zero beyond len: 16-byte blocks of two words, then the len & 15 tail.
constexpr uint64_t kMmC1 = 0x87c37b91114253d5ULL, kMmC2 = 0x4cf5ad432745937fULL;
NB_HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
NB_HD uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    return k ^ (k >> 33);
}
template <class LoadK>
NB_HD void mm3_x64_128(LoadK K, uint32_t len, uint32_t seed, uint64_t *o1, uint64_t *o2) {
    uint64_t h1 = seed, h2 = seed;
    const uint32_t nb = len >> 4, rem = len & 15;
    for (uint32_t i = 0; i < nb; ++i) {
        const uint64_t k1 = rotl64(K(2 * i) * kMmC1, 31) * kMmC2;
        h1 = (rotl64(h1 ^ k1, 27) + h2) * 5 + 0x52dce729;
        const uint64_t k2 = rotl64(K(2 * i + 1) * kMmC2, 33) * kMmC1;
        h2 = (rotl64(h2 ^ k2, 31) + h1) * 5 + 0x38495ab5;
    }
    if (rem > 8) {  // (the reference's switch falls through: k2 first, then k1)
        const uint64_t t = K(2 * nb + 1) & ((1ull << (8 * (rem - 8))) - 1);
        h2 ^= rotl64(t * kMmC2, 33) * kMmC1;
    }
    if (rem) {
        const uint64_t t = rem >= 8 ? K(2 * nb) : K(2 * nb) & ((1ull << (8 * rem)) - 1);
        h1 ^= rotl64(t * kMmC1, 31) * kMmC2;
    }
    h1 ^= len;
    h2 ^= len;
    h1 += h2;
    h2 += h1;
    h1 = fmix64(h1);
    h2 = fmix64(h2);
    h1 += h2;
    h2 += h1;
    *o1 = h1;
    *o2 = h2;
}

// ------------------------------------------------------------- fast mod ----
struct FastMod {
    uint32_t m;   // divisor (>= 1)
    uint32_t l;   // clz32(m)
    uint32_t d;   // m << l (top bit set)
    uint32_t v;   // floor((2^64-1)/d) - 2^32
    uint32_t fp;  // quotient through f64 (mod64 below): 0 off (m < 2^13),
                  // 1 for 2^13 <= m < 2^31, 2 for m >= 2^31
    uint32_t pad_;
    double inv;   // 1/m, correctly rounded
};

// fp_min: smallest m the f64 quotient is used for (>= 2^13; larger values, or
// ~0u, keep the integer remainder -- an A/B knob of the kernels' launcher).
inline FastMod make_fastmod(uint32_t m, uint32_t fp_min = 8192u) {
    FastMod f;
    f.m = m;
    uint32_t l = 0;
    while (l < 31 && !((m << l) & 0x80000000u)) ++l;
    f.l = l;
    f.d = m << l;
    f.v = (uint32_t)(~0ULL / f.d - (1ULL << 32));
    f.fp = (m >= 8192u && m >= fp_min) ? (m < 0x80000000u ? 1u : 2u) : 0u;
    f.pad_ = 0;
    f.inv = 1.0 / (double)m;
    return f;
}

// Remainder of (u1:u0) / d, requires u1 < d, d normalized.
NB_HD uint32_t rem_2by1(uint32_t u1, uint32_t u0, uint32_t d, uint32_t v) {
    // q = v*u1 + ((u1+1) << 32 | u0) mod 2^64; v*u1 + u0 < 2^64, so the high word
    // is hi(v*u1 + u0) + u1 + 1 (one 32x32+32 multiply-add, no 64-bit add)
    const uint64_t p = (uint64_t)v * u1 + u0;
    uint32_t q1 = (uint32_t)(p >> 32) + u1 + 1u, q0 = (uint32_t)p;
    uint32_t r = u0 - q1 * d;
    if (r > q0) r += d;
    if (r >= d) r -= d;
    return r;
}

NB_HD uint32_t mod64_int(uint64_t x, const FastMod &f) {
    uint32_t n2 = f.l ? (uint32_t)(x >> (64 - f.l)) : 0u;
    uint64_t xs = x << f.l;
    uint32_t r = rem_2by1(n2, (uint32_t)(xs >> 32), f.d, f.v);
    r = rem_2by1(r, (uint32_t)xs, f.d, f.v);
    return r >> f.l;
}

// x mod m through an f64 quotient (f.fp != 0, m >= 2^13; FMA and conversions are
// full rate on gfx950): xd = fl(x) is within 2^10 of x, and
// t = fl(xd * fl(1/m) + 2^52) holds q = rne(xd / m (1 + 2^-53)) in its low mantissa
// bits, with |q - x/m| < 2^10/m + (x/m) 2^-53 + 1/2 <= 3/8 + 1/2 < 1 (x/m < 2^51), so
// q = floor(x/m) or one more and x - q m lies in [-m, m).  m < 2^31: that fits a
// 32-bit two's complement value, corrected by one min (r + m < 2^32 when r >= 0,
// and wraps below r when r < 0).  m >= 2^31: the 64-bit difference, whose high
// word is 0 or ~0 (q < 2^52 from bits 0..51).  About 8 / 12 VALU instead of ~26.
NB_HD uint32_t mod64(uint64_t x, const FastMod &f) {
    if (f.fp) {  // kernel-uniform
        const double xd = __builtin_fma((double)(uint32_t)(x >> 32), 4294967296.0,
                                        (double)(uint32_t)x);
        const uint64_t tb = __builtin_bit_cast(uint64_t, __builtin_fma(xd, f.inv, 4503599627370496.0));
        const uint32_t ql = (uint32_t)tb;
        if (f.fp == 1) {
            const uint32_t r = (uint32_t)x - ql * f.m, u = r + f.m;
            return r < u ? r : u;
        }
        const uint32_t qh = (uint32_t)(tb >> 32) & 0xFFFFFu;
        const uint64_t r = x - ((uint64_t)ql * f.m + ((uint64_t)(qh * f.m) << 32));
        return (uint32_t)r + ((uint32_t)(r >> 32) & f.m);
    }
    return mod64_int(x, f);
}

// (a + b) mod m for a, b < m without 32-bit overflow.
NB_HD uint32_t addmod(uint32_t a, uint32_t b, uint32_t m) {
    return a >= m - b ? a - (m - b) : a + b;
}
// The same for any m < 2^32 in four VALU ops (add with carry, sub, min, select):
// without a carry min(t, t - m) picks the reduced value (t - m wraps when t < m);
// with one the true sum is t + 2^32 >= m, reduced to t - m (mod 2^32).
NB_HD uint32_t addmod_fast(uint32_t a, uint32_t b, uint32_t m) {
    const uint32_t t = a + b, u = t - m;
    const uint32_t mn = t < u ? t : u;
    return t < a ? u : mn;
}
NB_HD uint32_t submod(uint32_t a, uint32_t b, uint32_t m) {
    return a >= b ? a - b : a + (m - b);
}

// ------------------------------------------------- per-filter constants ----
constexpr int kMaxPrefixWords = 2;  // to_string(uint64) has <= 20 digits

struct FilterConsts {
    FastMod fm;
    uint32_t k;
    uint32_t c64;          // 2^64 mod m
    uint32_t plen;         // D = number of decimal digits of h2_seed
    uint32_t pwords;       // D / 8 whole prefix words
    uint32_t prem;         // r = D % 8 leftover prefix bytes
    uint32_t flavor;
    uint64_t pre_d[kMaxPrefixWords];  // libstdc++: pre-mixed whole prefix words
    uint64_t pre_tail;     // the r leftover prefix bytes, little-endian
    uint64_t fnv_pre;      // FNV-1a state after all D prefix bytes
    uint64_t h2_init_fixed; // libstdc++ h2 state after the whole prefix words, for
                            // keys of length fixed_len (fixed-length layouts only)
    uint32_t fixed_len;
    uint32_t mm3_seed;      // NB_FLAVOR_MURMUR3_X64_128: (uint32_t)h2_seed
};

inline FilterConsts make_consts(uint32_t m, uint32_t k, uint64_t seed, uint32_t flavor) {
    FilterConsts c{};
    c.fm = make_fastmod(m);
    c.k = k;
    c.c64 = (uint32_t)((~0ULL % m + 1) % m);
    char dig[24];
    int n = 0;
    {
        char tmp[24];
        uint64_t s = seed;
        do { tmp[n++] = (char)('0' + s % 10); s /= 10; } while (s);
        for (int i = 0; i < n; ++i) dig[i] = tmp[n - 1 - i];
    }
    c.plen = (uint32_t)n;
    c.pwords = (uint32_t)n / 8;
    c.prem = (uint32_t)n % 8;
    c.flavor = flavor;
    for (uint32_t w = 0; w < c.pwords; ++w) {
        uint64_t x = 0;
        for (int b = 0; b < 8; ++b) x |= (uint64_t)(uint8_t)dig[8 * w + b] << (8 * b);
        c.pre_d[w] = shift_mix(x * kMul) * kMul;
    }
    uint64_t t = 0;
    for (uint32_t b = 0; b < c.prem; ++b) t |= (uint64_t)(uint8_t)dig[8 * c.pwords + b] << (8 * b);
    c.pre_tail = t;
    uint64_t h = kFnvBasis;
    for (int i = 0; i < n; ++i) h = fnv_step(h, (uint8_t)dig[i]);
    c.fnv_pre = h;
    c.fixed_len = 0;
    c.h2_init_fixed = 0;
    c.mm3_seed = (uint32_t)seed;
    return c;
}

// libstdc++ h2 state once the whole prefix words are mixed, for a key of `len`
// bytes (the initial state depends on the total length len + D).
inline uint64_t h2_state_after_prefix(const FilterConsts &c, uint64_t len) {
    uint64_t g = kStdSeed ^ ((len + c.plen) * kMul);
    for (uint32_t w = 0; w < c.pwords; ++w) g = (g ^ c.pre_d[w]) * kMul;
    return g;
}

inline void set_fixed_len(FilterConsts &c, uint32_t len) {
    c.fixed_len = len;
    c.h2_init_fixed = h2_state_after_prefix(c, len);
}

// Index generator of one key: r_i = (h1 + i*h2 mod 2^64) mod m, incrementally
// (rewrite 2 above).  The two step sizes s = h2 mod m and s2 = (h2 - 2^64) mod m
// are kept biased by -m (mod 2^32): r + (a - m) carries out of 32 bits exactly
// when r + a >= m, so a step is one 64-bit add, one select on its carry, and a
// modular add of three ops (add with carry-out, add m, select) for any m < 2^32.
struct IndexGen {
    uint64_t x, h2;
    uint32_t r, sb, s2b;  // r = current index; sb = s - m, s2b = s2 - m (mod 2^32)
    NB_HD void start(uint64_t h1_, uint64_t h2_, const FilterConsts &c) {
        x = h1_;
        h2 = h2_;
        r = mod64(h1_, c.fm);
        const uint32_t s = mod64(h2_, c.fm);
        sb = s - c.fm.m;
        s2b = submod(s, c.c64, c.fm.m) - c.fm.m;
    }
    NB_HD void next(const FilterConsts &c) {
        const uint64_t nx = x + h2;
        const uint32_t t = r + (nx < x ? s2b : sb);
        r = t < r ? t : t + c.fm.m;  // carry: r + a >= m, t = r + a - m
        x = nx;
    }
};


// ------------------------------------------------- word-stream hashing ----
// Both hashes of one key computed from its bytes viewed as 8-byte little-endian
// words K_j (zero beyond len).  h2 hashes to_string(seed) ++ key: its whole
// prefix words are pre-mixed (pre_d), and stream word j is the r = D%8 leftover
// prefix bytes spliced in front of the key: S_j = K_{j-1} >> (64-8r) | K_j << 8r.

NB_HD uint64_t mask_bytes(uint64_t w, int nbytes) {
    return nbytes >= 8 ? w : (nbytes <= 0 ? 0ull : (w & ((1ull << (8 * nbytes)) - 1)));
}

// Bytes [a, a+8) of the 16-byte pair lo:hi; a8 = 8*a, a in [0, 8).
NB_HD uint64_t funnel(uint64_t lo, uint64_t hi, uint32_t a8) {
    return a8 ? (lo >> a8) | (hi << (64 - a8)) : lo;
}

struct LsxState {
    uint64_t h1, h2, kprev;
};

NB_HD void lsx_begin(const FilterConsts &c, LsxState &s, uint32_t len) {
    s.h1 = lsx_init(len);
    uint64_t g = lsx_init((uint64_t)len + c.plen);
    for (int w = 0; w < kMaxPrefixWords; ++w)
        if ((uint32_t)w < c.pwords) g = (g ^ c.pre_d[w]) * kMul;
    s.h2 = g;
    s.kprev = c.prem ? c.pre_tail << (64 - 8 * c.prem) : 0;
}

// Same, with the h2 prefix state precomputed on the host (fixed-length keys).
NB_HD void lsx_begin_fixed(const FilterConsts &c, LsxState &s, uint32_t len) {
    s.h1 = lsx_init(len);
    s.h2 = c.h2_init_fixed;
    s.kprev = c.prem ? c.pre_tail << (64 - 8 * c.prem) : 0;
}

// Feed key word j (zero beyond len) into both hashes.
NB_HD void lsx_consume(const FilterConsts &c, LsxState &s, uint32_t j, uint64_t kw,
                       uint32_t len) {
    if (j < (len >> 3)) s.h1 = lsx_round(s.h1, kw);
    else s.h1 = lsx_tail(s.h1, kw);  // only reached when len & 7 != 0
    const uint32_t r8 = 8 * c.prem;
    const uint64_t sw = r8 ? (s.kprev >> (64 - r8)) | (kw << r8) : kw;
    s.kprev = kw;
    const uint32_t slen = len + c.prem;
    if (j < (slen >> 3)) s.h2 = lsx_round(s.h2, sw);
    else if (slen & 7) s.h2 = lsx_tail(s.h2, sw);
}

NB_HD void lsx_end(const FilterConsts &c, LsxState &s, uint32_t len, uint64_t *h1,
                   uint64_t *h2) {
    const uint32_t nk = (len + 7) >> 3;
    const uint32_t slen = len + c.prem;
    if (((slen + 7) >> 3) > nk) {  // one more stream word: the last key word's high bytes
        const uint64_t sw = s.kprev >> (64 - 8 * c.prem);
        if (nk < (slen >> 3)) s.h2 = lsx_round(s.h2, sw);
        else s.h2 = lsx_tail(s.h2, sw);
    }
    *h1 = lsx_final(s.h1);
    *h2 = lsx_final(s.h2);
}

NB_HD void fnv_consume(uint64_t &h1, uint64_t &h2, uint64_t kw, int nbytes) {
    for (int b = 0; b < 8; ++b) {
        if (b < nbytes) {
            const uint32_t byte = (uint32_t)(kw >> (8 * b)) & 0xffu;
            h1 = fnv_step(h1, byte);
            h2 = fnv_step(h2, byte);
        }
    }
}

// Hash a key whose first byte sits at byte a (0..7) of aligned word Q(0);
// Q(j) returns aligned word j.  Only words holding at least one key byte are read.
template <int FLAVOR, class LoadQ, bool FIXED_LEN = false>
NB_HD void hash_aligned_words(const FilterConsts &c, LoadQ Q, uint32_t a, uint32_t len,
                              uint64_t *h1, uint64_t *h2) {
    const uint32_t nq = (a + len + 7) >> 3;
    const uint32_t nk = (len + 7) >> 3;
    if (FLAVOR == 2) {  // MurmurHash3_x64_128 (non-parity flavour)
        auto K = [&](uint32_t j) {
            const uint64_t lo = j < nq ? Q(j) : 0, hi = j + 1 < nq ? Q(j + 1) : 0;
            return mask_bytes(funnel(lo, hi, 8 * a), (int)(len - 8 * j));
        };
        mm3_x64_128(K, len, c.mm3_seed, h1, h2);
        return;
    }
    uint64_t qcur = nq ? Q(0) : 0;
    if (FLAVOR == 1) {
        uint64_t f1 = kFnvBasis, f2 = c.fnv_pre;
        for (uint32_t j = 0; j < nk; ++j) {
            const uint64_t qnext = (j + 1 < nq) ? Q(j + 1) : 0;
            const uint64_t kw = funnel(qcur, qnext, 8 * a);
            qcur = qnext;
            fnv_consume(f1, f2, kw, (int)(len - 8 * j));
        }
        *h1 = f1;
        *h2 = f2;
    } else {
        LsxState s;
        if (FIXED_LEN) lsx_begin_fixed(c, s, len);
        else lsx_begin(c, s, len);
        for (uint32_t j = 0; j < nk; ++j) {
            const uint64_t qnext = (j + 1 < nq) ? Q(j + 1) : 0;
            const uint64_t kw = mask_bytes(funnel(qcur, qnext, 8 * a), (int)(len - 8 * j));
            qcur = qnext;
            lsx_consume(c, s, j, kw, len);
        }
        lsx_end(c, s, len, h1, h2);
    }
}

// ------------------------------------------- dword-stream libstdc++ path ----
// The same two hashes for a key read as 32-bit dwords (the LDS-staged keys of the
// bin kernel): two v_alignbit_b32 per key word instead of a 64-bit funnel shift,
// no per-word length masks (whole words in the loop, one masked tail after it),
// and the h2 stream's seed-prefix splice as two more alignbits with a
// kernel-uniform shift (prefix class PC: 0 for D % 8 == 0, 1 for 1..4, 2 for 5..7).

// ({hi, lo} >> (s & 31))[31:0]: v_alignbit_b32 on the device.
NB_HD uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t s) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, s);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (s & 31));
#endif
}
NB_HD uint64_t pack64(uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); }

// Stream word = the previous key word's top p bytes ++ this key word's low 8 - p
// bytes, i.e. ({kw, kwp} >> (64 - 8p))[63:0] (p = D % 8, uniform).
template <int PC>
NB_HD uint64_t lsx_splice(uint64_t kwp, uint64_t kw, uint32_t p) {
    const uint32_t pl = (uint32_t)kwp, ph = (uint32_t)(kwp >> 32);
    const uint32_t l = (uint32_t)kw, h = (uint32_t)(kw >> 32);
    if (PC == 0) return kw;
    if (PC == 1) return pack64(alignbit(l, ph, 32 - 8 * p), alignbit(h, l, 32 - 8 * p));
    return pack64(alignbit(ph, pl, 64 - 8 * p), alignbit(l, ph, 64 - 8 * p));
}

// h1 = H(key), h2 = H(to_string(seed) ++ key) for a key of len bytes starting at
// bit sh (0, 8, 16, 24) of dword D(0); D(i) returns dword i, and reads run up to
// 12 bytes past the key's last byte.  h0 = lsx_init(len); g0: h2's state after the
// whole prefix words (lsx_h2_start(c, len), or c.h2_init_fixed for fixed-length
// keys) -- both per length, so a kernel may take them from a table.
template <int PC, class LoadD>
NB_HD void lsx_hash_dwords(const FilterConsts &c, LoadD D, uint32_t sh, uint32_t len, uint64_t h0,
                           uint64_t g0, uint64_t *h1o, uint64_t *h2o) {
    const uint32_t L8 = len >> 3, rem = len & 7, p = c.prem;
    auto mask = [](uint64_t x, uint32_t nb) { return x & ((1ull << (8 * nb)) - 1); };
    uint64_t h = h0, g = g0;
    uint64_t kwp = PC ? c.pre_tail << (64 - 8 * p) : 0;  // key word -1 as the splice sees it
    uint32_t d0 = D(0), d1 = D(1);
    for (uint32_t j = 0; j < L8; ++j) {  // whole key words and whole stream words
        const uint32_t d2 = D(2 * j + 2), d3 = D(2 * j + 3);
        const uint64_t kw = pack64(alignbit(d1, d0, sh), alignbit(d2, d1, sh));
        h = lsx_round(h, kw);
        g = lsx_round(g, lsx_splice<PC>(kwp, kw, p));
        kwp = kw;
        d0 = d2;
        d1 = d3;
    }
    // key word L8 (its first rem bytes are the key's; the rest is read past it)
    const uint64_t kwt = pack64(alignbit(d1, d0, sh), alignbit(D(2 * L8 + 2), d1, sh));
    if (rem) h = lsx_tail(h, mask(kwt, rem));
    // stream word L8 holds p + rem valid bytes: a whole round when that reaches 8,
    // then word L8 + 1 holds the rest (p + rem - 8, from kwt alone)
    // (one straight-line step with selects: its lanes' p + rem differ, and
    // divergent branches would run every case for the whole wave)
    const uint32_t sv = p + rem;
    const uint64_t s8 = lsx_splice<PC>(kwp, kwt, p);
    const uint64_t x = sv >= 8 ? shift_mix(s8 * kMul) * kMul : mask(s8, sv);
    if (sv) g = (g ^ x) * kMul;  // a whole round (sv >= 8) or the tail
    if (sv > 8) g = lsx_tail(g, mask(lsx_splice<PC>(kwt, 0, p), sv - 8));
    *h1o = lsx_final(h);
    *h2o = lsx_final(g);
}

// g0 for a variable-length key (lsx_begin's h2 state).
NB_HD uint64_t lsx_h2_start(const FilterConsts &c, uint32_t len) {
    uint64_t g = lsx_init((uint64_t)len + c.plen);
    for (int w = 0; w < kMaxPrefixWords; ++w)
        if ((uint32_t)w < c.pwords) g = (g ^ c.pre_d[w]) * kMul;
    return g;
}

// ------------------------------------------------------------- Merkle ----
// MerkleTree (reference MerkleTree/merkle.cpp:7-55) hashes with the same
// std::hash<std::string> as the filter, over decimal strings: a leaf is
// to_string(H(record)), a parent to_string(H(left ++ right)) (merkle.cpp:26-32,48).

// H(bytes) alone (no seed prefix): the filter's h1 (hash_aligned_words' first half).
template <int FLAVOR, class LoadQ>
NB_HD uint64_t hash1_aligned_words(LoadQ Q, uint32_t a, uint32_t len) {
    const uint32_t nq = (a + len + 7) >> 3;
    const uint32_t nk = (len + 7) >> 3;
    uint64_t qcur = nq ? Q(0) : 0;
    uint64_t h = FLAVOR == 1 ? kFnvBasis : lsx_init(len);
    for (uint32_t j = 0; j < nk; ++j) {
        const uint64_t qnext = (j + 1 < nq) ? Q(j + 1) : 0;
        const uint64_t kw = mask_bytes(funnel(qcur, qnext, 8 * a), (int)(len - 8 * j));
        qcur = qnext;
        if (FLAVOR == 1) {
            for (int b = 0; b < 8; ++b)
                if (b < (int)(len - 8 * j)) h = fnv_step(h, (uint32_t)(kw >> (8 * b)) & 0xffu);
        } else {
            h = (j < (len >> 3)) ? lsx_round(h, kw) : lsx_tail(h, kw);
        }
    }
    return FLAVOR == 1 ? h : lsx_final(h);
}

// Four decimal digits of y < 10^4 as ASCII bytes, most significant first (LE u32).
NB_HD uint32_t dec4(uint32_t y) {
    const uint32_t a = y / 100, b = y - a * 100;
    const uint32_t a1 = a / 10, a0 = a - a1 * 10, b1 = b / 10, b0 = b - b1 * 10;
    return (a1 | (a0 << 8) | (b1 << 16) | (b0 << 24)) + 0x30303030u;
}
// Eight decimal digits of c < 10^8, most significant first (LE u64).
NB_HD uint64_t dec8(uint32_t c) {
    const uint32_t hi = c / 10000, lo = c - hi * 10000;
    return (uint64_t)dec4(hi) | ((uint64_t)dec4(lo) << 32);
}

// to_string(x) (what `stringstream << size_t` writes, merkle.cpp:29-31): its
// D = 1..20 ASCII digits left-aligned in w[0..2] (byte i = character i, zero
// bytes after the last digit).  Returns D.
NB_HD uint32_t u64_to_dec(uint64_t x, uint64_t w[3]) {
    const uint64_t q = x / 100000000ull;
    const uint32_t c0 = (uint32_t)(x - q * 100000000ull);
    const uint32_t c2 = (uint32_t)(q / 100000000ull);  // < 1845
    const uint32_t c1 = (uint32_t)(q - (uint64_t)c2 * 100000000ull);
    const uint64_t d1 = dec8(c1), d0 = dec8(c0);
    // the 20-character zero-padded string: c2 (4) | c1 (8) | c0 (8)
    const uint64_t p0 = (uint64_t)dec4(c2) | (d1 << 32);
    const uint64_t p1 = (d1 >> 32) | (d0 << 32);
    const uint64_t p2 = d0 >> 32;
    // leading '0' characters to drop: the first non-'0' byte (the last one kept)
    const uint64_t z0 = p0 ^ 0x3030303030303030ull, z1 = p1 ^ 0x3030303030303030ull;
    const uint64_t z2 = (p2 ^ 0x30303030ull) & 0xffffffffull;
    uint32_t z;
    if (z0) z = (uint32_t)(__builtin_ctzll(z0) >> 3);
    else if (z1) z = 8 + (uint32_t)(__builtin_ctzll(z1) >> 3);
    else if (z2) z = 16 + (uint32_t)(__builtin_ctzll(z2) >> 3);
    else z = 19;  // x == 0: "0"
    // shift left by z bytes (selects, not an indexed array: no scratch on the device)
    const uint32_t zq = z >> 3, zr = 8 * (z & 7);
    auto pick = [&](uint32_t i) -> uint64_t { return i == 0 ? p0 : i == 1 ? p1 : i == 2 ? p2 : 0; };
    for (uint32_t j = 0; j < 3; ++j) {
        const uint64_t lo = pick(j + zq), hi = pick(j + zq + 1);
        w[j] = zr ? (lo >> zr) | (hi << (64 - zr)) : lo;
    }
    return 20 - z;
}

// H(to_string(l) ++ to_string(r)): a Merkle parent (merkle.cpp:44-48).
template <int FLAVOR>
NB_HD uint64_t hash_dec_pair(uint64_t l, uint64_t r) {
    uint64_t wl[3], wr[3];
    const uint32_t dl = u64_to_dec(l, wl), dr = u64_to_dec(r, wr);
    const uint32_t len = dl + dr, q = dl >> 3, s = 8 * (dl & 7);
    // r's characters shifted to byte offset dl: sr[j] lands in word q + j
    const uint64_t sr0 = wr[0] << s, sr1 = s ? (wr[1] << s) | (wr[0] >> (64 - s)) : wr[1],
                   sr2 = s ? (wr[2] << s) | (wr[1] >> (64 - s)) : wr[2],
                   sr3 = s ? wr[2] >> (64 - s) : 0;
    auto pick = [&](uint32_t i) -> uint64_t {  // sr[i], zero outside 0..3
        return i == 0 ? sr0 : i == 1 ? sr1 : i == 2 ? sr2 : i == 3 ? sr3 : 0;
    };
    uint64_t S[5];
    for (uint32_t j = 0; j < 5; ++j) S[j] = (j < 3 ? wl[j] : 0) | (j >= q ? pick(j - q) : 0);
    uint64_t h = FLAVOR == 1 ? kFnvBasis : lsx_init(len);
    for (uint32_t j = 0; j < 5; ++j) {
        if (8 * j >= len) break;
        if (FLAVOR == 1) {
            for (uint32_t b = 0; b < 8 && 8 * j + b < len; ++b)
                h = fnv_step(h, (uint32_t)(S[j] >> (8 * b)) & 0xffu);
        } else {
            h = (j < (len >> 3)) ? lsx_round(h, S[j]) : lsx_tail(h, S[j]);
        }
    }
    return FLAVOR == 1 ? h : lsx_final(h);
}

// -------------------------------------------------------- host reference ----
// Scalar host evaluation over a contiguous key (used for the single-key probe of
// the drop-in class; the batch paths run on the device).
inline void key_hashes_host(const FilterConsts &c, const uint8_t *p, uint64_t len,
                            uint64_t *h1o, uint64_t *h2o) {
    auto ld = [](const uint8_t *q, uint64_t nb) {
        uint64_t r = 0;
        for (uint64_t b = 0; b < nb; ++b) r |= (uint64_t)q[b] << (8 * b);
        return r;
    };
    if (c.flavor == 2) {
        auto K = [&](uint32_t j) {
            uint64_t w = 0;
            for (uint64_t b = 0; b < 8 && 8ull * j + b < len; ++b) w |= (uint64_t)p[8ull * j + b] << (8 * b);
            return w;
        };
        mm3_x64_128(K, (uint32_t)len, c.mm3_seed, h1o, h2o);
        return;
    }
    if (c.flavor == 1) {
        uint64_t a = kFnvBasis, b = c.fnv_pre;
        for (uint64_t i = 0; i < len; ++i) { a = fnv_step(a, p[i]); b = fnv_step(b, p[i]); }
        *h1o = a; *h2o = b;
        return;
    }
    uint64_t h = lsx_init(len);
    uint64_t whole = len & ~7ULL;
    for (uint64_t o = 0; o < whole; o += 8) h = lsx_round(h, ld(p + o, 8));
    if (len & 7) h = lsx_tail(h, ld(p + whole, len & 7));
    *h1o = lsx_final(h);
    // h2 over prefix ++ key, with the whole prefix words pre-mixed.
    uint64_t total = c.plen + len;
    uint64_t g = lsx_init(total);
    for (uint32_t w = 0; w < c.pwords; ++w) g = (g ^ c.pre_d[w]) * kMul;
    // stream = r prefix bytes ++ key bytes
    uint64_t slen = c.prem + len;
    uint64_t swhole = slen & ~7ULL;
    auto sbyte = [&](uint64_t i) -> uint64_t {
        return i < c.prem ? (c.pre_tail >> (8 * i)) & 0xff : p[i - c.prem];
    };
    for (uint64_t o = 0; o < swhole; o += 8) {
        uint64_t w = 0;
        for (int b = 0; b < 8; ++b) w |= sbyte(o + b) << (8 * b);
        g = lsx_round(g, w);
    }
    if (slen & 7) {
        uint64_t w = 0;
        for (uint64_t b = 0; b < (slen & 7); ++b) w |= sbyte(swhole + b) << (8 * b);
        g = lsx_tail(g, w);
    }
    *h2o = lsx_final(g);
}

}  // namespace nb
