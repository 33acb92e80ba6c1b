// Host check of bloom_math.h against plain 64-bit arithmetic and the oracle:
// fast remainder, incremental indices, and both hash flavours (with the seed
// prefix splice).  Built and run by tests/test_math_host.py (no GPU needed).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>
#include "../../nasp-key-value-engine_amd/csrc/bloom_math.h"
extern "C" {
#include "../../oracle/bloom_oracle.h"
}

int main() {
    std::mt19937_64 rng(12345);
    long bad = 0;
    std::vector<uint32_t> ms = {1u, 2u, 3u, 7u, 20u, 64u, 47926u, 95850584u, 958505838u,
                                1492685679u, 2147483648u, 2147483659u, 3000000019u,
                                4294967288u, 4294967295u};
    for (int t = 0; t < 2000; ++t) ms.push_back((uint32_t)(rng() >> (rng() % 32)) | 1u);
    for (uint32_t v : {8191u, 8192u, 8193u, 12289u, 65537u, 2147483647u, 2147483649u, 4294967291u})
        ms.push_back(v);
    for (uint32_t m : ms) {
        // the default (f64 quotient from m >= 2^13) and the integer remainder only
        for (uint32_t fp_min : {8192u, ~0u}) {
            nb::FastMod f = nb::make_fastmod(m, fp_min);
            for (int t = 0; t < 4000; ++t) {
                uint64_t x = rng();
                if (t < 8) x = t < 4 ? (uint64_t)t : ~0ull - (uint64_t)(t - 4);
                if (t >= 2000) {
                    // x = q m + r with r at the ends and the middle of [0, m): the
                    // quotient estimate's rounding boundaries, up to q = floor(2^64-1 / m)
                    const uint64_t qmax = ~0ull / m;
                    const uint64_t q = t < 2100 ? qmax - (uint64_t)(t - 2000) : (qmax == ~0ull ? rng() : rng() % (qmax + 1));
                    const uint32_t rs[] = {0u, 1u, m - 1, m / 2, m / 2 + 1, m / 2 - 1 + (m == 1)};
                    x = q * m + rs[t % 6] % m;
                    if (x / m != q) x = q * m;  // past 2^64 - 1
                }
                if (nb::mod64(x, f) != (uint32_t)(x % m)) ++bad;
            }
        }
        // incremental indices vs direct
        nb::FilterConsts c = nb::make_consts(m, 10, 17027509906831645879ull, 0);
        for (int t = 0; t < 200; ++t) {
            uint64_t h1 = rng(), h2 = rng();
            if (t == 0) h1 = ~0ull, h2 = ~0ull;  // a wrap on every step
            if (t == 1) h1 = 0, h2 = 1ull << 63;
            nb::IndexGen g;  // the kernels' generator
            g.start(h1, h2, c);
            for (uint32_t i = 0; i < 40; ++i) {
                if (i) g.next(c);
                if (g.r != (uint32_t)((h1 + (uint64_t)i * h2) % m)) ++bad;
            }
        }
        // modular add of the index step, including sums that carry out of 32 bits
        for (int t = 0; t < 2000; ++t) {
            uint32_t a = (uint32_t)(rng() % m), b = (uint32_t)(rng() % m);
            if (t == 0) a = b = m - 1;
            if (nb::addmod_fast(a, b, m) != (uint32_t)(((uint64_t)a + b) % m)) ++bad;
        }
    }
    printf("mod/incremental mismatches: %ld\n", bad);
    long hbad = 0;
    uint64_t seeds[] = {0ull, 5ull, 12345678ull, 123456789ull, 1234567890123456ull,
                        17027509906831645879ull, 18446744073709551615ull, 99999999ull,
                        // D % 8 = 2, 3, 5, 6, 7 (every prefix class of the dword path)
                        12ull, 123ull, 1234567890123ull, 12345678901234ull, 123456789012345ull,
                        1234567ull};
    for (uint64_t seed : seeds) {
        for (int fl = 0; fl < 2; ++fl) {
            nb::FilterConsts c = nb::make_consts(1000003u, 7, seed, (uint32_t)fl);
            for (int t = 0; t < 3000; ++t) {
                uint8_t buf[100];
                size_t len = rng() % 90;
                for (size_t b = 0; b < len; ++b) buf[b] = (uint8_t)rng();
                uint64_t h1, h2;
                nb::key_hashes_host(c, buf, len, &h1, &h2);
                // the device's word-stream path, at every misalignment a = 0..7
                alignas(8) uint8_t arena[128 + 16];
                uint32_t a = (uint32_t)(rng() % 8);
                for (size_t b = 0; b < sizeof arena; ++b) arena[b] = (uint8_t)rng();  // junk around
                for (size_t b = 0; b < len; ++b) arena[8 + a + b] = buf[b];
                const uint64_t *q = reinterpret_cast<const uint64_t *>(arena + 8);
                uint64_t g1, g2;
                if (fl) nb::hash_aligned_words<1>(c, [q](uint32_t j) { return q[j]; }, a, (uint32_t)len, &g1, &g2);
                else nb::hash_aligned_words<0>(c, [q](uint32_t j) { return q[j]; }, a, (uint32_t)len, &g1, &g2);
                if (g1 != h1 || g2 != h2) ++hbad;
                // fixed-length form: h2 prefix state precomputed on the host
                nb::FilterConsts cf = c;
                nb::set_fixed_len(cf, (uint32_t)len);
                if (fl == 0) {
                    auto load = [q](uint32_t j) { return q[j]; };
                    nb::hash_aligned_words<0, decltype(load), true>(cf, load, a, (uint32_t)len,
                                                                    &g1, &g2);
                    if (g1 != h1 || g2 != h2) ++hbad;
                }
                if (fl == 0) {
                    // the dword-stream path of the staged bin kernel (prefix class of
                    // D % 8), key at byte offset 0..3 of a dword, junk around it
                    alignas(4) uint8_t dw[128 + 32];
                    const uint32_t b = (uint32_t)(rng() % 4);
                    for (size_t q = 0; q < sizeof dw; ++q) dw[q] = (uint8_t)rng();
                    for (size_t q = 0; q < len; ++q) dw[b + q] = buf[q];
                    const uint32_t *d32 = reinterpret_cast<const uint32_t *>(dw);
                    auto D = [d32](uint32_t i) { return d32[i]; };
                    const uint32_t pc = c.prem == 0 ? 0 : c.prem <= 4 ? 1 : 2;
                    for (int fixed = 0; fixed < 2; ++fixed) {
                        const uint64_t g0 = fixed ? cf.h2_init_fixed : nb::lsx_h2_start(c, (uint32_t)len);
                        if (pc == 0) nb::lsx_hash_dwords<0>(c, D, 8 * b, (uint32_t)len, nb::lsx_init(len), g0, &g1, &g2);
                        else if (pc == 1) nb::lsx_hash_dwords<1>(c, D, 8 * b, (uint32_t)len, nb::lsx_init(len), g0, &g1, &g2);
                        else nb::lsx_hash_dwords<2>(c, D, 8 * b, (uint32_t)len, nb::lsx_init(len), g0, &g1, &g2);
                        if (g1 != h1 || g2 != h2) ++hbad;
                    }
                }
                for (uint32_t i = 0; i < 3; ++i) {
                    uint32_t want = orc_index(fl, buf, len, i, 1000003u, seed);
                    if ((uint32_t)((h1 + (uint64_t)i * h2) % 1000003u) != want) ++hbad;
                }
            }
        }
    }
    printf("hash mismatches: %ld\n", hbad);

    // Merkle helpers (MerkleTree/merkle.cpp:26-32,48): to_string(x) of every digit
    // count, single-string hash at every misalignment, and the parent hash
    // H(to_string(l) ++ to_string(r)) against the oracle's snprintf restatement.
    long mbad = 0;
    std::vector<uint64_t> xs = {0ull, 1ull, 9ull, 10ull, 99ull, 100ull, 12345678ull, 99999999ull,
                                100000000ull, 10000000000000000ull, 1844674407370955161ull,
                                9999999999999999999ull, 10000000000000000000ull, ~0ull};
    for (uint64_t p10 = 1; p10 < 10000000000000000000ull; p10 *= 10) {
        xs.push_back(p10);
        xs.push_back(p10 - 1);
        xs.push_back(p10 + 1);
    }
    for (int t = 0; t < 20000; ++t) xs.push_back(rng() >> (rng() % 64));
    for (uint64_t x : xs) {
        uint64_t w[3];
        const uint32_t d = nb::u64_to_dec(x, w);
        char want[32];
        const int wl = snprintf(want, sizeof want, "%llu", (unsigned long long)x);
        char got[25] = {0};
        for (int b = 0; b < 24; ++b) got[b] = (char)(w[b / 8] >> (8 * (b % 8)));
        if ((int)d != wl || std::string(got, d) != std::string(want, wl)) ++mbad;
        for (int b = d; b < 24; ++b)
            if (got[b]) { ++mbad; break; }  // zero bytes after the digits
    }
    for (int fl = 0; fl < 2; ++fl) {
        for (int t = 0; t < 20000; ++t) {
            const uint64_t l = xs[rng() % xs.size()], r = xs[rng() % xs.size()];
            char buf[48];
            const int n = snprintf(buf, sizeof buf, "%llu%llu", (unsigned long long)l,
                                   (unsigned long long)r);
            const uint64_t want = orc_hash(fl, reinterpret_cast<const uint8_t *>(buf), (size_t)n);
            const uint64_t got = fl ? nb::hash_dec_pair<1>(l, r) : nb::hash_dec_pair<0>(l, r);
            if (got != want) ++mbad;
        }
        for (int t = 0; t < 3000; ++t) {
            const size_t len = rng() % 100;
            alignas(8) uint8_t arena[128 + 16];
            const uint32_t a = (uint32_t)(rng() % 8);
            for (size_t b = 0; b < sizeof arena; ++b) arena[b] = (uint8_t)rng();
            const uint64_t *q = reinterpret_cast<const uint64_t *>(arena + 8);
            auto load = [q](uint32_t j) { return q[j]; };
            const uint64_t got = fl ? nb::hash1_aligned_words<1>(load, a, (uint32_t)len)
                                    : nb::hash1_aligned_words<0>(load, a, (uint32_t)len);
            if (got != orc_hash(fl, arena + 8 + a, len)) ++mbad;
        }
    }
    printf("merkle mismatches: %ld\n", mbad);
    return (bad || hbad || mbad) ? 1 : 0;
}
