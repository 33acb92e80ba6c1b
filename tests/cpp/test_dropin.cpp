// Drop-in class test: drives nasp-key-value-engine_amd/host/BloomFilter the way
// the reference's callers do and checks every image bit for bit against the
// oracle (oracle/bloom_oracle.c).  Runs with or without a GPU: batches of at
// least BloomFilter::hostBatchLimit() keys are built on the device when one is
// visible (checked), smaller ones -- and every batch on a GPU-less host, after
// one std::cerr line per failed device build -- on the host.
//   1. reference test program flow (BloomFilter/main.cpp:28-117): BF(20, 0.05),
//      10 names added, membership of added / absent names, BF(10, 0.1) round trip;
//   2. SSTable::build usage (SSTable/SSTable.cpp:28-35): BF(records.size(), 0.01),
//      add() per record key, copy-assign into a member, serialize();
//   3. TypesManager usage (System/TypesManager.cpp:74-107): deserialize, add,
//      serialize (accumulate), then probe;
//   4. the reference's committed MSVC filters with the FNV flavour;
//   5. device / host placement: a large batch reaches the GPU (when there is
//      one), a TypesManager round trip launches no device build.
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/nasp_bloom.h"
#include "../../nasp-key-value-engine_amd/host/BloomFilter.h"
extern "C" {
#include "../../oracle/bloom_oracle.h"
}

static int failures = 0;
#define EXPECT(cond, msg)                                     \
    do {                                                      \
        if (!(cond)) {                                        \
            std::printf("FAIL: %s (line %d)\n", msg, __LINE__); \
            ++failures;                                       \
        }                                                     \
    } while (0)

static std::vector<uint8_t> oracle_image(const std::vector<std::string> &keys, uint32_t m,
                                         uint32_t k, double p, uint32_t tc, uint64_t seed,
                                         int flavor, const std::vector<uint64_t> *start = nullptr) {
    std::vector<uint8_t> buf;
    std::vector<uint64_t> offs{0};
    for (auto &s : keys) {
        buf.insert(buf.end(), s.begin(), s.end());
        offs.push_back(buf.size());
    }
    buf.resize(buf.size() + 16);
    std::vector<uint64_t> words = start ? *start : std::vector<uint64_t>((m + 63) / 64 + 1, 0);
    orc_build(flavor, buf.data(), offs.data(), 0, keys.size(), m, k, seed, words.data());
    std::vector<uint8_t> img(orc_serialized_size(m));
    orc_serialize(m, k, p, tc, seed, words.data(), img.data());
    return img;
}

static std::vector<uint8_t> bytes_of(const std::vector<std::byte> &v) {
    return std::vector<uint8_t>(reinterpret_cast<const uint8_t *>(v.data()),
                                reinterpret_cast<const uint8_t *>(v.data()) + v.size());
}

static void header(const std::vector<uint8_t> &img, uint32_t *m, uint32_t *k, double *p,
                   uint32_t *tc, uint64_t *seed) {
    std::memcpy(m, img.data(), 4);
    std::memcpy(k, img.data() + 4, 4);
    std::memcpy(p, img.data() + 8, 8);
    std::memcpy(tc, img.data() + 16, 4);
    std::memcpy(seed, img.data() + 20, 8);
}

int main() {
    const bool gpu = nb_device_count() > 0;
    std::printf("devices: %d\n", nb_device_count());
    // 1. reference test program flow
    {
        BloomFilter bf(20, 0.05);
        std::vector<std::string> added = {"Ana", "Marko", "Jelena", "Nikola", "Maja",
                                          "Stefan", "Marina", "Petar", "Ivana", "Luka"};
        for (auto &e : added) bf.add(e);
        for (auto &e : added) EXPECT(bf.possiblyContains(e), "added name must be present");
        auto img = bytes_of(bf.serialize());
        uint32_t m, k, tc; double p; uint64_t seed;
        header(img, &m, &k, &p, &tc, &seed);
        EXPECT(m == orc_size_of_bitset(20, 0.05) && k == orc_num_hashes(20, m), "m/k formulas");
        EXPECT(seed == orc_seed_from_time(tc), "seed from timeConst");
        EXPECT(img == oracle_image(added, m, k, p, tc, seed, 0), "BF(20,0.05) image");
        // absent names: same answers as the oracle's probe
        std::vector<std::string> absent = {"Anja", "Marija", "Jovan", "Nina", "Milan", "Stefania",
                                           "Marin", "Pera", "Iva", "Lukas", "Bogdan", "Elena"};
        std::vector<uint64_t> words((m + 63) / 64 + 1, 0);
        std::memcpy(words.data(), img.data() + 28, img.size() - 28);
        for (auto &e : absent) {
            uint8_t o = 0;
            orc_probe(0, reinterpret_cast<const uint8_t *>(e.data()), nullptr, (uint32_t)e.size(), 1,
                      m, k, seed, words.data(), &o);
            EXPECT(bf.possiblyContains(e) == (o != 0), "absent-name answer matches oracle");
        }
        BloomFilter original(10, 0.1);
        for (const char *e : {"Jedan", "Dva", "Tri"}) original.add(e);
        BloomFilter restored = BloomFilter::deserialize(original.serialize());
        for (const char *e : {"Jedan", "Dva", "Tri", "Cetiri"})
            EXPECT(original.possiblyContains(e) == restored.possiblyContains(e), "round trip");
        EXPECT(bytes_of(original.serialize()) == bytes_of(restored.serialize()), "round trip image");
    }
    // 2. SSTable::build usage: 50k sorted records, copy-assign, serialize
    {
        std::vector<std::string> recs;
        for (int i = 0; i < 50000; ++i) {
            char b[32];
            std::snprintf(b, sizeof b, "user%012d", i);
            recs.push_back(b);
        }
        BloomFilter member;
        BloomFilter bf(recs.size(), 0.01);
        for (auto &r : recs) bf.add(r);
        member = bf;  // bloom_ = bf (SSTable.cpp:35)
        auto img = bytes_of(member.serialize());
        uint32_t m, k, tc; double p; uint64_t seed;
        header(img, &m, &k, &p, &tc, &seed);
        EXPECT(img == oracle_image(recs, m, k, p, tc, seed, 0), "SSTable-style build image");
        EXPECT(member.lastBuildOnDevice() == gpu, "50k-key batch built on the GPU iff one is visible");
        int present = 0;
        for (auto &r : recs) present += member.possiblyContains(r);
        EXPECT(present == (int)recs.size(), "no false negatives");
    }
    // 3. TypesManager usage: deserialize -> add -> serialize accumulates
    {
        const uint64_t launches = nb_device_build_count();
        BloomFilter bf(1000, 0.01);
        bf.add("alpha");
        auto first = bf.serialize();
        BloomFilter again = BloomFilter::deserialize(first);
        again.add("beta");
        again.add(std::string("\0gamma", 6));
        auto img = bytes_of(again.serialize());
        uint32_t m, k, tc; double p; uint64_t seed;
        header(img, &m, &k, &p, &tc, &seed);
        EXPECT(img == oracle_image({"alpha", "beta", std::string("\0gamma", 6)}, m, k, p, tc, seed, 0),
               "accumulate after deserialize");
        EXPECT(again.possiblyContains("alpha") && again.possiblyContains("beta"), "accumulated keys");
        EXPECT(!again.lastBuildOnDevice() && nb_device_build_count() == launches,
               "TypesManager round trip stays on the host (no device build)");
        BloomFilter def;
        EXPECT(def.possiblyContains("anything"), "default filter answers true");
    }
    // 4. an MSVC-written filter (level_0/filter_0.sst payload) with the FNV flavour
    {
        const uint8_t img0[31] = {0x14, 0, 0, 0, 7, 0, 0, 0, 0x7b, 0x14, 0xae, 0x47, 0xe1, 0x7a,
                                  0x84, 0x3f, 0xb7, 0x0f, 0x3f, 0x68, 0xb7, 0x1c, 0x25, 0x6e,
                                  0x0b, 0xde, 0x4d, 0xec, 0x2a, 0x2a, 0x0a};
        std::vector<std::byte> v(31);
        std::memcpy(v.data(), img0, 31);
        BloomFilter::setDefaultFlavor(NB_FLAVOR_MSVC_FNV1A);
        BloomFilter f = BloomFilter::deserialize(v);
        EXPECT(f.possiblyContains("test") && f.possiblyContains("test2"), "MSVC filter members");
        BloomFilter rebuilt = BloomFilter::deserialize(v);
        rebuilt.add("test");
        rebuilt.add("test2");
        EXPECT(bytes_of(rebuilt.serialize()) == std::vector<uint8_t>(img0, img0 + 31),
               "re-adding the members leaves the MSVC image unchanged");
        BloomFilter::setDefaultFlavor(NB_FLAVOR_LIBSTDCXX);
    }
    // 5. the host/device cut-over at hostBatchLimit() keys, both flavours, mixed
    //    key lengths (offsets chunk) and one length (fixed chunk), empty keys
    for (int flavor = 0; flavor < 2; ++flavor) {
        BloomFilter::setDefaultFlavor(flavor);
        for (uint64_t n : {BloomFilter::hostBatchLimit() - 1, BloomFilter::hostBatchLimit()}) {
            for (int mixed = 0; mixed < 2; ++mixed) {
                std::vector<std::string> keys;
                for (uint64_t i = 0; i < n; ++i) {
                    char b[48];
                    const int l = std::snprintf(b, sizeof b, "k%015llu", (unsigned long long)i * 7919);
                    keys.emplace_back(b, mixed ? (size_t)(i % 23) : (size_t)l);
                }
                BloomFilter bf((unsigned)n, 0.01);
                const uint64_t before = nb_device_build_count();
                for (auto &x : keys) bf.add(x);
                auto img = bytes_of(bf.serialize());
                uint32_t m, k, tc; double p; uint64_t seed;
                header(img, &m, &k, &p, &tc, &seed);
                EXPECT(img == oracle_image(keys, m, k, p, tc, seed, flavor), "cut-over image");
                const bool dev = n >= BloomFilter::hostBatchLimit() && gpu;
                EXPECT(bf.lastBuildOnDevice() == dev, "batch placement");
                EXPECT((nb_device_build_count() > before) == dev, "device builds only for large batches");
            }
        }
    }
    BloomFilter::setDefaultFlavor(NB_FLAVOR_LIBSTDCXX);
    // 6. a batch of several chunks (16 MB / 1M keys each): 16-byte keys, then mixed
    //    lengths from inside the third chunk on -- streamed chunk by chunk to the
    //    device builder, or (no GPU) built on the host chunk by chunk
    std::vector<std::string> big;
    for (uint64_t i = 0; i < 2'600'000; ++i) {
        char b[40];
        std::snprintf(b, sizeof b, "%016llx", (unsigned long long)(i * 0x9E3779B97F4A7C15ull));
        big.emplace_back(b, i < 2'300'000 ? 16 : 1 + i % 29);
    }
    {
        BloomFilter bf((unsigned)big.size(), 0.01);
        for (auto &x : big) bf.add(x);
        BloomFilter member;
        member = bf;
        auto img = bytes_of(member.serialize());
        uint32_t m, k, tc; double p; uint64_t seed;
        header(img, &m, &k, &p, &tc, &seed);
        EXPECT(img == oracle_image(big, m, k, p, tc, seed, 0), "multi-chunk streamed image");
        EXPECT(member.lastBuildOnDevice() == gpu, "multi-chunk batch on the GPU iff one is visible");
        // 7. copies share the words until one side changes: adding to the copy leaves
        //    the original's image alone (copy on write)
        BloomFilter copy = member;
        std::vector<std::string> extra(big.begin(), big.begin() + 10);
        for (auto &x : extra) x += "-more";
        for (auto &x : extra) copy.add(x);
        EXPECT(bytes_of(member.serialize()) == img, "original unchanged after its copy grew");
        std::vector<std::string> both = big;
        both.insert(both.end(), extra.begin(), extra.end());
        EXPECT(bytes_of(copy.serialize()) == oracle_image(both, m, k, p, tc, seed, 0), "copy image");
        // 8. a moved-from filter is a default one; both can be reused
        BloomFilter moved = std::move(copy);
        EXPECT(copy.possiblyContains("anything") && copy.serialize().size() == 28, "moved-from is default");
        copy = BloomFilter(100, 0.01);
        copy.add("x");
        EXPECT(copy.possiblyContains("x"), "moved-from filter reusable");
        EXPECT(bytes_of(moved.serialize()) == oracle_image(both, m, k, p, tc, seed, 0), "moved-to image");
        // pending keys move with the object
        BloomFilter half((unsigned)big.size(), 0.01);
        for (size_t i = 0; i < 1'500'000; ++i) half.add(big[i]);
        BloomFilter half2(std::move(half));
        for (size_t i = 1'500'000; i < big.size(); ++i) half2.add(big[i]);
        auto himg = bytes_of(half2.serialize());
        header(himg, &m, &k, &p, &tc, &seed);
        EXPECT(himg == oracle_image(big, m, k, p, tc, seed, 0), "moved mid-stream image");
    }
    // 9. device failures (fault injection, GPU only): a failure while keys stream is
    //    rebuilt on the host from the retained chunks; past retainBytes() it throws
    if (gpu) {
        std::vector<std::string> keys(big.begin(), big.begin() + 50'000);
        BloomFilter bf((unsigned)keys.size(), 0.01);
        nb_set_knob("NB_FAIL_BUILDS", 1);
        for (auto &x : keys) bf.add(x);
        auto img = bytes_of(bf.serialize());
        uint32_t m, k, tc; double p; uint64_t seed;
        header(img, &m, &k, &p, &tc, &seed);
        EXPECT(img == oracle_image(keys, m, k, p, tc, seed, 0), "injected failure: host rebuild image");
        EXPECT(!bf.lastBuildOnDevice(), "injected failure: built on the host");
        // accumulate-after-deserialize with a failure on the second of three chunks
        BloomFilter base = BloomFilter::deserialize(bf.serialize());
        for (size_t i = 0; i < 1'200'000; ++i) base.add(big[i]);
        nb_set_knob("NB_FAIL_BUILDS", 1);  // the chunk handed off next (at 2M keys) fails
        for (size_t i = 1'200'000; i < big.size(); ++i) base.add(big[i]);
        std::vector<std::string> all = keys;
        all.insert(all.end(), big.begin(), big.end());
        EXPECT(bytes_of(base.serialize()) == oracle_image(all, m, k, p, tc, seed, 0),
               "mid-stream failure: host rebuild from the deserialized bits");
        // nothing retained: the failure is reported, not hidden
        const uint64_t keep = BloomFilter::retainBytes();
        BloomFilter::setRetainBytes(0);
        BloomFilter lost((unsigned)big.size(), 0.01);
        for (size_t i = 0; i < 1'200'000; ++i) lost.add(big[i]);
        nb_set_knob("NB_FAIL_BUILDS", 1);
        bool threw = false;
        try {
            for (size_t i = 1'200'000; i < big.size(); ++i) lost.add(big[i]);
            (void)lost.serialize();
        } catch (const std::runtime_error &e) {
            threw = std::strstr(e.what(), "injected") != nullptr;
        }
        EXPECT(threw, "failure past the retention budget throws with the device error");
        BloomFilter::setRetainBytes(keep);
        nb_set_knob("NB_FAIL_BUILDS", 0);
        BloomFilter again((unsigned)keys.size(), 0.01);
        for (auto &x : keys) again.add(x);
        (void)again.serialize();
        EXPECT(again.lastBuildOnDevice(), "the next filter is built on the device again");
    }
    nb_shutdown();
    std::printf(failures ? "FAILED %d\n" : "drop-in OK\n", failures);
    return failures ? 1 : 0;
}
