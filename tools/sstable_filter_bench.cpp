// sstable_filter_bench.cpp -- host-to-host rate of SSTable::build's filter block
// through the drop-in class (reference SSTable/SSTable.cpp:28-35):
//
//   BloomFilter bf(records.size(), 0.01);
//   for (const auto& r : records) bf.add(r.key);   // keys packed into pinned chunks,
//   bloom_ = bf;                                    // uploaded + built while packing
//   ... writeBloomToFile: bf.serialize()            // filter downloaded, image made
//
// Keys are std::strings already in host memory (the memtable's records), the
// result is the serialized image in host memory: packing, H2D, build, D2H and
// serialize are all inside the timed region.  Prints one JSON line.
//   usage: sstable_filter_bench [n_keys=10000000] [key_len=16] [reps=3]
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../include/nasp_bloom.h"
#include "../nasp-key-value-engine_amd/host/BloomFilter.h"

static uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 10000000;
    const size_t len = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 16;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 3;
    if (nb_device_count() == 0) {
        std::printf("{\"error\": \"no GPU\"}\n");
        return 77;
    }
    std::vector<std::string> keys(n);
    for (size_t i = 0; i < n; ++i) {
        keys[i].resize(len);
        for (size_t b = 0; b < len; b += 8) {
            const uint64_t w = splitmix64(i * ((len + 7) / 8) + b / 8);
            for (size_t j = 0; j < 8 && b + j < len; ++j) keys[i][b + j] = (char)(w >> (8 * j));
        }
    }
    // the CPU floor: packing the same std::string keys into one contiguous buffer
    double pack_best = 1e30;
    {
        std::vector<uint8_t> packed(n * len + 64);
        for (int r = 0; r < reps; ++r) {
            const auto t0 = std::chrono::steady_clock::now();
            size_t o = 0;
            for (const std::string &k : keys) {
                std::memcpy(packed.data() + o, k.data(), k.size());
                o += k.size();
            }
            const auto t1 = std::chrono::steady_clock::now();
            pack_best = std::min(pack_best, std::chrono::duration<double>(t1 - t0).count());
            if (packed[o / 2] == 0xAB && packed[1] == 0xCD) std::printf(" ");  // keep the copy
        }
    }
    double best = 1e30, ph[3] = {0, 0, 0};  // phases of the best rep: add loop, copy-assign, serialize
    size_t img_bytes = 0;
    bool ok = true, on_dev = true;
    auto secs = [](auto a, auto b) { return std::chrono::duration<double>(b - a).count(); };
    for (int r = 0; r < reps + 1; ++r) {  // first rep warms the library's pools
        const auto t0 = std::chrono::steady_clock::now();
        BloomFilter bf((unsigned)n, 0.01);
        for (const std::string &k : keys) bf.add(k);
        const auto t1 = std::chrono::steady_clock::now();
        BloomFilter member;
        member = bf;  // SSTable.cpp:35 (bloom_ = bf): the pending keys are built here
        const auto t2 = std::chrono::steady_clock::now();
        const std::vector<std::byte> img = member.serialize();
        const auto t3 = std::chrono::steady_clock::now();
        const double s = secs(t0, t3);
        if (r > 0 && s < best) {
            best = s;
            ph[0] = secs(t0, t1);
            ph[1] = secs(t1, t2);
            ph[2] = secs(t2, t3);
        }
        img_bytes = img.size();
        on_dev = on_dev && member.lastBuildOnDevice();
        for (size_t i = 0; i < n; i += n / 1000 + 1) ok = ok && member.possiblyContains(keys[i]);
    }
    std::printf("{\"keys\": %zu, \"key_bytes\": %zu, \"ms\": %.3f, \"value\": %.3f, "
                "\"unit\": \"Mkeys/s\", \"pack_only_ms\": %.3f, \"phases_ms\": {\"ctor_and_adds\": %.3f, "
                "\"copy_assign_build\": %.3f, \"serialize\": %.3f}, \"image_bytes\": %zu, "
                "\"built_on_device\": %s, \"sampled_keys_found\": %s, "
                "\"note\": \"drop-in BloomFilter: ctor + add() per std::string key + copy-assign "
                "+ serialize(), host memory to host memory, best of %d\"}\n",
                n, len, best * 1e3, n / best / 1e6, pack_best * 1e3, ph[0] * 1e3, ph[1] * 1e3,
                ph[2] * 1e3, img_bytes, on_dev ? "true" : "false", ok ? "true" : "false", reps);
    nb_shutdown();
    return ok ? 0 : 1;
}
