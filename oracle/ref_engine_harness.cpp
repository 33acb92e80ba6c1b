// ref_engine_harness.cpp -- drives the reference engine's SSTable writer and LSM
// compaction (our code; the engine sources are compiled where they lie).
//
// Built twice (oracle/Makefile `ref-engine`, nasp-key-value-engine_amd/Makefile
// `engine-dropin`):
//   * against the reference BloomFilter.cpp  -> oracle/_ref/ref_engine
//   * against the MI355X drop-in class       -> nasp-key-value-engine_amd/build/engine_dropin
// Both write real SSTables through SSTManager::write (SSTable/SSTManager.cpp:274-359),
// so the filter files on disk come from SSTable::build (SSTable/SSTable.cpp:28-35)
// and writeBloomToFile (SSTableRaw.cpp:534-567 / SSTableComp.cpp:469-504).
// tests/test_engine_dropin.py checks every filter file against the oracle and the
// drop-in run against the reference run.
//
// usage: engine <data_dir> <raw|comp> <n_records> <block_size> [tiered|leveled]
//   writes one level-1 SSTable of n records ("user%012d" keys); with `tiered` or
//   `leveled`, writes three overlapping tables and runs
//   LSMManager::triggerCompactionCheck: size-tiered (LSM/LSMManager.cpp:203-233,
//   the level is merged into one level-2 table) or leveled (LSMManager.cpp:146-196,
//   multiplier 2: two level-1 tables are merged one by one into level 2).
// Prints "engine_ms <t>" on stderr: the time spent inside SSTManager::write and the
// compaction (records are generated outside the clock; the drop-in build starts HIP
// first).  NB_ENGINE_TIME (seconds) fixes the clock the filters' timeConst comes from
// (BloomFilter.cpp:37): runs of both binaries then write byte-identical files.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <vector>

// time() for this executable's own code (the BloomFilter constructors compiled
// into it resolve to this definition before libc's).
extern "C" time_t time(time_t *out) {
    const char *fixed = std::getenv("NB_ENGINE_TIME");
    const time_t v = fixed && *fixed
                         ? (time_t)std::strtoll(fixed, nullptr, 10)
                         : (time_t)std::chrono::duration_cast<std::chrono::seconds>(
                               std::chrono::system_clock::now().time_since_epoch())
                               .count();
    if (out) *out = v;
    return v;
}

#ifdef NB_ENGINE_DROPIN  // the drop-in build: HIP starts before the clock, as in a running engine
extern "C" int nb_device_count(void);
extern "C" unsigned long long nb_device_build_count(void);
extern "C" unsigned long long nb_device_merkle_count(void);
#endif

#include "Config.h"
#include "LSMManager.h"
#include "SSTManager.h"
#include "block-manager.h"

static std::vector<Record> records(int first, int n) {
    std::vector<Record> out;
    out.reserve(n);
    for (int i = 0; i < n; ++i) {
        char k[32], v[32];
        std::snprintf(k, sizeof k, "user%012d", first + i);
        std::snprintf(v, sizeof v, "value-%d", first + i);
        Record r{};
        r.key = k;
        r.value = v;
        r.key_size = r.key.size();
        r.value_size = r.value.size();
        r.timestamp = 1000000ull + (unsigned long long)(first + i);
        r.tombstone = std::byte{0};
        out.push_back(r);
    }
    return out;
}

int main(int argc, char **argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s <dir> <raw|comp> <n> <block_size> [tiered|leveled]\n", argv[0]);
        return 2;
    }
    Config::data_directory = argv[1];
    Config::compress_sstable = std::strcmp(argv[2], "comp") == 0;
    Config::sstable_single_file = false;
    const int n = std::atoi(argv[3]);
    Config::block_size = std::atoi(argv[4]);
    const bool tiered = argc > 5 && std::strcmp(argv[5], "tiered") == 0;
    const bool leveled = argc > 5 && std::strcmp(argv[5], "leveled") == 0;
    Config::compaction_strategy = leveled ? "leveled" : "tiered";
    Config::max_levels = 4;
    Config::max_number_of_sstable_on_level = 3;
    Config::l0_compaction_trigger = 2;
    Config::level_size_multiplier = 2;

#ifdef NB_ENGINE_DROPIN
    (void)nb_device_count();
#endif
    Block_manager bm;
    SSTManager sst(&bm);
    double ms = 0;  // engine time only: records are generated outside the clock
    auto timed = [&ms](auto &&fn) {
        const auto t0 = std::chrono::steady_clock::now();
        fn();
        ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    };
    if (!tiered && !leveled) {
        std::vector<Record> recs = records(0, n);
        timed([&] { sst.write(recs, 1); });
    } else {
        for (int t = 0; t < 3; ++t) {  // overlapping ranges
            std::vector<Record> recs = records(t * (n / 2), n);
            timed([&] { sst.write(recs, 1); });
        }
        LSMManager lsm(&sst);
        timed([&] { lsm.triggerCompactionCheck(); });
    }
    std::printf("engine done\n");
    std::fprintf(stderr, "engine_ms %.3f\n", ms);
#ifdef NB_ENGINE_DROPIN  // which flushes reached the GPU (filters, Merkle trees)
    std::fprintf(stderr, "device_builds %llu device_merkles %llu\n", nb_device_build_count(),
                 nb_device_merkle_count());
#endif
    return 0;
}
