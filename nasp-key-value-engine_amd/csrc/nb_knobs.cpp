// nb_knobs.cpp -- storage of the library's switches (nb_knobs.h) and their C ABI
// (nb_set_knob / nb_get_knob, include/nasp_bloom.h).  The only getenv of the
// library: each NB_* variable is read once, on first use.
#include "nb_knobs.h"

#include <atomic>
#include <cstdlib>
#include <cstring>

#include "../../include/nasp_bloom.h"

int nb_internal_fail(int code, const char *msg);  // bloom_kernels.hip: the error slot

namespace {

struct KnobDef {
    const char *name;
    uint64_t dflt;
};

constexpr KnobDef kDefs[nb::kKnobCount] = {
    {"NB_BUILD_PATH", 0},    {"NB_PACK", 1},        {"NB_TILE_BITS", 0},
    {"NB_SHARDS", 8},        {"NB_CHUNK_KEYS", 0},  {"NB_TWO_LEVEL", 1},
    {"NB_PACK5", 1},         {"NB_ENTRY32", 0},     {"NB_RANK", 1},
    {"NB_FIXED32", 1},       {"NB_FPMOD", 1},       {"NB_KEXACT", 1},
    {"NB_BIN_WIDE", 1},      {"NB_SHARDED_STAGE", 0},
    {"NB_OVERLAP", 6},       {"NB_SUBPASSES", 0},
    {"NB_TILE_COUNT", 0},
    {"NB_PROBE_PATH", 0},    {"NB_PROBE_CHUNK", 0}, {"NB_PROBE_TILED_PCT", 0},
    {"NB_PROBE_SPLIT_PCT", 0}, {"NB_PROBE_ENTRY", 0},
    {"NB_PROBE_BIN_GRID", 0}, {"NB_PROBE_HOST_PICK", 0},
    {"NB_PROBE_KPT", 0},
    {"NB_FAIL_BUILDS", 0},   {"NB_FAIL_MERKLES", 0},
};

// path knobs also take their names from the environment
uint64_t parse(int id, const char *s) {
    if (id == nb::kKnobBuildPath) {
        if (!std::strcmp(s, "atomic")) return 1;
        if (!std::strcmp(s, "tiled")) return 2;
        if (!std::strcmp(s, "auto")) return 0;
    }
    if (id == nb::kKnobProbePath) {
        if (!std::strcmp(s, "lane")) return 1;
        if (!std::strcmp(s, "tiled")) return 2;
        if (!std::strcmp(s, "split")) return 3;
        if (!std::strcmp(s, "auto")) return 0;
    }
    return std::strtoull(s, nullptr, 10);
}

struct Knobs {
    std::atomic<uint64_t> v[nb::kKnobCount];
    Knobs() {
        for (int i = 0; i < nb::kKnobCount; ++i) {
            const char *e = std::getenv(kDefs[i].name);
            v[i].store(e && *e ? parse(i, e) : kDefs[i].dflt, std::memory_order_relaxed);
        }
    }
};

Knobs &knobs() {
    static Knobs k;  // thread-safe one-time initialisation
    return k;
}

int find(const char *name) {
    if (!name) return -1;
    for (int i = 0; i < nb::kKnobCount; ++i)
        if (!std::strcmp(kDefs[i].name, name)) return i;
    return -1;
}

}  // namespace

namespace nb {

uint64_t knob(Knob k) { return knobs().v[k].load(std::memory_order_relaxed); }

bool knob_take(Knob k) {
    std::atomic<uint64_t> &a = knobs().v[k];
    uint64_t c = a.load(std::memory_order_relaxed);
    while (c && !a.compare_exchange_weak(c, c - 1, std::memory_order_relaxed)) {
    }
    return c != 0;
}

}  // namespace nb

extern "C" {

int nb_set_knob(const char *name, uint64_t value) {
    const int i = find(name);
    if (i < 0) return nb_internal_fail(NB_ERR_ARG, "unknown knob");
    knobs().v[i].store(value, std::memory_order_relaxed);
    return NB_OK;
}

int nb_get_knob(const char *name, uint64_t *value) {
    const int i = find(name);
    if (i < 0 || !value) return nb_internal_fail(NB_ERR_ARG, "unknown knob or NULL value");
    *value = knobs().v[i].load(std::memory_order_relaxed);
    return NB_OK;
}

}  // extern "C"
