// ref_murmur3_harness.cpp -- extern "C" shim around the REAL reference
// MurmurHash3_x64_128 (/root/reference/MurmurHash3/MurmurHash3.cpp:255-332),
// compiled where it lies (recipe: oracle/Makefile target `ref`; output only into
// oracle/_ref/).  TEST INFRASTRUCTURE ONLY: pins the oracle's restatement of the
// non-parity NB_FLAVOR_MURMUR3_X64_128 (tests/golden/gen_murmur3_golden.py).
#include <cstdint>

#include "MurmurHash3.h"

extern "C" void ref_murmur3_x64_128(const void *key, int len, uint32_t seed, uint64_t *out) {
    MurmurHash3_x64_128(key, len, seed, out);
}
