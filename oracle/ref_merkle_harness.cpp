// ref_merkle_harness.cpp -- extern "C" shim around the REAL reference MerkleTree,
// compiled from /root/reference/MerkleTree/merkle.cpp where it lies (recipe:
// oracle/Makefile target `ref`; output only into oracle/_ref/).
//
// TEST INFRASTRUCTURE ONLY: pins the oracle's Merkle restatement, generates the
// golden Merkle vectors (tests/golden/gen_golden.py) and is bench.py's Merkle
// cpu_baseline.  This file is our own code; no reference source is copied.
//
// Records go into MerkleTree(const std::vector<std::string>&) exactly as
// SSTable::build (SSTable/SSTable.cpp:29-40) and SSTableRaw::writeDataMetaFiles
// (SSTableRaw.cpp:238,392-397) build them.
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "MerkleTree.h"

namespace {

std::vector<std::string> records(const uint8_t *data, const uint64_t *offs, uint32_t rec_len,
                                 uint64_t n) {
    std::vector<std::string> v;
    v.reserve(n);
    for (uint64_t i = 0; i < n; ++i) {
        const char *p = reinterpret_cast<const char *>(data);
        if (offs) v.emplace_back(p + offs[i], offs[i + 1] - offs[i]);
        else v.emplace_back(p + i * (uint64_t)rec_len, rec_len);
    }
    return v;
}

}  // namespace

extern "C" {

// Root (decimal string, NUL-terminated, <= 63 chars) and the leaves parsed back to
// their size_t hashes.  Returns 0, or -1 if the reference threw (n == 0).
int ref_merkle(const uint8_t *data, const uint64_t *offs, uint32_t rec_len, uint64_t n,
               char *root_out, uint64_t *leaves_out) {
    try {
        MerkleTree t(records(data, offs, rec_len, n));
        const std::string root = t.getRootHash();
        std::strncpy(root_out, root.c_str(), 63);
        root_out[63] = 0;
        if (leaves_out) {
            const std::vector<std::string> lv = t.getLeaves();
            for (size_t i = 0; i < lv.size(); ++i) leaves_out[i] = std::strtoull(lv[i].c_str(), nullptr, 10);
        }
        return 0;
    } catch (...) {
        return -1;
    }
}

// Seconds spent in the MerkleTree constructor alone (records already built).
double ref_merkle_timed(const uint8_t *data, const uint64_t *offs, uint32_t rec_len, uint64_t n,
                        char *root_out) {
    const std::vector<std::string> v = records(data, offs, rec_len, n);
    const auto t0 = std::chrono::steady_clock::now();
    MerkleTree t(v);
    const auto t1 = std::chrono::steady_clock::now();
    std::strncpy(root_out, t.getRootHash().c_str(), 63);
    root_out[63] = 0;
    return std::chrono::duration<double>(t1 - t0).count();
}

// generateProof(record `target`) (merkle.cpp:57-84): siblings parsed to hashes,
// is_right flags; returns the proof length, or -1 if the reference threw.
int ref_merkle_proof(const uint8_t *data, const uint64_t *offs, uint32_t rec_len, uint64_t n,
                     uint64_t target, uint64_t *siblings, uint8_t *is_right, int cap) {
    try {
        const std::vector<std::string> v = records(data, offs, rec_len, n);
        MerkleTree t(v);
        const auto proof = t.generateProof(v[target]);
        int i = 0;
        for (const auto &pr : proof) {
            if (i >= cap) break;
            siblings[i] = std::strtoull(pr.first.c_str(), nullptr, 10);
            is_right[i] = pr.second ? 1 : 0;
            ++i;
        }
        return i;
    } catch (...) {
        return -1;
    }
}

// verifyProof (merkle.cpp:86-102) of `data` against a root string.
int ref_merkle_verify(const char *root, const uint8_t *rec, uint64_t len, const uint64_t *siblings,
                      const uint8_t *is_right, int np) {
    std::vector<std::pair<std::string, bool>> proof;
    for (int i = 0; i < np; ++i) proof.push_back({std::to_string(siblings[i]), is_right[i] != 0});
    return MerkleTree::verifyProof(root, std::string(reinterpret_cast<const char *>(rec), len), proof)
               ? 1
               : 0;
}

}  // extern "C"
