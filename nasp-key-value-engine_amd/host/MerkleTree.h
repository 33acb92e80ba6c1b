// MerkleTree.h -- drop-in replacement for the reference class
// (reference MerkleTree/MerkleTree.h:10-36), backed by the MI355X Merkle kernels
// (nb_merkle, include/nasp_bloom.h).
//
// Same public surface and strings, so SSTable::build (SSTable/SSTable.cpp:37-42),
// SSTableRaw/SSTableComp's writers and validators (SSTableRaw.cpp:67,394-397,959;
// SSTableComp.cpp:325-327,838) compile unchanged:
//   - leaves are to_string(std::hash<std::string>(record)) (merkle.cpp:13-15,26-32);
//   - a parent is hash(left + right) of the children's decimal strings, the last
//     node of an odd level paired with itself (merkle.cpp:41-52);
//   - generateProof / verifyProof walk the levels exactly as merkle.cpp:57-102.
// What changes inside: the whole tree (every level) is computed in one call and
// kept as the hash values; strings are made when a caller asks for them.  A flush
// of at least hostRecordLimit() records (4 096) is built on the GPU (nb_merkle);
// a smaller one -- e.g. the reference's tiny-config flushes of two records -- on
// the host with the Merkle kernels' own hashing (nb_merkle_cpu), with no device
// call.  If the device build fails (no GPU, a device error) the tree is built on
// the host after one std::cerr line (once per process when there is no GPU), in
// the reference's error style (SSTableComp.cpp:543): the constructor throws only
// what the reference throws (no data).
#pragma once

// the reference header's includes are kept (its callers rely on them transitively)
#include <cstdint>
#include <functional>
#include <iomanip>
#include <sstream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

class MerkleTree {
private:
    std::vector<uint64_t> tree;      // every level's hashes, leaves first, root last
    std::vector<uint64_t> level_at;  // first node of each level in `tree`
    std::vector<uint64_t> level_n;   // nodes per level
    bool on_device = false;          // the tree was built on the GPU

    // MerkleTree::hash (merkle.cpp:26-32): decimal string of std::hash<std::string>
    static std::string hash(const std::string &data);

public:
    // builds the tree of `data` (merkle.cpp:7-19); std::invalid_argument on no data
    MerkleTree(const std::vector<std::string> &data);

    // the root's decimal hash (merkle.cpp:22-24)
    std::string getRootHash() const;

    // the leaves' decimal hashes (MerkleTree.h:28)
    std::vector<std::string> getLeaves() const;

    // sibling path of the first leaf equal to hash(data) (merkle.cpp:57-84)
    std::vector<std::pair<std::string, bool>> generateProof(const std::string &data) const;

    // recomputes the root along `proof` (merkle.cpp:86-102)
    static bool verifyProof(const std::string &rootHash, const std::string &data,
                            const std::vector<std::pair<std::string, bool>> &proof);

    // ---- extensions (not in the reference) ----
    // std::hash flavour (NB_FLAVOR_LIBSTDCXX default; NB_FLAVOR_MSVC_FNV1A for
    // trees written by the authors' Windows build) and device for new trees.
    static void setDefaultFlavor(int flavor);
    static void setDefaultDevice(int device);
    // Trees of fewer records than this are built on the host (default 4 096).
    static void setHostRecordLimit(uint64_t records);
    static uint64_t hostRecordLimit();
    bool builtOnDevice() const { return on_device; }
};
