// MerkleTree.cpp -- the drop-in MerkleTree over the C ABI (include/nasp_bloom.h).
// See MerkleTree.h for the contract; reference behaviour cited per method.
#include "MerkleTree.h"

#include <atomic>
#include <cstring>
#include <iostream>
#include <mutex>

#include "../../include/nasp_bloom.h"

namespace {
int g_flavor = NB_FLAVOR_LIBSTDCXX;
int g_device = 0;
std::atomic<uint64_t> g_host_limit{4096};
std::once_flag g_nodev_note;

uint64_t std_hash(const std::string &s) {
    return nb_std_hash(reinterpret_cast<const uint8_t *>(s.data()), s.size(), g_flavor);
}
}  // namespace

void MerkleTree::setDefaultFlavor(int flavor) { g_flavor = flavor; }
void MerkleTree::setDefaultDevice(int device) { g_device = device; }
void MerkleTree::setHostRecordLimit(uint64_t records) { g_host_limit = records; }
uint64_t MerkleTree::hostRecordLimit() { return g_host_limit; }

// merkle.cpp:26-32
std::string MerkleTree::hash(const std::string &data) { return std::to_string(std_hash(data)); }

// merkle.cpp:7-19: leaves, then the levels (buildTree, merkle.cpp:34-55) -- on the
// GPU for a flush of at least hostRecordLimit() records, else (and whenever the
// device build fails) on the host with the kernels' own hashing (nb_merkle_cpu)
MerkleTree::MerkleTree(const std::vector<std::string> &data) {
    if (data.empty()) throw std::invalid_argument("Podaci za Merkle stablo ne smeju biti prazni.");
    const uint64_t n = data.size();
    std::vector<uint64_t> offs(n + 1, 0);
    for (uint64_t i = 0; i < n; ++i) offs[i + 1] = offs[i] + data[i].size();
    std::vector<uint8_t> bytes(offs[n] + 16, 0);
    for (uint64_t i = 0; i < n; ++i)
        if (!data[i].empty()) std::memcpy(bytes.data() + offs[i], data[i].data(), data[i].size());
    tree.assign(nb_merkle_tree_size(n), 0);
    uint64_t root = 0;
    int rc = NB_ERR_UNSUPPORTED;
    on_device = false;
    if (n >= g_host_limit) {
        rc = nb_merkle(bytes.data(), offs.data(), 0, n, g_flavor, tree.data(), nullptr, &root, g_device);
        if (rc == NB_ERR_NODEV) {
            std::call_once(g_nodev_note, [] {
                std::cerr << "[MerkleTree] GPU build failed (no HIP device visible); building "
                             "trees on the host\n";
            });
        } else if (rc != NB_OK) {  // the reference's error style (SSTableComp.cpp:543): report, carry on
            std::cerr << "[MerkleTree] GPU build failed (" << nb_last_error() << "); building " << n
                      << " records on the host\n";
        }
        on_device = rc == NB_OK;
    }
    if (rc != NB_OK &&
        nb_merkle_cpu(bytes.data(), offs.data(), 0, n, g_flavor, tree.data(), nullptr, &root) != NB_OK)
        throw std::runtime_error(std::string("nasp_bloom: nb_merkle_cpu failed: ") + nb_last_error());
    for (uint64_t at = 0, c = n;; c = (c + 1) / 2) {
        level_at.push_back(at);
        level_n.push_back(c);
        at += c;
        if (c == 1) break;
    }
}

std::string MerkleTree::getRootHash() const { return std::to_string(tree.back()); }

std::vector<std::string> MerkleTree::getLeaves() const {
    std::vector<std::string> out;
    out.reserve(level_n[0]);
    for (uint64_t i = 0; i < level_n[0]; ++i) out.push_back(std::to_string(tree[i]));
    return out;
}

// merkle.cpp:57-84: the first leaf equal to hash(data), then its siblings upward
std::vector<std::pair<std::string, bool>> MerkleTree::generateProof(const std::string &data) const {
    const uint64_t h = std_hash(data);
    uint64_t index = 0;
    while (index < level_n[0] && tree[index] != h) ++index;
    if (index == level_n[0]) throw std::invalid_argument("Podatak nije pronadjen u Merkle stablu.");
    std::vector<std::pair<std::string, bool>> proof;
    for (size_t level = 0; level + 1 < level_n.size(); ++level) {
        const bool isRight = index % 2 == 1;
        const uint64_t sibling = isRight ? index - 1 : index + 1;
        if (sibling < level_n[level])
            proof.push_back({std::to_string(tree[level_at[level] + sibling]), isRight});
        index /= 2;
    }
    return proof;
}

// merkle.cpp:86-102
bool MerkleTree::verifyProof(const std::string &rootHash, const std::string &data,
                             const std::vector<std::pair<std::string, bool>> &proof) {
    std::string computedHash = hash(data);
    for (const auto &pair : proof)
        computedHash = pair.second ? hash(pair.first + computedHash) : hash(computedHash + pair.first);
    return computedHash == rootHash;
}
