"""Merkle path without a GPU: the oracle's restatement (oracle/bloom_oracle.c
orc_merkle) and the library's host std::hash (nb_std_hash) against the golden
vectors made by the REAL reference MerkleTree (tests/golden/gen_merkle_golden.py),
the Python mirror's proof logic on oracle trees, and the tree-size formula."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from merkle_records import record_set


@pytest.fixture(scope="module")
def mg():
    return json.load(open(os.path.join(GOLDEN, "merkle_vectors.json")))


def test_oracle_merkle_matches_reference(oracle, mg):
    for t in mg["trees"]:
        buf, offs = record_set(t["recipe"], t["n"])
        root, leaves, tree = oracle.merkle(0, buf, offs, 0, t["n"], want_tree=True)
        assert str(root) == t["root"], (t["recipe"], t["n"])
        assert int(tree[-1]) == root
        if "leaves" in t:
            assert [str(int(x)) for x in leaves] == t["leaves"]


def test_oracle_proofs_match_reference(oracle, mg):
    """generateProof (merkle.cpp:57-84) walked over the oracle's levels."""
    for t in mg["trees"]:
        if "proofs" not in t:
            continue
        n = t["n"]
        buf, offs = record_set(t["recipe"], n)
        _, _, tree = oracle.merkle(0, buf, offs, 0, n, want_tree=True)
        levels, at, c = [], 0, n
        while True:
            levels.append((at, c))
            at += c
            if c == 1:
                break
            c = (c + 1) // 2
        for p in t["proofs"]:
            data = bytes(buf[int(offs[p["target"]]):int(offs[p["target"] + 1])])
            h = oracle.hash(0, data)
            index = int(np.nonzero(tree[:n] == np.uint64(h))[0][0])
            proof = []
            for lat, cnt in levels[:-1]:
                right = index % 2 == 1
                sib = index - 1 if right else index + 1
                if sib < cnt:
                    proof.append([str(int(tree[lat + sib])), right])
                index //= 2
            assert proof == p["proof"], (t["recipe"], n, p["target"])


def test_host_std_hash_matches_reference(built, oracle, mg):
    import nasp_bloom as nbm
    for h in mg["std_hash"]:
        assert str(nbm.std_hash(bytes.fromhex(h["hex"]))) == h["hash"]
    rng = np.random.default_rng(7)
    for _ in range(2000):
        s = rng.integers(0, 256, int(rng.integers(0, 90)), dtype=np.uint8).tobytes()
        for fl in (0, 1):
            assert nbm.std_hash(s, fl) == oracle.hash(fl, s)


def test_verify_proof_mirror(built, mg):
    """MerkleTree.verifyProof (merkle.cpp:86-102) is host logic: golden proofs verify,
    tampered data does not -- the reference's own answers."""
    import nasp_bloom as nbm
    for t in mg["trees"]:
        buf, offs = record_set(t["recipe"], t["n"])
        for p in t.get("proofs", []):
            data = bytes(buf[int(offs[p["target"]]):int(offs[p["target"] + 1])])
            proof = [(s, r) for s, r in p["proof"]]
            assert nbm.MerkleTree.verifyProof(t["root"], data, proof) == p["verifies"]
            assert nbm.MerkleTree.verifyProof(t["root"], data + b"x", proof) == p["tampered_verifies"]


def test_tree_size(built, oracle):
    import nasp_bloom as nbm
    for n in (1, 2, 3, 4, 5, 2047, 2048, 2049, 10**7):
        assert nbm.merkle_tree_size(n) == oracle.lib.orc_merkle_tree_size(n)
