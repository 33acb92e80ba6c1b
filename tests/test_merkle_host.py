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


def test_merkle_cpu_matches_reference(built, oracle, mg):
    """nb_merkle_cpu (the drop-in MerkleTree's host path: small flushes, no GPU) --
    the product's own hashing (bloom_math.h), checked against the REAL reference's
    roots and leaves and against the oracle's every level, both flavours."""
    import nasp_bloom as nbm
    for t in mg["trees"]:
        buf, offs = record_set(t["recipe"], t["n"])
        root, tree = nbm.merkle_cpu(buf, offs, 0, t["n"])
        assert str(root) == t["root"], (t["recipe"], t["n"])
        if "leaves" in t:
            assert [str(int(x)) for x in tree[:t["n"]]] == t["leaves"]
        for fl in (0, 1):
            r, _, want = oracle.merkle(fl, buf, offs, 0, t["n"], want_tree=True)
            r2, got = nbm.merkle_cpu(buf, offs, 0, t["n"], fl)
            assert r2 == r
            np.testing.assert_array_equal(got, want)


def test_merkle_cpu_reads_only_record_bytes(built, oracle):
    """Records at every misalignment in a buffer with no slack: the host path reads
    the record bytes only (the byte-safe word loader), fixed and variable layout."""
    import nasp_bloom as nbm
    rng = np.random.default_rng(3)
    for shift in range(8):
        n, rl = 37, 13
        raw = rng.integers(0, 256, shift + n * rl, dtype=np.uint8)
        data = raw[shift:]  # a view: starts at a misaligned address, ends at the allocation
        r, tree = nbm.merkle_cpu(data, None, rl, n)
        ro, _, want = oracle.merkle(0, np.concatenate([data, np.zeros(16, np.uint8)]), None, rl, n,
                                    want_tree=True)
        assert r == ro
        np.testing.assert_array_equal(tree, want)


def test_merkle_mirror_small_tree_on_host(built, mg):
    """The Python MerkleTree mirror builds small trees on the host (no device call)."""
    import nasp_bloom as nbm
    t = next(t for t in mg["trees"] if t["n"] < nbm.MerkleTree.HOST_RECORD_LIMIT and "leaves" in t)
    buf, offs = record_set(t["recipe"], t["n"])
    recs = [bytes(buf[int(offs[i]):int(offs[i + 1])]) for i in range(t["n"])]
    before = nbm.device_merkle_count()
    tree = nbm.MerkleTree(recs)
    assert tree.getRootHash() == t["root"] and tree.getLeaves() == t["leaves"]
    assert not tree.on_device and nbm.device_merkle_count() == before


def test_merkle_errors_without_device(built):
    import nasp_bloom as nbm
    with pytest.raises(nbm.NaspBloomError):
        nbm.merkle_cpu(np.zeros(4, np.uint8), None, 4, 0)  # no records: the reference throws
    with pytest.raises(nbm.NaspBloomError):
        nbm.merkle_cpu(np.zeros(4, np.uint8), None, 4, 1, 2)  # Merkle stays a std::hash flavour


def test_merkle_dropin_cxx_without_gpu(tmp_path, built):
    """The C++ drop-in MerkleTree program (tests/cpp/test_merkle_dropin.cpp) with no
    device visible: every tree built on the host (nb_merkle_cpu), one note per
    process on stderr, every string equal to the oracle's."""
    import subprocess
    from test_gpu_merkle import build_merkle_dropin
    exe = build_merkle_dropin(tmp_path)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="")
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "devices: 0" in out.stdout and "merkle drop-in OK" in out.stdout
    assert out.stderr.count("[MerkleTree] GPU build failed (no HIP device visible)") == 1
