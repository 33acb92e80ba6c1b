"""Deterministic Merkle record sets shared by the golden generator
(tests/golden/gen_merkle_golden.py) and the tests, so the fixture stores only
what the reference computed.

  podatak: the reference's own MerkleTree/main.cpp data ("Podatak1".."Podatak4")
  engine : key ++ value as SSTableRaw::writeDataMetaFiles builds them
           (SSTableRaw.cpp:238; keys/values as oracle/ref_engine_harness.cpp writes)
  random : nasp_bloom.synth.var_keys(n, 0, 60, seed=n) -- 0..60 random bytes
"""
import numpy as np


def pack(recs):
    offs = np.zeros(len(recs) + 1, dtype=np.uint64)
    if recs:
        offs[1:] = np.cumsum([len(r) for r in recs], dtype=np.uint64)
    buf = np.frombuffer(b"".join(recs) + b"\0" * 16, dtype=np.uint8).copy()
    return buf, offs


def record_set(recipe, n):
    if recipe == "podatak":
        return pack([b"Podatak%d" % (i + 1) for i in range(n)])
    if recipe == "engine":
        return pack([b"user%012d" % i + b"value-%d" % i for i in range(n)])
    if recipe == "random":
        from nasp_bloom import synth
        return synth.var_keys(n, 0, 60, seed=n)
    raise ValueError(recipe)
