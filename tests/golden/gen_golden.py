#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (run in the build container).

Sources of truth:
  * msvc_filters.json   -- the six serialized filters committed in the reference
    (`NASP key-value-engine/level_0/filter_{0..4}.sst`,
    `NASP key-value-engine/data/level_0/filter_0.sst`), written by the authors'
    MSVC build (std::hash = FNV-1a).  Their keys are "test" and "test2"
    (`level_0/sstable_N.sst`, `index_N.sst`).  Stored as data (hex), not source.
  * libstdcxx_vectors.json -- outputs of the REAL reference BloomFilter.cpp
    compiled here with GCC 11.4 (oracle/_ref/libref_bloom.so, recipe
    oracle/Makefile `ref`): serialized images, probe answers, m/k formulas and
    set-bit positions for large m.

Needs /root/reference (build container only); the GPU box only reads the JSON.
"""
from __future__ import annotations

import glob
import json
import os
import random
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
from oracle_ctypes import RefLib, build_oracle, pack_keys  # noqa: E402

REF_ROOT = "/root/reference/NASP key-value-engine"
SEED = 17027509906831645879  # h2_seed of level_0/filter_0.sst
TC = 1748963255              # its timeConst


def msvc_filters():
    out = []
    files = sorted(glob.glob(os.path.join(REF_ROOT, "level_0", "filter_*.sst")))
    files.append(os.path.join(REF_ROOT, "data", "level_0", "filter_0.sst"))
    for f in files:
        raw = open(f, "rb").read()
        out.append({
            "file": os.path.relpath(f, os.path.dirname(REF_ROOT)),
            "framing": "u64 length prefix (SSTableRaw legacy *.sst)",
            "bytes_hex": raw.hex(),
            "keys_hex": [b"test".hex(), b"test2".hex()],
            "flavor": "msvc_fnv1a",
        })
    return out


def set_bits(bits_bytes: bytes) -> list[int]:
    bits = np.unpackbits(np.frombuffer(bits_bytes, dtype=np.uint8), bitorder="little")
    return np.nonzero(bits)[0].tolist()


def image_record(img: bytes) -> dict:
    """Serialized image as header hex + sorted set-bit positions (compact for big m)."""
    return {"header_hex": img[:28].hex(), "image_len": len(img), "bits": set_bits(img[28:])}


def rand_keys(rng, n, lo, hi):
    return [bytes(rng.randrange(256) for _ in range(rng.randrange(lo, hi + 1))) for _ in range(n)]


def main():
    build_oracle(ref=True)
    ref = RefLib()
    rng = random.Random(0x5EED)

    cases = []
    # edge-case key sets
    edge = [b"", b"\0", b"\0\0\0\0\0\0\0\0", b"a", b"test", b"test2", b"Ana", b"Marko",
            b"a\0b", bytes(range(256))[:80]]
    edge += [bytes([0x41 + (i % 26)] * L) for i, L in enumerate(range(1, 81))]
    key_sets = {
        "edge": edge,
        "fixed16": [rng.randbytes(16) for _ in range(200)],
        "var8_64": rand_keys(rng, 200, 8, 64),
        "ascii_sorted": [b"user%012d" % i for i in range(150)],
        "var0_80": rand_keys(rng, 120, 0, 80),
    }
    ms = [1, 7, 20, 64, 65, 47926, 1000003, 95850584 // 1000]
    ks = [1, 3, 7, 10]
    seeds = [(SEED, TC), (0, 0), (5, 5), (18446744073709551615, 1)]
    for name, keys in key_sets.items():
        for mi, m in enumerate(ms):
            for k in (ks[mi % 4], ks[(mi + 2) % 4]):
                seed, tc = seeds[rng.randrange(len(seeds))]
                buf, offs = pack_keys(keys)
                img = ref.build(buf, offs, 0, len(keys), m, k, 0.01, tc, seed)
                cases.append({"keys": name, "m": m, "k": k, "p": 0.01, "time_const": tc,
                              "seed": str(seed), **image_record(img)})

    # probe answers: filter from half of the keys, probe all + absent keys
    probes = []
    for name in ("fixed16", "var8_64", "edge"):
        keys = key_sets[name]
        ins = keys[::2]
        q = keys + rand_keys(rng, 100, 0, 40)
        for m, k in ((47926, 3), (2000, 7), (64, 10)):
            bi, oi = pack_keys(ins)
            img = ref.build(bi, oi, 0, len(ins), m, k, 0.1, TC, SEED)
            bq, oq = pack_keys(q)
            ans = ref.probe(img, bq, oq, 0, len(q))
            probes.append({"keys": name, "inserted": "even", "m": m, "k": k,
                           **image_record(img), "query_hex": [x.hex() for x in q],
                           "answer": ans.tolist()})

    # accumulate: add keys2 into a deserialized filter (TypesManager.cpp:84-86)
    accum = []
    for m, k in ((47926, 3), (1000003, 7)):
        k1, k2 = key_sets["var8_64"][:100], key_sets["var8_64"][100:]
        b1, o1 = pack_keys(k1)
        img1 = ref.build(b1, o1, 0, len(k1), m, k, 0.01, TC, SEED)
        b2, o2 = pack_keys(k2)
        img2 = ref.build(b2, o2, 0, len(k2), m, k, 0.01, TC, SEED, initial=img1)
        accum.append({"m": m, "k": k, "first": image_record(img1), "final": image_record(img2)})

    # m / k formulas (BloomFilter.cpp:192-199), including the 32-bit wrap
    formulas = []
    for n in [1, 2, 3, 10, 20, 100, 1000, 10000, 12345, 10**6, 10**7, 10**8, 10**9, 2**32 - 1]:
        for p in [0.5, 0.1, 0.05, 0.01, 0.001, 1e-6]:
            m = ref.size_of_bitset(n, p)
            formulas.append({"n": n, "p": p, "m": m, "k": ref.num_hashes(n, m) if m else None})

    # set-bit positions for large m (single key per filter; m up to 2^32-8, the
    # largest m the reference's serialize() can represent)
    big = []
    for m in (2**31 + 11, 3000000019, 2**32 - 8):
        for key in (b"", b"test", rng.randbytes(16), rng.randbytes(37)):
            for k in (7, 10):
                buf, offs = pack_keys([key])
                img = ref.build(buf, offs, 0, 1, m, k, 0.01, TC, SEED)
                pos = set_bits(img[28:])
                big.append({"m": m, "k": k, "seed": str(SEED), "key_hex": key.hex(),
                            "bits": pos, "image_len": len(img)})

    json.dump({"generator": "tests/golden/gen_golden.py", "flavor": "libstdcxx (GCC 11.4.0)",
               "key_sets": {k: [x.hex() for x in v] for k, v in key_sets.items()},
               "build_cases": cases, "probe_cases": probes, "accumulate_cases": accum,
               "formulas": formulas, "large_m": big},
              open(os.path.join(HERE, "libstdcxx_vectors.json"), "w"))
    json.dump({"generator": "tests/golden/gen_golden.py", "filters": msvc_filters()},
              open(os.path.join(HERE, "msvc_filters.json"), "w"), indent=1)
    print("wrote", len(cases), "build cases,", len(probes), "probe cases,", len(big), "large-m cases")


if __name__ == "__main__":
    main()
