#!/usr/bin/env python3
"""Generate tests/golden/murmur3_vectors.json from the REAL reference
MurmurHash3_x64_128 (/root/reference/MurmurHash3/MurmurHash3.cpp:255-332) compiled
here by oracle/Makefile `ref` (oracle/_ref/libref_murmur3.so).  Pins the oracle's
restatement behind the non-parity NB_FLAVOR_MURMUR3_X64_128.  Build container only.
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
from oracle_ctypes import RefMurmur3, murmur3_x64_128  # noqa: E402


def main():
    ref = RefMurmur3()
    rng = random.Random(3)
    cases = []
    for seed in (0, 1, 0x9747B28C, 0xFFFFFFFF, 17027509906831645879 & 0xFFFFFFFF):
        for n in list(range(0, 50)) + [63, 64, 65, 100, 255]:
            data = bytes(rng.randrange(256) for _ in range(n))
            h1, h2 = murmur3_x64_128(ref.lib, data, seed, "ref_murmur3_x64_128")
            cases.append({"key": data.hex(), "seed": seed, "h1": str(h1), "h2": str(h2)})
    out = {"generator": "tests/golden/gen_murmur3_golden.py",
           "source": "reference MurmurHash3/MurmurHash3.cpp:255-332 compiled by oracle/Makefile ref",
           "cases": cases}
    json.dump(out, open(os.path.join(HERE, "murmur3_vectors.json"), "w"), indent=0)
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
