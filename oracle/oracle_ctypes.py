"""ctypes bindings for the oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  The product path (nasp-key-value-engine_amd/) never does.

  Oracle  -> oracle/build/liboracle.so  : CPU restatement (bloom_oracle.c)
  RefLib  -> oracle/_ref/libref_bloom.so: the reference BloomFilter.cpp compiled here
  RefMerkle -> oracle/_ref/libref_merkle.so: the reference MerkleTree/merkle.cpp compiled here
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "build", "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref_bloom.so")
REF_MERKLE_SO = os.path.join(HERE, "_ref", "libref_merkle.so")

LIBSTDCXX = 0
MSVC_FNV1A = 1

_u8p = C.POINTER(C.c_uint8)
_u64p = C.POINTER(C.c_uint64)


def build_oracle(ref: bool | None = None) -> None:
    """Compile liboracle.so (and, when /root/reference exists, the _ref shim)."""
    subprocess.check_call(["make", "-s", "-C", HERE, "all"])
    if ref is None:
        ref = os.path.isdir("/root/reference/BloomFilter")
    if ref:
        subprocess.check_call(["make", "-s", "-C", HERE, "ref"])


def _ptr(a: np.ndarray | None, t=_u8p):
    if a is None:
        return None
    return a.ctypes.data_as(t)


def pack_keys(keys: list[bytes]) -> tuple[np.ndarray, np.ndarray]:
    """list of bytes -> (packed u8 buffer, u64 offsets[n+1])."""
    offs = np.zeros(len(keys) + 1, dtype=np.uint64)
    if keys:
        offs[1:] = np.cumsum([len(k) for k in keys], dtype=np.uint64)
    buf = np.frombuffer(b"".join(keys), dtype=np.uint8).copy() if keys else np.zeros(1, np.uint8)
    if buf.size == 0:
        buf = np.zeros(1, np.uint8)
    return buf, offs


class Oracle:
    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build_oracle(ref=False)
        lib = C.CDLL(path)
        lib.orc_hash.restype = C.c_uint64
        lib.orc_hash.argtypes = [C.c_int, _u8p, C.c_size_t]
        lib.orc_size_of_bitset.restype = C.c_uint32
        lib.orc_size_of_bitset.argtypes = [C.c_uint32, C.c_double]
        lib.orc_num_hashes.restype = C.c_uint32
        lib.orc_num_hashes.argtypes = [C.c_uint32, C.c_uint32]
        lib.orc_seed_from_time.restype = C.c_uint64
        lib.orc_seed_from_time.argtypes = [C.c_uint32]
        lib.orc_murmur3_x64_128.restype = None
        lib.orc_murmur3_x64_128.argtypes = [_u8p, C.c_size_t, C.c_uint32, _u64p]
        lib.orc_index.restype = C.c_uint32
        lib.orc_index.argtypes = [C.c_int, _u8p, C.c_size_t, C.c_uint32, C.c_uint32, C.c_uint64]
        lib.orc_build.restype = C.c_int
        lib.orc_build.argtypes = [C.c_int, _u8p, _u64p, C.c_uint32, C.c_uint64, C.c_uint32,
                                  C.c_uint32, C.c_uint64, _u64p]
        lib.orc_probe.restype = C.c_int
        lib.orc_probe.argtypes = [C.c_int, _u8p, _u64p, C.c_uint32, C.c_uint64, C.c_uint32,
                                  C.c_uint32, C.c_uint64, _u64p, _u8p]
        lib.orc_serialized_size.restype = C.c_size_t
        lib.orc_serialized_size.argtypes = [C.c_uint32]
        lib.orc_serialize.restype = C.c_size_t
        lib.orc_serialize.argtypes = [C.c_uint32, C.c_uint32, C.c_double, C.c_uint32,
                                      C.c_uint64, _u64p, _u8p]
        lib.orc_merkle.restype = C.c_uint64
        lib.orc_merkle.argtypes = [C.c_int, _u8p, _u64p, C.c_uint32, C.c_uint64, _u64p, _u64p]
        lib.orc_merkle_tree_size.restype = C.c_uint64
        lib.orc_merkle_tree_size.argtypes = [C.c_uint64]
        self.lib = lib

    def hash(self, flavor: int, key: bytes) -> int:
        a = np.frombuffer(key + b"\0", dtype=np.uint8)
        return self.lib.orc_hash(flavor, _ptr(a), len(key))

    def size_of_bitset(self, n: int, p: float) -> int:
        return self.lib.orc_size_of_bitset(n, p)

    def num_hashes(self, n: int, m: int) -> int:
        return self.lib.orc_num_hashes(n, m)

    def seed_from_time(self, tc: int) -> int:
        return self.lib.orc_seed_from_time(tc)

    def index(self, flavor: int, key: bytes, i: int, m: int, seed: int) -> int:
        a = np.frombuffer(key + b"\0", dtype=np.uint8)
        return self.lib.orc_index(flavor, _ptr(a), len(key), i, m, seed)

    def build(self, flavor, keys_u8, offsets, key_len, n, m, k, seed, words=None):
        if words is None:
            words = np.zeros((m + 63) // 64 or 1, dtype=np.uint64)
        rc = self.lib.orc_build(flavor, _ptr(keys_u8), _ptr(offsets, _u64p), key_len, n, m, k,
                                seed, _ptr(words, _u64p))
        if rc != 0:
            raise ValueError(f"orc_build rc={rc}")
        return words

    def probe(self, flavor, keys_u8, offsets, key_len, n, m, k, seed, words):
        out = np.zeros(max(n, 1), dtype=np.uint8)
        rc = self.lib.orc_probe(flavor, _ptr(keys_u8), _ptr(offsets, _u64p), key_len, n, m, k,
                                seed, _ptr(words, _u64p), _ptr(out))
        if rc != 0:
            raise ValueError(f"orc_probe rc={rc}")
        return out[:n]

    def serialize(self, m, k, p, tc, seed, words) -> bytes:
        out = np.zeros(self.lib.orc_serialized_size(m), dtype=np.uint8)
        n = self.lib.orc_serialize(m, k, p, tc, seed, _ptr(words, _u64p), _ptr(out))
        return out[:n].tobytes()

    def merkle(self, flavor, data_u8, offsets, rec_len, n, want_tree=False):
        """-> (root hash, leaf hashes[n], every level [tree size] or None)"""
        leaves = np.zeros(max(n, 1), dtype=np.uint64)
        tree = np.zeros(self.lib.orc_merkle_tree_size(n), dtype=np.uint64) if want_tree else None
        root = self.lib.orc_merkle(flavor, _ptr(data_u8), _ptr(offsets, _u64p), rec_len, n,
                                   _ptr(leaves, _u64p), _ptr(tree, _u64p))
        return int(root), leaves[:n], tree


def murmur3_x64_128(lib, data: bytes, seed: int, fn: str = "orc_murmur3_x64_128"):
    """(h1, h2) of MurmurHash3_x64_128 through the oracle (default) or the reference
    shim (lib = RefMurmur3().lib, fn = "ref_murmur3_x64_128")."""
    buf = np.frombuffer(data, dtype=np.uint8).copy() if data else np.zeros(1, np.uint8)
    out = np.zeros(2, dtype=np.uint64)
    getattr(lib, fn)(_ptr(buf), len(data), seed, _ptr(out, _u64p))
    return int(out[0]), int(out[1])


class RefMurmur3:
    """The reference MurmurHash3.cpp compiled here (oracle/_ref/libref_murmur3.so)."""

    def __init__(self, path: str = os.path.join(os.path.dirname(REF_SO), "libref_murmur3.so")):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.lib = C.CDLL(path)
        self.lib.ref_murmur3_x64_128.restype = None
        self.lib.ref_murmur3_x64_128.argtypes = [_u8p, C.c_int, C.c_uint32, _u64p]


class RefLib:
    """The reference BloomFilter.cpp compiled here (oracle/_ref)."""

    def __init__(self, path: str = REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        lib = C.CDLL(path)
        lib.ref_std_hash.restype = C.c_uint64
        lib.ref_std_hash.argtypes = [_u8p, C.c_uint64]
        lib.ref_ctor_params.restype = C.c_int
        lib.ref_ctor_params.argtypes = [C.c_uint32, C.c_double, C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_uint64)]
        lib.ref_size_of_bitset.restype = C.c_uint32
        lib.ref_size_of_bitset.argtypes = [C.c_uint32, C.c_double]
        lib.ref_num_hashes.restype = C.c_uint32
        lib.ref_num_hashes.argtypes = [C.c_uint32, C.c_uint32]
        lib.ref_build.restype = C.c_int
        lib.ref_build.argtypes = [_u8p, _u64p, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32,
                                  C.c_double, C.c_uint32, C.c_uint64, _u8p, _u8p]
        lib.ref_probe.restype = C.c_int
        lib.ref_probe.argtypes = [_u8p, C.c_uint64, _u8p, _u64p, C.c_uint32, C.c_uint64, _u8p]
        lib.ref_build_timed.restype = C.c_double
        lib.ref_build_timed.argtypes = [_u8p, _u64p, C.c_uint32, C.c_uint64, C.c_uint32,
                                        C.c_uint32, C.c_uint64, _u8p, C.c_uint64]
        lib.ref_default_contains.restype = C.c_int
        lib.ref_default_contains.argtypes = [_u8p, C.c_uint64]
        self.lib = lib

    def std_hash(self, key: bytes) -> int:
        a = np.frombuffer(key + b"\0", dtype=np.uint8)
        return self.lib.ref_std_hash(_ptr(a), len(key))

    def ctor_params(self, n: int, p: float):
        m, k, tc, seed = C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_uint64()
        self.lib.ref_ctor_params(n, p, C.byref(m), C.byref(k), C.byref(tc), C.byref(seed))
        return m.value, k.value, tc.value, seed.value

    def size_of_bitset(self, n, p):
        return self.lib.ref_size_of_bitset(n, p)

    def num_hashes(self, n, m):
        return self.lib.ref_num_hashes(n, m)

    def build(self, keys_u8, offsets, key_len, n, m, k, p, tc, seed, initial: bytes | None = None):
        size = 28 + ((m + 7) & 0xFFFFFFFF) // 8
        out = np.zeros(size, dtype=np.uint8)
        init = None
        if initial is not None:
            init = np.frombuffer(initial, dtype=np.uint8).copy()
        self.lib.ref_build(_ptr(keys_u8), _ptr(offsets, _u64p), key_len, n, m, k, p, tc, seed,
                           _ptr(init), _ptr(out))
        return out.tobytes()

    def build_timed(self, keys_u8, offsets, key_len, n, m, k, seed,
                    want_image: bool = True) -> tuple[float, bytes | None]:
        """Seconds spent in the reference add() loop, and the serialized image
        (skipped with want_image=False).  Releases the GIL while it runs."""
        if not want_image:
            secs = self.lib.ref_build_timed(_ptr(keys_u8), _ptr(offsets, _u64p), key_len, n, m, k,
                                            seed, None, 0)
            return secs, None
        size = 28 + ((m + 7) & 0xFFFFFFFF) // 8
        out = np.zeros(size, dtype=np.uint8)
        secs = self.lib.ref_build_timed(_ptr(keys_u8), _ptr(offsets, _u64p), key_len, n, m, k,
                                        seed, _ptr(out), size)
        return secs, out.tobytes()

    def probe(self, image: bytes, keys_u8, offsets, key_len, n):
        img = np.frombuffer(image, dtype=np.uint8).copy()
        out = np.zeros(max(n, 1), dtype=np.uint8)
        self.lib.ref_probe(_ptr(img), len(image), _ptr(keys_u8), _ptr(offsets, _u64p), key_len,
                           n, _ptr(out))
        return out[:n]

    def default_contains(self, key: bytes) -> bool:
        a = np.frombuffer(key + b"\0", dtype=np.uint8)
        return bool(self.lib.ref_default_contains(_ptr(a), len(key)))


class RefMerkle:
    """The reference MerkleTree/merkle.cpp compiled here (oracle/_ref)."""

    def __init__(self, path: str = REF_MERKLE_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        lib = C.CDLL(path)
        lib.ref_merkle.restype = C.c_int
        lib.ref_merkle.argtypes = [_u8p, _u64p, C.c_uint32, C.c_uint64, C.c_char_p, _u64p]
        lib.ref_merkle_timed.restype = C.c_double
        lib.ref_merkle_timed.argtypes = [_u8p, _u64p, C.c_uint32, C.c_uint64, C.c_char_p]
        lib.ref_merkle_proof.restype = C.c_int
        lib.ref_merkle_proof.argtypes = [_u8p, _u64p, C.c_uint32, C.c_uint64, C.c_uint64, _u64p,
                                         _u8p, C.c_int]
        lib.ref_merkle_verify.restype = C.c_int
        lib.ref_merkle_verify.argtypes = [C.c_char_p, _u8p, C.c_uint64, _u64p, _u8p, C.c_int]
        self.lib = lib

    def merkle(self, data_u8, offsets, rec_len, n):
        """-> (root string, leaf hashes[n])"""
        root = C.create_string_buffer(64)
        leaves = np.zeros(max(n, 1), dtype=np.uint64)
        rc = self.lib.ref_merkle(_ptr(data_u8), _ptr(offsets, _u64p), rec_len, n, root,
                                 _ptr(leaves, _u64p))
        if rc != 0:
            raise ValueError("reference MerkleTree threw")
        return root.value.decode(), leaves[:n]

    def merkle_timed(self, data_u8, offsets, rec_len, n):
        root = C.create_string_buffer(64)
        t = self.lib.ref_merkle_timed(_ptr(data_u8), _ptr(offsets, _u64p), rec_len, n, root)
        return t, root.value.decode()

    def proof(self, data_u8, offsets, rec_len, n, target):
        sib = np.zeros(64, dtype=np.uint64)
        right = np.zeros(64, dtype=np.uint8)
        np_ = self.lib.ref_merkle_proof(_ptr(data_u8), _ptr(offsets, _u64p), rec_len, n, target,
                                        _ptr(sib, _u64p), _ptr(right), 64)
        if np_ < 0:
            raise ValueError("reference generateProof threw")
        return [(int(sib[i]), bool(right[i])) for i in range(np_)]

    def verify(self, root: str, rec: bytes, proof) -> bool:
        a = np.frombuffer(rec + b"\0", dtype=np.uint8)
        sib = np.array([p[0] for p in proof] or [0], dtype=np.uint64)
        right = np.array([1 if p[1] else 0 for p in proof] or [0], dtype=np.uint8)
        return bool(self.lib.ref_merkle_verify(root.encode(), _ptr(a), len(rec), _ptr(sib, _u64p),
                                               _ptr(right), len(proof)))
