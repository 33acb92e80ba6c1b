"""Python surface over the C ABI.

Device entry points take torch tensors that already live on the GPU (the
device-resident hot path); host entry points take numpy arrays.  The
`BloomFilter` class mirrors the reference class (BloomFilter/BloomFilter.h:24-41)
with the same names, argument meaning and semantics:
  - default-constructed filter: possiblyContains() is True (BloomFilter.cpp:26,67-80)
  - add() after deserialize() ORs into the existing bits (TypesManager.cpp:84-86)
  - serialize() is byte-identical to the reference image (BloomFilter.cpp:88-129)
Adds are batched inside the object and built on the GPU when the filter is read.
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np

from ._lib import BUILD_OVERWRITE, FLAVOR_LIBSTDCXX, NaspBloomError, check, lib


def nwords(m: int) -> int:
    """u64 words holding m bits (the device/host filter layout)."""
    return (int(m) + 63) // 64


def size_of_bitset(n: int, p: float) -> int:
    return int(lib().nb_size_of_bitset(n, p))


def num_hashes(n: int, m: int) -> int:
    return int(lib().nb_num_hashes(n, m))


def seed_from_time(time_const: int) -> int:
    return int(lib().nb_seed_from_time(time_const))


def std_hash(data: bytes, flavor: int = FLAVOR_LIBSTDCXX) -> int:
    """std::hash<std::string> of the flavour (host function of the library)."""
    return int(lib().nb_std_hash(data, len(data), flavor))


# named values of the path knobs (include/nasp_bloom.h nb_set_knob)
_KNOB_NAMES = {"NB_BUILD_PATH": {"auto": 0, "atomic": 1, "tiled": 2},
               "NB_PROBE_PATH": {"auto": 0, "lane": 1, "tiled": 2, "split": 3}}


def set_knob(name: str, value) -> None:
    """nb_set_knob: one of the library's A/B / fault-injection switches, for the
    whole process (thread-safe; the environment is read only once, at first use)."""
    if isinstance(value, str):
        value = _KNOB_NAMES.get(name, {}).get(value, None) if not value.isdigit() else int(value)
        if value is None:
            raise NaspBloomError(f"bad value for knob {name}")
    check(lib().nb_set_knob(name.encode(), int(value)), f"nb_set_knob({name})")


def get_knob(name: str) -> int:
    v = C.c_uint64()
    check(lib().nb_get_knob(name.encode(), C.byref(v)), f"nb_get_knob({name})")
    return int(v.value)


class knobs:
    """Context manager: set knobs for a block, restore the previous values after
    (`with knobs(NB_BUILD_PATH="tiled", NB_CHUNK_KEYS=70000): ...`)."""

    def __init__(self, **kv):
        self.kv = kv
        self.saved = {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.saved.setdefault(k, get_knob(k))
            set_knob(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.saved.items():
            set_knob(k, v)


def _stream_handle(stream) -> int | None:
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    return getattr(stream, "cuda_stream", stream)


def _check_device_args(keys, offsets, words, key_len=0, n=0):
    """Host-side shape checks before a kernel reads the tensors (no device sync:
    the last offset itself is the caller's contract)."""
    if not keys.is_cuda or not words.is_cuda:
        raise NaspBloomError("device entry points need CUDA (HIP) tensors")
    if offsets is not None and not offsets.is_cuda:
        raise NaspBloomError("offsets must be on the device")
    if not words.is_contiguous() or not keys.is_contiguous():
        raise NaspBloomError("keys and words must be contiguous")
    if offsets is None:
        if keys.numel() * keys.element_size() < n * key_len:
            raise NaspBloomError(f"keys tensor holds fewer than n * key_len = {n * key_len} bytes")
    elif n:
        if offsets.element_size() != 8 or not offsets.is_contiguous():
            raise NaspBloomError("offsets must be a contiguous 64-bit tensor")
        if offsets.numel() < n + 1:
            raise NaspBloomError(f"offsets tensor needs n + 1 = {n + 1} entries")


def build_device(keys, offsets, key_len: int, n: int, m: int, k: int, seed: int, flavor: int,
                 words, stream=None, overwrite: bool = False) -> None:
    """OR the k bits of n device-resident keys into `words` (int64/uint64 cuda tensor);
    with overwrite=True, `words` becomes the filter of this batch alone."""
    _check_device_args(keys, offsets, words, key_len, n)
    if words.numel() * words.element_size() < nwords(m) * 8:
        raise NaspBloomError("words tensor smaller than ceil(m/64) u64 words")
    rc = lib().nb_build_device_ex(keys.data_ptr(),
                                  offsets.data_ptr() if offsets is not None else None,
                                  key_len, n, m, k, seed, flavor, words.data_ptr(),
                                  BUILD_OVERWRITE if overwrite else 0, _stream_handle(stream))
    check(rc, "nb_build_device_ex")


def probe_device(keys, offsets, key_len: int, n: int, m: int, k: int, seed: int, flavor: int,
                 words, out, stream=None) -> None:
    """out[i] (uint8 cuda tensor) = 1 if all k bits of key i are set."""
    _check_device_args(keys, offsets, words, key_len, n)
    if k and words.numel() * words.element_size() < nwords(m) * 8:
        raise NaspBloomError("words tensor smaller than ceil(m/64) u64 words")
    if not out.is_cuda or out.numel() * out.element_size() < n:
        raise NaspBloomError("out must be a device tensor of at least n bytes")
    rc = lib().nb_probe_device(keys.data_ptr(), offsets.data_ptr() if offsets is not None else None,
                               key_len, n, m, k, seed, flavor, words.data_ptr(), out.data_ptr(),
                               _stream_handle(stream))
    check(rc, "nb_probe_device")


def or_merge_device(dst, src, nwords_: int, nsrc: int, src_stride: int, stream=None) -> None:
    rc = lib().nb_or_merge_device(dst.data_ptr(), src.data_ptr(), nwords_, nsrc, src_stride,
                                  _stream_handle(stream))
    check(rc, "nb_or_merge_device")


def _np_ptr(a):
    return None if a is None else a.ctypes.data


def build_host(keys: np.ndarray, offsets: np.ndarray | None, key_len: int, n: int, m: int, k: int,
               seed: int, flavor: int, words: np.ndarray, device: int = 0) -> None:
    """Host buffers in, host words OR-accumulated out (H2D + kernel + D2H)."""
    assert words.dtype == np.uint64 and words.flags.c_contiguous
    rc = lib().nb_build(_np_ptr(keys), _np_ptr(offsets), key_len, n, m, k, seed, flavor,
                        _np_ptr(words), device)
    check(rc, "nb_build")


def build_cpu(keys: np.ndarray, offsets: np.ndarray | None, key_len: int, n: int, m: int, k: int,
              seed: int, flavor: int, words: np.ndarray) -> None:
    """nb_build_cpu: the same build on the calling CPU thread (the drop-in classes'
    small-batch / no-device path); keys need the aligned-word slack
    the packers here add."""
    assert words.dtype == np.uint64 and words.flags.c_contiguous
    rc = lib().nb_build_cpu(_np_ptr(keys), _np_ptr(offsets), key_len, n, m, k, seed, flavor,
                            _np_ptr(words))
    check(rc, "nb_build_cpu")


def probe_cpu(keys: np.ndarray, offsets: np.ndarray | None, key_len: int, n: int, m: int, k: int,
              seed: int, flavor: int, words: np.ndarray) -> np.ndarray:
    """nb_probe_cpu: possiblyContains for a (small) batch on the calling CPU thread."""
    out = np.zeros(max(n, 1), dtype=np.uint8)
    rc = lib().nb_probe_cpu(_np_ptr(keys), _np_ptr(offsets), key_len, n, m, k, seed, flavor,
                            _np_ptr(words), _np_ptr(out))
    check(rc, "nb_probe_cpu")
    return out[:n]


def device_build_count() -> int:
    """Device builds this process has enqueued (nb_device_build_count)."""
    return int(lib().nb_device_build_count())


def device_merkle_count() -> int:
    """Device Merkle trees this process has built (nb_device_merkle_count)."""
    return int(lib().nb_device_merkle_count())


def build_host_sharded(keys: np.ndarray, offsets: np.ndarray | None, key_len: int, n: int, m: int,
                       k: int, seed: int, flavor: int, words: np.ndarray, nshards: int = 0) -> None:
    """nb_build over `nshards` key ranges (0: one per visible device), shard s on
    device s % device_count, partials OR-merged over xGMI into the host words."""
    assert words.dtype == np.uint64 and words.flags.c_contiguous
    rc = lib().nb_build_sharded(_np_ptr(keys), _np_ptr(offsets), key_len, n, m, k, seed, flavor,
                                _np_ptr(words), nshards)
    check(rc, "nb_build_sharded")


def probe_host(keys: np.ndarray, offsets: np.ndarray | None, key_len: int, n: int, m: int, k: int,
               seed: int, flavor: int, words: np.ndarray, device: int = 0) -> np.ndarray:
    out = np.zeros(max(n, 1), dtype=np.uint8)
    rc = lib().nb_probe(_np_ptr(keys), _np_ptr(offsets), key_len, n, m, k, seed, flavor,
                        _np_ptr(words), _np_ptr(out), device)
    check(rc, "nb_probe")
    return out[:n]


class Builder:
    """Streaming host builder (nb_builder_*): keys packed into pinned chunks whose
    upload and device build overlap further packing; finish() returns the filter
    words.  init_words: host words the keys OR into (None = a fresh filter)."""

    def __init__(self, m: int, k: int, seed: int, flavor: int = FLAVOR_LIBSTDCXX,
                 init_words: np.ndarray | None = None, device: int = 0):
        self.m = m
        self._h = C.c_void_p()
        if init_words is not None:
            assert init_words.dtype == np.uint64 and init_words.size >= nwords(m)
        check(lib().nb_builder_create(m, k, seed, flavor, _np_ptr(init_words), device,
                                      C.byref(self._h)), "nb_builder_create")

    def add(self, key: bytes) -> None:
        check(lib().nb_builder_add(self._h, key, len(key)), "nb_builder_add")

    def add_batch(self, keys: np.ndarray, offsets: np.ndarray | None, key_len: int, n: int) -> None:
        check(lib().nb_builder_add_batch(self._h, _np_ptr(keys), _np_ptr(offsets), key_len, n),
              "nb_builder_add_batch")

    def add_batch_async(self, keys: np.ndarray, offsets: np.ndarray | None, key_len: int,
                        n: int) -> None:
        """nb_builder_add_batch_async: the buffers must stay untouched (and alive) until
        sync_uploads(), finish() or close() returns."""
        check(lib().nb_builder_add_batch_async(self._h, _np_ptr(keys), _np_ptr(offsets), key_len, n),
              "nb_builder_add_batch_async")

    def sync_uploads(self) -> None:
        check(lib().nb_builder_sync_uploads(self._h), "nb_builder_sync_uploads")

    def finish(self, words: np.ndarray | None = None) -> np.ndarray:
        if words is None:
            words = np.zeros(max(nwords(self.m), 1), dtype=np.uint64)
        check(lib().nb_builder_finish(self._h, _np_ptr(words)), "nb_builder_finish")
        return words

    def close(self) -> None:
        if self._h:
            check(lib().nb_builder_destroy(self._h), "nb_builder_destroy")
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def serialize(m: int, k: int, p: float, time_const: int, seed: int, words: np.ndarray) -> bytes:
    size = lib().nb_serialized_size(m)
    out = np.zeros(size, dtype=np.uint8)
    w = words if words.size else np.zeros(1, np.uint64)
    n = lib().nb_serialize(m, k, p, time_const, seed, _np_ptr(w), _np_ptr(out))
    return out[:n].tobytes()


def deserialize(img: bytes):
    """-> (m, k, p, time_const, seed, words)"""
    buf = np.frombuffer(img, dtype=np.uint8).copy()
    m, k, tc, seed = C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_uint64()
    p = C.c_double()
    rc = lib().nb_deserialize(_np_ptr(buf), len(img), C.addressof(m), C.addressof(k),
                              C.addressof(p), C.addressof(tc), C.addressof(seed), None)
    check(rc, "nb_deserialize(header)")
    words = np.zeros(max(nwords(m.value), 1), dtype=np.uint64)
    rc = lib().nb_deserialize(_np_ptr(buf), len(img), None, None, None, None, None, _np_ptr(words))
    check(rc, "nb_deserialize")
    return m.value, k.value, p.value, tc.value, seed.value, words


def _pack(keys: list[bytes]):
    offs = np.zeros(len(keys) + 1, dtype=np.uint64)
    if keys:
        offs[1:] = np.cumsum([len(x) for x in keys], dtype=np.uint64)
    flat = b"".join(keys)
    buf = np.frombuffer(flat + b"\0" * 16, dtype=np.uint8).copy()
    return buf, offs


class BloomFilter:
    """Mirror of the reference `BloomFilter` (BloomFilter/BloomFilter.h:12-42)."""

    BATCH_LIMIT = 1 << 20  # pending keys before an automatic build
    HOST_BATCH_LIMIT = 4096  # smaller batches are built on the host (nb_build_cpu)

    def __init__(self, n: int | None = None, falsePositiveRate: float | None = None, *,
                 flavor: int = FLAVOR_LIBSTDCXX, device: int = 0, time_const: int | None = None):
        self.flavor = flavor
        self.device = device
        self.last_on_device = False
        self._pending: list[bytes] = []
        if n is None:  # BloomFilter() -- BloomFilter.cpp:26: no closures, no bits
            self.m, self.k, self.p, self.timeConst, self.h2_seed = 0, 0, 0.0, 0, 0
            self.words = np.zeros(1, dtype=np.uint64)
            return
        self.m = self.calculateSizeOfBitSet(n, falsePositiveRate)
        self.k = self.calculateNumberOfHashFunctions(n, self.m)
        self.p = float(falsePositiveRate)
        self.timeConst = (int(time.time()) if time_const is None else int(time_const)) & 0xFFFFFFFF
        self.h2_seed = seed_from_time(self.timeConst)
        self.words = np.zeros(max(nwords(self.m), 1), dtype=np.uint64)

    # -- reference static helpers (BloomFilter.cpp:192-199)
    @staticmethod
    def calculateSizeOfBitSet(expectedElements: int, falsePositiveRate: float) -> int:
        return size_of_bitset(expectedElements, falsePositiveRate)

    @staticmethod
    def calculateNumberOfHashFunctions(expectedElements: int, m: int) -> int:
        return num_hashes(expectedElements, m)

    # -- batching
    def _flush(self) -> None:
        if not self._pending:
            return
        keys, self._pending = self._pending, []
        if self.k == 0:
            return  # no closures: add() sets nothing (BloomFilter.cpp:82-86)
        buf, offs = _pack(keys)
        self.last_on_device = False
        if len(keys) >= self.HOST_BATCH_LIMIT:
            try:
                build_host(buf, offs, 0, len(keys), self.m, self.k, self.h2_seed, self.flavor,
                           self.words, self.device)
                self.last_on_device = True
                return
            except NaspBloomError as e:  # the reference's error style: report, carry on
                import sys
                print(f"[BloomFilter] GPU build failed ({e}); building {len(keys)} keys on the host",
                      file=sys.stderr)
        build_cpu(buf, offs, 0, len(keys), self.m, self.k, self.h2_seed, self.flavor, self.words)

    def add(self, elem: bytes | str) -> None:
        self._pending.append(elem.encode() if isinstance(elem, str) else bytes(elem))
        if len(self._pending) >= self.BATCH_LIMIT:
            self._flush()

    def add_batch(self, elems) -> None:
        for e in elems:
            self._pending.append(e.encode() if isinstance(e, str) else bytes(e))
        if len(self._pending) >= self.BATCH_LIMIT:
            self._flush()

    def possiblyContains(self, elem: bytes | str) -> bool:
        return bool(self.possiblyContainsBatch([elem])[0])

    def possiblyContainsBatch(self, elems) -> np.ndarray:
        self._flush()
        keys = [e.encode() if isinstance(e, str) else bytes(e) for e in elems]
        if self.k == 0:
            return np.ones(len(keys), dtype=np.uint8)
        buf, offs = _pack(keys)
        if len(keys) < self.HOST_BATCH_LIMIT:  # single-key lookups stay on the host
            return probe_cpu(buf, offs, 0, len(keys), self.m, self.k, self.h2_seed, self.flavor,
                             self.words)
        return probe_host(buf, offs, 0, len(keys), self.m, self.k, self.h2_seed, self.flavor,
                          self.words, self.device)

    def serialize(self) -> bytes:
        self._flush()
        return serialize(self.m, self.k, self.p, self.timeConst, self.h2_seed, self.words)

    @staticmethod
    def deserialize(data: bytes, *, flavor: int = FLAVOR_LIBSTDCXX, device: int = 0) -> "BloomFilter":
        bf = BloomFilter(flavor=flavor, device=device)
        bf.m, bf.k, bf.p, bf.timeConst, bf.h2_seed, bf.words = deserialize(data)
        return bf

    def copy(self) -> "BloomFilter":
        self._flush()
        bf = BloomFilter(flavor=self.flavor, device=self.device)
        bf.m, bf.k, bf.p, bf.timeConst, bf.h2_seed = self.m, self.k, self.p, self.timeConst, self.h2_seed
        bf.words = self.words.copy()
        return bf


# ------------------------------------------------------------------ Merkle --

def merkle_tree_size(n: int) -> int:
    return int(lib().nb_merkle_tree_size(n))


def merkle_device(data, offsets, rec_len: int, n: int, flavor: int, tree, stream=None) -> None:
    """Every level of the Merkle tree of n device-resident records into `tree`
    (merkle_tree_size(n) int64/uint64 cuda words; leaves first, root last)."""
    if not data.is_cuda or not tree.is_cuda or (offsets is not None and not offsets.is_cuda):
        raise NaspBloomError("merkle_device needs CUDA (HIP) tensors")
    if tree.numel() * tree.element_size() < merkle_tree_size(n) * 8:
        raise NaspBloomError("tree tensor smaller than merkle_tree_size(n) words")
    check(lib().nb_merkle_device(data.data_ptr(), offsets.data_ptr() if offsets is not None else None,
                                 rec_len, n, flavor, tree.data_ptr(), _stream_handle(stream)),
          "nb_merkle_device")


def merkle_host(data: np.ndarray, offsets: np.ndarray | None, rec_len: int, n: int,
                flavor: int = FLAVOR_LIBSTDCXX, device: int = 0, want_tree: bool = True):
    """-> (root hash, tree words or None).  tree[:n] are the leaves."""
    tree = np.zeros(merkle_tree_size(n), dtype=np.uint64) if want_tree else None
    root = C.c_uint64()
    check(lib().nb_merkle(_np_ptr(data), _np_ptr(offsets), rec_len, n, flavor, _np_ptr(tree), None,
                          C.addressof(root), device), "nb_merkle")
    return int(root.value), tree


def merkle_cpu(data: np.ndarray, offsets: np.ndarray | None, rec_len: int, n: int,
               flavor: int = FLAVOR_LIBSTDCXX, want_tree: bool = True):
    """nb_merkle_cpu: the same tree on the calling CPU thread (small flushes, no GPU)."""
    tree = np.zeros(merkle_tree_size(n), dtype=np.uint64) if want_tree else None
    root = C.c_uint64()
    check(lib().nb_merkle_cpu(_np_ptr(data), _np_ptr(offsets), rec_len, n, flavor, _np_ptr(tree),
                              None, C.addressof(root)), "nb_merkle_cpu")
    return int(root.value), tree


class MerkleTree:
    """Mirror of the reference MerkleTree (MerkleTree/MerkleTree.h:10-36): trees of at
    least HOST_RECORD_LIMIT records are built on the GPU, smaller ones -- and any
    whose device build fails, after a note on stderr -- on the host with the same
    hashing (nb_merkle_cpu); strings are the decimal hashes the reference stores."""

    HOST_RECORD_LIMIT = 4096

    def __init__(self, data, *, flavor: int = FLAVOR_LIBSTDCXX, device: int = 0):
        recs = [d.encode() if isinstance(d, str) else bytes(d) for d in data]
        if not recs:
            raise ValueError("Merkle tree of no data (merkle.cpp:8-10 throws)")
        self.flavor = flavor
        buf, offs = _pack(recs)
        self._n = len(recs)
        self.on_device = False
        if self._n >= self.HOST_RECORD_LIMIT:
            try:
                _, self._tree = merkle_host(buf, offs, 0, self._n, flavor, device)
                self.on_device = True
            except NaspBloomError as e:  # the reference's error style: report, carry on
                import sys
                print(f"[MerkleTree] GPU build failed ({e}); building {self._n} records on the host",
                      file=sys.stderr)
        if not self.on_device:
            _, self._tree = merkle_cpu(buf, offs, 0, self._n, flavor)
        self._levels = []
        at, c = 0, self._n
        while True:
            self._levels.append((at, c))
            at += c
            if c == 1:
                break
            c = (c + 1) // 2

    def _hash(self, data: bytes) -> str:  # merkle.cpp:26-32
        return str(std_hash(data, self.flavor))

    def getRootHash(self) -> str:
        return str(int(self._tree[-1]))

    def getLeaves(self) -> list[str]:
        return [str(int(x)) for x in self._tree[: self._n]]

    def generateProof(self, data) -> list[tuple[str, bool]]:  # merkle.cpp:57-84
        h = std_hash(data.encode() if isinstance(data, str) else bytes(data), self.flavor)
        hits = np.nonzero(self._tree[: self._n] == np.uint64(h))[0]
        if hits.size == 0:
            raise ValueError("record not in the Merkle tree (merkle.cpp:63-65 throws)")
        index = int(hits[0])
        proof = []
        for at, cnt in self._levels[:-1]:
            is_right = index % 2 == 1
            sib = index - 1 if is_right else index + 1
            if sib < cnt:
                proof.append((str(int(self._tree[at + sib])), is_right))
            index //= 2
        return proof

    @staticmethod
    def verifyProof(rootHash: str, data, proof, flavor: int = FLAVOR_LIBSTDCXX) -> bool:
        h = lambda s: str(std_hash(s.encode(), flavor))  # noqa: E731
        d = data.encode() if isinstance(data, str) else bytes(data)
        computed = str(std_hash(d, flavor))
        for sib, is_right in proof:  # merkle.cpp:90-99
            computed = h(sib + computed) if is_right else h(computed + sib)
        return computed == rootHash
