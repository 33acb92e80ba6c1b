"""nasp_bloom -- Python binding of the MI355X-native SSTable Bloom-filter path.

The product is libnasp_bloom.so (HIP kernels for gfx950 behind the C ABI in
include/nasp_bloom.h) and the C++ drop-in class host/BloomFilter.h.  This package
is the Python binding used by tests/ and bench.py:

  build_device / probe_device  -- device-resident batch build / probe on torch tensors
  build_host / probe_host      -- host-buffer entry points (H2D + kernel + D2H)
  Builder                      -- streaming host builder: pinned chunks, packing /
                                  upload / device build overlapped (nb_builder_*)
  BloomFilter                  -- mirror of the reference class surface
                                  (reference BloomFilter/BloomFilter.h:24-41)
  MerkleTree, merkle_device    -- the SSTable Merkle tree on the GPU (nb_merkle*; small
                                  trees on the host, merkle_cpu), mirror of the reference
                                  class (MerkleTree/MerkleTree.h:10-36)
  set_knob / get_knob / knobs  -- the library's A/B and fault-injection switches
  distributed                  -- multi-GPU: independent filters / cooperative OR-merge
"""
from ._lib import (FLAVOR_LIBSTDCXX, FLAVOR_MSVC_FNV1A, FLAVOR_MURMUR3_X64_128,  # noqa: F401
                   NaspBloomError, lib)
from .api import (BloomFilter, Builder, MerkleTree, build_device, merkle_device, merkle_host,  # noqa: F401
                  merkle_tree_size, std_hash, build_host, build_host_sharded, deserialize, nwords, or_merge_device,  # noqa: F401
                  probe_device, probe_host, build_cpu, probe_cpu, device_build_count, seed_from_time, serialize, size_of_bitset,
                  num_hashes, merkle_cpu, device_merkle_count, set_knob, get_knob, knobs)
