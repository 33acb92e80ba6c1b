"""Multi-process (world sizes 2-4, gloo, CPU) tests of the multi-GPU host logic in
nasp_bloom/distributed.py: key sharding, the all-to-all + OR reduce-scatter that
replaces the missing RCCL bitwise-OR, and the all-gather.  The per-rank build
step is the oracle here (test-side builder: no GPU in this container); on the
GPU the same code runs with the HIP build and merge kernels."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ORACLE, PKG

SEED = 17027509906831645879


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _oracle_build(keys, offsets, key_len, n, m, k, seed, flavor, partial):
    from oracle_ctypes import Oracle
    w = partial.numpy().view(np.uint64)
    kb = keys.numpy()
    ob = offsets.numpy().view(np.uint64) if offsets is not None else None
    Oracle().build(flavor, kb, ob, key_len, n, m, k, seed, words=w)


def _reduce_or(x):
    out = x[0].clone()
    for r in range(1, x.shape[0]):
        out |= x[r]
    return out


def _worker(rank, world, port, n, m, k, var, result_dir):
    for p in (PKG, ORACLE):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from nasp_bloom import distributed as D
    from nasp_bloom import synth
    if var:
        buf, offs = synth.var_keys(n, 0, 40)
    else:
        buf, offs = synth.fixed_keys(n, 16), None
    b, e = D.shard_range(n, rank, world)
    if var:
        kb = torch.from_numpy(buf.copy())
        ob = torch.from_numpy(offs[b:e + 1].view(np.int64).copy())
        key_len = 0
    else:
        kb = torch.from_numpy(buf[b * 16:e * 16 + 16].copy())
        ob = None
        key_len = 16
    merge = lambda dst, recv, nsrc, stride: dst.__ior__(_reduce_or(recv.view(nsrc, stride)))
    full = D.build_cooperative(kb, ob, key_len, e - b, m, k, SEED, 0, build_fn=_oracle_build,
                               merge_fn=merge)
    owned = D.merge_partials(_partial(kb, ob, key_len, e - b, m, k, world), m, all_gather=False,
                             merge_fn=merge)
    np.save(os.path.join(result_dir, f"full{rank}.npy"), full.numpy())
    np.save(os.path.join(result_dir, f"owned{rank}.npy"), owned.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _partial(kb, ob, key_len, n, m, k, world):
    from nasp_bloom import distributed as D
    S = D.slice_words(m, world)
    p = torch.zeros(world * S, dtype=torch.int64)
    _oracle_build(kb, ob, key_len, n, m, k, SEED, 0, p)
    return p


@pytest.mark.parametrize("var,m,k,world", [(True, 1_000_003, 7, 2), (False, 95_851, 10, 2),
                                           (True, 64, 3, 2), (False, 95_851, 7, 3),
                                           (True, 200_003, 7, 4), (False, 95_851, 7, 1)])
def test_cooperative_or_merge_gloo(tmp_path, oracle, var, m, k, world):
    """World sizes 2-4 (uneven key shards, word slices that do not divide m), and
    world size 1 (the partial is returned as the filter, no collective)."""
    from nasp_bloom import distributed as D
    from nasp_bloom import synth
    n = 30_011
    mp.spawn(_worker, args=(world, _free_port(), n, m, k, var, str(tmp_path)), nprocs=world)
    if var:
        buf, offs = synth.var_keys(n, 0, 40)
        want = oracle.build(0, buf, offs, 0, n, m, k, SEED)
    else:
        buf = synth.fixed_keys(n, 16)
        want = oracle.build(0, buf, None, 16, n, m, k, SEED)
    nw = (m + 63) // 64
    S = D.slice_words(m, world)
    for r in range(world):
        full = np.load(tmp_path / f"full{r}.npy").view(np.uint64)
        np.testing.assert_array_equal(full[:nw], want[:nw])
        assert not full[nw:].any()
        owned = np.load(tmp_path / f"owned{r}.npy").view(np.uint64)
        ref = np.zeros(world * S, np.uint64)
        ref[:nw] = want[:nw]
        np.testing.assert_array_equal(owned, ref[r * S:(r + 1) * S])


def test_shard_ranges_cover_exactly():
    from nasp_bloom import distributed as D
    for n in (0, 1, 7, 1000, 1_000_000_007):
        for w in (1, 2, 3, 8):
            rs = [D.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(e - b for b, e in rs) - min(e - b for b, e in rs) <= 1
