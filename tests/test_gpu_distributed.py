"""The cooperative build (C5's shape) end to end through the HIP path
at world sizes 2 and 3: gloo ranks that share cuda:0 each build their key shard's
partial filter with the HIP build (build_fn default), exchange word slices through
host copies (comm_device="cpu": RCCL will not put two ranks on one GPU) and OR
them with the HIP nb_or_merge_device kernel (merge_fn default) -- the exact
sequence an 8-GPU run executes over RCCL, minus the transport.  Every rank's
filter, and the owned slices downloaded to host memory (host_out), are bit-exact
against the oracle.  Uneven shards, both key layouts."""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import ORACLE, PKG

pytestmark = pytest.mark.gpu

SEED = 17027509906831645879


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _keys(n, var):
    from nasp_bloom import synth
    if var:
        return synth.var_keys(n, 0, 40)
    return synth.fixed_keys(n, 32, seed=44), None


def _worker(rank, world, port, n, m, k, var, result_dir):
    for p in (PKG, ORACLE):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from nasp_bloom import distributed as D
    dev = torch.device("cuda", 0)
    buf, offs = _keys(n, var)
    b, e = D.shard_range(n, rank, world)
    if var:
        kb = torch.from_numpy(buf).to(dev)
        ob = torch.from_numpy(offs[b:e + 1].view(np.int64).copy()).to(dev)
        key_len = 0
    else:
        kb = torch.from_numpy(buf[b * 32:e * 32].copy()).to(dev)
        ob, key_len = None, 32
    full = D.build_cooperative(kb, ob, key_len, e - b, m, k, SEED, 0, comm_device="cpu")
    S = D.slice_words(m, world)
    host = torch.empty(S, dtype=torch.int64).pin_memory()
    owned = D.build_cooperative(kb, ob, key_len, e - b, m, k, SEED, 0, comm_device="cpu",
                                host_out=host)
    torch.cuda.synchronize()
    np.save(os.path.join(result_dir, f"full{rank}.npy"), full.cpu().numpy())
    np.save(os.path.join(result_dir, f"owned{rank}.npy"), owned.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("var,m,k,world", [(False, 2**32 - 1, 10, 2), (True, 9_585_059, 7, 3),
                                           (False, 95_850_587, 7, 3), (True, 1_000_003, 10, 2)])
def test_cooperative_merge_hip_path(tmp_path, oracle, var, m, k, world):
    import torch
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from nasp_bloom import distributed as D
    n = 600_011
    mp.spawn(_worker, args=(world, _free_port(), n, m, k, var, str(tmp_path)), nprocs=world)
    buf, offs = _keys(n, var)
    want = oracle.build(0, buf, offs, 0 if var else 32, n, m, k, SEED)
    nw = (m + 63) // 64
    S = D.slice_words(m, world)
    ref = np.zeros(world * S, np.uint64)
    ref[:nw] = want[:nw]
    for r in range(world):
        full = np.load(tmp_path / f"full{r}.npy").view(np.uint64)
        np.testing.assert_array_equal(full, ref)
        owned = np.load(tmp_path / f"owned{r}.npy").view(np.uint64)
        np.testing.assert_array_equal(owned, ref[r * S:(r + 1) * S])
