#!/usr/bin/env python3
"""Diagnostic: the auto probe over present / absent / 30 % / 80 % present batches of
the graph test's shape (n = 4.2M, m = 40 250 003, k = 7), first as direct calls, then
replayed from one captured graph (argv[1] == "graph"), printing each step."""
import sys

import numpy as np
import torch

sys.path.insert(0, "nasp-key-value-engine_amd")
sys.path.insert(0, "oracle")
import nasp_bloom as nbm  # noqa: E402
from nasp_bloom import synth  # noqa: E402
from oracle_ctypes import Oracle  # noqa: E402

SEED = 17027509906831645879
mode = sys.argv[1] if len(sys.argv) > 1 else "direct"
path = sys.argv[2] if len(sys.argv) > 2 else "auto"  # NB_PROBE_PATH of every call
nbm.set_knob("NB_PROBE_PATH", {"auto": 0, "lane": 1, "tiled": 2, "split": 3}[path])
dev = torch.device("cuda", 0)
n, m, k = 4_200_000, 40_250_003, 7
orc = Oracle()
base = synth.fixed_keys(n, 16, seed=71)
words_np = orc.build(0, base, None, 16, n, m, k, SEED)
other = synth.fixed_keys(n, 16, seed=72)


def mixed(pc):
    b = other.copy()
    bv, pv = b[:n * 16].reshape(n // 10, 10, 16), base[:n * 16].reshape(n // 10, 10, 16)
    bv[:, :pc // 10] = pv[:, :pc // 10]
    return b


kt = torch.from_numpy(base).to(dev)
words = torch.from_numpy(words_np.view(np.int64)).to(dev)
out = torch.zeros(n, dtype=torch.uint8, device=dev)
st = torch.cuda.Stream(device=dev)
seq = (("present", base), ("absent", other), ("p30", mixed(30)), ("p80", mixed(80)))
with torch.cuda.stream(st):
    nbm.probe_device(kt, None, 16, n, m, k, SEED, 0, words, out, stream=st)
st.synchronize()
print("warm-up ok", flush=True)
g = None
if mode == "graph":
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        nbm.probe_device(kt, None, 16, n, m, k, SEED, 0, words, out, stream=st)
    print("captured", flush=True)
bad = 0
for name, keys in seq:
    kt.copy_(torch.from_numpy(keys))
    out.fill_(7)
    torch.cuda.synchronize()
    print("running", name, flush=True)
    if g is not None:
        g.replay()
    else:
        with torch.cuda.stream(st):
            nbm.probe_device(kt, None, 16, n, m, k, SEED, 0, words, out, stream=st)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    want = orc.probe(0, keys, None, 16, n, m, k, SEED, words_np)
    ok = np.array_equal(got, want)
    bad += not ok
    print(name, "ok" if ok else f"MISMATCH {(got != want).sum()}", flush=True)
sys.exit(1 if bad else 0)
