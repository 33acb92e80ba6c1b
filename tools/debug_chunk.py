"""Debug helper: find which keys of a var-length build are wrong (GPU)."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, "nasp-key-value-engine_amd"); sys.path.insert(0, "oracle")
import nasp_bloom as nbm
from nasp_bloom import synth
from oracle_ctypes import Oracle
SEED = 17027509906831645879
o = Oracle()
dev = torch.device("cuda:0")
n = int(os.environ.get("N", "1000000")); m = int(os.environ.get("M", "9585059"))
buf, offs = synth.var_keys(n)
want = o.build(0, buf, offs, 0, n, m, 7, SEED)
for mode in os.environ.get("MODES", "0 2 1").split():
    for chunk in ["0", "999999", "100000"]:
        os.environ["NB_VAR_MODE"] = mode
        os.environ["NB_CHUNK_KEYS"] = chunk
        kt = torch.from_numpy(buf).to(dev); ot = torch.from_numpy(offs.view(np.int64)).to(dev)
        w = torch.zeros(nbm.nwords(m), dtype=torch.int64, device=dev)
        nbm.build_device(kt, ot, 0, n, m, 7, SEED, 0, w)
        torch.cuda.synchronize()
        got = w.cpu().numpy().view(np.uint64)
        bad = np.nonzero(got != want)[0]
        missing = int(np.unpackbits((want & ~got).view(np.uint8)).sum())
        extra = int(np.unpackbits((got & ~want).view(np.uint8)).sum())
        out = np.zeros(n, np.uint8)
        msg = ""
        if len(bad):
            pr = torch.zeros(n, dtype=torch.uint8, device=dev)
            nbm.probe_device(kt, ot, 0, n, m, 7, SEED, 0, w, pr)
            fn = np.nonzero(pr.cpu().numpy() == 0)[0]
            msg = f" false-negative keys: {len(fn)} first {fn[:10].tolist()} lens {[int(offs[i+1]-offs[i]) for i in fn[:10]]}"
        print(f"mode {mode} chunk {chunk}: bad words {len(bad)} missing bits {missing} extra bits {extra}{msg}", flush=True)
