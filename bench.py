#!/usr/bin/env python3
"""bench.py -- device-resident Bloom-filter build throughput (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c4|c2|c3|c1|c5|merkle]

Default workload: C4's per-GPU shard, 100M x 16 B keys, k = 7 (m = 958,505,838):
the shape the north star's target ("100M x 16B keys at k=7") is quoted on, and
at N GPUs exactly BASELINE config 4 (one independent SSTable filter per GPU).

One step = one pass of the hot path over one batch: build a fresh filter from
every key of the batch (hash + index + bit scatter + filter store; the library's
overwrite mode, so no separate clear pass), keys already resident in HBM.  N > 1 (one rank
per GPU: `--gpus N` starts the N ranks itself as a torch.distributed.run child process
when no launcher is around it, and refuses a launcher's WORLD_SIZE != N): every rank builds
its own independent filter over its own keys (the compaction fan-out, C4) --
weak scaling, no data-path collective.  `value` = all keys of all ranks / the
max-over-ranks time of the K timed steps.

Extra fields: `roofline` (the build call's kernels, HIP-event timed on their own
stream; achieved = algorithmic bytes / average build time; traffic
and valu_frac from the committed rocprofv3 PMC summaries of the current kernel
source) and, on rank 0 at N = 1, `cpu_baseline` (the reference BloomFilter.cpp
compiled here, timed on a bounded sample of the same workload: 1 pinned core, or
for C4 8 concurrent builds on 8 pinned cores) and `c2` (BASELINE config 2's
device-resident rate, the round-1 headline, measured in the same run).
"""
from __future__ import annotations

import argparse
import contextlib
import glob
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "nasp-key-value-engine_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def algorithmic_bytes(n, key_len, total_key_bytes, m, var_len):
    """keys read once, offsets read once, the filter written once."""
    return total_key_bytes + (8 * (n + 1) if var_len else 0) + (m + 7) // 8


@contextlib.contextmanager
def pinned_one_core():
    """Run the calling thread on one core (the 1-core CPU reference,
    taskset-style); the previous affinity is restored afterwards."""
    allowed = os.sched_getaffinity(0)
    core = min(allowed)
    os.sched_setaffinity(0, {core})
    try:
        yield core
    finally:
        os.sched_setaffinity(0, allowed)


def cpu_baseline(wl, keys_np, offs_np, key_len, budget_s=12.0, threads=1):
    """The reference add() loop (oracle/_ref: BloomFilter.cpp compiled here) on a
    bounded prefix sample of this workload, 1 thread.  Falls back to the oracle
    restatement (kind "port") if the reference build is absent.  threads > 1
    (C4, SURVEY §8d: one independent filter per core): that many concurrent
    builds of the same sample, each thread pinned to its own core; the rate is
    threads x sample / the slowest thread's add() loop."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    try:
        from oracle_ctypes import RefLib
        ref = RefLib()
        kind = "reference"
    except (FileNotFoundError, OSError):
        ref = None
        kind = "port"
    from nasp_bloom.synth import H2_SEED
    # calibrate on 100k keys, then size the sample to ~budget_s
    n_cal = min(100_000, wl.n)

    def run(nk):
        if ref is not None:
            return ref.build_timed(keys_np, offs_np, key_len, nk, wl.m, wl.k, H2_SEED,
                                   want_image=False)[0]
        from oracle_ctypes import Oracle
        t0 = time.perf_counter()
        Oracle().build(0, keys_np, offs_np, key_len, nk, wl.m, wl.k, H2_SEED)
        return time.perf_counter() - t0

    with pinned_one_core() as core:
        t_cal = run(n_cal)
        n_s = int(min(wl.n, max(n_cal, n_cal * budget_s / max(t_cal, 1e-9))))
        if threads <= 1 or ref is None:
            t = run(n_s)
    try:
        cpu_model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:  # noqa: BLE001
        cpu_model = "unknown"
    if threads > 1 and ref is not None:
        import threading
        cores = sorted(os.sched_getaffinity(0))[:threads]
        secs = [0.0] * len(cores)

        def worker(i):
            os.sched_setaffinity(0, {cores[i]})  # this thread only
            secs[i] = ref.build_timed(keys_np, offs_np, key_len, n_s, wl.m, wl.k, H2_SEED,
                                      want_image=False)[0]
        th = [threading.Thread(target=worker, args=(i,)) for i in range(len(cores))]
        for x in th:
            x.start()
        for x in th:
            x.join()
        t = max(secs)
        return {"value": round(len(cores) * n_s / t / 1e6, 4), "unit": "Mkeys/s",
                "cores": len(cores), "kind": kind,
                "sample": f"{len(cores)} concurrent reference add() loops, one per pinned core "
                          f"(cpus {cores[0]}-{cores[-1]}), each over the first {n_s} keys of "
                          f"{wl.name} into its own m={wl.m}, k={wl.k} filter; slowest {t:.1f} s "
                          f"({cpu_model})"}
    return {"value": round(n_s / t / 1e6, 4), "unit": "Mkeys/s", "cores": 1, "kind": kind,
            "sample": f"first {n_s} keys of {wl.name} into the same m={wl.m}, k={wl.k} filter; "
                      f"reference add() loop, {t:.1f} s, 1 thread pinned to cpu {core} ({cpu_model})"}


def host_path_rate(wl, keys_np, offs_np, key_len, seed, flavor, reps=3):
    """Host-memory-to-host-memory rates, reported beside `value`,
    never as it:
      value        -- nb_build: current words up, keys up chunk by chunk (pageable,
                      straight from the caller's buffer) with each chunk's build
                      overlapping the next upload, words down
      fresh_filter -- the streaming builder on a fresh filter (no words upload):
                      what SSTable::build's new filter costs from packed keys
      dropin_class -- the C++ drop-in class end to end (ctor, add() per std::string
                      key into pinned chunks, copy-assign, serialize), C2's key count"""
    import subprocess
    import nasp_bloom as nbm
    words = np.zeros(nbm.nwords(wl.m), dtype=np.uint64)

    def best_of(fn):
        fn()  # warm the pools
        t = 1e30
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            t = min(t, time.perf_counter() - t0)
        return t

    def via_nb_build():
        nbm.build_host(keys_np, offs_np, key_len, wl.n, wl.m, wl.k, seed, flavor, words)

    def via_builder():
        with nbm.Builder(wl.m, wl.k, seed, flavor) as b:
            b.add_batch(keys_np, offs_np, key_len, wl.n)
            b.finish(words)

    t_build, t_fresh = best_of(via_nb_build), best_of(via_builder)
    key_bytes = int(offs_np[-1]) + 8 * (wl.n + 1) if offs_np is not None else wl.n * key_len
    out = {"value": round(wl.n / t_build / 1e6, 3), "unit": "Mkeys/s", "ms": round(t_build * 1e3, 3),
           "h2d_bytes": key_bytes + nbm.nwords(wl.m) * 8, "d2h_bytes": nbm.nwords(wl.m) * 8,
           "fresh_filter": {"value": round(wl.n / t_fresh / 1e6, 3), "ms": round(t_fresh * 1e3, 3),
                            "h2d_bytes": key_bytes},
           "note": "nb_build from pageable host buffers, chunked upload overlapped with the "
                   "device build; best of %d" % reps}
    exe = os.path.join(REPO, "nasp-key-value-engine_amd", "build", "sstable_filter_bench")
    if offs_np is None and os.path.exists(exe):
        # 10M std::string keys at most (C4's 100M would hold ~5 GB of strings)
        r = subprocess.run([exe, str(min(wl.n, 10_000_000)), str(key_len), str(reps)],
                           capture_output=True, text=True, timeout=300)
        if r.returncode == 0:
            out["dropin_class"] = json.loads(r.stdout.strip().splitlines()[-1])
        else:
            out["dropin_class"] = {"error": (r.stdout + r.stderr)[-300:]}
    return out


def c2_rate(nbm, synth, dev, stream, flavor, steps=20):
    """BASELINE config 2 (10M x 16 B, k = 7, one filter) device-resident, the same
    timing as `value`: reported beside the C4 headline."""
    import torch
    wl = synth.C2
    keys_np, _, kl = synth.keys_for(wl)
    keys = torch.from_numpy(keys_np).to(dev)
    words = torch.zeros(nbm.nwords(wl.m), dtype=torch.int64, device=dev)

    def step():
        with torch.cuda.stream(stream):
            nbm.build_device(keys, None, kl, wl.n, wl.m, wl.k, synth.H2_SEED, flavor, words,
                             stream=stream, overwrite=True)
    for _ in range(3):
        step()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    ms = ev0.elapsed_time(ev1) / steps
    B = algorithmic_bytes(wl.n, kl, wl.n * kl, wl.m, False)
    return {"workload": wl.name, "value": round(wl.n * steps / el / 1e6, 3), "unit": "Mkeys/s",
            "kernel_ms": round(ms, 5), "frac": round(B / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
            "algorithmic_bytes_per_launch": B}


def probe_rates(wl, keys, offs, key_len, seed, flavor, words, stream, dev, reps=5):
    """Batch possiblyContains (nb_probe_device, BloomFilter.cpp:67-80) over the filter
    just built: the batch's own keys (every one present) and as many absent keys
    (their positive rate is the filter's measured false-positive rate), on each
    probe path (NB_PROBE_PATH): `auto` (the library's default: a sampled prefix picks
    the path on the device), `lane` (one lane per key, k gathers with early exit),
    `tiled` (lookups binned by filter tile and tested in LDS) and `split` (the tiled
    path in two rounds: two indices of every key, then the rest of the keys still
    present).  Fixed-length keys also get a mixed batch, `p30`: 3 of every 10 keys
    present, the rest absent (LSM point lookups over one level's SSTables are mostly
    misses).  Reported beside `value`."""
    import torch
    import nasp_bloom as nbm
    from nasp_bloom import synth
    a_np, a_offs, _ = synth.keys_for(wl, seed=synth.SEED + 1000)
    absent = torch.from_numpy(a_np).to(dev)
    a_o = torch.from_numpy(a_offs.view(np.int64)).to(dev) if a_offs is not None else None
    out_t = torch.empty(wl.n, dtype=torch.uint8, device=dev)
    batches = [("present", keys, offs), ("absent", absent, a_o)]
    nb = wl.n * key_len
    if offs is None and a_o is None and wl.n % 10 == 0 and min(keys.numel(), absent.numel()) >= nb:
        mixed = absent.clone()  # (the key buffers carry a few bytes of tail padding)
        mv, kv = mixed[:nb].view(wl.n // 10, 10, key_len), keys[:nb].view(wl.n // 10, 10, key_len)
        mv[:, :3] = kv[:, :3]
        batches.append(("p30", mixed, None))
    res = {}
    # SURVEY §8(d)'s probe row: keys (and offsets) read once, the filter read once, one
    # answer byte written per key; traffic from the committed PMC summary of the probe
    # kernels at the current kernel source (tools/profile_probe.sh), C4 only
    B = (int(offs[-1].item()) + 8 * (wl.n + 1) if offs is not None else wl.n * key_len) + (wl.m + 7) // 8 + wl.n
    ppmc = latest_profile("c4_probe", "pmc") if wl.name == "c4_100M_x16B_k7_per_gpu" else None
    for path, extra in (("auto", {}), ("lane", {}), ("tiled", {}), ("split", {}),
                        ("auto_host_pick", {"NB_PROBE_HOST_PICK": 1})):
        r = {}
        with nbm.knobs(NB_PROBE_PATH=path.split("_")[0], **extra):
            for name, kk, oo in batches:
                with torch.cuda.stream(stream):
                    nbm.probe_device(kk, oo, key_len, wl.n, wl.m, wl.k, seed, flavor, words, out_t,
                                     stream=stream)
                # wall clock between device synchronisations: what a caller sees (with
                # NB_PROBE_HOST_PICK=1 the auto path blocks the host on its sample, and
                # HIP events around the calls would miss that)
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for _ in range(reps):
                    with torch.cuda.stream(stream):
                        nbm.probe_device(kk, oo, key_len, wl.n, wl.m, wl.k, seed, flavor, words, out_t,
                                         stream=stream)
                torch.cuda.synchronize(dev)
                ms = (time.perf_counter() - t0) * 1e3 / reps
                r[name] = {"value": round(wl.n / (ms * 1e-3) / 1e6, 3), "unit": "Mkeys/s",
                           "ms": round(ms, 4), "positive_rate": round(float(out_t.float().mean()), 6)}
                pm = ((ppmc or {}).get("paths", {}).get(path, {}).get(name) or {})
                r[name]["roofline"] = {
                    "bound": "hbm", "achieved": round(B / (ms * 1e-3) / 1e9, 2), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(B / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                    "algorithmic_bytes": B, "traffic": pm.get("hbm_bytes_per_call"),
                    "device_us": pm.get("device_us_per_call")}
        res[path] = r
    res["note"] = ("auto = the default (lane kernel on a 4 096-key sample, whose hit count picks lane, "
                   "split or tiled for the rest on the device: every path launched, the closed ones "
                   "return at once; no host wait); auto_host_pick = the same choice read back on the "
                   "host, which then launches only the chosen path (NB_PROBE_HOST_PICK=1, rounds 3-5: "
                   "blocks the caller on the sample); absent keys from another seed; p30 = keys 0-2 of every 10 "
                   "present, the rest absent; ms = wall clock per call over 5 back-to-back calls "
                   "between device synchronisations; roofline: algorithmic bytes (keys + filter + "
                   "answers) / ms, traffic and device_us from the committed probe PMC summary ("
                   + ((ppmc or {}).get("source") or "none at the current kernel source") + ")")
    return res


def latest_profile(workload_name, kind="pmc"):
    """The committed profile summary of this workload for the current kernel
    source: kind "pmc" = per-launch HBM bytes (profiles/*_pmc_*.json, written by
    tools/pmc_traffic.py), "sq" = VALU counters (profiles/*_sq_*.json, written by
    tools/sq_summary.py); None when none matches the kernel source hash."""
    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", f"*_{kind}_*.json"))):
        try:
            d = json.load(open(f))
        except Exception:  # noqa: BLE001
            continue
        if d.get("workload") == workload_name and d.get("kernel_source_sha") == kernel_sha():
            best = dict(d, source=d.get("source") or os.path.relpath(f, REPO))
    return best


def valu_frac_of(sq):
    """Build-weighted VALU fraction of the build kernels from an SQ summary:
    sum of VALU floors (SQ_INSTS_VALU x 4 cycles / 1024 SIMDs / effective clock)
    over the sum of the kernels' durations (tools/sq_summary.py)."""
    if not sq:
        return None
    ks = [v for k, v in sq.get("kernels", {}).items() if k in sq.get("build_kernels", [])]
    if not ks or any("valu_floor_us" not in v for v in ks):
        return None
    return round(sum(v["valu_floor_us"] for v in ks) / sum(v["avg_duration_us"] for v in ks), 4)


def steady_state(step, stream, dev, n):
    """Diagnostic beside `value`, never it: n more builds right after the timed ones,
    each bracketed by its own HIP events on the build stream.  The build time follows
    the chip's clock, which the power controller pulls down for the first ~25 builds
    after any idle gap and then raises again (profiles/r04_c4_dispatch_clock.txt,
    DESIGN.md §6): the timed K steps after W warmup steps sit in that ramp, the last
    builds here show the settled rate."""
    import torch
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    evs[0].record(stream)
    for i in range(n):
        step()
        evs[i + 1].record(stream)
    torch.cuda.synchronize(dev)
    ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(n)]
    last = ms[-20:]
    return {"build_ms": [round(x, 4) for x in ms], "last20_mean_ms": round(sum(last) / len(last), 5),
            "last20_min_ms": round(min(last), 5),
            "note": "per-build device time of 40 builds after the timed steps (events per build); "
                    "the build time tracks the DVFS clock -- not the contract value"}


def rank_diag(per_rank, key):
    """N > 1 self-diagnosis: the world size and the backend the
    process group reports, each rank's own numbers, and the min / max of `key`."""
    import torch.distributed as dist
    import torch
    vals = [r[key] for r in per_rank]
    backend = str(dist.get_backend())
    nccl = None
    if backend == "nccl":
        try:
            v = torch.cuda.nccl.version()
            nccl = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
        except Exception:  # noqa: BLE001
            nccl = "unknown"
    return {"world_size": dist.get_world_size(), "backend": backend, "rccl_version": nccl,
            f"{key}_min": min(vals), f"{key}_max": max(vals), "per_rank": per_rank}


def reduce_device(dev):
    """Where the max-over-ranks timing tensor lives: the GPU for RCCL, the host for
    the gloo rehearsal (NB_BENCH_BACKEND)."""
    return dev if os.environ.get("NB_BENCH_BACKEND", "nccl") == "nccl" else "cpu"


def kernel_sha():
    import hashlib
    h = hashlib.sha256()
    for f in ("csrc/bloom_kernels.hip", "csrc/bloom_math.h"):
        h.update(open(os.path.join(REPO, "nasp-key-value-engine_amd", f), "rb").read())
    return h.hexdigest()[:16]


# The JSON line is the only thing bench.py writes to stdout: everything else written
# to file descriptor 1 -- e.g. the RCCL banner its communicator prints on init, or
# library notes -- is sent to stderr, and the line goes to a saved copy of stdout.
_JSON_OUT = None


def emit(obj):
    out = _JSON_OUT or sys.stdout
    out.write(json.dumps(obj) + "\n")
    out.flush()


def launch_plan(gpus, argv, env):
    """What `bench.py --gpus N` does before anything touches torch or the GPU:
      ("run", None)       -- this process is the (only) rank: N = 1 without a launcher,
                             or one rank of an external torch.distributed.run whose
                             WORLD_SIZE equals N;
      ("launch", cmd)     -- N > 1 and no launcher around us: start N ranks through
                             torch.distributed.run as a CHILD process (never an exec)
                             with the same arguments; the parent relays the rank-0 JSON
                             line and exits with the child's code;
      ("error", message)  -- WORLD_SIZE is set and differs from N, or N < 1."""
    if gpus < 1:
        return "error", f"--gpus must be >= 1 (got {gpus})"
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            return "error", (f"WORLD_SIZE={ws} from the launcher but --gpus {gpus}: "
                             "refusing to report a line for the wrong GPU count")
        return "run", None
    if gpus == 1:
        return "run", None
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:  # a free rendezvous port
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + list(argv)
    return "launch", cmd


def run_launcher(cmd, json_out):
    """Runs the N-rank child and relays its output: the rank-0 JSON line (the only
    stdout line that parses as a JSON object) to our stdout, everything else to stderr,
    line by line as it arrives.  Returns the child's exit code."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=None, env=env, text=True, bufsize=1)
    for line in p.stdout:
        s = line.strip()
        if s.startswith("{"):
            try:
                json.loads(s)
                json_out.write(s + "\n")
                json_out.flush()
                continue
            except ValueError:
                pass
        sys.stderr.write(line)
        sys.stderr.flush()
    return p.wait()


def main():
    global _JSON_OUT
    sys.stdout.flush()
    _JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c4", choices=["c1", "c2", "c3", "c4", "c5", "merkle"],
                    help="c1-c4: an independent filter per GPU (weak scaling); c5: one "
                         "cooperative filter over all GPUs (strong scaling, RCCL OR-merge); "
                         "merkle: the SSTable Merkle tree of C2's 10M x 16 B records per GPU")
    ap.add_argument("--flavor", type=int, default=0, help="0 libstdc++ (default), 1 MSVC FNV-1a")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the host-buffer (H2D + build + D2H) rate measurement")
    ap.add_argument("--no-probe", action="store_true", help="skip the batch-probe rates")
    ap.add_argument("--no-c2", action="store_true", help="skip the extra C2 line of the c4 run")
    ap.add_argument("--no-steady", action="store_true",
                    help="skip the per-build steady-state series after the timed steps")
    ap.add_argument("--no-rank-share", action="store_true",
                    help="c5 at N=1: skip the per-rank (1B/8 keys) partial-build line")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="print the launch decision for --gpus as JSON and exit (no GPU use)")
    args = ap.parse_args()

    # --gpus N: N ranks, one per GPU.  Decided before torch is imported: with no
    # launcher around us the ranks are a torch.distributed.run child process
    argv = [a for a in sys.argv[1:] if a != "--launch-dry-run"]
    action, what = launch_plan(args.gpus, argv, os.environ)
    if args.launch_dry_run:
        emit({"action": action, "detail": what, "gpus": args.gpus})
        return 0
    if action == "error":
        sys.stderr.write(f"bench.py: {what}\n")
        return 2
    if action == "launch":
        return run_launcher(what, _JSON_OUT)

    import torch
    import torch.distributed as dist
    import nasp_bloom as nbm
    from nasp_bloom import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # NB_BENCH_BACKEND=gloo with more ranks than GPUs: a rehearsal of the N > 1 path
    # on a one-GPU box (ranks share the device; RCCL refuses two ranks per GPU).
    # The driver's runs use the defaults: RCCL, one rank per GPU.
    backend = os.environ.get("NB_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    elif world > torch.cuda.device_count():  # (counting devices does not initialise HIP)
        raise SystemExit(f"bench.py: {world} ranks over RCCL need {world} GPUs, "
                         f"{torch.cuda.device_count()} visible (NB_BENCH_BACKEND=gloo rehearses "
                         "more ranks than GPUs)")
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    nbm.lib()  # fail loudly if the HIP library is missing

    if args.workload == "merkle":
        return bench_merkle(args, world, rank, dev)
    wl = synth.WORKLOADS[args.workload]
    if args.workload == "c5":
        return bench_cooperative(args, wl, world, rank, dev)
    # each rank: its own independent key set (distinct generator seed) and filter
    keys_np, offs_np, key_len = synth.keys_for(wl, seed=synth.SEED + rank)
    var_len = offs_np is not None
    total_key_bytes = int(offs_np[-1]) if var_len else wl.n * key_len
    keys = torch.from_numpy(keys_np).to(dev)
    offs = torch.from_numpy(offs_np.view(np.int64)).to(dev) if var_len else None
    words = torch.zeros(nbm.nwords(wl.m), dtype=torch.int64, device=dev)
    stream = torch.cuda.Stream(device=dev)
    seed = synth.H2_SEED

    def step():
        with torch.cuda.stream(stream):
            # a fresh filter per step (overwrite mode: no separate clear pass)
            nbm.build_device(keys, offs, key_len, wl.n, wl.m, wl.k, seed, args.flavor, words,
                             stream=stream, overwrite=True)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # correctness guard (cheap): every key of the batch must probe positive
    probe_out = torch.empty(wl.n, dtype=torch.uint8, device=dev)
    nbm.probe_device(keys, offs, key_len, wl.n, wl.m, wl.k, seed, args.flavor, words, probe_out)
    torch.cuda.synchronize(dev)
    if int(probe_out.min()) != 1:
        raise SystemExit("build produced a false negative -- refusing to report")
    del probe_out

    # HIP events on the build stream bracket the K builds (one pair: per-step
    # event packets would put a ~10 us bubble between builds); kern_ms is the
    # average device time of one build call
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps

    ranks = None
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=reduce_device(dev))
        per = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(per, t)
        ranks = rank_diag([{"elapsed_s": round(float(x[0]), 5), "kern_ms": round(float(x[1]), 5)}
                           for x in per], "kern_ms")
        elapsed = max(float(x[0]) for x in per)
        kern_ms = max(float(x[1]) for x in per)

    total_keys = wl.n * args.steps * world
    value = total_keys / elapsed / 1e6
    B = algorithmic_bytes(wl.n, key_len, total_key_bytes, wl.m, var_len)
    achieved = B / (kern_ms * 1e-3) / 1e9
    pmc = latest_profile(wl.name, "pmc")
    sq = latest_profile(wl.name, "sq")
    roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": (pmc or {}).get("hbm_bytes_per_launch"),
                "kernel": "bloom_bin_kernel+bloom_tile_or_kernel (one build call)", "kernel_ms": round(kern_ms, 5),
                "algorithmic_bytes_per_launch": B,
                "traffic_source": (pmc or {}).get("source"),
                "valu_frac": valu_frac_of(sq),
                "valu_source": (sq or {}).get("source")}

    out = {"metric": "bloom-filter build Mkeys/s (device-resident, k=7), 1/2/4/8 GPU",
           "value": round(value, 3), "unit": "Mkeys/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 5),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
           "data": "synthetic (splitmix64 keys, seed 0x5EED+rank)",
           "config": {"workload": wl.name, "keys_per_gpu": wl.n,
                      "key_bytes": key_len if key_len else f"{wl.lo}-{wl.hi} (var)",
                      "m": wl.m, "k": wl.k, "h2_seed": seed,
                      "flavor": ["libstdc++", "msvc-fnv1a"][args.flavor],
                      "parallelism": f"independent filter per GPU x{world}"},
           "roofline": roofline}
    if ranks is not None:
        out["ranks"] = ranks
    if world == 1 and not args.no_steady:
        out["steady_state"] = steady_state(step, stream, dev, 40)
    if rank == 0 and world == 1 and args.workload == "c4" and not args.no_c2:
        out["c2"] = c2_rate(nbm, synth, dev, stream, args.flavor)
    if rank == 0 and world == 1 and not args.no_probe:
        out["probe"] = probe_rates(wl, keys, offs, key_len, seed, args.flavor, words, stream, dev)
    if rank == 0 and world == 1 and not args.no_host_path:
        out["host_path"] = host_path_rate(wl, keys_np, offs_np, key_len, seed, args.flavor)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(wl, keys_np, offs_np, key_len, args.cpu_budget,
                                           threads=8 if args.workload == "c4" else 1)
    if rank == 0:
        emit(out)
    if world > 1:
        dist.destroy_process_group()


def bench_merkle(args, world, rank, dev):
    """The Merkle tree SSTable::build makes on the same flush (SSTable.cpp:29-40):
    every level of the tree of C2's 10M x 16-byte records, device-resident, one
    independent tree per rank (weak scaling).  Algorithmic bytes: records read once,
    every node written once and every non-root node read once by its parent."""
    import torch
    import torch.distributed as dist
    import nasp_bloom as nbm
    from nasp_bloom import synth
    wl = synth.C2
    keys_np, _, kl = synth.keys_for(wl, seed=synth.SEED + rank)
    data = torch.from_numpy(keys_np).to(dev)
    tsize = nbm.merkle_tree_size(wl.n)
    tree = torch.empty(tsize, dtype=torch.int64, device=dev)
    stream = torch.cuda.Stream(device=dev)

    def step():
        with torch.cuda.stream(stream):
            nbm.merkle_device(data, None, kl, wl.n, 0, tree, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from oracle_ctypes import Oracle
    root, _, _ = Oracle().merkle(0, keys_np, None, kl, wl.n)
    if int(tree[-1].item()) & 0xFFFFFFFFFFFFFFFF != root:
        raise SystemExit("Merkle root differs from the oracle -- refusing to report")
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=reduce_device(dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    B = wl.n * kl + 8 * tsize + 8 * (tsize - 1)
    achieved = B / (kern_ms * 1e-3) / 1e9
    out = {"metric": "Merkle tree build Mrecords/s (device-resident), 1/2/4/8 GPU",
           "value": round(wl.n * args.steps * world / elapsed / 1e6, 3), "unit": "Mrecords/s",
           "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(elapsed / args.steps * 1e3, 5), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u64",
           "data": "synthetic (splitmix64 records, seed 0x5EED+rank)",
           "config": {"workload": "merkle_c2_10M_x16B", "records_per_gpu": wl.n, "record_bytes": kl,
                      "tree_nodes": tsize, "parallelism": f"independent tree per GPU x{world}"},
           "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                        "kernel": "merkle_leaf_kernel + merkle_level_kernel (one tree)",
                        "kernel_ms": round(kern_ms, 5), "algorithmic_bytes_per_launch": B}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            from oracle_ctypes import RefMerkle
            ref = RefMerkle()
            n_cal = 200_000
            with pinned_one_core() as core:
                t_cal, _ = ref.merkle_timed(keys_np, None, kl, n_cal)
                n_s = int(min(wl.n, max(n_cal, n_cal * args.cpu_budget / max(t_cal, 1e-9))))
                t_s, _ = ref.merkle_timed(keys_np, None, kl, n_s)
            out["cpu_baseline"] = {"value": round(n_s / t_s / 1e6, 4), "unit": "Mrecords/s",
                                   "cores": 1, "kind": "reference",
                                   "sample": f"first {n_s} records: reference MerkleTree(data) "
                                             f"constructor, {t_s:.1f} s, 1 thread pinned to cpu {core}"}
        except FileNotFoundError:
            pass
    if rank == 0:
        emit(out)
    if world > 1:
        dist.destroy_process_group()


def bench_cooperative(args, wl, world, rank, dev):
    """C5: 1B x 32B keys, k=10, m=2^32-1, one filter built by all ranks: each rank
    builds a full-size partial filter from its key range, then the all-to-all +
    OR-merge into owned word slices (nasp_bloom.distributed; one rank: no collective).  Keys are generated on the
    device (32 GB in total) -- only the build is timed."""
    import torch
    import torch.distributed as dist
    import nasp_bloom as nbm
    from nasp_bloom import distributed as D
    from nasp_bloom import synth
    if world == 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    b, e = D.shard_range(wl.n, rank, world)
    n = e - b
    g = torch.Generator(device=dev).manual_seed(synth.SEED + rank)
    keys = torch.randint(0, 256, (n * wl.key_len + 16,), dtype=torch.uint8, device=dev, generator=g)
    seed = synth.H2_SEED
    stream = torch.cuda.current_stream(dev)

    # the gloo rehearsal (NB_BENCH_BACKEND) exchanges the slices through host copies
    comm = None if os.environ.get("NB_BENCH_BACKEND", "nccl") == "nccl" else "cpu"

    def step(host_out=None):
        # each rank ends with its owned word slice (no all-gather of the whole filter
        # to every rank: the filter is written out slice by slice)
        return D.build_cooperative(keys, None, wl.key_len, n, wl.m, wl.k, seed, args.flavor,
                                   all_gather=False, host_out=host_out, comm_device=comm)

    # correctness guard (untimed): the all-gathered filter has no false negative
    full = D.build_cooperative(keys, None, wl.key_len, n, wl.m, wl.k, seed, args.flavor,
                               comm_device=comm)
    torch.cuda.synchronize(dev)
    out = torch.empty(n, dtype=torch.uint8, device=dev)
    nbm.probe_device(keys, None, wl.key_len, n, wl.m, wl.k, seed, args.flavor, full, out)
    torch.cuda.synchronize(dev)
    if int(out.min()) != 1:
        raise SystemExit("cooperative build produced a false negative -- refusing to report")
    del out, full
    for _ in range(args.warmup):
        step()

    def timed(nsteps, host_out=None):
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(nsteps):
            step(host_out)
        torch.cuda.synchronize(dev)
        dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=reduce_device(dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    elapsed = timed(args.steps)
    # the same step ending in host memory: each owner downloads its slice into pinned
    # memory (never `value`)
    host = torch.empty(D.slice_words(wl.m, world), dtype=torch.int64).pin_memory()
    step(host)
    host_steps = max(1, min(args.steps, 3))
    host_ms = timed(host_steps, host) / host_steps * 1e3
    value = wl.n * args.steps / elapsed / 1e6
    B = algorithmic_bytes(wl.n, wl.key_len, wl.n * wl.key_len, wl.m, False)
    achieved = B / (elapsed / args.steps) / 1e9 / world  # per GPU
    res = {"metric": "bloom-filter build Mkeys/s (device-resident, k=10 cooperative), 1/2/4/8 GPU",
           "value": round(value, 3), "unit": "Mkeys/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
           "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u64",
           "data": "synthetic (device-generated random 32-byte keys)",
           "config": {"workload": wl.name, "keys_total": wl.n, "key_bytes": wl.key_len, "m": wl.m,
                      "k": wl.k, "h2_seed": seed, "parallelism": (f"cooperative x{world}: key shards + all-to-all OR "
                                      "reduce-scatter; each rank keeps its owned slice") if world > 1 else
                      "one rank: its partial is the whole filter, no collective"},
           "host_ending": {"ms_per_step": round(host_ms, 4),
                           "value": round(wl.n / (host_ms * 1e-3) / 1e6, 3), "unit": "Mkeys/s",
                           "note": "the same step plus each owner's D2H of its word slice into "
                                   "pinned host memory (the filter ends in host memory)"},
           "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                        "kernel": "whole cooperative step per GPU (build + merge collectives)",
                        "algorithmic_bytes_per_launch": B}}
    if world == 1:
        # the one-rank step is the build alone: its measured HBM bytes per step (every
        # bin / re-bin / tile pass) from the committed PMC summary of these kernels
        pmc = latest_profile(wl.name, "pmc")
        res["roofline"]["traffic"] = (pmc or {}).get("hbm_bytes_per_launch")
        res["roofline"]["traffic_source"] = (pmc or {}).get("source")
    if world > 1:
        # one instrumented step (untimed above): per rank, the build, all-to-all, OR
        # kernel and D2H of its owned slice, from events on the step's stream
        marks = []
        D.build_cooperative(keys, None, wl.key_len, n, wl.m, wl.k, seed, args.flavor,
                            all_gather=False, host_out=host, comm_device=comm, marks=marks)
        mine = D.phase_ms(marks)
        names = ("build", "all_to_all", "or_merge", "d2h")
        t = torch.tensor([mine.get(x, -1.0) for x in names], dtype=torch.float64, device=reduce_device(dev))
        per = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(per, t)
        res["ranks"] = rank_diag([{x: round(float(v), 4) for x, v in zip(names, p)} for p in per],
                                 "build")
        res["ranks"]["comm_device"] = comm or "gpu (RCCL over xGMI)"
    if world == 1 and not args.no_rank_share:
        res["per_rank_at_8"] = rank_share_rate(nbm, wl, keys, seed, args.flavor, dev, stream)
    if rank == 0:
        emit(res)
    dist.destroy_process_group()


def rank_share_rate(nbm, wl, keys, seed, flavor, dev, stream, world=8, steps=3):
    """What one rank of an 8-GPU C5 step builds: its 1/8 key range (125M x 32 B)
    into the full-size partial filter (m = 2^32-1, k = 10, overwrite), device-resident
    and timed on its own -- the merge collectives are not in this number."""
    import torch
    from nasp_bloom import distributed as D
    b, e = D.shard_range(wl.n, 0, world)
    n = e - b
    words = torch.empty(nbm.nwords(wl.m), dtype=torch.int64, device=dev)

    def step():
        nbm.build_device(keys, None, wl.key_len, n, wl.m, wl.k, seed, flavor, words,
                         stream=stream, overwrite=True)
    step()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    ms = ev0.elapsed_time(ev1) / steps
    B = algorithmic_bytes(n, wl.key_len, n * wl.key_len, wl.m, False)
    return {"keys": n, "ms": round(ms, 4), "value": round(n / (ms * 1e-3) / 1e6, 3),
            "unit": "Mkeys/s", "frac": round(B / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
            "note": "one rank's share of an 8-GPU C5 step: 1B/8 keys into the full "
                    "2^32-1-bit partial filter, one pass (merge collectives not included)"}


if __name__ == "__main__":
    sys.exit(main() or 0)
