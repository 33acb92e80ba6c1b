"""Multi-GPU builds over torch.distributed (backend "nccl" = RCCL over xGMI).

Two shapes:

* Independent filters (C4, the compaction fan-out): every rank builds its own
  SSTable's filter from its own keys.  No collective on the data path -- see
  `build_independent`.

* One cooperative filter (C5, 1B keys into m = 2^32-1 bits): keys are split into
  contiguous ranges, one per rank; each rank builds a full-size partial filter
  from its range (the OR of the partial filters is exactly the filter of all
  keys, because a Bloom filter is an OR of its keys' bits).  RCCL has no bitwise-
  OR reduction (ncclRedOp_t is sum/prod/max/min/avg), so the merge is a
  reduce-scatter built by hand: one all-to-all of equal word slices (rank j
  receives slice j of every partial; over the xGMI full mesh each peer pair uses
  its own link, (W-1)/W of the filter per rank instead of a ring's 2(W-1)/W over
  one link), then a local W-way OR kernel (nb_or_merge_device) into the owned
  slice, then optionally an all-gather of the owned slices so every rank holds
  the whole filter.

The collective logic takes its build/merge steps as parameters so the same code
is exercised by world-size-2 gloo tests on CPU (tests/test_distributed.py, with
the oracle as the test-side builder); on the GPU the defaults are the HIP kernels.
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist

from .api import build_device, nwords, or_merge_device


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous key range [begin, end) of `rank` (sizes differ by at most 1)."""
    q, r = divmod(n, world)
    begin = rank * q + min(rank, r)
    return begin, begin + q + (1 if rank < r else 0)


def slice_words(m: int, world: int) -> int:
    """Words per rank slice (the filter's ceil(m/64) words padded to world*S)."""
    nw = nwords(m)
    return (nw + world - 1) // world


def _hip_merge(dst: torch.Tensor, recv: torch.Tensor, nsrc: int, stride: int) -> None:
    or_merge_device(dst, recv, dst.numel(), nsrc, stride)


def _mark(marks: list | None, name: str, device, stream=None) -> None:
    """Phase boundary of an instrumented step (bench.py's N > 1 diagnostics): a timing
    event recorded on `stream` (default: the current stream of `device`), appended as
    (name, event)."""
    if marks is not None and torch.device(device).type == "cuda":
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(stream if stream is not None else torch.cuda.current_stream(device))
        marks.append((name, ev))


def phase_ms(marks: list) -> dict:
    """Milliseconds between consecutive marks, keyed by the later mark's name
    (synchronises on the last event)."""
    if not marks:
        return {}
    marks[-1][1].synchronize()
    return {name: round(prev.elapsed_time(ev), 4)
            for (_, prev), (name, ev) in zip(marks[:-1], marks[1:])}


def merge_partials(partial: torch.Tensor, m: int, group=None, all_gather: bool = True,
                   merge_fn: Callable | None = None, exchange_single: bool = False,
                   comm_device=None, marks: list | None = None) -> torch.Tensor:
    """OR-merge every rank's full-size partial filter (int64 tensor of >= world*S
    words, padding zero).  Returns the whole merged filter (all_gather=True) or this
    rank's owned slice of S words (words [rank*S, (rank+1)*S) of the filter).  With
    one rank the partial already is the filter and no collective runs
    (exchange_single=True forces the all-to-all / OR / all-gather sequence anyway, for
    tests of the RCCL path on a one-GPU box).  comm_device: where the exchanged
    slices live for the collectives (default: the partial's device, i.e. RCCL over
    xGMI); "cpu" routes them through host copies, so a gloo group -- e.g. ranks that
    share one GPU -- runs the same sequence with the HIP build and OR kernels.
    marks: a list that receives a timing event after each phase ("all_to_all",
    "or_merge", "all_gather"), see phase_ms."""
    world = dist.get_world_size(group)
    S = slice_words(m, world)
    if partial.numel() < world * S:
        raise ValueError("partial filter must be padded to world * slice_words(m) words")
    if world == 1 and not exchange_single:
        return partial[:S]
    cd = partial.device if comm_device is None else torch.device(comm_device)
    send = partial[: world * S].contiguous()
    send_c = send if cd == send.device else send.to(cd)
    recv_c = torch.empty_like(send_c)
    dist.all_to_all_single(recv_c, send_c, group=group)     # recv[j*S:(j+1)*S] = slice of rank j
    recv = recv_c if cd == partial.device else recv_c.to(partial.device)
    _mark(marks, "all_to_all", partial.device)
    owned = torch.zeros(S, dtype=partial.dtype, device=partial.device)
    (merge_fn or _hip_merge)(owned, recv, world, S)
    _mark(marks, "or_merge", partial.device)
    if not all_gather:
        return owned
    owned_c = owned if cd == partial.device else owned.to(cd)
    full_c = torch.empty(world * S, dtype=partial.dtype, device=cd)
    dist.all_gather_into_tensor(full_c, owned_c, group=group)
    full = full_c if cd == partial.device else full_c.to(partial.device)
    _mark(marks, "all_gather", partial.device)
    return full


def build_cooperative(keys: torch.Tensor, offsets: torch.Tensor | None, key_len: int, n: int,
                      m: int, k: int, seed: int, flavor: int, group=None,
                      all_gather: bool = True, build_fn: Callable | None = None,
                      merge_fn: Callable | None = None, stream=None,
                      exchange_single: bool = False, comm_device=None,
                      host_out: torch.Tensor | None = None,
                      marks: list | None = None) -> torch.Tensor:
    """Cooperative single-filter build.  `keys`/`offsets` hold THIS rank's key range
    (offsets relative to `keys`, n+1 entries; or fixed key_len).  Every rank passes
    the same (m, k, seed, flavor).  all_gather=False leaves each rank with its owned
    slice only (words [rank*S, (rank+1)*S), S = slice_words(m, world)); with
    `host_out` (a host tensor of >= S int64 words, pinned for an asynchronous copy)
    that slice is downloaded into it -- the filter then ends in host memory, each
    owner holding its part of SSTable::build's filter block (per-slice
    D2H instead of an all-gather).  The call returns once that download has landed
    (an event recorded behind the copy is waited for), so the caller may write the
    returned host slice to disk at once.  marks: timing events after each phase
    ("build", then merge_partials' phases, then "d2h"), see phase_ms."""
    world = dist.get_world_size(group)
    S = slice_words(m, world)
    if build_fn is None:
        # the device build overwrites the filter's words; only the slice padding needs zeros
        partial = torch.empty(world * S, dtype=torch.int64, device=keys.device)
        partial[nwords(m):].zero_()
    else:  # a test-side builder may OR into the words
        partial = torch.zeros(world * S, dtype=torch.int64, device=keys.device)
    # the build runs on `stream` when one is given; the merge's collectives and OR
    # kernel on the current stream, which waits for the build first (a caller's
    # non-current build stream is joined, not raced)
    side = stream is not None and keys.is_cuda and stream != torch.cuda.current_stream(keys.device)
    if side:
        # the other direction too: the side stream waits for the current
        # stream's work -- the keys' producer and the padding memset above -- and the
        # caching allocator learns that `partial` is in use on it
        stream.wait_stream(torch.cuda.current_stream(keys.device))
        partial.record_stream(stream)
    _mark(marks, "start", keys.device, stream if side else None)
    if build_fn is None:
        build_device(keys, offsets, key_len, n, m, k, seed, flavor, partial, stream=stream,
                     overwrite=True)
    else:
        build_fn(keys, offsets, key_len, n, m, k, seed, flavor, partial)
    if side:
        torch.cuda.current_stream(keys.device).wait_stream(stream)
    _mark(marks, "build", keys.device)
    out = merge_partials(partial, m, group=group, all_gather=all_gather and host_out is None,
                         merge_fn=merge_fn, exchange_single=exchange_single,
                         comm_device=comm_device, marks=marks)
    if host_out is not None:
        if host_out.numel() < out.numel():
            raise ValueError("host_out holds fewer words than the owned slice")
        host_out[: out.numel()].copy_(out, non_blocking=host_out.is_pinned())
        if host_out.is_pinned() and out.is_cuda:
            # the copy is asynchronous: wait for it before the host words are handed
            # back -- so bench.py's host_ending phase is a synchronous D2H
            landed = torch.cuda.Event()
            landed.record(torch.cuda.current_stream(out.device))
            landed.synchronize()
        _mark(marks, "d2h", out.device)
        return host_out[: out.numel()]
    return out


def build_independent(keys: torch.Tensor, offsets: torch.Tensor | None, key_len: int, n: int,
                      m: int, k: int, seed: int, flavor: int, words: torch.Tensor,
                      stream=None) -> None:
    """One SSTable filter per rank: a plain device build, no collective."""
    build_device(keys, offsets, key_len, n, m, k, seed, flavor, words, stream=stream,
                 overwrite=True)
