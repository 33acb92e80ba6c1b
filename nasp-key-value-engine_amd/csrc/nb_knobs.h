// nb_knobs.h -- the library's A/B and diagnostic switches.  None of them changes a
// filter's bits; they select between equivalent build paths (for same-box A/Bs and
// for the parity tests that pin every path), or inject device failures (for the
// drop-in classes' fallback tests).
//
// The process environment is read once, the first time any knob is consulted
// (nb_knobs.cpp holds the library's only getenv); afterwards nb_set_knob()
// (include/nasp_bloom.h) changes a value in place.  Values are atomics, so a
// build running on another thread sees either the old or the new value, never a
// torn one -- unlike getenv racing setenv.
#pragma once

#include <stdint.h>

namespace nb {

enum Knob : int {
    kKnobBuildPath,     // NB_BUILD_PATH     0 auto | 1 "atomic" | 2 "tiled"
    kKnobPack,          // NB_PACK           1: packed 21-bit bucket entries (0: 32-bit)
    kKnobTileBits,      // NB_TILE_BITS      0: tile-size policy, else log2 bits per tile
    kKnobShards,        // NB_SHARDS         bucket cursor shards (8)
    kKnobChunkKeys,     // NB_CHUNK_KEYS     0: chunk policy, else keys per bin/tile pass
    kKnobTwoLevel,      // NB_TWO_LEVEL      1: super tiles + re-bin for T > 2048 tiles
    kKnobPack5,         // NB_PACK5          1: pass-1 entries five per 16 bytes
    kKnobEntry32,       // NB_ENTRY32        1: 32-bit entries instead of u16 for small tiles
    kKnobRank,          // NB_RANK           1: indices + ranks kept in registers (k <= 16)
    kKnobFixed32,       // NB_FIXED32        1: register path for 16-byte-aligned 32-byte keys
    kKnobFpMod,         // NB_FPMOD          1: f64-quotient remainders
    kKnobKExact,        // NB_KEXACT         1: bin kernels specialised for k = 7 / 10
    kKnobBinWide,       // NB_BIN_WIDE       1: bin blocks by shape (2 304 keys for 16-byte
                        //                   keys at k = 7 -- 1 024, three per CU, when the
                        //                   filter has <= 384 tiles -- and 1 792 for
                        //                   32-byte keys at k = 10 -- 1 152, three per CU,
                        //                   for <= 384 tiles or two-level pass 1); 2 / 3:
                        //                   force 1 024 / 2 304, 4: force 1 152; 0: the
                        //                   2 048-key (1 024 for k = 10) blocks
    kKnobShardedStage,  // NB_SHARDED_STAGE  1: nb_build_sharded stages every merge source
    kKnobOverlap,       // NB_OVERLAP        bit field (default 6): & 3 == 1: two-level
                        //                   sub-passes pipelined over two streams (sub-pass
                        //                   s's re-bin beside sub-pass s+1's bin kernel),
                        //                   & 3 == 2: the same, the second stream at high
                        //                   priority; + 4: a pass's first bin kernel does
                        //                   not wait for the previous pass's tile kernel;
                        //                   0: no pipelining
    kKnobSubpasses,     // NB_SUBPASSES      bin + re-bin sub-passes per tile pass (0: 2 for
                        //                   multi-pass builds, 1 for a single pass)
    kKnobTileCount,     // NB_TILE_COUNT     0: counted-tile policy (single-level packed path:
                        //                   a whole number of tile-kernel rounds), 1:
                        //                   power-of-two tiles only, else that many tiles
    kKnobProbePath,     // NB_PROBE_PATH     0 auto | 1 "lane" (one lane per key) | 2 "tiled"
                        //                   | 3 "split" (the tiled probe in two rounds)
    kKnobProbeChunk,    // NB_PROBE_CHUNK    0: tiled-probe pass policy, else keys per pass
    kKnobProbeTiledPct, // NB_PROBE_TILED_PCT auto: the tiled path from this % of the sample
                        //                   present; 0 (default): the policy -- 65 % (55 %
                        //                   for k > 8, 40 % for variable-length keys) when
                        //                   the split path takes part, else 30 %
    kKnobProbeSplitPct, // NB_PROBE_SPLIT_PCT auto, k > 2: the split path from this % present
                        //                   up to the tiled threshold; 0 (default): the
                        //                   policy, 7 % for 16-/32-byte keys at k <= 8, 18 %
                        //                   otherwise; > 100, or >= the tiled threshold:
                        //                   never split (the two-way choice at 30 %)
    kKnobProbeEntry,    // NB_PROBE_ENTRY    tiled-probe bucket entries: 32 = a 32-bit word
                        //                   per lookup (key-in-block id | in-tile offset)
                        //                   behind one header word per run holding the bin
                        //                   block; 64 = key << 32 | offset (rounds 3-5);
                        //                   0 (default): 32 for the one-round tiled path,
                        //                   64 for the split path
    kKnobProbeBinGrid,  // NB_PROBE_BIN_GRID auto's gated tiled-probe bin kernels: blocks per
                        //                   CU of their looping grid (0: the policy, 2)
    kKnobProbeHostPick, // NB_PROBE_HOST_PICK auto outside stream capture: 0 (default) the
                        //                   sample's count stays on the device and every
                        //                   path is launched gated (no host wait); 1: the
                        //                   host reads the count back and launches only
                        //                   the chosen path (rounds 3-5)
    kKnobProbeKPT,      // NB_PROBE_KPT      one-round E32 tiled probe: keys per bin thread
                        //                   (0 the policy: 2 at k = 7 when two blocks fit a
                        //                   CU; 1 / 2 force, 2 at k = 7 only)
    kKnobFailBuilds,    // NB_FAIL_BUILDS    fault injection: the next N device builds fail
                        //                   with NB_ERR_HIP before launching anything
    kKnobFailMerkles,   // NB_FAIL_MERKLES   the same for device Merkle trees
    kKnobCount
};

uint64_t knob(Knob k);
// Fault injection: true (and one injected failure consumed) when the knob is > 0.
bool knob_take(Knob k);

}  // namespace nb
