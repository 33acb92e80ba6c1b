#!/usr/bin/env python3
"""Summarise a rocprofv3 SQ-counter pass of the build kernels (tools/gpu_baseline.sh,
tools/profile_round.sh) into per-kernel averages and a VALU roofline.

  python tools/sq_summary.py <tag> <workload key> <run_counter_collection.csv>
      -> profiles/<tag>_sq_<workload>.json (read by bench.py for roofline.valu_frac)

SQ_INSTS_VALU counts wave-level VALU instructions (summed over the chip).  A wave64
VALU instruction holds its SIMD for 4 cycles, so the VALU floor of a launch is
  SQ_INSTS_VALU x 4 / (1 024 SIMDs x f_clk)
and valu_frac = that floor / the launch's duration.  f_clk is the effective clock
of the launch, GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md, DVFS);
SQ_ACTIVE_INST_VALU (quad-cycles per wave) gives the issue-side view beside it.
"""
import csv
import json
import re
import sys
from collections import defaultdict

SIMDS = 1024


def short(name):
    m = re.search(r"([A-Za-z_][A-Za-z_0-9]*(<[^()]*>)?)\(", name)
    return m.group(1) if m else name


def summarise(path, keys_per_build):
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        name = short(r["Kernel_Name"])
        if "bloom_" not in name:
            continue
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[name][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {}
    for name, cs in acc.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        t = sum(dur[name].values()) / len(dur[name])
        d = {"dispatches": len(dur[name]), "avg_duration_us": round(t * 1e6, 2)}
        d.update({c: round(v, 1) for c, v in avg.items()})
        if "GRBM_GUI_ACTIVE" in avg and t > 0:
            f = avg["GRBM_GUI_ACTIVE"] / 8 / t
            d["eff_clock_ghz"] = round(f / 1e9, 3)
            if "SQ_INSTS_VALU" in avg:
                floor = avg["SQ_INSTS_VALU"] * 4 / (SIMDS * f)
                d["valu_floor_us"] = round(floor * 1e6, 2)
                d["valu_frac"] = round(floor / t, 4)
        if "SQ_INSTS_VALU" in avg and keys_per_build:
            d["valu_insts_per_key_lane"] = round(avg["SQ_INSTS_VALU"] * 64 / keys_per_build, 1)
        if "SQ_ACTIVE_INST_VALU" in avg and "SQ_WAVE_CYCLES" in avg and avg["SQ_WAVE_CYCLES"]:
            d["valu_active_per_wave_cycle"] = round(avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"], 4)
        if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_INSTS_LDS" in avg and avg["SQ_INSTS_LDS"]:
            d["lds_conflict_cycles_per_inst"] = round(avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_INSTS_LDS"], 3)
        out[name] = d
    return out


def main(tag, wl_key, path):
    import os
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "nasp-key-value-engine_amd"))
    sys.path.insert(0, repo)
    from nasp_bloom import synth
    from bench import kernel_sha
    wl = synth.WORKLOADS[wl_key]
    ks = summarise(path, wl.n)
    # one bench build = the bin kernel (+ re-bin) + the overwrite-mode tile kernel
    used = [k for k in ks if "bloom_bin_kernel" in k or "bloom_rebin_kernel" in k
            or ("tile_or" in k and "true" in k)]
    floor = sum(ks[k].get("valu_floor_us", 0) for k in used)
    dur = sum(ks[k]["avg_duration_us"] for k in used)
    out = {"workload": wl.name, "kernel_source_sha": kernel_sha(), "build_kernels": used,
           "valu_frac_build": round(floor / dur, 4) if dur else None, "kernels": ks,
           "source": f"profiles/{tag}_sq_{wl_key}.json (rocprofv3 --pmc SQ_* pass, "
                     "tools/sq_summary.py)"}
    dst = os.path.join(repo, "profiles", f"{tag}_sq_{wl_key}.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(dst, out["valu_frac_build"])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
