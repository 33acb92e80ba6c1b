#!/usr/bin/env python3
"""profiles/INDEX.md: one line per file under profiles/ that the docs or the code
cite (README.md, INTEGRATION.md, tools/README.md, bench.py, tests/,
tools/), with the first place that cites it; `--prune` deletes the uncited ones.

A citation is a profile file name with or without the `profiles/` prefix; shell
brace lists (`r05z_{pmc,sq}_c4.json`) and `*` globs are expanded against profiles/.
bench.py's read-back of the PMC / SQ summaries (`*_pmc_*.json`, `*_sq_*.json`
matching the current kernel source hash) counts as a citation of those files.

  python tools/profile_index.py [--prune]
"""
import argparse
import fnmatch
import glob
import json
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(REPO, "profiles")
SOURCES = ["DESIGN.md", "README.md", "INTEGRATION.md", "tools/README.md", "bench.py",
           "__graft_entry__.py"] + sorted(glob.glob(os.path.join(REPO, "tests", "*.py"))) + \
    sorted(glob.glob(os.path.join(REPO, "tools", "*.py"))) + sorted(glob.glob(os.path.join(REPO, "tools", "*.sh")))
TOKEN = re.compile(r"(?:profiles/)?(r0\d[\w{},.*-]*)")


def expand(tok):
    m = re.search(r"\{([^{}]*)\}", tok)
    if not m:
        return [tok]
    out = []
    for alt in m.group(1).split(","):
        out += expand(tok[:m.start()] + alt + tok[m.end():])
    return out


def kernel_sha():
    import hashlib
    h = hashlib.sha256()
    for f in ("csrc/bloom_kernels.hip", "csrc/bloom_math.h"):
        h.update(open(os.path.join(REPO, "nasp-key-value-engine_amd", f), "rb").read())
    return h.hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prune", action="store_true")
    args = ap.parse_args()
    files = sorted(f for f in os.listdir(PROF) if f != "INDEX.md")
    cited = {}
    for src in SOURCES:
        path = src if os.path.isabs(src) else os.path.join(REPO, src)
        if not os.path.exists(path):
            continue
        rel = os.path.relpath(path, REPO)
        for ln, line in enumerate(open(path, errors="replace"), 1):
            for tok in TOKEN.findall(line):
                for pat in expand(tok.rstrip(".,;:)")):
                    pats = [pat, pat + ".*"] if "." not in pat.split("/")[-1] else [pat]
                    for p in pats:
                        for f in fnmatch.filter(files, p):
                            cited.setdefault(f, f"{rel}:{ln}")
    sha = kernel_sha()
    for f in files:  # bench.py's read-back of the current kernels' counter summaries
        if re.search(r"_(pmc|sq)_.*\.json$", f) and f not in cited:
            try:
                if json.load(open(os.path.join(PROF, f))).get("kernel_source_sha") == sha:
                    cited[f] = "bench.py latest_profile (current kernel source)"
            except Exception:  # noqa: BLE001
                pass
    lines = ["# profiles/ index", "",
             "Every file kept here is cited by the docs or read by the code; the first citing",
             "place is listed (regenerate with `python tools/profile_index.py`).  Recipes:",
             "`tools/README.md`; a file's name starts with the round (`r06*` = round 6).", "",
             "| file | cited at |", "|---|---|"]
    lines += [f"| `{f}` | {cited[f]} |" for f in files if f in cited]
    open(os.path.join(PROF, "INDEX.md"), "w").write("\n".join(lines) + "\n")
    unc = [f for f in files if f not in cited]
    print(f"{len(cited)} cited, {len(unc)} uncited of {len(files)}")
    if args.prune:
        for f in unc:
            p = os.path.join(PROF, f)
            if os.path.isdir(p):
                import shutil
                shutil.rmtree(p)
            else:
                os.remove(p)
        print("pruned", len(unc))
    else:
        for f in unc[:400]:
            print("uncited:", f)


if __name__ == "__main__":
    main()
