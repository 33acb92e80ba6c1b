"""bench.py's inputs travel to the GPU box: the committed profile summaries it
reads back (roofline.traffic / valu_frac, profiles/*_pmc_*.json and *_sq_*.json)
must not be excluded from the gpurun snapshot by .gpurunignore."""
import fnmatch
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_profiles_read_by_bench_travel():
    pats = [l.strip() for l in open(os.path.join(REPO, ".gpurunignore")) if l.strip()]
    for rel in ("profiles/r02c_pmc_c4.json", "profiles/r02c_sq_c4.json"):
        for p in pats:
            anchored = p.startswith("./")
            pat = p[2:] if anchored else p
            hit = fnmatch.fnmatch(rel, pat) or (anchored and (rel == pat or rel.startswith(pat + "/"))) \
                or (not anchored and fnmatch.fnmatch(os.path.basename(rel), pat))
            assert not hit, f".gpurunignore pattern {p!r} drops {rel}, which bench.py reads"
