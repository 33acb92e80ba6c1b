"""Static instruction mix of one bin-kernel instantiation per phase (diagnostic).
Copies csrc/bloom_kernels.hip with asm markers at the phase boundaries, compiles
it for gfx950 to assembly and counts VALU/SALU/LDS/VMEM instructions per region.
usage: python tools/phase_asm.py [mangled-name-substring]"""
import collections
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "nasp-key-value-engine_amd", "csrc")


def main():
    want = sys.argv[1] if len(sys.argv) > 1 else "bloom_bin_kernelILi0ELi2ELi2EtLi1024ELb0ELi8E"
    s = open(os.path.join(CSRC, "bloom_kernels.hip")).read()
    s = s.replace('#include "nb_knobs.h"', f'#include "{CSRC}/nb_knobs.h"')
    s = s.replace('#include "bloom_math.h"', f'#include "{CSRC}/bloom_math.h"')
    s = s.replace('#include "../../include/nasp_bloom.h"', f'#include "{REPO}/include/nasp_bloom.h"')
    s = s.replace("    if (NB_DIAG_STOP(1)) return;", '    asm volatile(";NBMARK phase2");\n    if (NB_DIAG_STOP(1)) return;')
    s = s.replace("    if (NB_DIAG_STOP(2)) return;", '    asm volatile(";NBMARK phase3");\n    if (NB_DIAG_STOP(2)) return;')
    s = s.replace("    if (NB_DIAG_STOP(3)) return;", '    asm volatile(";NBMARK phase4");\n    if (NB_DIAG_STOP(3)) return;')
    os.makedirs("/tmp/nbasm", exist_ok=True)
    open("/tmp/nbasm/k.hip", "w").write(s)
    subprocess.check_call(["hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                           "-S", "/tmp/nbasm/k.hip", "-o", "/tmp/nbasm/k.s"])
    asm = open("/tmp/nbasm/k.s").read()
    m = re.search(r"^(_Z\S*%s\S*):" % re.escape(want), asm, re.M)
    body = asm[m.end():asm.index(".Lfunc_end", m.end())]
    region, cnt = "phase1", collections.Counter()
    for line in body.split("\n"):
        t = line.strip()
        if "NBMARK" in t:
            region = t.split()[-1]
            continue
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        op = t.split()[0]
        cls = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") else
               "lds" if op.startswith("ds_") else
               "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "other")
        cnt[(region, cls)] += 1
        if op in ("v_mul_lo_u32", "v_mad_u64_u32", "v_mul_hi_u32"):
            cnt[(region, "mul")] += 1
    print(m.group(1))
    for k in sorted(cnt):
        print(f"  {k[0]:7s} {k[1]:5s} {cnt[k]}")


if __name__ == "__main__":
    main()
