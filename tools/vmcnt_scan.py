#!/usr/bin/env python3
"""Find loads that a kernel waits for in series: per function of a gfx950 assembly listing (hipcc
--save-temps), count the global / buffer / flat loads (not LDS-DMA) followed within three instructions by
`s_waitcnt vmcnt(0)`. A high count marks a kernel whose loads hipcc's vmcnt bookkeeping serialises (a load in
a per-lane branch waited for inside the branch, constants behind a full drain): DESIGN.md §8 item 5.

    cd /tmp/x && hipcc -O3 -std=c++17 --offload-arch=gfx950 --save-temps -c .../csrc/norm.hip
    python3 tools/vmcnt_scan.py /tmp/x/*-hip-amdgcn-amd-amdhsa-gfx950.s [--top 4]
"""
import re
import sys


def scan(path):
    s = open(path).read()
    out = []
    for m in re.finditer(r"^(_Z\S+):", s, re.M):
        body = s[m.end():]
        body = body[:body.find(".Lfunc_end")]
        lines = [l.strip() for l in body.split("\n") if l.strip() and not l.strip().startswith((".", ";"))]
        n = 0
        for i, l in enumerate(lines):
            if l.startswith(("global_load", "buffer_load", "flat_load")) and " lds" not in l:
                if any(i + k < len(lines) and lines[i + k].startswith("s_waitcnt") and "vmcnt(0)" in lines[i + k]
                       for k in range(1, 4)):
                    n += 1
        out.append((n, m.group(1)))
    return sorted(out, reverse=True)


if __name__ == "__main__":
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 4
    for f in [a for a in sys.argv[1:] if a.endswith(".s")]:
        print(f.split("/")[-1], [(n, name[:90]) for n, name in scan(f)[:top]])
