#!/usr/bin/env python3
"""Audit the gfx950 code of libmme.so for two hazards that hipcc does not pad inside inline asm:
(1) the one round 5 found in the persistent fp8 GEMM (mx12): a VALU write of an SGPR (v_readlane / v_readfirstlane: SGPR-spill reloads, uniform values) followed, within
5 wait states, by a VMEM instruction that reads that SGPR (descriptor, soffset or saddr). The hardware needs
the 5 wait states; hipcc inserts them for the instructions it generates, but not for an inline-asm consumer,
so a hit in the final code object is always an unpadded inline-asm load (stale soffset -> wrong data, on
some waves of some launches); (2) an SALU write of M0 immediately followed by an LDS-DMA load, which
takes its LDS destination from M0 and needs one wait state after the write.

    python tools/asm_hazard_audit.py [path/to/libmme.so]        # exit 1 on any hit
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
VMEM = re.compile(r"^(buffer_|global_|flat_|scratch_)")


def code_objects(lib: str, tmp: str):
    """The gfx950 code objects bundled in `lib` (extracted into tmp)."""
    dst = os.path.join(tmp, os.path.basename(lib))
    shutil.copy(lib, dst)
    subprocess.run([OBJDUMP, "--offloading", dst], check=True, capture_output=True, cwd=tmp)
    return sorted(os.path.join(tmp, f) for f in os.listdir(tmp) if "amdgcn" in f and "gfx950" in f)


def _sgprs(operands: str):
    out = set(int(x) for x in re.findall(r"\bs(\d+)\b", operands))
    for a, b in re.findall(r"s\[(\d+):(\d+)\]", operands):
        out.update(range(int(a), int(b) + 1))
    return out


def audit_text(text: str):
    """[(function, instruction index, 'v_readlane ... -> vmem ...')] for every unpadded pair in a disassembly
    (llvm-objdump -d) or compiler assembly listing."""
    lines, fn = [], "?"
    for raw in text.split("\n"):
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", raw) or re.match(r"^(_Z\S+):", raw)
        if m:
            fn = m.group(1)
            continue
        ins = raw.split("//")[0].strip()
        if not ins or ins.startswith((";", ".")) or ins.endswith(":"):
            continue
        lines.append((fn, ins))
    hits = []
    for i, (fn, ins) in enumerate(lines):
        # an SALU write of M0 directly followed by an LDS-DMA load (which takes its LDS base from M0): 1 wait state
        if re.match(r"s_(mov|add|sub)_[ub]32 m0\b", ins) and i + 1 < len(lines):
            nxt = lines[i + 1][1]
            if re.match(r"(buffer_load_\w+ .* lds$|global_load_lds_)", nxt):
                hits.append((fn, i, f"{ins}  ->  {nxt}"))
        m = re.match(r"v_read(?:first)?lane_b32 s(\d+)", ins)
        if not m:
            continue
        sg, waits = int(m.group(1)), 0
        for j in range(i + 1, min(i + 8, len(lines))):
            fn2, nxt = lines[j]
            op, _, rest = nxt.partition(" ")
            if VMEM.match(op) and sg in _sgprs(rest):
                hits.append((fn, i, f"{ins}  ->  {nxt}"))
                break
            if re.match(r"s(\d+)\b", rest) and int(re.match(r"s(\d+)", rest).group(1)) == sg and not VMEM.match(op):
                break  # the SGPR is rewritten first
            n = re.match(r"s_nop (\d+)", nxt)
            waits += int(n.group(1)) + 1 if n else 1
            if waits >= 5:
                break
    return hits


def audit_lib(lib: str):
    hits = []
    with tempfile.TemporaryDirectory() as tmp:
        for obj in code_objects(lib, tmp):
            dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", obj], check=True, capture_output=True, text=True).stdout
            hits += audit_text(dis)
    return hits


if __name__ == "__main__":
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(root, "multimodal-embedding_amd", "mme", "libmme.so")
    hits = audit_lib(lib)
    for fn, i, what in hits[:40]:
        print(f"{fn[:90]}  #{i}: {what}")
    print(f"{len(hits)} unpadded hazard pairs (VALU SGPR write -> VMEM read, M0 write -> LDS-DMA) in {lib}")
    sys.exit(1 if hits else 0)
