#!/usr/bin/env python3
"""Audit the gfx950 code of libmme.so for two hazards that hipcc does not pad inside inline asm:
(1) the one round 5 found in the persistent fp8 GEMM (mx12): a VALU write of an SGPR (v_readlane / v_readfirstlane: SGPR-spill reloads, uniform values; also v_cmp_*_e64 into SGPRs and VOP3b carry-outs) followed, across branches, within
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


# VALU instructions whose SECOND operand is an SGPR (pair) they write: the VOP3b carry / scale outputs
CARRY_OUT = re.compile(r"^v_(add|sub|subrev)_co_u32|^v_(addc|subb|subbrev)_co_u32|^v_div_scale_|^v_mad_(u64_u32|i64_i32)")
BRANCH = re.compile(r"^s_(branch|cbranch_\w+)$")


def _valu_sgpr_writes(op: str, rest: str):
    """SGPRs a VALU instruction writes: its destination (v_readlane / v_readfirstlane / v_cmp_*_e64 /
    v_cndmask ... with an SGPR first operand) or a VOP3b carry-out (second operand)."""
    if not op.startswith("v_"):
        return set()
    ops = [o.strip() for o in rest.split(",")]
    out = set()
    if ops and re.fullmatch(r"s(\d+)|s\[\d+:\d+\]", ops[0]):
        out |= _sgprs(ops[0])
    if CARRY_OUT.match(op) and len(ops) > 1 and re.fullmatch(r"s(\d+)|s\[\d+:\d+\]", ops[1]):
        out |= _sgprs(ops[1])
    return out


def _parse(text: str):
    """[(function, address or None, instruction)] plus {label or address: index} for branch targets."""
    lines, fn, targets = [], "?", {}
    for raw in text.split("\n"):
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", raw) or re.match(r"^(_Z\S+):", raw)
        if m:
            fn = m.group(1)
            continue
        lab = re.match(r"^\s*(\.?L\w+):", raw)
        if lab:
            targets[lab.group(1)] = len(lines)
            continue
        code, _, comment = raw.partition("//")
        ins = code.strip()
        if not ins or ins.startswith((";", ".")) or ins.endswith(":"):
            continue
        am = re.match(r"\s*([0-9A-Fa-f]{6,}):", comment)
        addr = int(am.group(1), 16) if am else None
        if addr is not None:
            targets[addr] = len(lines)
        lines.append((fn, addr, ins))
    return lines, targets


def _branch_target(lines, targets, i):
    """Index of the instruction a branch at i jumps to (objdump: pc + 4 + 4 * simm16; listing: a label)."""
    _, addr, ins = lines[i]
    arg = ins.split(None, 1)[1].strip() if " " in ins else ""
    if re.fullmatch(r"-?\d+", arg) and addr is not None:
        imm = int(arg)
        imm = imm - 65536 if imm >= 32768 else imm   # objdump prints simm16 unsigned
        return targets.get(addr + 4 + 4 * imm)
    return targets.get(arg)


def audit_text(text: str):
    """[(function, instruction index, 'writer ... -> vmem ...')] for every unpadded pair in a disassembly
    (llvm-objdump -d, branch targets from the encoded offsets) or a compiler assembly listing (labels).

    Hazard 1: a VALU instruction writing an SGPR (v_readlane / v_readfirstlane, v_cmp_*_e64 into an SGPR
    pair, VOP3b carry-outs) followed within 5 wait states by a VMEM instruction that reads it. Each
    instruction issued is one wait state, s_nop N is N + 1. The scan FOLLOWS control flow: an
    unconditional branch continues at its target, a conditional one on both paths, so a VMEM read at a
    branch target is seen; a branch whose target cannot be resolved is reported as a hit (unknown).
    Hazard 2: an SALU write of M0 directly followed by an LDS-DMA load (one wait state)."""
    lines, targets = _parse(text)
    hits = []
    for i, (fn, _, ins) in enumerate(lines):
        if re.match(r"s_(mov|add|sub)_[ub]32 m0\b", ins) and i + 1 < len(lines):
            nxt = lines[i + 1][2]
            if re.match(r"(buffer_load_\w+ .* lds$|global_load_lds_)", nxt):
                hits.append((fn, i, f"{ins}  ->  {nxt}"))
        op, _, rest = ins.partition(" ")
        written = _valu_sgpr_writes(op, rest)
        if not written:
            continue
        work, seen, found = [(i + 1, 0)], set(), None
        while work and found is None:
            j, waits = work.pop()
            while j is not None and j < len(lines) and waits < 5 and (j, waits) not in seen:
                seen.add((j, waits))
                nxt = lines[j][2]
                op2, _, rest2 = nxt.partition(" ")
                if VMEM.match(op2) and written & _sgprs(rest2):
                    found = f"{ins}  ->  {nxt}"
                    break
                if op2 == "s_endpgm":
                    break
                dst = re.match(r"(s\d+|s\[\d+:\d+\])", rest2)
                if dst and not VMEM.match(op2) and not op2.startswith(("s_cmp", "s_bitcmp")) and \
                        _sgprs(dst.group(1)) >= written:
                    break  # every written SGPR is overwritten first
                n = re.match(r"s_nop (\d+)", nxt)
                waits += int(n.group(1)) + 1 if n else 1
                if BRANCH.match(op2):
                    t = _branch_target(lines, targets, j)
                    if t is None:
                        found = f"{ins}  ->  {nxt} (branch target unresolved)"
                        break
                    if op2 == "s_branch":
                        j = t
                        continue
                    work.append((t, waits))
                j += 1
        if found:
            hits.append((fn, i, found))
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
