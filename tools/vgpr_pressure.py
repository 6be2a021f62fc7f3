#!/usr/bin/env python3
"""VGPR pressure map of one kernel of a gfx950 assembly listing (build diagnostic).

Backward liveness over the listing's basic blocks (labels, s_branch / s_cbranch_*), VGPR
operands only: the first operand of a VALU / load instruction is its definition, the rest are
uses (stores, v_cmp to SGPR / vcc and v_readlane define no VGPR).  A definition under a partial
exec mask is treated as a full one, so the figure is a lower bound in divergent code, but its
peaks are where the register allocator's pressure is.  Source lines come from the .loc
directives (compile with -gline-tables-only).

usage: vgpr_pressure.py LISTING.s KERNEL_SUBSTRING [--top N] [--min LIVE]
  -> the source lines (file:line) of the instructions with the most live VGPRs, and the
     per-line maximum of live VGPRs, highest first
"""
import collections
import re
import sys

REG1 = re.compile(r"\bv(\d+)\b")
REGN = re.compile(r"\bv\[(\d+):(\d+)\]")
NODEF = ("global_store", "buffer_store", "scratch_store", "flat_store", "ds_write", "ds_store", "v_cmp", "v_readlane",
         "v_readfirstlane", "s_", "global_atomic", "buffer_atomic", "ds_add", "ds_max", "ds_min")
DEFUSE = ("v_writelane",)


def regs(op):
    out = set()
    for a, b in REGN.findall(op):
        out.update(range(int(a), int(b) + 1))
    for a in REG1.findall(op):
        out.add(int(a))
    return out


def parse(path, kern):
    files, fn, loc = {}, None, None
    insts, labels = [], {}
    for line in open(path):
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', line)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
            continue
        m = re.match(r"^(_Z\S+):", line)
        if m:
            if fn and kern in fn:
                break
            fn = m.group(1)
            continue
        if fn is None or kern not in fn:
            continue
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
        if m:
            loc = "%s:%s" % (files.get(m.group(1), m.group(1)), m.group(2))
            continue
        m = re.match(r"^(\.LBB\S+):", line)
        if m:
            labels[m.group(1)] = len(insts)
            continue
        s = line.split(";")[0].strip()
        if not s or s.startswith("."):
            continue
        parts = s.split(None, 1)
        mn, ops = parts[0], (parts[1] if len(parts) > 1 else "")
        opl = [o.strip() for o in ops.split(",")]
        d, u = set(), set()
        if mn.startswith(DEFUSE):
            d = regs(opl[0]); u = set().union(*[regs(o) for o in opl])
        elif mn.startswith(NODEF) or not opl or not opl[0]:
            u = set().union(*[regs(o) for o in opl]) if opl else set()
        else:
            d = regs(opl[0]); u = set().union(*[regs(o) for o in opl[1:]]) if len(opl) > 1 else set()
            if mn.startswith("v_swap"):
                u |= d
        tgt = None
        if mn.startswith("s_branch") or mn.startswith("s_cbranch"):
            tgt = opl[0]
        insts.append((mn, d, u, tgt, loc))
    return insts, labels


def liveness(insts, labels):
    n = len(insts)
    succ = []
    for i, (mn, d, u, tgt, loc) in enumerate(insts):
        s = []
        if tgt in labels:
            s.append(labels[tgt])
        if not (mn.startswith("s_branch") or mn.startswith("s_endpgm") or mn.startswith("s_setpc")) and i + 1 < n:
            s.append(i + 1)
        succ.append(s)
    live_in = [set() for _ in range(n)]
    changed = True
    while changed:
        changed = False
        for i in range(n - 1, -1, -1):
            out = set()
            for j in succ[i]:
                out |= live_in[j]
            new = (out - insts[i][1]) | insts[i][2]
            if new != live_in[i]:
                live_in[i] = new
                changed = True
    return live_in


def main():
    path, kern = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    insts, labels = parse(path, kern)
    live = liveness(insts, labels)
    per = collections.defaultdict(int)
    for i, (mn, d, u, tgt, loc) in enumerate(insts):
        per[loc] = max(per[loc], len(live[i]))
    print("%d instructions, peak live VGPRs %d" % (len(insts), max(len(x) for x in live)))
    for loc, v in sorted(per.items(), key=lambda kv: -kv[1])[:top]:
        print("%5d  %s" % (v, loc))


if __name__ == "__main__":
    main()
