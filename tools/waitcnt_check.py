"""Static vmcnt check of gfx950 assembly (round 6, the packed-fp32 divergence of DESIGN.md §6).

For every kernel in a `hipcc -S` listing, a forward dataflow over its basic blocks tracks the
VGPRs that an outstanding VMEM load still has to write: each VMEM instruction ages the loads
before it by one, `s_waitcnt vmcnt(N)` retires every load with N or more VMEM instructions
issued after it (gfx9 returns them in order), and the blocks' states merge conservatively (a
register is pending if it is pending on any incoming path, at its youngest age).  Any
instruction that reads or writes a pending VGPR is reported: a missing wait.

usage: python tools/waitcnt_check.py FILE.s [--only SUBSTR] [--mnemonic-stats]"""
from __future__ import annotations

import re
import sys
from collections import Counter

VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
MAXAGE = 64


def vregs(text):
    out = set()
    for m in VREG.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def is_vmem(op):
    return op.startswith(("buffer_", "global_", "flat_", "scratch_"))


def split_operands(rest):
    rest = rest.split(";")[0].strip()
    parts, depth, cur = [], 0, ""
    for ch in rest:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur.strip())
    return parts


def parse_kernels(path, only=None):
    kernels, cur, name = {}, None, None
    for ln in open(path):
        ln = ln.rstrip("\n")
        m = re.match(r"^(_Z\S+|[A-Za-z_]\w*):\s*(;.*)?$", ln)
        if m and not ln.startswith("."):
            name = m.group(1)
            cur = [] if (only is None or only in name) else None
            if cur is not None:
                kernels[name] = cur
            continue
        if ln.startswith(".Lfunc_end"):
            cur = None
            continue
        if cur is not None:
            cur.append(ln)
    return kernels


def blocks_of(lines):
    blocks, labels = [], {}
    cur = {"label": None, "insts": []}
    for ln in lines:
        s = ln.strip()
        lm = re.match(r"^(\.LBB\w+):", s)
        if lm:
            blocks.append(cur)
            cur = {"label": lm.group(1), "insts": []}
            labels[lm.group(1)] = len(blocks)
            continue
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        cur["insts"].append((op, s))
        if op.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc")):
            blocks.append(cur)
            cur = {"label": None, "insts": []}
    blocks.append(cur)
    blocks = [b for b in blocks if b["insts"] or b["label"]]
    labels = {b["label"]: i for i, b in enumerate(blocks) if b["label"]}
    succ = []
    for i, b in enumerate(blocks):
        last = b["insts"][-1] if b["insts"] else ("", "")
        op = last[0]
        tgt = re.search(r"(\.LBB\w+)", last[1])
        if op == "s_branch":
            succ.append([labels[tgt.group(1)]] if tgt else [])
        elif op.startswith("s_cbranch"):
            succ.append(([labels[tgt.group(1)]] if tgt else []) + ([i + 1] if i + 1 < len(blocks) else []))
        elif op.startswith(("s_endpgm", "s_setpc")):
            succ.append([])
        else:
            succ.append([i + 1] if i + 1 < len(blocks) else [])
    return blocks, succ


def step(state, op, s, report=None):
    """Apply one instruction to `state` (dict vgpr -> age); report hazards via report(reg_set)."""
    rest = s[len(op):]
    ops = split_operands(rest)
    if op == "s_waitcnt":
        m = re.search(r"vmcnt\((\d+)\)", s)
        if m:
            n = int(m.group(1))
            for r in [r for r, a in state.items() if a >= n]:
                del state[r]
        return
    if op.startswith("s_") and not op.startswith("s_waitcnt"):
        return
    touched = vregs(rest.split(";")[0])
    is_load = is_vmem(op) and (("load" in op and " lds" not in s) or
                               ("atomic" in op and (" glc" in s or " sc0" in s)))
    if is_load and ops:
        # a load may overwrite a register an older load still has to write: loads return in order
        touched = vregs(",".join(ops[1:]))
    if report is not None:
        bad = {r for r in touched if r in state}
        if bad:
            report(bad)
    if is_vmem(op):
        for r in list(state):
            state[r] += 1
            if state[r] >= MAXAGE:
                del state[r]
        if is_load and ops:
            for r in vregs(ops[0]):
                state[r] = 0


def merge(a, b):
    out = dict(a)
    for r, x in b.items():
        out[r] = min(out.get(r, MAXAGE), x)
    return out


def check_kernel(lines):
    blocks, succ = blocks_of(lines)
    n = len(blocks)
    inn = [None] * n
    inn[0] = {}
    work = [0]
    while work:
        i = work.pop()
        st = dict(inn[i])
        for op, s in blocks[i]["insts"]:
            step(st, op, s)
        for j in succ[i]:
            new = st if inn[j] is None else merge(inn[j], st)
            if inn[j] is None or new != inn[j]:
                inn[j] = new
                work.append(j)
    hazards = []
    for i in range(n):
        if inn[i] is None:
            continue
        st = dict(inn[i])
        for op, s in blocks[i]["insts"]:
            step(st, op, s, report=lambda bad, s=s, op=op: hazards.append((op, s, sorted(bad))))
    return hazards


def main():
    path = sys.argv[1]
    only = None
    if "--only" in sys.argv:
        only = sys.argv[sys.argv.index("--only") + 1]
    kernels = parse_kernels(path, only)
    total = Counter()
    nk = 0
    for name, lines in kernels.items():
        hz = check_kernel(lines)
        nk += 1
        for op, s, regs in hz:
            total[op] += 1
        if hz:
            print(f"{name[:90]}: {len(hz)} reads/writes of VGPRs with a load pending")
            for op, s, regs in hz[:6]:
                print(f"    {s[:110]}   pending v{regs}")
    print(f"{nk} kernels; hazards by mnemonic: {dict(total)}")


if __name__ == "__main__":
    main()
