"""Static instruction budget of a kernel's gfx950 assembly by line range (round 6).

usage: python tools/isa_budget.py FILE.s START:END[:LABEL[:MULT]] ...
Counts VALU / SALU / MFMA / LDS / VMEM / SMEM / DPP / branch instructions in each range,
multiplied by MULT (e.g. a loop body's trip count)."""
import re
import sys


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith(("s_waitcnt", "s_barrier", "s_nop", "s_cbranch", "s_branch", "s_setprio")):
        return "ctl"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return None


def main():
    lines = open(sys.argv[1]).read().split("\n")
    tot = {}
    for spec in sys.argv[2:]:
        parts = spec.split(":")
        a, b = int(parts[0]), int(parts[1])
        label = parts[2] if len(parts) > 2 else spec
        mult = float(parts[3]) if len(parts) > 3 else 1.0
        cnt = {}
        for ln in lines[a - 1:b]:
            s = ln.strip()
            if not s or s.startswith((";", ".")) or s.endswith(":"):
                continue
            op = s.split()[0]
            c = classify(op)
            if c is None:
                continue
            cnt[c] = cnt.get(c, 0) + mult
            if "_dpp" in op or " row_" in s or "quad_perm" in s:
                cnt["dpp"] = cnt.get("dpp", 0) + mult
        for k, v in cnt.items():
            tot[k] = tot.get(k, 0) + v
        print(f"{label:28s} " + " ".join(f"{k}={v:g}" for k, v in sorted(cnt.items())))
    print(f"{'TOTAL':28s} " + " ".join(f"{k}={v:g}" for k, v in sorted(tot.items())))


if __name__ == "__main__":
    main()
