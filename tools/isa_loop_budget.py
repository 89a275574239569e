"""Per-item instruction budget of a kernel in gfx950 assembly (round 6): extracts the kernel
named by a substring, weights each basic block by TRIP^(loop depth - 1) (the item loop is
depth 1, the chunk loop depth 2), and counts instruction classes.

usage: python tools/isa_loop_budget.py FILE.s NAME_SUBSTRING [TRIP=4] [BASE=1]
(BASE: the loop depth counted once, i.e. the item loop's; 0 when the compiler does not
annotate the item loop as a loop)"""
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from isa_budget import classify  # noqa: E402


def kernel_lines(path, sub):
    lines = open(path).read().split("\n")
    out, on = [], False
    for ln in lines:
        if not on and re.match(r"^_Z\S*:", ln) and sub in ln.split(":")[0]:
            on = True
        elif on and ln.startswith(".Lfunc_end"):
            break
        if on:
            out.append(ln)
    return out


def main():
    path, sub = sys.argv[1], sys.argv[2]
    trip = float(sys.argv[3]) if len(sys.argv) > 3 else 4.0
    base = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    depth = 0
    cnt = {}
    for ln in kernel_lines(path, sub):
        s = ln.strip()
        if ln and not ln[0].isspace() and (s.endswith(":") or ":" in s.split(";")[0]) or s.startswith("; %bb"):
            m = re.search(r"Depth=(\d+)", ln)
            depth = int(m.group(1)) if m else 0
            continue
        if not s or s.startswith((";", ".")):
            continue
        c = classify(s.split()[0])
        if c is None:
            continue
        w = trip ** max(depth - base, 0)
        cnt[c] = cnt.get(c, 0) + w
        if "_dpp" in s.split()[0] or "row_" in s or "quad_perm" in s:
            cnt["dpp"] = cnt.get("dpp", 0) + w
    print(" ".join(f"{k}={v:g}" for k, v in sorted(cnt.items())))


if __name__ == "__main__":
    main()
