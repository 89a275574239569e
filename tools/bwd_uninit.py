"""Which backward scratch region is read before it is written (the first-call difference found
by tools/bwd_nondet.py: run 0 of a process differs, runs 1.. agree)?  For each region of the
backward scratch (bptt.hip BpttLayout, then warp_cost.hip CostBwdLayout) the whole scratch is
zeroed, that region filled with NaN bytes, and the backward run once: a region whose NaNs reach
dL/dref, dL/dx or the parameter gradients is read before this run writes it."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402

from aarmvs import _lib, ops, synthetic as syn  # noqa: E402

B, N, H, W, D = 1, 3, 96, 128, 20
nsrc, HW, G = N - 1, H * W, 16


def al(x):
    return (x + 255) // 256 * 256


def regions():
    px = [HW, HW // 4, HW // 16, HW // 4, HW]
    hid = [16, 16, 16, 16, 8]
    sizes = []
    for k in range(5):
        sizes += [(f"gh{k}", B * px[k] * hid[k] * 4), (f"gc{k}", B * px[k] * hid[k] * 4),
                  (f"gz{k}", G * B * px[k] * 4 * hid[k] * 4)]
    sizes += [("zmax", 5 * G * 4), ("gr0", B * (HW // 4) * 64), ("gr1", B * HW * 64), ("gr0b", B * (HW // 4) * 64)]
    for q in range(2):
        for k in range(2):
            sizes.append((f"gskip{q}{k}", B * px[k] * 64))
    sizes += [("gpool0", B * (HW // 4) * 64), ("gpool1", B * (HW // 16) * 64),
              ("gu0", G * B * (HW // 4) * 64), ("gu1", G * B * HW * 64), ("gx", G * B * HW * 32 * 4)]
    nblk = min(512, (HW + 1023) // 1024)
    sizes += [("gnb_part0", G * B * nblk * 36 * 8), ("gnb_part1", G * B * nblk * 36 * 8)]
    raw = _lib.lib().aarmvs_param_count()
    sizes += [("gacc", raw * 8)]
    out, off = [], 0
    for name, n in sizes:
        out.append((name, off, n))
        off = al(off + n)
    return out


sc = syn.scene(B, N, H, W, D, seed=3)
P = {k: torch.from_numpy(v).cuda() for k, v in syn.sweep_weights(5).items()}
sw = ops.DepthSweep(P, "cuda")
f = torch.from_numpy(sc["features"]).cuda()
proj = torch.from_numpy(sc["proj_matrices"])
dv = torch.from_numpy(sc["depth_values"])
ref, srcs = f[0], [f[v] for v in range(1, N)]
rec = sw.record_buffers(B, H, W, D, "cuda", nsrc=nsrc)
rel = sw.relative(proj[:, 0], [proj[:, v] for v in range(1, N)], B)
cost = torch.empty(B, D, H, W, device="cuda")
sw(ref, srcs, proj[:, 0], [proj[:, v] for v in range(1, N)], dv, want_depth=False, cost_out=cost,
   rel=rel, record=rec)
torch.manual_seed(0)
g = torch.randn_like(cost)
total = _lib.lib().aarmvs_backward_scratch_bytes(B, H, W, nsrc)
key = ("bwd", B, H, W, nsrc)
regs = regions()
bend = regs[-1][1] + regs[-1][2]
regs.append(("bptt_tail(wpart,rseg)", al(bend), 0))
import bwd_nondet as BN  # noqa: E402  (cost layout)
CL, cbytes = BN.cost_layout()
breg = total - cbytes
regs[-1] = ("bptt_tail(wpart,rseg)", al(bend), breg - al(bend))
for k, (o, n) in CL.items():
    regs.append(("cost:" + k, breg + o, n))
for name, off, n in regs:
    s = torch.zeros(total, dtype=torch.uint8, device="cuda")
    s[off: off + n] = 0xFF
    sw._ws[key] = s
    g_ref, g_src, g_par, g_x = sw.backward(ref, srcs, rel, dv, rec, g, want_grad_x=True)
    torch.cuda.synchronize()
    bad = {nm: int((~torch.isfinite(t)).sum()) for nm, t in
           (("ref", g_ref), ("x", g_x), ("params", torch.cat([v.reshape(-1) for v in g_par.values()])),
            ("src", torch.stack(g_src)))}
    flag = "READ-BEFORE-WRITE" if any(bad.values()) else "ok"
    print(f"{name:24s} {n:>10d} B  {flag}  {bad if any(bad.values()) else ''}", flush=True)
