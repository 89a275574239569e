"""Run-to-run bisection of the backward's nondeterminism: one recorded
forward, then the backward R times on the same inputs and record; per run a SHA-256 of
dL/dref, the parameter gradients, dL/dx and of the cost-slice backward's scratch buffers left
by the last group (the omega weights wo, dL/dt1, dL/do, the per-view dL/dref accumulators grefv
and the source-feature accumulators gsrc8).  Prints which digests vary across runs.
usage: python tools/bwd_nondet.py [R] [D]   (AARMVS_BWD_PIPE=0 for the one-stream schedule)"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")]
import torch  # noqa: E402

from aarmvs import _lib, ops, synthetic as syn  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 8
B, N, H, W = 1, 3, 96, 128
D = int(sys.argv[2]) if len(sys.argv) > 2 else 20
nsrc, HW, G = N - 1, 96 * 128, 16


def al(x):
    return (x + 255) // 256 * 256


def cost_layout():
    pblk = max(1, min((HW + 4095) // 4096, 64))
    nt = ((W + 15) // 16) * ((H + 15) // 16)
    sizes = [("go", G * B * nsrc * HW * 4), ("wo", G * B * nsrc * HW * 4), ("gt1", G * B * nsrc * HW * 16),
             ("gsum", G * B * nsrc * 6 * 8), ("part", G * B * nsrc * pblk * 32 * 8),
             ("wpart", 4 * nsrc * B * nt * 288 * 4), ("wseg", 64 * 1152 * 8),
             ("gsrc8", nsrc * B * 32 * HW * 4), ("grefv", nsrc * B * 32 * HW * 4),
             ("gsrc64", nsrc * B * 32 * HW * 8), ("gmax", 256)]
    off, L = 0, {}
    for k, n in sizes:
        L[k] = (off, n)
        off = al(off + n)
    return L, off


def bptt_sets():
    """Offsets of the two group buffer sets in the backward scratch (bptt.hip bptt_layout)."""
    hid = [16, 16, 16, 16, 8]
    px = [HW, HW // 4, HW // 16, HW // 4, HW]
    off = 0
    for k in range(5):
        off = al(off + B * px[k] * hid[k] * 4)   # gh
        off = al(off + B * px[k] * hid[k] * 4)   # gc
    nblk = min(512, (HW + 1023) // 1024)
    sets = []
    for q in range(2):
        d = {}
        for k in range(5):
            d[f"gz{k}"] = (off, G * B * px[k] * 4 * hid[k] * 4)
            off = al(off + G * B * px[k] * 4 * hid[k] * 4)
        d["zmax"] = (off, 5 * G * 4)
        off = al(off + 5 * G * 4)
        zp_n = (B * px[0] * 4 + 255) // 256   # bptt.hip: the largest gate grid
        d["zpart"] = (off, 5 * G * zp_n * 4)
        off = al(off + 5 * G * zp_n * 4)
        d["gu0"] = (off, G * B * (HW // 4) * 64)
        off = al(off + G * B * (HW // 4) * 64)
        d["gu1"] = (off, G * B * HW * 64)
        off = al(off + G * B * HW * 64)
        d["gx"] = (off, G * B * HW * 128)
        off = al(off + G * B * HW * 128)
        for j in range(2):
            d[f"gnb{j}"] = (off, G * B * nblk * 36 * 8)
            off = al(off + G * B * nblk * 36 * 8)
        sets.append(d)
    return sets


def where(a, b):
    """Where run b differs from run 0: dL/dx per plane (count, max |diff|, pixels), dL/dref
    per channel, dL/dsrc per view, and the parameter tensors that differ."""
    x0, x1 = a["x"], b["x"]   # [D][B][H][W][32]
    dx = (x0 != x1)
    if dx.any():
        planes = dx.reshape(dx.shape[0], -1).sum(1)
        pl = [(int(i), int(planes[i]), float((x0[i] - x1[i]).abs().max())) for i in range(len(planes)) if planes[i]]
        top = pl[-1][0]
        xm = float(x0[top].abs().max())
        rel = ((x0[top] - x1[top]).abs() / x0[top].abs().clamp_min(xm * 1e-3)).max()
        print(f"   x: {len(pl)} planes differ, d = {[p[0] for p in pl]}; top plane {pl[-1]}; "
              f"max {max(p[2] for p in pl):.2e}; top plane max|x| {xm:.2e}, max rel diff {float(rel):.2e}",
              flush=True)
        i = pl[0][0]
        idx = dx[i].nonzero()[:8].tolist()
        print("   x first plane diffs at [b,y,x,c]:", idx, flush=True)
    for name in ("ref", "src"):
        t0, t1 = a[name], b[name]
        m = t0 != t1
        if m.any():
            nz = m.nonzero()
            print(f"   {name}: n={int(m.sum())} max={float((t0 - t1).abs().max()):.3e} "
                  f"first={nz[:6].tolist()}", flush=True)
    ps = [k for k in a["params"] if not torch.equal(a["params"][k], b["params"][k])]
    if ps:
        print(f"   params differ: {len(ps)} tensors, e.g. {ps[:3]}", flush=True)


def main():
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
    CL, cbytes = cost_layout()
    total = _lib.lib().aarmvs_backward_scratch_bytes(B, H, W, nsrc)
    breg = total - cbytes
    runs = []
    for r in range(R):
        g_ref, g_src, g_par, g_x = sw.backward(ref, srcs, rel, dv, rec, g, want_grad_x=True)
        torch.cuda.synchronize()
        scratch = sw._ws[("bwd", B, H, W, nsrc)]
        d = {}
        for name, ts in (("ref", [g_ref]), ("params", [g_par[k] for k in sorted(g_par)]), ("x", [g_x]),
                         ("src", g_src)):
            h = hashlib.sha256()
            for t in ts:
                h.update(t.detach().cpu().contiguous().numpy().tobytes())
            d[name] = h.hexdigest()[:12]
        for k in ("wo", "gt1", "go", "grefv", "gsrc8", "gsum"):
            o, n = CL[k]
            d["s:" + k] = hashlib.sha256(scratch[breg + o: breg + o + n].cpu().numpy().tobytes()).hexdigest()[:12]
        for q, st in enumerate(bptt_sets()):
            for name in ("zmax", "gz0", "gz4", "gx"):
                o, n = st[name]
                d[f"b{q}:{name}"] = hashlib.sha256(scratch[o: o + n].cpu().numpy().tobytes()).hexdigest()[:8]
        o, n = bptt_sets()[0]["zmax"]
        zm = scratch[o: o + n].cpu().view(torch.float32).reshape(5, G)
        if r == 0:
            zm0 = zm.clone()
        elif not torch.equal(zm, zm0):
            dd = (zm != zm0).nonzero().tolist()
            print("   zmax set 0 differs at (cell, slot):", dd[:10],
                  [(float(zm0[c, k]), float(zm[c, k])) for c, k in dd[:4]], flush=True)
        if os.environ.get("AARMVS_BWD_TRACE"):
            import ctypes
            import numpy as np
            buf = np.zeros((D, 32), dtype=np.uint64)
            lib = _lib.lib()
            lib.aarmvs_debug_bwd_trace.restype = ctypes.c_int
            lib.aarmvs_debug_bwd_trace(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(buf.nbytes))
            if r == 0:
                trace0 = buf.copy()
            else:
                diff = [(dd, sl) for dd in range(D - 1, -1, -1) for sl in range(32) if buf[dd, sl] != trace0[dd, sl]]
                if diff:
                    print(f"   trace: {len(diff)} entries differ; first (plane, slot): {diff[:6]}", flush=True)
        runs.append(d)
        print(r, " ".join(f"{k}={v}" for k, v in d.items()), flush=True)
        cur = {"x": g_x.detach().cpu().clone(), "ref": g_ref.detach().cpu().clone(),
               "src": torch.stack([t.detach().cpu() for t in g_src]),
               "params": {k: v.detach().cpu().clone() for k, v in g_par.items()}}
        if r == 0:
            first = cur
        else:
            where(first, cur)
    for k in runs[0]:
        vals = sorted(set(r[k] for r in runs))
        print(f"{k:8s} {'VARIES' if len(vals) > 1 else 'same'} ({len(vals)} distinct)")


if __name__ == "__main__":
    if os.environ.get("NONDET_STREAM") == "1":   # the library called on a created (non-null) stream
        with torch.cuda.stream(torch.cuda.Stream()):
            main()
    else:
        main()
