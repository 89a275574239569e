"""Schedule-1 divergence anatomy: how large the run-to-run differences of dL/dref and dL/dsrc
are when dL/dx and the parameter gradients are bit-equal, and where they sit (tiles, channels).
usage: python tools/bwd_sched1.py [D] [reps] [pipe]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")]
import torch  # noqa: E402

from aarmvs import ops, synthetic as syn  # noqa: E402

B, N, H, W = 1, 3, 96, 128
D = int(sys.argv[1]) if len(sys.argv) > 1 else 36
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 10
PIPE = sys.argv[3] if len(sys.argv) > 3 else "1"
nsrc = N - 1


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
    os.environ["AARMVS_BWD_PIPE"] = "0"
    r0, s0, p0, x0 = [t for t in sw.backward(ref, srcs, rel, dv, rec, g, want_grad_x=True)]
    r0 = r0.clone()
    s0 = [t.clone() for t in s0]
    x0 = x0.clone()
    p0 = {k: v.clone() for k, v in p0.items()}
    import hashlib
    dig = lambda ts: hashlib.sha256(b"".join(t.detach().cpu().contiguous().numpy().tobytes() for t in ts)).hexdigest()[:12]  # noqa: E731
    print(f"base (one-stream) digests: x={dig([x0])} ref={dig([r0])} src={dig(s0)} "
          f"params={dig([p0[k] for k in sorted(p0)])} cost={dig([cost])}", flush=True)
    os.environ["AARMVS_BWD_PIPE"] = PIPE
    for r in range(REPS):
        gr, gs, gp, gx = sw.backward(ref, srcs, rel, dv, rec, g, want_grad_x=True)
        torch.cuda.synchronize()
        xeq = torch.equal(gx, x0)
        peq = all(torch.equal(gp[k], p0[k]) for k in p0)
        dr = (gr - r0).abs()
        line = f"run {r}: x {'eq' if xeq else 'DIFF'} params {'eq' if peq else 'DIFF'}"
        if bool((dr != 0).any()):
            nz = (dr != 0).nonzero()
            rel_ = float(dr.max() / r0.abs().max())
            ch = sorted(set(nz[:, 1].tolist()))
            ys = nz[:, 2]
            xs = nz[:, 3]
            tiles = sorted(set(((ys // 16) * ((W + 15) // 16) + xs // 16).tolist()))
            line += (f" | ref: {len(nz)} elems differ, max {float(dr.max()):.3e} (rel to max|ref| {rel_:.2e}),"
                     f" channels {ch[:12]}{'...' if len(ch) > 12 else ''}, tiles {tiles[:12]}"
                     f"{'...' if len(tiles) > 12 else ''} of {((H + 15) // 16) * ((W + 15) // 16)}")
            # elementwise relative size of the differences
            rr = dr[dr != 0] / r0.abs()[dr != 0].clamp_min(1e-30)
            line += f", elem rel median {float(rr.median()):.2e} max {float(rr.max()):.2e}"
            if len(nz) <= 64:
                idx = nz.tolist()
                line += "\n      ref diffs [b,c,y,x] base -> run: " + "; ".join(
                    f"{tuple(i)} {float(r0[tuple(i)]):.6e} -> {float(gr[tuple(i)]):.6e}" for i in idx[:20])
        else:
            line += " | ref eq"
        for v in range(nsrc):
            ds = (gs[v] - s0[v]).abs()
            if bool((ds != 0).any()):
                line += f" | src{v}: {int((ds != 0).sum())} differ, max {float(ds.max()):.3e} rel {float(ds.max() / s0[v].abs().max()):.2e}"
        if not xeq:
            xd = (gx - x0).abs()
            pl = [d for d in range(D) if bool((xd[d] != 0).any())]
            line += f" | x planes {pl[-1]}..{pl[0]}, max {float(xd.max()):.2e}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
