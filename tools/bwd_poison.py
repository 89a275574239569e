"""Uninitialised-read probe of the sweep backward (VERDICT r4 'next' item 1): the backward's
scratch (and, separately, the sweep workspace) is filled with a poison pattern before each
backward call; any output that depends on a value the call did not write first changes with
the pattern (NaN / huge / zero / one).  Run per stream schedule (AARMVS_BWD_PIPE 0, 3, 1).
usage: python tools/bwd_poison.py [D] [reps]"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")]
import torch  # noqa: E402

from aarmvs import ops, synthetic as syn  # noqa: E402

B, N, H, W = 1, 3, 96, 128
D = int(sys.argv[1]) if len(sys.argv) > 1 else 36
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 4
nsrc = N - 1
PATTERNS = {"none": None, "zero": 0x00000000, "nan": 0xFFFFFFFF, "huge": 0x7F7F7F7F, "one": 0x3F800000}


def digest(ts):
    h = hashlib.sha256()
    for t in ts:
        h.update(t.detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()[:12]


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
    sw.backward(ref, srcs, rel, dv, rec, g, want_grad_x=True)   # allocates the scratch
    torch.cuda.synchronize()
    scratch = sw._ws[("bwd", B, H, W, nsrc)]
    wsp = sw.workspace(B, H, W, nsrc)
    base = None
    for pipe in ("0", "3", "1"):
        os.environ["AARMVS_BWD_PIPE"] = pipe
        for target in ("scratch", "workspace"):
            for pname, pat in PATTERNS.items():
                if target == "workspace" and pname == "none":
                    continue
                seen = {}
                for r in range(REPS):
                    if pat is not None:
                        buf = scratch if target == "scratch" else wsp
                        n4 = buf.numel() // 4
                        buf[: n4 * 4].view(torch.int32).fill_(pat - (1 << 32) if pat >= (1 << 31) else pat)
                    gr, gs, gp, gx = sw.backward(ref, srcs, rel, dv, rec, g, want_grad_x=True)
                    torch.cuda.synchronize()
                    outs = {"x": [gx], "ref": [gr], "src": gs, "par": [gp[k] for k in sorted(gp)]}
                    dg = " ".join(f"{k}={digest(v)}" for k, v in outs.items())
                    nan = sum(int((~torch.isfinite(t)).sum()) for v in outs.values() for t in v)
                    if base is None:
                        base = dg
                    key = (dg, nan)
                    seen[key] = seen.get(key, 0) + 1
                    if dg != base and nan == 0:
                        xd = (gx - base_x).abs()
                        pl = [d for d in range(D) if bool((xd[d] != 0).any())]
                        print(f"      differs: planes {pl[-3:] if pl else []} (first in backward order "
                              f"{pl[-1] if pl else None}), max |dx| {float(xd.max()):.3e}", flush=True)
                    if r == 0 and pipe == "0" and pname == "none" and target == "scratch":
                        base_x = gx.clone()
                for (dg, nan), cnt in seen.items():
                    tag = "BASE" if dg == base else "DIFF"
                    print(f"pipe={pipe} {target:9s} poison={pname:5s} {cnt}x {tag} nonfinite={nan} {dg}",
                          flush=True)


if __name__ == "__main__":
    main()
