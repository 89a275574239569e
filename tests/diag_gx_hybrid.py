"""CPU-side split of the HIP dL/dx error (no GPU) into what the backward's arithmetic adds and
what the forward's recorded values add: from tests/diag_gx_dump.py's dump (the GPU's record:
cost slices and every plane's regulariser state, its dL/dcost and its dL/dx), the float64 BPTT
is run plane by plane AT THE GPU'S RECORDED STATES (local autograd of one oracle unet_step per
plane, gradients chained backward) -> gx_hyb.  Then
   e_bwd = gx_gpu - gx_hyb    (the HIP backward's arithmetic)
   e_fwd = gx_hyb - gx64      (the HIP forward's values, float64 backward)
are projected on K_d = dx_d/dtheta (tests/diag_gx_corr.py) for an omega parameter theta.
usage: python tests/diag_gx_hybrid.py gpurun_out/<dump>.npz [param]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from aarmvs import _lib, synthetic as syn  # noqa: E402
from oracle import sweep_oracle as orc  # noqa: E402
import test_gpu_bptt as T  # noqa: E402

torch.set_num_threads(8)

# EMUL=dgrad: the hybrid's cell convs take their input gradient as the HIP dgrad forms it --
# gz (per plane and cell scaled to [2^14, 2^15)) and the weights split into fp16 hi + lo,
# three products (hi hi, lo hi, hi lo), lo lo dropped -- in float64 otherwise.
EMUL = os.environ.get("EMUL", "")


def split16(t, per_sample=False):
    a = t.abs().amax() if not per_sample else t.abs().amax()
    e = int(np.floor(np.log2(float(a)))) - 14 if float(a) > 0 else 0
    v = t * 2.0 ** -e
    hi = v.to(torch.float16).double()
    lo = (v - hi).to(torch.float16).double()
    return hi * 2.0 ** e, lo * 2.0 ** e


class EmulConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inp, w, b):
        ctx.save_for_backward(inp, w)
        return torch.nn.functional.conv2d(inp, w, b, padding=1)

    @staticmethod
    def backward(ctx, gz):
        inp, w = ctx.saved_tensors
        gh, gl = split16(gz)
        wh, wl = split16(w)
        ci = lambda g, ww: torch.nn.grad.conv2d_input(inp.shape, ww, g, padding=1)  # noqa: E731
        gin = ci(gh, wh) + ci(gl, wh) + ci(gh, wl) if "lolo" not in EMUL else ci(gh + gl, wh + wl)
        gw = torch.nn.grad.conv2d_weight(inp, w.shape, gz, padding=1)
        return gin, gw, gz.sum(dim=(0, 2, 3))


if EMUL.startswith("dgrad"):
    def _cell(x, h, c, w, b):
        z = EmulConv.apply(torch.cat([x, h], 1), w, b)
        i, f, o, g = torch.split(z, h.shape[1], dim=1)
        c2 = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
        return torch.sigmoid(o) * torch.tanh(c2), c2
    orc.lstm_cell = _cell
dump = np.load(sys.argv[1])
pname = sys.argv[2] if len(sys.argv) > 2 else "omega.reweight_network.2.bias"
L = _lib.lib()
shapes = [(1, 3, 32, 48, 6), (2, 4, 24, 40, 5)]
CELLS = [(16, 1), (16, 2), (16, 4), (16, 2), (8, 1)]


def parse_state(flat, B, H, W):
    st, off = [], 0
    for hid, s in CELLS:
        n = B * (H // s) * (W // s) * hid
        pair = []
        for _ in (0, 1):
            pair.append(torch.from_numpy(flat[off:off + n].reshape(B, H // s, W // s, hid)).permute(0, 3, 1, 2).double())
            off += -(-n // 64) * 64
        st.append(tuple(pair))
    return st


for i, (B, N, H, W, D) in enumerate(shapes):
    sc = syn.scene(B, N, H, W, D, seed=11 + D)
    P = {k: torch.from_numpy(v) for k, v in syn.sweep_weights(6).items()}
    P64 = {k: v.double() for k, v in P.items()}
    feats = torch.from_numpy(sc["features"])
    proj = torch.from_numpy(sc["proj_matrices"])
    dv = torch.from_numpy(sc["depth_values"])
    R = torch.randn(B, D, H, W, generator=torch.Generator().manual_seed(5))
    _, _, _, gx64 = T._oracle_grads(feats, proj, dv, P, R, torch.float64)
    gx64 = np.stack([g.numpy() for g in gx64])
    gxg = dump[f"gx{i}"].astype(np.float64)
    gcost = torch.from_numpy(dump[f"gcost{i}"]).double()
    xs = torch.from_numpy(dump[f"rec_x{i}"].reshape(D, B, H, W, 32)).permute(0, 1, 4, 2, 3).double()
    slab = L.aarmvs_train_record_bytes(B, H, W, 1) // 4
    sflat = dump[f"rec_state{i}"]
    states = [parse_state(sflat[d * slab:(d + 1) * slab], B, H, W) for d in range(D + 1)]
    # float64 BPTT at the GPU's recorded points
    g_next = [(torch.zeros_like(h), torch.zeros_like(c)) for h, c in states[0]]
    gx_hyb = np.zeros_like(gxg)
    for d in reversed(range(D)):
        x = xs[d].clone().requires_grad_(True)
        st = [(h.clone().requires_grad_(True), c.clone().requires_grad_(True)) for h, c in states[d]]
        cost, new = orc.unet_step(x, st, P64)
        obj = (cost.squeeze(1) * gcost[:, d]).sum()
        for (h, c), (gh, gc) in zip(new, g_next):
            obj = obj + (h * gh).sum() + (c * gc).sum()
        leaves = [x] + [t for pair in st for t in pair]
        grads = torch.autograd.grad(obj, leaves)
        gx_hyb[d] = grads[0].numpy()
        g_next = [(grads[1 + 2 * k], grads[2 + 2 * k]) for k in range(5)]
    rels = [orc.relative_projection(proj[:, v], proj[:, 0]) for v in range(1, N)]
    fd = feats.double()
    K = []
    for d in range(D):
        def f(b):
            Q = dict(P64)
            Q[pname] = b
            return orc.cost_slice(fd[0], [fd[v] for v in range(1, N)], rels, dv[:, d], Q, fast=True)
        _, t = torch.func.jvp(f, (P64[pname],), (torch.ones_like(P64[pname]),))
        K.append(t.numpy())
    K = np.stack(K)
    g_true = float((gx64 * K).sum())
    nrm = np.linalg.norm(gx64)
    print(f"shape {i} {(B, N, H, W, D)}: {pname} via dL/dx {g_true:.6e}")
    print(f"  (EMUL={EMUL!r})")
    for tag, e in (("total gpu-64", gxg - gx64), ("bwd gpu-hyb", gxg - gx_hyb), ("fwd hyb-64", gx_hyb - gx64)):
        pe = e * K
        print(f"  {tag:14s} L2 {np.linalg.norm(e) / nrm:.3e}  projection {pe.sum() / abs(g_true):+.3e}  per plane "
              + " ".join(f"{pe[d].sum() / abs(g_true):+.1e}" for d in range(D)))
