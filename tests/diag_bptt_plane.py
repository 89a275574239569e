"""Per-tensor bisection of the HIP backward of ONE plane (D = 1): every intermediate gradient
the backward leaves in its scratch (cell gate gradients dL/dz, dL/d relu(GN(u_j)), dL/du_j,
dL/d maxpool(h), dL/dx, dL/d previous state) against float64 autograd of the oracle's
unet_step AT THE GPU'S RECORDED FORWARD VALUES (so only the backward's arithmetic differs),
next to float32 autograd at the same point.  Reported per tensor: relative L2 error and the
error's component along the tensor itself (<e, g> / <g, g>: a relative scale bias).
Runs on the GPU box (the CPU part is one plane at 32x48)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from aarmvs import _lib  # noqa: E402
from oracle import sweep_oracle as orc  # noqa: E402
import test_gpu_bptt as T  # noqa: E402

G, C, HID = 16, 32, (16, 16, 16, 16, 8)
B, N, H, W, D = [int(v) for v in os.environ.get("SHAPE", "1,3,32,48,1").split(",")]


def al256(x):
    return (x + 255) // 256 * 256


def layout():
    HW = H * W
    px = [HW, HW // 4, HW // 16, HW // 4, HW]
    off, L = 0, {}

    def take(name, nbytes):
        nonlocal off
        L[name] = (off, nbytes)
        off = al256(off + nbytes)
    for k in range(5):
        take(f"gh{k}", B * px[k] * HID[k] * 4)
        take(f"gc{k}", B * px[k] * HID[k] * 4)
        take(f"gz{k}", G * B * px[k] * 4 * HID[k] * 4)
    take("zmax", 5 * G * 4)
    take("gr0", B * (HW // 4) * 16 * 4)
    take("gr1", B * HW * 16 * 4)
    take("gr0b", B * (HW // 4) * 16 * 4)
    for q in range(2):
        for k in range(2):
            take(f"gskip{q}{k}", B * px[k] * 16 * 4)
    take("gpool0", B * (HW // 4) * 16 * 4)
    take("gpool1", B * (HW // 16) * 16 * 4)
    take("gu0", G * B * (HW // 4) * 16 * 4)
    take("gu1", G * B * HW * 16 * 4)
    take("gx", G * B * HW * C * 4)
    return L


sc, P, feats, proj, dv, sw, args = T._setup(B, N, H, W, D, 11 + D, 6)
cost, rec, rel = T._record_forward(sw, args, B, H, W, D)
R = torch.randn(B, D, H, W, generator=torch.Generator().manual_seed(5))
prob = torch.softmax(cost, dim=1)
Rd = R.to("cuda")
gcost = (prob * (Rd - (Rd * prob).sum(dim=1, keepdim=True))) if D > 1 else torch.randn(B, D, H, W, device="cuda")
_, _, _, gxo = sw.backward(args[0], args[1], rel, dv, rec, gcost, regulariser_only=True, want_grad_x=True)
torch.cuda.synchronize()
scratch = sw._ws[("bwd", B, H, W, N - 1)].cpu().numpy()
Lay = layout()


def sget(name, shape, plane_slot=None):
    off, nb = Lay[name]
    a = scratch[off: off + nb].view(np.float32)
    if plane_slot is not None:
        n = int(np.prod(shape))
        a = a[plane_slot * n: (plane_slot + 1) * n]
    return a.reshape(shape).astype(np.float64)


# the GPU's recorded forward values of the last plane (D - 1), and its state before it
d = D - 1
xs = torch.from_numpy(rec["x"].view(torch.float32).cpu().numpy()[d * B * H * W * C:(d + 1) * B * H * W * C]
                      .reshape(B, H, W, C)).permute(0, 3, 1, 2).double()
slab = _lib.lib().aarmvs_train_record_bytes(B, H, W, 1) // 4
sflat = rec["state"].view(torch.float32).cpu().numpy()[d * slab:(d + 1) * slab]
st, off = [], 0
for k, s in enumerate((1, 2, 4, 2, 1)):
    pair = []
    for _ in range(2):
        n = B * (H // s) * (W // s) * HID[k]
        pair.append(torch.from_numpy(sflat[off:off + n].reshape(B, H // s, W // s, HID[k])).permute(0, 3, 1, 2).double())
        off += -(-n // 64) * 64
    st.append(pair)


def plane_grads(dtype):
    Pd = {k: v.to(dtype) for k, v in P.items()}
    x = xs.detach().to(dtype).clone().requires_grad_(True)
    hp = [p[0].detach().to(dtype).clone().requires_grad_(True) for p in st]
    cp = [p[1].detach().to(dtype).clone().requires_grad_(True) for p in st]
    keep = {}

    def cell(k, inp):
        z = F.conv2d(inp, Pd[f"cost_regularization.cell_list.{k}.conv.weight"],
                     Pd[f"cost_regularization.cell_list.{k}.conv.bias"], padding=1)
        z.retain_grad()
        keep[f"z{k}"] = z
        i, f, o, g = torch.split(z, HID[k], dim=1)
        c2 = torch.sigmoid(f) * cp[k] + torch.sigmoid(i) * torch.tanh(g)
        return torch.sigmoid(o) * torch.tanh(c2)

    def dec(j, h):
        kk = f"cost_regularization.deconv_{j}."
        u = F.conv_transpose2d(h, Pd[kk + "conv.weight"], Pd[kk + "conv.bias"], stride=2, padding=1, output_padding=1)
        u.retain_grad()
        keep[f"u{j}"] = u
        r = F.relu(orc.group_norm(u, 2, Pd[kk + "gn.weight"], Pd[kk + "gn.bias"]))
        r.retain_grad()
        keep[f"r{j}"] = r
        return r
    h0 = cell(0, torch.cat([x, hp[0]], 1))
    p0 = F.max_pool2d(h0, 2, 2)
    p0.retain_grad()
    keep["p0"] = p0
    h1 = cell(1, torch.cat([p0, hp[1]], 1))
    p1 = F.max_pool2d(h1, 2, 2)
    p1.retain_grad()
    keep["p1"] = p1
    h2 = cell(2, torch.cat([p1, hp[2]], 1))
    h3 = cell(3, torch.cat([dec(0, h2), h1, hp[3]], 1))
    h4 = cell(4, torch.cat([dec(1, h3), h0, hp[4]], 1))
    cst = F.conv2d(h4, Pd["cost_regularization.conv_0.weight"], Pd["cost_regularization.conv_0.bias"], padding=1)
    (cst.squeeze(1) * gcost[:, d].cpu().to(dtype)).sum().backward()
    out = {f"gz{k}": keep[f"z{k}"].grad for k in range(5)}
    out.update({f"gu{j}": keep[f"u{j}"].grad for j in range(2)})
    out.update({f"gr{j}": keep[f"r{j}"].grad for j in range(2)})
    out.update({"gpool0": keep["p0"].grad, "gpool1": keep["p1"].grad, "gx": x.grad})
    out.update({f"gh{k}": hp[k].grad for k in range(5)})
    out.update({f"gc{k}": cp[k].grad for k in range(5)})
    return {k: v.double().permute(0, 2, 3, 1).numpy() for k, v in out.items()}   # NHWC


g64 = plane_grads(torch.float64)
g32 = plane_grads(torch.float32)
slot = d % G
res = [1, 2, 4, 2, 1]
gpu = {}
for k in range(5):
    hk, wk = H // res[k], W // res[k]
    z = sget(f"gz{k}", (B, hk, wk, 4 * HID[k]), slot)
    gpu[f"gz{k}"] = z
    if D == 1:
        gpu[f"gh{k}"] = sget(f"gh{k}", (B, hk, wk, HID[k]))
        gpu[f"gc{k}"] = sget(f"gc{k}", (B, hk, wk, HID[k]))
gpu["gu0"] = sget("gu0", (B, H // 2, W // 2, 16), slot)
gpu["gu1"] = sget("gu1", (B, H, W, 16), slot)
gpu["gr1"] = sget("gr1", (B, H, W, 16))
gpu["gr0"] = sget("gr0" if d % 2 == 0 else "gr0b", (B, H // 2, W // 2, 16))
gpu["gpool0"] = sget("gpool0", (B, H // 2, W // 2, 16))
gpu["gpool1"] = sget("gpool1", (B, H // 4, W // 4, 16))
gpu["gx"] = gxo[d].double().cpu().numpy()
print(f"shape {(B, N, H, W, D)}: last plane's backward, relative L2 / scale bias <e,g>/<g,g> vs float64 at the GPU's forward point")
for k in ["gz4", "gr1", "gu1", "gz3", "gr0", "gu0", "gz2", "gpool1", "gz1", "gpool0", "gz0", "gx"] + \
        [f"g{t}{k}" for k in range(5) for t in "hc"]:
    if k not in gpu:
        continue
    ref = g64[k]
    nr = np.linalg.norm(ref)
    for tag, g in (("gpu", gpu[k]), ("cpu32", g32[k])):
        e = g - ref
        print(f"  {k:7s} {tag:5s} L2 {np.linalg.norm(e) / nr:.3e}  bias {float((e * ref).sum()) / nr ** 2:+.3e}")

# projection of the last plane's dL/dx error on K = dx/dtheta (tests/diag_gx_corr.py)
rels = [orc.relative_projection(proj[:, v], proj[:, 0]) for v in range(1, N)]
P64 = {k: v.double() for k, v in P.items()}
fd = feats.double()


def fwd_inter(x):
    """float64 forward of the plane from x (state fixed at the GPU's), every intermediate the
    backward leaves a gradient for (NCHW)."""
    Pd = P64
    hp = [p[0] for p in st]
    cp = [p[1] for p in st]
    out = {}

    def cell(k, inp):
        z = F.conv2d(inp, Pd[f"cost_regularization.cell_list.{k}.conv.weight"],
                     Pd[f"cost_regularization.cell_list.{k}.conv.bias"], padding=1)
        out[f"gz{k}"] = z
        i, f_, o, g = torch.split(z, HID[k], dim=1)
        c2 = torch.sigmoid(f_) * cp[k] + torch.sigmoid(i) * torch.tanh(g)
        return torch.sigmoid(o) * torch.tanh(c2)

    def dec(j, h):
        kk = f"cost_regularization.deconv_{j}."
        u = F.conv_transpose2d(h, Pd[kk + "conv.weight"], Pd[kk + "conv.bias"], stride=2, padding=1, output_padding=1)
        out[f"gu{j}"] = u
        r = F.relu(orc.group_norm(u, 2, Pd[kk + "gn.weight"], Pd[kk + "gn.bias"]))
        out[f"gr{j}"] = r
        return r
    h0 = cell(0, torch.cat([x, hp[0]], 1))
    p0 = F.max_pool2d(h0, 2, 2)
    out["gpool0"] = p0
    h1 = cell(1, torch.cat([p0, hp[1]], 1))
    p1 = F.max_pool2d(h1, 2, 2)
    out["gpool1"] = p1
    h2 = cell(2, torch.cat([p1, hp[2]], 1))
    h3 = cell(3, torch.cat([dec(0, h2), h1, hp[3]], 1))
    cell(4, torch.cat([dec(1, h3), h0, hp[4]], 1))
    return out


for pname in ("omega.reweight_network.2.bias", "omega.reweight_network.1.stem.2.weight"):
    def f(b):
        Q = dict(P64)
        Q[pname] = b
        return orc.cost_slice(fd[0], [fd[v] for v in range(1, N)], rels, dv[:, d], Q, fast=True)
    _, K = torch.func.jvp(f, (P64[pname],), (torch.ones_like(P64[pname]),))
    K = K.permute(0, 2, 3, 1).numpy()
    gt = float((g64["gx"] * K).sum())
    ab = float(np.abs(g64["gx"] * K).sum())
    print(f"  <gx,K> {pname}: {gt:+.4e} (sum|.| {ab:.3e})  gpu err {float(((gpu['gx'] - g64['gx']) * K).sum()) / abs(gt):+.3e}"
          f"  cpu32 err {float(((g32['gx'] - g64['gx']) * K).sum()) / abs(gt):+.3e}")
    if D == 1:
        # <dL/dT, dT/dx K> = <dL/dx, K> for every intermediate T on the way from the cost to x:
        # where the GPU's error projection departs from float32's is where it enters
        _, tang = torch.func.jvp(fwd_inter, (xs,), (torch.from_numpy(K).permute(0, 3, 1, 2).contiguous(),))
        for t in ["gz4", "gr1", "gu1", "gz3", "gr0", "gu0", "gz2", "gpool1", "gz1", "gpool0", "gz0"]:
            tv = tang[t].permute(0, 2, 3, 1).numpy()
            if t not in gpu:
                continue
            print(f"      via {t:7s} float64 {float((g64[t] * tv).sum()):+.4e}  gpu err "
                  f"{float(((gpu[t] - g64[t]) * tv).sum()) / abs(gt):+.3e}  cpu32 err {float(((g32[t] - g64[t]) * tv).sum()) / abs(gt):+.3e}")
