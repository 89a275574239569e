"""Depth-map fusion (fusion.py) -- the oracle's known answers, the file formats, and (GPU)
the HIP filter against the oracle.

cv2 and plyfile are not installed in this image and the reference ships no fusion
fixtures: the cv2.remap restatement is checked against known answers of OpenCV's
published INTER_LINEAR algorithm (1/32-px coordinates, table weights, zero border), not
against cv2 itself (parity unpinned for that step)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "aa-rmvsnet_amd"))

from oracle import fusion_oracle as fo  # noqa: E402
from aarmvs import fusion, synthetic as syn  # noqa: E402


def test_remap_known_answers():
    src = np.arange(12, dtype=np.float32).reshape(3, 4)
    mx = np.array([[0, 1, 2.5, 3, -1, 0.5]], np.float32)
    my = np.array([[0, 1, 0, 2, 0, 0.25]], np.float32)
    out = fo.remap_linear(src, mx, my)
    # integer points read the pixel; (2.5, 0) averages 2 and 3; (3, 2) = 11 (right tap outside,
    # weight 0); (-1, 0): all taps outside but the right one, weight 0 -> 0; (0.5, 0.25)
    # bilinear with 1/32 weights
    want = [0.0, 5.0, 2.5, 11.0, 0.0, 0.75 * (0.5 * 0 + 0.5 * 1) + 0.25 * (0.5 * 4 + 0.5 * 5)]
    np.testing.assert_allclose(out[0], np.array(want, np.float32), rtol=0, atol=1e-6)
    # coordinates are rounded to 1/32 px (half to even): 0.015625 = 0.5/32 -> 0
    out = fo.remap_linear(src, np.array([[0.015625, 0.046875]], np.float32), np.zeros((1, 2), np.float32))
    np.testing.assert_array_equal(out[0], np.array([0.0, 2 / 32], np.float32))
    # non-finite coordinates read the border value
    out = fo.remap_linear(src, np.array([[np.inf, np.nan]], np.float32), np.zeros((1, 2), np.float32))
    np.testing.assert_array_equal(out[0], np.zeros(2, np.float32))


def test_filter_core_on_a_consistent_scene():
    depths, cams, conf = syn.fusion_views(48, 64, 4, seed=3)
    photo, geo, final, avg = fo.filter_depth_core(depths[0], conf, cams[0], depths[1:], cams[1:], 0.35)
    assert photo.dtype == bool and geo.dtype == bool and avg.dtype == np.float64
    np.testing.assert_array_equal(final, photo & geo)
    assert geo.mean() > 0.6          # the views see one surface
    good = geo & (depths[0] > 0)
    rel = np.abs(avg[good] - depths[0][good]) / depths[0][good]
    assert np.median(rel) < 2e-3     # averaged with consistent reprojections


def test_pfm_cam_pair_roundtrip(tmp_path):
    img = np.random.default_rng(0).random((5, 7)).astype(np.float32)
    fusion.save_pfm(str(tmp_path / "d.pfm"), img)
    back, scale = fusion.read_pfm(str(tmp_path / "d.pfm"))
    np.testing.assert_array_equal(back, img)
    assert scale == 1.0
    rgb = np.random.default_rng(1).random((4, 3, 3)).astype(np.float32)
    fusion.save_pfm(str(tmp_path / "c.pfm"), rgb)
    np.testing.assert_array_equal(fusion.read_pfm(str(tmp_path / "c.pfm"))[0], rgb)
    # a cam.txt in the DTU / MVSNet layout (extrinsic, 4 rows; intrinsic, 3 rows; depth range)
    cam = ("extrinsic\n1 0 0 10\n0 1 0 20\n0 0 1 30\n0 0 0 1\n\nintrinsic\n"
           "361.54 0 82.9\n0 360.4 66.4\n0 0 1\n\n425 2.5\n")
    (tmp_path / "00000000_cam.txt").write_text(cam)
    K, E = fusion.read_camera_parameters(str(tmp_path / "00000000_cam.txt"), scale=2.0, index=3, flag=0)
    assert K.dtype == np.float32 and E.dtype == np.float32
    np.testing.assert_allclose(E[:3, 3], [10, 20, 30])
    np.testing.assert_allclose(K[0], np.array([361.54 * 2, 0, 82.9 * 2 - 3], np.float32))
    (tmp_path / "pair.txt").write_text("2\n0\n3 1 2.5 2 1.0 5 0.3\n1\n1 0 9.0\n")
    assert fusion.read_pair_file(str(tmp_path / "pair.txt")) == [(0, [1, 2, 5]), (1, [0])]
    xyz = np.arange(12, dtype=np.float32).reshape(4, 3)
    fusion.write_ply(str(tmp_path / "p.ply"), xyz, np.full((4, 3), 7, np.uint8))
    raw = (tmp_path / "p.ply").read_bytes()
    head, body = raw.split(b"end_header\n", 1)
    assert b"element vertex 4" in head and len(body) == 4 * 15


def test_camera_pack_layout():
    _, cams, _ = syn.fusion_views(8, 8, 3)
    p = fusion.pack_cameras(cams[0], cams[1:])
    assert p.dtype == np.float32 and p.size == 18 + 42 * 3
    np.testing.assert_array_equal(p[:9], np.linalg.inv(cams[0][0]).ravel())
    np.testing.assert_array_equal(p[18 + 18:18 + 30], np.matmul(cams[1][1], np.linalg.inv(cams[0][1]))[:3].ravel())


def _fma(a, b, c):
    from fractions import Fraction
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def test_numpy_matmul_is_an_fma_chain():
    """The fusion kernel's float64 projections (csrc/fusion.hip mrow) assume numpy's matmul of
    a float32 3x3 / 4x4 camera matrix with a float64 [k, N] block rounds like
    fma(a_k, b_k, ... fma(a_1, b_1, a_0 * b_0)): check that on this host's BLAS exactly."""
    rng = np.random.default_rng(5)
    for k in (3, 4):
        A = rng.standard_normal((3, k)).astype(np.float32)
        B = rng.standard_normal((k, 700)) * 613.7
        C = np.matmul(A, B)
        for r in range(3):
            for j in range(0, 700, 7):
                s = float(A[r, 0]) * B[0, j]
                for q in range(1, k):
                    s = _fma(float(A[r, q]), B[q, j], s)
                assert s == C[r, j], (k, r, j)


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,nsrc,seed", [(96, 128, 10, 0), (75, 101, 4, 1), (40, 52, 1, 2),
                                           (300, 400, 10, 3)])
def test_gpu_filter_matches_oracle(H, W, nsrc, seed):
    import torch
    depths, cams, conf = syn.fusion_views(H, W, nsrc, seed=seed)
    photo, geo, final, avg = fo.filter_depth_core(depths[0], conf, cams[0], depths[1:], cams[1:], 0.35)
    dev = torch.device("cuda")
    t = [torch.from_numpy(d).to(dev) for d in depths]
    g = fusion.filter_depth_core(t[0], torch.from_numpy(conf).to(dev), cams[0], t[1:], cams[1:], 0.35)
    gp, gg, gf, ga = (x.cpu().numpy() for x in g)
    # bit-exact: the kernel evaluates numpy's float64 chains in numpy's order (OpenBLAS
    # dgemm's per-k fma chain, first product unfused; tests/test_fusion.py
    # ::test_numpy_matmul_is_an_fma_chain pins that order on the host running the oracle)
    np.testing.assert_array_equal(gp, photo)
    np.testing.assert_array_equal(gg, geo)
    np.testing.assert_array_equal(gf, final)
    np.testing.assert_array_equal(ga, avg)


@pytest.mark.gpu
def test_gpu_filter_rejects_bad_input():
    import torch
    from aarmvs._lib import AarmvsError
    depths, cams, conf = syn.fusion_views(16, 16, 2)
    with pytest.raises(AarmvsError):
        fusion.filter_depth_core(torch.from_numpy(depths[0]), torch.from_numpy(conf), cams[0],
                                 [torch.from_numpy(d) for d in depths[1:]], cams[1:], 0.35)


def test_crop_params_and_resize_identity():
    # DTU eval: 1200x1600 images, 1184x1600 depth maps -> scale 1, crop 8 rows top and bottom
    assert fusion.crop_params((1200, 1600), (1184, 1600)) == (1.0, 8, 8, 1)
    # a 2x downscale that crops columns
    s, i, ip, f = fusion.crop_params((600, 820), (300, 400))
    assert (s, i, ip, f) == (0.5, 5, 5, 0)
    img = np.random.default_rng(0).random((6, 8, 3)).astype(np.float32)
    np.testing.assert_array_equal(fusion.resize_linear(img, 8, 6), img)
    half = fusion.resize_linear(img, 4, 3)                  # INTER_AREA path: 2x2 means
    np.testing.assert_allclose(half[1, 2], img[2:4, 4:6].mean((0, 1)), rtol=1e-6)
    up = fusion.resize_linear(img[:, :, 0], 16, 12)          # bilinear, clamped borders
    assert up.shape == (12, 16) and up[0, 0] == img[0, 0, 0] and up[-1, -1] == img[-1, -1, 0]


def _write_scan(root, H, W, nsrc, pad):
    """A scan folder in the DTU layout: pair.txt, cams/, images/ (pad extra rows top and
    bottom: the driver's crop), depth_est_0/ and confidence_0/ PFMs."""
    from PIL import Image
    depths, cams, conf = syn.fusion_views(H, W, nsrc, seed=11)
    n = nsrc + 1
    scan, out = root / "scan1", root / "out"
    for d in ("cams", "images"):
        (scan / d).mkdir(parents=True, exist_ok=True)
    for d in ("depth_est_0", "confidence_0"):
        (out / d).mkdir(parents=True, exist_ok=True)
    rng = np.random.default_rng(3)
    pair, images, cam_texts, dmaps, confs = [], {}, {}, {}, {}
    for v in range(n):
        K, E = cams[v]
        K = K.copy()
        K[1, 2] += pad                      # the image has pad more rows above the crop
        txt = ("extrinsic\n" + "\n".join(" ".join(repr(float(q)) for q in row) for row in E)
               + "\n\nintrinsic\n" + "\n".join(" ".join(repr(float(q)) for q in row) for row in K)
               + "\n\n425 2.5\n")
        (scan / "cams" / "{:0>8}_cam.txt".format(v)).write_text(txt)
        cam_texts[v] = txt
        img = (rng.random((H + 2 * pad, W, 3)) * 255).astype(np.uint8)
        Image.fromarray(img).save(str(scan / "images" / "{:0>8}.jpg".format(v)), format="PNG")
        images[v] = np.array(Image.open(str(scan / "images" / "{:0>8}.jpg".format(v))), np.float32) / 255.0
        cv = np.roll(conf, 7 * v, axis=1) if v else conf
        fusion.save_pfm(str(out / "depth_est_0" / "{:0>8}.pfm".format(v)), depths[v])
        fusion.save_pfm(str(out / "confidence_0" / "{:0>8}.pfm".format(v)), cv)
        dmaps[v], confs[v] = depths[v], cv
        pair.append((v, [s for s in range(n) if s != v]))
    with open(scan / "pair.txt", "w") as f:
        f.write(f"{n}\n")
        for v, srcs in pair:
            f.write(f"{v}\n{len(srcs)} " + " ".join(f"{s} {9.0 - s:.1f}" for s in srcs) + "\n")
    return scan, out, (pair, images, cam_texts, dmaps, confs)


@pytest.mark.gpu
def test_gpu_filter_depth_scan_matches_oracle(tmp_path):
    """The per-scan driver (fusion.py:135-273): image crop and camera re-centring, the masks
    of every reference view (PNG files) and the scan's PLY, bit-exact vs the oracle."""
    from PIL import Image
    scan, out, (pair, images, cam_texts, dmaps, confs) = _write_scan(tmp_path, 48, 64, 3, 4)
    ply = tmp_path / "scan1.ply"
    npts = fusion.filter_depth(str(scan), str(out), str(ply), 0.35)
    masks, xyz, rgb = fo.filter_depth_scan(pair, images, cam_texts, dmaps, confs, 0.35)
    assert npts == xyz.shape[0] > 0
    for v, (photo, geo, final) in masks.items():
        for name, m in (("photo", photo), ("geo", geo), ("final", final)):
            png = np.array(Image.open(str(out / "mask" / "{:0>8}_{}.png".format(v, name))))
            np.testing.assert_array_equal(png, m.astype(np.uint8) * 255)
    head, body = ply.read_bytes().split(b"end_header\n", 1)
    assert f"element vertex {npts}".encode() in head
    v = np.frombuffer(body, dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"),
                                   ("red", "u1"), ("green", "u1"), ("blue", "u1")])
    np.testing.assert_array_equal(np.stack([v["x"], v["y"], v["z"]], 1), xyz)
    np.testing.assert_array_equal(np.stack([v["red"], v["green"], v["blue"]], 1), rgb)
