"""The drop-in ``datasets`` package (camera/pair files and the depth-hypothesis
recipes that decide which planes the sweep sees).

* The training loader against datasets.npz, made by running the reference's
  datasets/dtu_yao.py on the committed tiny DTU-format tree tests/golden/dtu_mini.
* The eval loaders' recipes (data_eval_transform.py:57-69,113-129 and the padding variant
  :60-81,126-145) against known answers: those reference modules import OpenCV, which is
  not installed, so they cannot be run here (parity pinned by known answers only).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

ROOT = os.path.join(GOLDEN, "dtu_mini")


def load():
    return np.load(os.path.join(GOLDEN, "datasets.npz"), allow_pickle=False)


@pytest.mark.parametrize("tag,kw,idxs", [("lin", {}, (0, 1, 5)),
                                          ("inv", {"inverse_depth": True, "fix_range": True}, (2, 7))])
def test_training_loader_matches_reference(tag, kw, idxs):
    from datasets import find_dataset_def
    g = load()
    ds = find_dataset_def("dtu_yao")(ROOT, os.path.join(ROOT, "scans.txt"), "train", 3, ndepths=48,
                                     light_idx=3, image_scale=0.25, **kw)
    assert len(ds) == int(g[f"{tag}:n"])
    for i in idxs:
        smp = ds[i]
        for k, v in smp.items():
            ref = g[f"{tag}:{i}:{k}"]
            if k == "name":
                assert os.path.relpath(v, ROOT) == str(ref)
            elif k == "imgs":   # per-image normalisation: float32 reductions may reorder
                np.testing.assert_allclose(v, ref, atol=1e-5, rtol=0)
            else:
                assert np.asarray(v).dtype == ref.dtype, k
                np.testing.assert_array_equal(v, ref, err_msg=k)


def test_flip_samples_are_descending():
    from datasets.dtu_yao import MVSDataset
    ds = MVSDataset(ROOT, os.path.join(ROOT, "scans.txt"), "train", 3, ndepths=16, light_idx=3)
    a, b = ds[0]["depth_values"], ds[1]["depth_values"]   # flip 1 then flip 0 (both=True)
    np.testing.assert_array_equal(a, b[::-1])
    assert np.all(np.diff(b) > 0)


def test_eval_recipes_known_answers(tmp_path):
    from datasets import cams
    D, dmin, dint = 8, 400.0, 2.5
    # inverse, endpoint=False: 1 / (1/dmin (1 - i/D)) = dmin D / (D - i)
    inv = cams.eval_depth_values(dmin, dint, D, inverse=True)
    np.testing.assert_allclose(inv, [dmin * D / (D - i) for i in range(D)], rtol=1e-6)
    assert inv.dtype == np.float32
    lin = cams.eval_depth_values(dmin, dint, D, inverse=False)
    np.testing.assert_array_equal(lin, np.float32(dmin) + np.float32(dint) * np.arange(D, dtype=np.float32))
    # padding loader: between depth_min and the file's depth_end, endpoint excluded
    pad = cams.padding_depth_values(dmin, 800.0, D, inverse=False)
    np.testing.assert_allclose(pad, dmin + (800.0 - dmin) * np.arange(D) / D, rtol=1e-7)
    padi = cams.padding_depth_values(dmin, 800.0, D, inverse=True)
    np.testing.assert_allclose(1.0 / padi, 1 / dmin + (1 / 800.0 - 1 / dmin) * np.arange(D) / D, rtol=1e-6)
    # training recipe: depth_end = dmin + (D - 1) interval, or 935 with fix_range
    tr, end = cams.train_depth_values(dmin, dint, D)
    assert end == dmin + (D - 1) * dint and tr[0] == dmin and tr[-1] == np.float32(end)
    tr, end = cams.train_depth_values(dmin, dint, D, inverse=True, fix_range=True, reverse=True)
    assert end == 935 and tr[0] == np.float32(935) and tr[-1] == np.float32(dmin)


def test_camera_file_variants(tmp_path):
    from datasets import cams
    K = np.array([[361.5, 0, 82.5], [0, 360.25, 66.5], [0, 0, 1]])
    E = np.eye(4)
    E[:3, 3] = [1.5, -2.0, 3.25]
    f = tmp_path / "00000000_cam.txt"
    cams.write_cam(f, K, E, 425.0, 2.5, depth_num=192, depth_max=935.0)
    K1, E1, dmin, dint = cams.read_cam(f, interval_scale=1.06)
    np.testing.assert_array_equal(K1, K.astype(np.float32))
    np.testing.assert_array_equal(E1, E.astype(np.float32))
    assert dmin == 425.0 and dint == 2.5 * 1.06
    K4, *_ = cams.read_cam(f, image_scale=1.0)        # training loader at full resolution
    np.testing.assert_array_equal(K4[:2], (K.astype(np.float32) * 4)[:2])
    Kp, _, _, _, dend = cams.read_cam(f, row_shift=4.0, with_depth_end=True)   # padding loader
    assert Kp[1, 2] == np.float32(66.5 + 4) and dend == 935.0
    P = cams.projection(K1, E1)
    np.testing.assert_allclose(P[:3], K1 @ E1[:3], rtol=1e-7)
    np.testing.assert_array_equal(P[3], E1[3])


def test_crop_and_scale_cameras():
    from datasets.preprocess import crop_mvs_input, scale_camera, scale_image
    K = np.array([[100.0, 0, 50], [0, 100, 40], [0, 0, 1]], dtype=np.float32)
    np.testing.assert_array_equal(scale_camera(K, 0.5), [[50, 0, 25], [0, 50, 20], [0, 0, 1]])
    imgs = np.zeros((2, 83, 101, 3), np.float32)
    out, cams_ = crop_mvs_input(imgs, [K.copy(), K.copy()], view_num=2, max_h=80, max_w=200,
                                base_image_size=8)
    # height cropped to max_h (start ceil(3/2) = 2); width rounded UP to 104 gives start
    # ceil(-3/2) = -1, and the reference's slice [-1:103] wraps to one column (kept as is)
    assert out.shape == (2, 80, 1, 3)
    assert cams_[0][1][2] == 38 and cams_[0][0][2] == 50 - int(np.ceil((101 - 104) / 2))
    assert scale_image(np.ones((8, 10, 3), np.float32), 0.5).shape == (4, 5, 3)


def test_eval_loader_end_to_end(tmp_path):
    """A tiny eval tree through data_eval_transform and its padding variant."""
    from PIL import Image
    from datasets import cams, find_dataset_def
    scan = tmp_path / "scanX"
    (scan / "images").mkdir(parents=True)
    (scan / "cams").mkdir()
    with open(scan / "pair.txt", "w") as f:
        f.write("3\n0\n2 1 9.0 2 8.0\n1\n2 0 9.0 2 8.0\n2\n0\n")
    rng = np.random.default_rng(0)
    for v in range(3):
        Image.fromarray(rng.integers(0, 256, (40, 56, 3), dtype=np.uint8)).save(scan / "images" / f"{v:0>8}.jpg")
        K = np.array([[50.0, 0, 28], [0, 50, 20], [0, 0, 1]])
        cams.write_cam(scan / "cams" / f"{v:0>8}_cam.txt", K, np.eye(4), 425.0, 2.5, 192, 935.0)
    (tmp_path / "list.txt").write_text("scanX\n")
    ds = find_dataset_def("data_eval_transform")(str(tmp_path), str(tmp_path / "list.txt"), "test", 3,
                                                 ndepths=16, max_h=32, max_w=48)
    assert len(ds) == 3
    s = ds[0]
    assert s["imgs"].shape == (3, 3, 32, 48) and s["proj_matrices"].shape == (3, 4, 4)
    np.testing.assert_allclose(s["depth_values"],
                               cams.eval_depth_values(425.0, 2.5 * 1.06, 16, inverse=True))
    assert s["filename"] == "scanX/{}/00000000{}"
    dp = find_dataset_def("data_eval_transform_padding")(str(tmp_path), str(tmp_path / "list.txt"),
                                                         "test", 3, ndepths=16, max_h=48, max_w=56,
                                                         adaptive_scaling=False)
    assert len(dp) == 2   # views without sources are skipped
    s = dp[0]
    assert s["imgs"].shape == (3, 3, 48, 56)
    np.testing.assert_allclose(s["depth_values"], cams.padding_depth_values(425.0, 935.0, 16))
