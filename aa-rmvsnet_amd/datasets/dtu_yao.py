"""DTU training loader (reference: datasets/dtu_yao.py), the input contract of config 4.

Same constructor, sample list and sample dict as the reference ``MVSDataset``; the camera
and depth-hypothesis logic lives in ``datasets.cams``.  Images are read with PIL,
resized by PIL's default filter like the reference (dtu_yao.py:84-90), and normalised
per image and channel (:99-104).
"""
from __future__ import annotations

import os

import numpy as np
from PIL import Image
from torch.utils.data import Dataset

from . import cams
from .data_io import read_pfm


def center_img(img, eps=1e-8):
    """(img - mean) / (std + eps) per channel over the image (dtu_yao.py:99-104)."""
    img = img.astype(np.float32)
    var = np.var(img, axis=(0, 1), keepdims=True)
    mean = np.mean(img, axis=(0, 1), keepdims=True)
    return (img - mean) / (np.sqrt(var) + eps)


class MVSDataset(Dataset):
    def __init__(self, datapath, listfile, mode, nviews, ndepths=192, interval_scale=1.06,
                 inverse_depth=False, origin_size=False, light_idx=-1, image_scale=0.25,
                 reverse=False, both=True, fix_range=False, **kwargs):
        super().__init__()
        assert mode in ("train", "val", "test")
        self.datapath, self.listfile, self.mode, self.nviews = datapath, listfile, mode, nviews
        self.ndepths, self.interval_scale, self.inverse_depth = ndepths, interval_scale, inverse_depth
        self.origin_size, self.light_idx, self.image_scale = origin_size, light_idx, image_scale
        self.reverse, self.both, self.fix_range = reverse, both, fix_range
        self.metas = self.build_list()

    def build_list(self):
        """(scan, light, ref_view, src_views, flip) for every scan x view x light; with
        ``both`` each sample appears with flip 1 (descending depths) before flip 0
        (dtu_yao.py:33-57)."""
        with open(self.listfile) as f:
            scans = [ln.rstrip() for ln in f.readlines()]
        pairs = cams.read_pair(os.path.join(self.datapath, "Cameras/pair.txt"))
        lights = range(7) if self.light_idx == -1 else [self.light_idx]
        metas = []
        for scan in scans:
            for ref, srcs in pairs:
                for light in lights:
                    if self.both:
                        metas.append((scan, light, ref, srcs, 1))
                    metas.append((scan, light, ref, srcs, 0))
        return metas

    def __len__(self):
        return len(self.metas)

    def read_cam_file(self, filename):
        return cams.read_cam(filename, self.interval_scale, image_scale=self.image_scale)

    def _load(self, filename):
        img = Image.open(filename)
        if self.image_scale != 1.0:
            w, h = img.size
            img = img.resize((int(self.image_scale * w), int(self.image_scale * h)))
        return np.array(img, dtype=np.float32)

    def read_img(self, filename):
        return self.center_img(self._load(filename))

    def read_original_img(self, filename):
        return self._load(filename)

    def center_img(self, img):
        return center_img(img)

    def read_depth(self, filename):
        return np.array(read_pfm(filename)[0], dtype=np.float32)

    def _paths(self, scan, vid, light):
        root = self.datapath
        img = os.path.join(root, f"Rectified/{scan}_train/rect_{vid + 1:0>3}_{light}_r5000.png")
        if self.image_scale == 1.0:
            depth = os.path.join(root, f"../640_depth/{scan}/depth_map_{vid:0>4}.pfm")
        elif self.image_scale == 0.5:
            depth = os.path.join(root, f"../320_depth/{scan}/depth_map_{vid:0>4}_4.pfm")
        else:
            depth = os.path.join(root, f"Depths/{scan}_train/depth_map_{vid:0>4}.pfm")
        cam = os.path.join(root, f"Cameras/train/{vid:0>8}_cam.txt")
        return img, depth, cam

    def __getitem__(self, idx):
        scan, light, ref_view, src_views, flip = self.metas[idx]
        view_ids = [ref_view] + src_views[:self.nviews - 1]
        imgs, originals, projs = [], [], []
        for i, vid in enumerate(view_ids):
            img_path, depth_path, cam_path = self._paths(scan, vid, light)
            imgs.append(self.read_img(img_path))
            originals.append(self.read_original_img(img_path))
            K, E, depth_min, depth_interval = self.read_cam_file(cam_path)
            projs.append(cams.projection(K, E))
            last_interval = depth_interval   # the reference returns the last view's (:180)
            if i == 0:
                depth_name = depth_path
                depth_values, depth_end = cams.train_depth_values(
                    depth_min, depth_interval, self.ndepths, inverse=self.inverse_depth,
                    fix_range=self.fix_range)
                depth = self.read_depth(depth_path)
                mask = np.array((depth >= depth_min) & (depth <= depth_end), dtype=np.float32)
        if (flip and self.both) or (self.reverse and not self.both):
            depth_values = depth_values[::-1].copy()
        return {"imgs": np.stack(imgs).transpose([0, 3, 1, 2]),
                "imgs_original": np.stack(originals).transpose([0, 3, 1, 2]),
                "proj_matrices": np.stack(projs),
                "depth": depth,
                "depth_values": depth_values,
                "mask": mask,
                "depth_interval": last_interval,
                "name": depth_name}
