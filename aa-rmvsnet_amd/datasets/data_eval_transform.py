"""Eval loader with adaptive rescale and centre crop (reference:
datasets/data_eval_transform.py), the input contract of the DTU / T&T eval configs.

Same constructor, sample list and sample dict as the reference ``MVSDataset``.  The
``padding`` subclass is datasets/data_eval_transform_padding.py.  Image resizing goes
through ``datasets.preprocess.scale_image`` (OpenCV is not in this image; see there).
"""
from __future__ import annotations

import os

import numpy as np
from PIL import Image
from torch.utils.data import Dataset

from . import cams
from .data_io import read_pfm
from .preprocess import crop_mvs_input, scale_mvs_input


class MVSDataset(Dataset):
    padding = False

    def __init__(self, datapath, listfile, mode, nviews, ndepths=192, interval_scale=1.06,
                 inverse_depth=True, adaptive_scaling=True, max_h=1200, max_w=1600,
                 sample_scale=1, base_image_size=8, **kwargs):
        super().__init__()
        assert mode == "test"
        self.datapath, self.listfile, self.mode, self.nviews = datapath, listfile, mode, nviews
        self.ndepths, self.interval_scale, self.inverse_depth = ndepths, interval_scale, inverse_depth
        self.adaptive_scaling, self.max_h, self.max_w = adaptive_scaling, max_h, max_w
        self.sample_scale, self.base_image_size = sample_scale, base_image_size
        self.metas = self.build_list()

    def build_list(self):
        """(scan, ref_view, src_views) per view of every scan's pair.txt
        (data_eval_transform.py:34-50); the padding loader skips views without sources."""
        with open(self.listfile) as f:
            scans = [ln.rstrip() for ln in f.readlines()]
        metas = []
        for scan in scans:
            for ref, srcs in cams.read_pair(os.path.join(self.datapath, f"{scan}/pair.txt")):
                if self.padding and not srcs:
                    continue
                metas.append((scan, ref, srcs))
        return metas

    def __len__(self):
        return len(self.metas)

    def read_cam_file(self, filename):
        return cams.read_cam(filename, self.interval_scale)

    def read_img(self, filename):
        return self.center_img(np.array(Image.open(filename), dtype=np.float32))

    def center_img(self, img):
        """(img - mean) / std per channel, no epsilon (data_eval_transform.py:78-82)."""
        img = img.astype(np.float32)
        var = np.var(img, axis=(0, 1), keepdims=True)
        mean = np.mean(img, axis=(0, 1), keepdims=True)
        return (img - mean) / np.sqrt(var)

    def read_depth(self, filename):
        return np.array(read_pfm(filename)[0], dtype=np.float32)

    def view_ids(self, ref_view, src_views):
        return [ref_view] + src_views[:self.nviews - 1]

    def depth_hypotheses(self, cam_path):
        K, E, depth_min, depth_interval = self.read_cam_file(cam_path)
        return K, E, cams.eval_depth_values(depth_min, depth_interval, self.ndepths,
                                            inverse=self.inverse_depth)

    def resize_scale(self, imgs):
        """The largest of max_h / H and max_w / W over the views (:136-152); the reference
        exits when that exceeds 1 (upscaling), which raises here."""
        if not self.adaptive_scaling:
            return 1
        hs = max(float(self.max_h) / imgs[v].shape[1] for v in range(self.nviews))
        ws = max(float(self.max_w) / imgs[v].shape[2] for v in range(self.nviews))
        if hs > 1 or ws > 1:
            raise ValueError("max_h, max_w should < W and H!")
        return ws if ws > hs else hs

    def __getitem__(self, idx):
        scan, ref_view, src_views = self.metas[idx]
        if self.nviews > len(src_views):
            self.nviews = len(src_views) + 1     # as the reference (:95-96), persistently
        vids = self.view_ids(ref_view, src_views)
        imgs, Ks, Es = [], [], []
        for i, vid in enumerate(vids):
            imgs.append(self.read_img(os.path.join(self.datapath, f"{scan}/images/{vid:0>8}.jpg")))
            cam_path = os.path.join(self.datapath, f"{scan}/cams/{vid:0>8}_cam.txt")
            K, E, dv = self.depth_hypotheses(cam_path)
            Ks.append(K)
            Es.append(E)
            if i == 0:
                depth_values = dv
        imgs = np.stack(imgs).transpose([0, 3, 1, 2])
        scale = self.resize_scale(imgs)
        imgs, Ks = scale_mvs_input(imgs.transpose(0, 2, 3, 1), Ks, scale=scale, view_num=self.nviews)
        imgs, Ks = crop_mvs_input(imgs, Ks, view_num=self.nviews, max_h=self.max_h, max_w=self.max_w,
                                  base_image_size=self.base_image_size)
        projs = np.stack([cams.projection(Ks[v], Es[v]) for v in range(self.nviews)])
        return {"imgs": imgs.transpose(0, 3, 1, 2),
                "proj_matrices": projs,
                "depth_values": depth_values,
                "filename": scan + "/{}/" + f"{vids[0]:0>8}" + "{}"}
