"""Eval loader with 4+4 rows of zero padding (reference:
datasets/data_eval_transform_padding.py): images padded to H + 8 rows (K[1,2] += 4), the
depth range read from the camera file's 4th depth field, hypotheses with
``endpoint=False``, and source views taken from both ends of the pair list.
"""
from __future__ import annotations

import numpy as np

from . import cams
from .data_eval_transform import MVSDataset as _EvalDataset


class MVSDataset(_EvalDataset):
    padding = True

    def read_cam_file(self, filename):
        """(K with K[1,2] + 4, E, depth_min, depth_interval, depth_end) (:60-81)."""
        return cams.read_cam(filename, self.interval_scale, row_shift=4.0, with_depth_end=True)

    def read_img(self, filename):
        from PIL import Image
        mat = np.array(Image.open(filename), dtype=np.float32)
        padded = np.zeros((mat.shape[0] + 8, mat.shape[1], mat.shape[2]))   # float64, as :87-90
        padded[4:-4, :, :] = mat
        return self.center_img(padded)

    def view_ids(self, ref_view, src_views):
        """The first (N-1)//2 and the last N//2 source views (:110-111)."""
        n = self.nviews
        return [ref_view] + src_views[:int((n - 1) / 2)] + src_views[len(src_views) - int(n / 2):]

    def depth_hypotheses(self, cam_path):
        K, E, depth_min, _, depth_end = self.read_cam_file(cam_path)
        return K, E, cams.padding_depth_values(depth_min, depth_end, self.ndepths,
                                               inverse=self.inverse_depth)
