"""Sharded multi-GPU inference driver (aarmvs.eval_sharded: eval.py's save_depth, SURVEY
§8e): every (scan, ref_view) sample is written by exactly one rank, and each written map
equals the drop-in model's own output for that sample.  Ranks are run one after another in
this process on the one device (the driver has no collective)."""
import numpy as np
import pytest
import torch

from datasets import cams, find_dataset_def
from aarmvs import eval_sharded, fusion

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _tree(tmp_path, nv=4):
    from PIL import Image
    scan = tmp_path / "scanX"
    (scan / "images").mkdir(parents=True)
    (scan / "cams").mkdir()
    with open(scan / "pair.txt", "w") as f:
        f.write(f"{nv}\n")
        for v in range(nv):
            srcs = [s for s in range(nv) if s != v]
            f.write(f"{v}\n{len(srcs)} " + " ".join(f"{s} {9.0 - s:.1f}" for s in srcs) + "\n")
    rng = np.random.default_rng(0)
    for v in range(nv):
        Image.fromarray(rng.integers(0, 256, (40, 56, 3), dtype=np.uint8)).save(
            scan / "images" / f"{v:0>8}.jpg", format="PNG")
        K = np.array([[50.0, 0, 28], [0, 50, 20], [0, 0, 1]])
        E = np.eye(4)
        E[0, 3] = -2.0 * v
        cams.write_cam(scan / "cams" / f"{v:0>8}_cam.txt", K, E, 425.0, 2.5, 192, 935.0)
    (tmp_path / "list.txt").write_text("scanX\n")
    return tmp_path


@pytest.mark.parametrize("numdepth", [16, 32])
def test_sharded_eval_writes_every_sample_once(tmp_path, numdepth):
    from models import EMVSNet
    root = _tree(tmp_path)
    args = eval_sharded.parse_args([
        "--testpath", str(root), "--testlist", str(root / "list.txt"), "--outdir", str(root / "out"),
        "--max_h", "32", "--max_w", "48", "--numdepth", str(numdepth), "--view_num", "3",
        "--interval_scale", "1.06"])
    torch.manual_seed(0)
    model = EMVSNet(disparity_level=32, image_scale=1.0, max_h=32, max_w=48, return_depth=True)
    written = []
    for rank in range(2):
        written += eval_sharded.save_depth(args, rank, 2, DEV, model=model)
    assert sorted(written) == sorted(set(written)) and len(written) == 4
    ds = find_dataset_def(args.dataset)(args.testpath, args.testlist, "test", 3, numdepth, 1.06,
                                        inverse_depth=False, adaptive_scaling=True, max_h=32,
                                        max_w=48, sample_scale=1, base_image_size=8)
    model = model.to(DEV).eval()
    for i in range(len(ds)):
        s = ds[i]
        with torch.no_grad():
            out = model(torch.from_numpy(s["imgs"])[None].to(DEV),
                        torch.from_numpy(s["proj_matrices"])[None].to(DEV),
                        torch.from_numpy(s["depth_values"])[None].to(DEV))
        f = root / "out" / s["filename"].format("depth_est_0", ".pfm")
        saved = fusion.read_pfm(str(f))[0]
        if numdepth == 32:   # the evidential head runs (B = 1, D = 32): gamma, as eval.py
            ev = out["evidential_prediction"].cpu().numpy()
            np.testing.assert_array_equal(saved, ev[0])
            assert (root / "out" / s["filename"].format("epistemic_0", ".pfm")).exists()
        else:
            np.testing.assert_array_equal(saved, out["depth"][0].cpu().numpy())
        conf = fusion.read_pfm(str(root / "out" / s["filename"].format("confidence_0", ".pfm")))[0]
        np.testing.assert_array_equal(conf, out["photometric_confidence"][0].cpu().numpy())


def test_sharded_eval_two_rank_processes_share_one_gpu(tmp_path):
    """``python -m aarmvs.eval_sharded`` as two rank processes (LOCAL_RANK 0 and 1) on the one
    GPU (AARMVS_SHARED_GPU=1: rank 1 maps to cuda:0 through local_device_index, as in
    train_ddp and bench.py): each writes its shard, together every sample once."""
    import os
    import subprocess
    import sys
    from conftest import ROOT
    root = _tree(tmp_path)
    cmd = [sys.executable, "-m", "aarmvs.eval_sharded", "--testpath", str(root), "--testlist",
           str(root / "list.txt"), "--outdir", str(root / "out"), "--max_h", "32", "--max_w", "48",
           "--numdepth", "16", "--view_num", "3", "--interval_scale", "1.06"]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", AARMVS_SHARED_GPU="1",
                   PYTHONPATH=os.pathsep.join([os.path.join(ROOT, "aa-rmvsnet_amd"), ROOT,
                                               os.environ.get("PYTHONPATH", "")]))
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
        assert p.returncode == 0, out[-3000:]
    assert "rank 0/2: 2 reference views written" in outs[0], outs[0][-2000:]
    assert "rank 1/2: 2 reference views written" in outs[1], outs[1][-2000:]
    pfms = sorted(p.name for p in (root / "out").rglob("*.pfm") if "depth_est_0" in str(p))
    assert len(pfms) == 4
