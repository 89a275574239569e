"""bench.py's multi-rank path as the driver's N-GPU run exercises it: ``--gpus N``
without a launcher spawns N rank processes (one per GPU), each sweeps its own reference
views, and rank 0 prints one JSON line with n_gpus = N and the aggregate over all ranks.

On a one-GPU box the ranks share the card under AARMVS_SHARED_GPU=1 (gloo for the timing
collectives, since RCCL refuses two ranks on one device); without the switch ``--gpus 2``
must refuse to oversubscribe (exit 2).
"""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--config", "dtu_eval_800x600_n5_d256", "--planes", "2", "--steps", "1", "--warmup", "1",
         "--no-cpu", "--no-e2e", "--no-fusion", "--no-train", "--no-kernel-timing"]


def _bench(args, extra_env=None, timeout=300):
    env = dict(os.environ, **(extra_env or {}))
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=timeout, cwd=ROOT)


def _line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_two_ranks_report_the_aggregate():
    one = _bench(["--gpus", "1"] + SMALL)
    assert one.returncode == 0, one.stderr[-3000:]
    two = _bench(["--gpus", "2"] + SMALL, {"AARMVS_SHARED_GPU": "1"})
    assert two.returncode == 0, two.stderr[-3000:]
    l1, l2 = _line(one.stdout), _line(two.stdout)
    assert l1["n_gpus"] == 1 and l2["n_gpus"] == 2
    assert l2["config"]["global_batch"] == 2 * l1["config"]["global_batch"]
    # value = hypotheses of all ranks over the max-over-ranks time
    hyp2 = 2 * 600 * 800 * 2
    assert abs(l2["value"] * l2["ms_per_step"] / 1e3 - hyp2) / hyp2 < 1e-2


def test_bench_refuses_to_oversubscribe_one_gpu():
    if torch.cuda.device_count() >= 2:
        pytest.skip("two or more GPUs visible: --gpus 2 is a real two-GPU run here")
    r = _bench(["--gpus", "2"] + SMALL)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])


TRAIN = ["--train", "--train-planes", "4", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-kernel-timing"]


def test_bench_train_mode_one_and_two_ranks():
    """``--train`` (config 4's DDP step, train.py:172, 288-307): one JSON line per run with
    n_gpus = N, samples/s = N x steps over the max-over-ranks time, finite loss and gradients,
    and (N > 1) the gradient all-reduce timed beside it."""
    one = _bench(["--gpus", "1"] + TRAIN)
    assert one.returncode == 0, one.stderr[-3000:]
    two = _bench(["--gpus", "2"] + TRAIN, {"AARMVS_SHARED_GPU": "1"}, timeout=600)
    assert two.returncode == 0, two.stderr[-3000:]
    l1, l2 = _line(one.stdout), _line(two.stdout)
    for ln, n in ((l1, 1), (l2, 2)):
        assert ln["n_gpus"] == n and ln["unit"] == "samples/s"
        assert ln["config"]["global_batch"] == n and ln["config"]["parallelism"] == f"ddp x{n}"
        assert ln["loss_and_grads_finite"]
        assert abs(ln["value"] * ln["ms_per_step"] / 1e3 - n) < 1e-2 * n
    assert l2["allreduce"]["params"] == l1["allreduce"]["params"] > 0
    assert l2["allreduce"]["ms"] > 0 and l2["allreduce"]["backend"] == "gloo"
