"""Host enqueue time vs device time of the library's training calls at config 4 (640x512,
N=3, D=192): the recorded forward sweep and aarmvs_sweep_backward, each timed from the call to
its return (host: every launch enqueued) and to the end of a device synchronisation, per
backward schedule (AARMVS_BWD_PIPE).  If the host time approaches the device time the step is
launch-bound.  usage: python tools/host_time.py [D]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")]
import torch  # noqa: E402

from aarmvs import ops, synthetic as syn  # noqa: E402

B, N, H, W = 1, 3, 512, 640
D = int(sys.argv[1]) if len(sys.argv) > 1 else 192
nsrc = N - 1


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
    g = torch.randn_like(cost)

    def fwd():
        sw(ref, srcs, proj[:, 0], [proj[:, v] for v in range(1, N)], dv, want_depth=False, cost_out=cost,
           rel=rel, record=rec)

    def bwd():
        sw.backward(ref, srcs, rel, dv, rec, g)

    for name, fn, modes in (("forward", fwd, ("0",)), ("backward", bwd, ("0", "3", "1"))):
        for m in modes:
            os.environ["AARMVS_BWD_PIPE"] = m
            fn()
            torch.cuda.synchronize()
            hs, ds = [], []
            for _ in range(3):
                t0 = time.perf_counter()
                fn()
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                hs.append(t1 - t0)
                ds.append(t2 - t0)
            print(f"{name:8s} pipe {m}: host enqueue {min(hs) * 1e3:7.2f} ms, to device end {min(ds) * 1e3:7.2f} ms "
                  f"({min(ds) / D * 1e3:.3f} ms per plane)", flush=True)


if __name__ == "__main__":
    main()
