"""Launch overhead of small sweeps (round 6): one eval sweep at a BASELINE
config (default config 1, 160x128, N=3, D=48) timed as ordinary stream launches and as a
replayed HIP graph of the same call (torch.cuda.CUDAGraph capture), with the outputs compared.
usage: [PROBE_OVERLAP=0] python tools/graph_probe.py [N H W D]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")]
import torch  # noqa: E402

from aarmvs import ops, synthetic as syn  # noqa: E402

N, H, W, D = (int(x) for x in sys.argv[1:5]) if len(sys.argv) >= 5 else (3, 128, 160, 48)
B = 1
sc = syn.scene(B, N, H, W, D, seed=0)
P = {k: torch.from_numpy(v).cuda() for k, v in syn.sweep_weights(1).items()}
sw = ops.DepthSweep(P, "cuda", overlap=os.environ.get("PROBE_OVERLAP", "1") == "1")
f = torch.from_numpy(sc["features"]).cuda()
proj = torch.from_numpy(sc["proj_matrices"])
dv = torch.from_numpy(sc["depth_values"]).cuda().float().contiguous()
ref, srcs = f[0].contiguous(), [f[v].contiguous() for v in range(1, N)]
rel = sw.relative(proj[:, 0], [proj[:, v] for v in range(1, N)], B)
cost = torch.empty(B, D, H, W, device="cuda")


def run():
    return sw(ref, srcs, None, [None] * (N - 1), dv, want_depth=True, cost_out=cost, rel=rel)


out = run()
torch.cuda.synchronize()
print("eager sweep done", flush=True)
eager_depth = out["depth"].clone()
eager_cost = cost.clone()
K = 30
for _ in range(3):
    run()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    run()
torch.cuda.synchronize()
t_eager = (time.perf_counter() - t0) / K

g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    run()   # warm-up on the capture stream
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
print("capturing", flush=True)
with torch.cuda.graph(g):
    gout = run()
torch.cuda.synchronize()
print("captured", flush=True)
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    g.replay()
torch.cuda.synchronize()
t_graph = (time.perf_counter() - t0) / K
same = torch.equal(gout["depth"], eager_depth) and torch.equal(cost, eager_cost)
hyp = B * H * W * D
print(f"{W}x{H} N={N} D={D}: eager {t_eager * 1e3:.3f} ms ({hyp / t_eager / 1e9:.3f} G hyp/s, "
      f"{t_eager / D * 1e6:.1f} us/plane); graph {t_graph * 1e3:.3f} ms ({hyp / t_graph / 1e9:.3f} G hyp/s, "
      f"{t_graph / D * 1e6:.1f} us/plane); outputs bit-identical: {same}", flush=True)
