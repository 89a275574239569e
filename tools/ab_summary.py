"""One row per bench.py line: headline value, ms/step, warp+aggregation and the main kernels'
average launch times (round-6 A/B helper).  usage: python tools/ab_summary.py LINE.json ..."""
import json
import sys

KS = ["omega_conv", "cost_x", "omega_stats1", "lstm_cell0", "lstm_cell1", "lstm_cell2", "lstm_cell3",
      "lstm_cell4", "deconv0", "deconv1", "head_wta"]
for path in sys.argv[1:]:
    try:
        d = json.loads(open(path).read().strip().split("\n")[-1])
    except Exception as e:  # noqa: BLE001
        print(path, "unreadable", e)
        continue
    k = d.get("kernels", {})
    wa = d.get("warp_aggregation", {})
    ks = " ".join(f"{n}={k[n]['avg_us']:.1f}" for n in KS if n in k)
    print(f"{path.split('/')[-1]:24s} {d['value'] / 1e9:.4f} G  {d['ms_per_step']:.1f} ms  "
          f"wa {wa.get('us_per_plane', 0):.1f} us/pl ({wa.get('frac', 0):.3f})  {ks}")
