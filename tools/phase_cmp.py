"""Side-by-side decoder phase clocks of two or more phases_*.json files."""
import json
import sys

ds = [json.load(open(f))["decoder_phase_clocks_per_frame"] for f in sys.argv[1:]]
keys = list(ds[-1].keys())
print(f"{'phase':24s}" + "".join(f"{f.split('/')[-1][7:-5]:>16s}" for f in sys.argv[1:]))
for k in keys:
    print(f"{k:24s}" + "".join(f"{d.get(k, 0):16.1f}" for d in ds))
clk = [k for k in keys if not k.startswith("n_") and k != "stream_clock_max_over_mean"]
print(f"{'TOTAL clocks':24s}" + "".join(f"{sum(d.get(k, 0) for k in clk):16.1f}" for d in ds))
