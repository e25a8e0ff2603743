"""Summary of the last tools/gpu/iter.sh run (gpurun_out/)."""
import json
import os

G = "gpurun_out"
print(open(os.path.join(G, "iter_tests.log")).read().strip().splitlines()[-1])
d = json.loads(open(os.path.join(G, "iter_bench.json")).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"value {d['value'] / 1e6:.2f} M reads/s  ms/step {d['ms_per_step']:.2f}  busy/step {r['kernel_busy_ms_per_step']:.2f}  "
      f"parity {d.get('parity')}")
if os.path.exists(os.path.join(G, "phase.json")):
    p = json.load(open(os.path.join(G, "phase.json")))
    c = p["cycles_per_read"]
    keys = ("setup", "lookup", "insert", "select", "rank", "fetch", "candlist", "stage", "lv_fwd", "lv_rev", "apply",
            "passloop", "writeback", "score", "cycles_per_read_total", "n_batch", "n_elems_forced")
    print("phase kernel_ms", round(p["kernel_ms"], 2), {k: round(c[k]) if c[k] > 100 else round(c[k], 2) for k in keys if k in c})
