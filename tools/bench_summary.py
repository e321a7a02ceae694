"""Print the headline of a bench.py JSON log: value, ms/step, roofline, kernel table."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print({k: d[k] for k in ("value", "ms_per_step", "final_loss")})
r = d.get("roofline") or {}
print("roofline", {k: r.get(k) for k in ("kernel", "bound", "achieved", "frac", "avg_ms", "traffic")})
for k, v in (d.get("kernels") or {}).items():
    print(f"  {k:28s} {v.get('avg_ms', 0):8.4f} ms/launch {v.get('ms_per_step', 0):8.4f} ms/step",
          {x: v[x] for x in ("hbm_frac", "mfma_frac") if x in v})
