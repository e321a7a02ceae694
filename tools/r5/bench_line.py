"""One-line digest of a bench.py JSON log: python tools/r5/bench_line.py LOG [label]."""
import json
import sys

line = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(line)
r = d.get("roofline") or {}
k = d.get("kernels") or {}
ks = " ".join(f"{n}={v.get('avg_ms')}" for n, v in list(k.items())[:6])
print(sys.argv[2] if len(sys.argv) > 2 else "", d.get("numerics"), d["value"], d["ms_per_step"],
      "| dom", r.get("kernel"), r.get("avg_ms"), r.get("frac"),
      "req", r.get("atomic_requests_before_after"), "nz", r.get("d_enc_nonzero_before_after"),
      "rows", r.get("d_enc_nonzero_rows_before_after"), "|", ks, flush=True)
