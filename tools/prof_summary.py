"""Summarise a tools/prof.sh run into profiles/.

    python tools/prof_summary.py gpurun_out/prof_v3 r01

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, copied), profiles/<tag>_summary.md
(per-kernel average duration and HBM traffic per launch) and updates
profiles/pmc_traffic.json, which bench.py reads for roofline.traffic.

HBM traffic per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes: rocprofv3 reports
both in KiB; on gfx950 FETCH_SIZE counts exactly half the bytes of wide coalesced reads
(MI355X_MICROARCH.md §HBM), hence the factor 2. That correction is calibrated for
streaming reads; for the gather-heavy hash kernels it is an upper-bound estimate.
"""

from __future__ import annotations

import collections
import csv
import hashlib
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "atmospheric-neural-rendering_amd", "csrc")
# bench.py kernel tag prefix -> the source file that defines it (PMC entries carry its
# sha1, and bench.py ignores an entry whose kernel source has changed since)
SOURCES = {"hash": ("hashgrid.hip", "hash_levels.h"), "field": ("field_fused.hip", "hash_levels.h"),
           "composite": ("composite.hip",), "sampler": ("sampler.hip",)}


def source_sha1(tag: str) -> str | None:
    files = SOURCES.get(tag.split("_")[0])
    if files is None:
        return None
    h = hashlib.sha1()
    for f in files:
        h.update(open(os.path.join(CSRC, f), "rb").read())
    return h.hexdigest()

# bench.py kernel tag -> substring of the mangled/demangled kernel name
TAGS = {  # prefixes: one instantiation of each per bench run (width / dtype follow --variant, --dtype)
    "hash_fwd": "hashgrid_fwd_planes_kernel<3, __half",
    "hash_fwd_v6": "hashgrid_fwd_v6_kernel<3,",
    "hash_field_fwd": "hf_fwd_kernel<64, 2",
    "hash_fwd_v1": "hashgrid_fwd_kernel<3,",
    # reference numerics (the headline): the row-bit walker over f16 rows (r06); the build
    # numerics' dense f32 walker beside it (bench.py's alt_numerics leg)
    "hash_bwd": "hashgrid_bwd_v2_kernel<3, __half, 3, 32, false, 6, true>",
    "hash_bwd_build": "hashgrid_bwd_v2_kernel<3, float, 3, 32, false, 6, false>",
    "hash_bwd_rtstride": "hashgrid_bwd_v2_kernel<3, float, 0, 0>",
    "field_fwd": "field::fwd_kernel<",
    # reference numerics: the pos pass (zero-colour tiles) and the list pass (r06)
    "field_bwd": "field::bwd_rt_kernel<64, 2, true, false, false, 4>",
    "field_bwd_list": "field::bwd_rt_kernel<64, 2, true, false, false, 3>",
    "field_bwd_build": "field::bwd_rt_kernel<64, 2, true, false, false, 0>",
    "field_bwd_lds": "field::bwd_kernel<",
    "composite_fwd": "rb::fwd_kernel<float, 4, 1, 4>",
    "composite_bwd": "rb::bwd_kernel<float, 4, 1, 4>",
    "sampler": "sample_uniform_bins_kernel",
}


def per_launch(path: str) -> dict[str, float]:
    """Median per launch over the second half of each kernel's launches: the bench
    network is dead for its first few AdamW steps (tools/liveness.py: no densities, no
    hash-grid gradients, the backward's atomics skipped), so early launches are not the
    steady state the timed region measures."""
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, v in agg.items():
        tail = sorted(v[len(v) // 2:])
        out[k] = tail[len(tail) // 2]
    return out


def main(src: str, tag: str, key_suffix: str = "baseline:8192x1024"):
    prof = os.path.join(ROOT, "profiles")
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    fetch = per_launch(os.path.join(src, "fetch", "run_counter_collection.csv"))
    write = per_launch(os.path.join(src, "write", "run_counter_collection.csv"))
    rows = list(csv.DictReader(open(stats)))
    pmc_path = os.path.join(prof, "pmc_traffic.json")
    pmc = json.load(open(pmc_path)) if os.path.exists(pmc_path) else {}
    lines = [f"# rocprofv3 summary ({tag})", "",
             "bench.py (config-3 train step, 8192 rays x 1024 samples), "
             "`rocprofv3 --kernel-trace --stats` plus separate `--pmc FETCH_SIZE` and "
             "`--pmc WRITE_SIZE` passes (tools/prof.sh). Traffic = (2*FETCH_SIZE + "
             "WRITE_SIZE) KiB per launch (gfx950 FETCH_SIZE half-count correction; the "
             "hash-grid forward's 4-B gathers are counted in full, so its calibrated "
             "traffic in profiles/pmc_traffic.json is FETCH + 6 B/sample + WRITE: "
             "profiles/r03_hash_levels.md).", "",
             "Steady avg = mean duration over the second half of each kernel's launches in "
             "the kernel trace (the bench network is alive from step ~7; the first steps' "
             "backward skips its zero-gradient atomics).", "",
             "| kernel | calls | avg us | steady avg us | % time | HBM traffic / launch (MB) |",
             "|---|---|---|---|---|---|"]
    steady = {}
    tpath = os.path.join(src, "trace", "run_kernel_trace.csv")
    if os.path.exists(tpath):
        durs = collections.defaultdict(list)
        for r in csv.DictReader(open(tpath)):
            durs[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for k, v in durs.items():
            tail = v[len(v) // 2:]
            steady[k] = sum(tail) / len(tail) / 1e3
    for r in rows[:25]:
        name = r["Name"]
        f = next((v for k, v in fetch.items() if k == name or k.startswith(name[:80])), None)
        w = next((v for k, v in write.items() if k == name or k.startswith(name[:80])), None)
        traffic = (2 * f + w) * 1024 / 1e6 if f is not None and w is not None else None
        short = name.replace("|", "/")[:90]
        sa = next((v for k, v in steady.items() if k == name or k.startswith(name[:80])), None)
        lines.append(f"| `{short}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{'' if sa is None else f'{sa:.1f}'} | {float(r['Percentage']):.1f} | "
                     f"{'' if traffic is None else f'{traffic:.1f}'} |")
    apath = os.path.join(src, "atomic", "run_counter_collection.csv")
    atomic = per_launch(apath) if os.path.exists(apath) else {}
    for t, pat in TAGS.items():
        f = next((v for k, v in fetch.items() if pat in k), None)
        w = next((v for k, v in write.items() if pat in k), None)
        a = next((v for k, v in atomic.items() if pat in k), None)
        if f is not None and w is not None:
            ent = {"bytes": round((2 * f + w) * 1024), "fetch_kib": round(f, 1),
                   "write_kib": round(w, 1), "source": tag}
            if t.startswith("hash_fwd"):
                # 4-B corner gathers: FETCH_SIZE counts the 64 B of each miss in full
                # (tools/ubench gather_calib, profiles/r03_hash_levels.md); only the
                # 12-B/sample coordinate stream is half-counted
                B, N = (int(v) for v in key_suffix.rsplit(":", 1)[1].split("x"))
                ent["bytes"] = round(f * 1024 + 6 * B * N + w * 1024)
                ent["calibration"] = ("FETCH_SIZE not doubled for the 4-B gathers; "
                                      "+6 B/sample for the half-counted coordinates")
            if a:  # TCC_EA0_ATOMIC_sum: memory-side atomic requests (64-B segments)
                ent["atomic_requests"] = round(a)
            ent["kernel_source_sha1"] = source_sha1(t)
            pmc[f"{t}:{key_suffix}"] = ent
    json.dump(pmc, open(pmc_path, "w"), indent=1, sort_keys=True)
    open(os.path.join(prof, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *sys.argv[3:4])
