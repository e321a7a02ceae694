"""Join tools/hash_level_probe.py's launch order with the rocprofv3 --pmc passes of
tools/archive/r3_hash_level_pmc.sh: per (grid, rep) duration, TCC hit/miss, FETCH_SIZE and
WRITE_SIZE per sample. FETCH_SIZE is printed raw and calibrated: 4-B gathers count one
64-B unit per TCC miss (profiles/r03_gather_calib), the 12-B/sample coordinate stream is
half-counted (MI355X_MICROARCH.md), so calibrated fetch = raw + 6 B/sample.

    python tools/hash_level_table.py gpurun_out/r4c [--md]
"""

import collections
import csv
import json
import sys


def per(d, f):
    rows = list(csv.DictReader(open(f"{d}/{f}/run_counter_collection.csv")))
    agg = collections.OrderedDict()
    for r in rows:
        if "hashgrid_fwd" not in r["Kernel_Name"]:
            continue
        e = agg.setdefault(int(r["Dispatch_Id"]),
                           {"dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [agg[k] for k in sorted(agg)]


def main():
    d = sys.argv[1]
    rec = json.load(open(f"{d}/levels.json"))
    hit, fe, wr = per(d, "hit"), per(d, "fetch"), per(d, "write")
    M = rec["samples"]
    groups = collections.OrderedDict()
    for o, h, f, w in zip(rec["launch_order"], hit, fe, wr):
        if o[0] == "warmup" or o[1] == 0:
            continue  # cold L2 / first touch
        g = groups.setdefault(str(o[0]), collections.defaultdict(list))
        g["ms"].append(h["dur"])
        g["hit"].append(h["TCC_HIT_sum"] / M)
        g["miss"].append(h["TCC_MISS_sum"] / M)
        g["fetch"].append(f["FETCH_SIZE"] * 1024 / M)
        g["write"].append(w["WRITE_SIZE"] * 1024 / M)
    newc = {f"level{r['level']}": r["new_cell_fraction"] for r in rec["levels"]}
    print("| grid | new cells / sample | ms (PMC run) | TCC hit / sample | TCC miss / sample "
          "| FETCH raw B / sample | fetch calibrated B / sample | WRITE B / sample |")
    print("|---|---|---|---|---|---|---|---|")
    for k, g in groups.items():
        av = {n: sum(v) / len(v) for n, v in g.items()}
        nc = newc.get(k)
        if nc is None and k.startswith("level"):
            nc = sum(newc[f"level{x}"] for x in k[5:].split("_"))
        if k == "full":
            nc = sum(newc.values())
        print(f"| {k} | {nc:.3f} | {av['ms']:.3f} | {av['hit']:.2f} | {av['miss']:.3f} | "
              f"{av['fetch']:.1f} | {av['fetch'] + 6:.1f} | {av['write']:.1f} |")


if __name__ == "__main__":
    main()
