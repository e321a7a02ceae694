"""One bench step's kernel timeline from a rocprofv3 kernel trace (run_kernel_trace.csv):
start / end / duration relative to the step's sampler launch, with the queue, so the
side-stream (surface branch) overlap is visible. Prints the last complete step.

    python tools/step_timeline.py <trace_dir> [--steps 2]
"""

import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--steps", type=int, default=1)
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "sample_uniform_bins" in r["Kernel_Name"]]
    for k in range(len(starts) - 1 - a.steps, len(starts) - 1):
        i0, i1 = starts[k], starts[k + 1]
        t0 = int(rows[i0]["Start_Timestamp"])
        span = (int(rows[i1]["Start_Timestamp"]) - t0) / 1000
        print(f"== step: {span:.1f} us (sampler to sampler)")
        lo = i0
        while lo > 0 and int(rows[lo - 1]["End_Timestamp"]) > t0:
            lo -= 1
        for r in rows[lo:i1]:
            st = (int(r["Start_Timestamp"]) - t0) / 1000
            en = (int(r["End_Timestamp"]) - t0) / 1000
            print(f"{st:9.1f} {en:9.1f} {en - st:8.1f} q{r['Queue_Id']} {r['Kernel_Name'][:80]}")


if __name__ == "__main__":
    main()
