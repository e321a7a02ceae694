"""Per-kernel steady-state counter table from tools/sq_bench.sh output.

    python tools/pmc_table.py gpurun_out/sq_bench [kernel-substring ...]

Each counter: median over the second half of the kernel's launches (bench.py settles the
reference numerics for 150 steps first, so that half is the settled state)."""

from __future__ import annotations

import collections
import csv
import glob
import os
import sys

KERNELS = {"hash_fwd": "hashgrid_fwd_planes_kernel<",
           "hash_bwd": "hashgrid_bwd_v2_kernel<3, __half, 3, 32, false, 6, true>",
           "hash_bwd_build": "hashgrid_bwd_v2_kernel<3, float, 3, 32",
           "field_fwd": "field::fwd_kernel<64, 2",
           "hash_field_fwd": "hf_fwd_kernel<64, 2",
           "field_bwd": "field::bwd_rt_kernel<64, 2, true, false, false, 4>",
           "field_bwd_list": "field::bwd_rt_kernel<64, 2, true, false, false, 3>",
           "field_bwd_build": "field::bwd_rt_kernel<64, 2, true, false, false, 0>",
           "sampler": "sample_uniform_bins_kernel",
           "comp_fwd": "ref16::fwd_kernel<",
           "comp_bwd": "ref16::bwd_kernel<",
           "nerf_nt_p256": "nerfmlp::nt_kernel<1, 4, 4, 4, 2>",
           "nerf_nt_2x2": "nerfmlp::nt_kernel<2, 2, 4, 4, 2>",
           "nerf_dw": "nerfmlp::dw_kernel("}


def main(src):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(src, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            for tag, pat in KERNELS.items():
                if pat in r["Kernel_Name"]:
                    vals[tag][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for tag in KERNELS:
        if tag not in vals:
            continue
        print(f"== {tag}")
        med = {}
        for c, v in vals[tag].items():
            tail = sorted(v[len(v) // 2:])
            med[c] = tail[len(tail) // 2]
        for c in sorted(med):
            print(f"  {c:34s} {med[c]:.4g}")
        wc = med.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in med:
                    print(f"  {c + ' / WAVE_CYCLES':34s} {med[c] / wc:.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
