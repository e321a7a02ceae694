"""FETCH_SIZE / TCC calibration for 4-B random gathers (the hash-grid forward's corner
loads), run under rocprofv3 --pmc (tools/pmc_gather.sh). Each launch makes a known number
of 4-B gathers into a table of a given size; the printed table lists them so the PMC
rows (one per launch, in this order) can be divided by the gather count.

    python tools/ubench/gather_calib.py [--out gpurun_out/gather_calib.json]
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from peaks import LIB  # noqa: E402

SIZES_MB = [1, 2, 16, 24, 96, 1024]   # one fine level (f16) ~2 MB, the table 24 MB, HBM 1 GB
BLOCKS, ITERS = 4096, 64              # 1,048,576 lanes x 64 = 67 M gathers per launch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    lib = ctypes.CDLL(LIB)
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.ub_gather.argtypes = [vp, i64, i32, i32, ctypes.c_uint32, vp, vp]
    dev = torch.device("cuda:0")
    sink = torch.zeros(256, dtype=torch.int32, device=dev)
    rows = []
    for mb in SIZES_MB:
        n = mb * (1 << 20) // 4
        table = torch.randint(0, 1 << 30, (n,), dtype=torch.int32, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        for r in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert lib.ub_gather(table.data_ptr(), n, ITERS, BLOCKS, 1234 + r, sink.data_ptr(),
                                 st) == 0
            e1.record()
            torch.cuda.synchronize()
            g = BLOCKS * 256 * ITERS
            rows.append({"table_mb": mb, "rep": r, "gathers": g, "requested_bytes": 4 * g,
                         "ms": e0.elapsed_time(e1),
                         "g_gathers_s": g / (e0.elapsed_time(e1) * 1e-3) / 1e9})
            print(json.dumps(rows[-1]), flush=True)
        del table
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        json.dump(rows, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
