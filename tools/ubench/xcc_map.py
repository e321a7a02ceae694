"""Observed workgroup -> XCD placement (ub_xcc_map): for grids of 4096 x 256-thread
workgroups, with and without a per-(b % 8) imbalance, print how often blocks b and b + 8k
land on the XCD that block b % 8 got. Measurement aid for the XCD-affine hash forward.

    python tools/ubench/xcc_map.py
"""

import collections
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from peaks import LIB  # noqa: E402


def main():
    lib = ctypes.CDLL(LIB)
    lib.ub_xcc_map.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev).cuda_stream
    for blocks, spin in [(4096, 0), (4096, 2000), (4096, 20000), (16384, 2000)]:
        out = torch.full((blocks,), -1, dtype=torch.int32, device=dev)
        assert lib.ub_xcc_map(out.data_ptr(), blocks, spin, st) == 0
        torch.cuda.synchronize()
        x = out.cpu().tolist()
        first = x[:8]
        same = sum(1 for b, v in enumerate(x) if v == first[b % 8]) / blocks
        per_res = {r: dict(collections.Counter(x[r::8]).most_common(3)) for r in range(8)}
        print(json.dumps({"blocks": blocks, "spin": spin, "first8": first,
                          "frac_on_xcd_of_b_mod_8": round(same, 4),
                          "xcc_counts": dict(collections.Counter(x)),
                          "per_residue_top": per_res}), flush=True)


if __name__ == "__main__":
    main()
