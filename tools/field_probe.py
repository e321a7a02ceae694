"""Standalone driver for the fused field kernels at bench size (profiling aid).

    python tools/field_probe.py [--rays 8192] [--samples 1024] [--width 64] [--iters 3]

Runs anr_ingp_field_pack / _fwd / _bwd on random inputs of the bench shape so rocprofv3
passes (--kernel-trace, --pmc SQ_*) see only these kernels. Prints per-kernel HIP-event
averages.
"""

from __future__ import annotations

import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "atmospheric-neural-rendering_amd"))

import torch  # noqa: E402

from atmonr_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=8192)
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--width", type=int, default=64)
    ap.add_argument("--nhd", type=int, default=2)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--bf16", action="store_true", help="bf16 MFMA operands (configs[4])")
    ap.add_argument("--fwd-mode", type=int, default=1,
                    help="anr_ingp_field_force_fwd: 1 uniform-tile form (default), 0 general")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    M = args.rays * args.samples
    lib = _lib.load()
    lib.anr_ingp_field_force_fwd(args.fwd_mode)
    pd_ = _lib.mlp_desc(32, 16, args.width, 1, False)
    dd_ = _lib.mlp_desc(19, 4, args.width, args.nhd, False)
    pdesc, ddesc = ctypes.byref(pd_), ctypes.byref(dd_)
    pp = torch.randn(lib.anr_mlp_n_params(pdesc), device=dev) * 0.2
    pdir = torch.randn(lib.anr_mlp_n_params(ddesc), device=dev) * 0.15
    enc = (torch.rand(M, 32, device=dev) * 2 - 1).half()
    dirs = torch.nn.functional.normalize(torch.randn(args.rays, 3, device=dev), dim=1)
    dcol = torch.randn(M, 4, device=dev) * 1e-3
    dsig = torch.randn(M, device=dev) * 1e-3
    packed = torch.empty(lib.anr_ingp_field_packed_size(pdesc, ddesc), device=dev,
                         dtype=torch.float16)
    sigma = torch.empty(M, device=dev)
    color = torch.empty(M, 4, device=dev)
    d_enc = torch.empty(M, 32, device=dev)
    g_pos = torch.zeros_like(pp)
    g_dir = torch.zeros_like(pdir)
    code = _lib.BF16 if args.bf16 else _lib.F16
    ws_bytes = lib.anr_ingp_field_bwd_workspace_bytes(pdesc, ddesc, code, M)
    ws = torch.empty(max(1, ws_bytes // 4), device=dev)
    s = _lib.stream(dev)
    timer = _lib.KernelTimer()
    with timer:
        for _ in range(args.iters):
            _lib.call("anr_ingp_field_pack", pdesc, ddesc, code, pp.data_ptr(),
                      pdir.data_ptr(), packed.data_ptr(), s, tag="pack")
            _lib.call("anr_ingp_field_fwd", pdesc, ddesc, code, packed.data_ptr(),
                      enc.data_ptr(), 32, dirs.data_ptr(), args.samples, M, sigma.data_ptr(),
                      color.data_ptr(), 4, s, tag="field_fwd")
            _lib.call("anr_ingp_field_bwd", pdesc, ddesc, code, packed.data_ptr(),
                      enc.data_ptr(), 32, dirs.data_ptr(), args.samples, M, dsig.data_ptr(),
                      dcol.data_ptr(), 4, d_enc.data_ptr(), 32, g_pos.data_ptr(),
                      g_dir.data_ptr(), ws.data_ptr(), ws_bytes, s, tag="field_bwd")
    torch.cuda.synchronize()
    for k, v in timer.summary().items():
        print(f"{k:12s} avg {v['avg_ms']:.4f} ms  ({v['launches']} calls)")
    print("finite:", bool(torch.isfinite(d_enc).all()), bool(torch.isfinite(g_dir).all()))
    # equal checksums across library builds = the same forward outputs (A/B runs)
    print(f"checksum sigma {sigma.double().sum().item()!r} color {color.double().sum().item()!r} "
          f"d_enc {d_enc.double().abs().sum().item()!r}")
    if hasattr(lib, "anr_debug_field_stamps"):  # FIELD_STAMP builds: per-stage cycles
        buf = (ctypes.c_ulonglong * 16)()
        lib.anr_debug_field_stamps(buf)
        names = ["prefetch", "fwd", "D2", "D1", "D0", "P1", "P0+enc"]
        tiles = max(1, buf[8])
        tot = sum(buf[k] for k in range(7))
        print(f"stamps over {buf[8]} tiles (wave 0), cycles/tile (s_memtime ticks):")
        for k, n in enumerate(names):
            print(f"  {n:9s} {buf[k] / tiles:9.0f}  {100 * buf[k] / max(1, tot):5.1f}%")


if __name__ == "__main__":
    main()
