"""Throughput of the AtmoNeRF dense-layer kernels (csrc/nerf_mlp.hip) at the fine model's
bench shape (4,096 rays x 192 samples = 786,432 rows), against torch's library GEMMs on
the same operands. HIP events around 10 launches each after 3 warm-ups.

    python tools/r5/nerf_gemm_probe.py
"""

from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "atmospheric-neural-rendering_amd")]

import torch  # noqa: E402

from atmonr_amd import _lib  # noqa: E402


def timed(fn, reps=10, warm=3):
    for _ in range(warm):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    dev = torch.device("cuda")
    M = 786432
    st = _lib.stream(dev)
    lib = _lib.load()
    shapes = [(256, 256), (76, 256), (332, 256), (256, 260), (280, 128), (128, 4)]
    args = [a for a in sys.argv[1:] if a != "--zeros"]
    zeros = "--zeros" in sys.argv   # all-zero operands: the clock / data-toggling check
    if args:   # e.g. "256x256" (q x n): only that shape (counter passes)
        shapes = [tuple(int(v) for v in a.split("x")) for a in args]
    for (q, n) in shapes:
        x = torch.randn(M, q, device=dev)
        w = torch.randn(n, q, device=dev) * 0.05
        b = torch.randn(n, device=dev)
        ld = (n + 3) // 4 * 4
        y = torch.empty(M, ld, device=dev)
        g = torch.randn(M, ld, device=dev)
        g[:, n:] = 0
        wt = torch.zeros(q, ld, device=dev)
        wt[:, :n] = w.t()
        dxo = torch.empty(M, q, device=dev)
        dw = torch.zeros(n, q, device=dev)
        db = torch.zeros(n, device=dev)
        ws = torch.empty(lib.anr_nerf_linear_dw_workspace(M, n, q) // 4 + 4, device=dev)
        fl = 2.0 * M * n * q
        if zeros:
            for t in (x, w, b, g, wt):
                t.zero_()
        bits = torch.empty(M, (n + 63) // 64, dtype=torch.int64, device=dev)
        mb = torch.full((M, (q + 63) // 64), 0x5555555555555555, dtype=torch.int64, device=dev)
        pq = q // 64 * 64   # the masked part of dX must be whole 64-column words
        t_f = timed(lambda: _lib.call("anr_nerf_linear_fwd", _lib.ptr(x), q, q, None, 0, 0, M,
                                      _lib.ptr(w), n, _lib.ptr(b), 1, _lib.ptr(y), ld,
                                      _lib.ptr(bits), st))
        t_x = timed(lambda: _lib.call("anr_nerf_linear_dx", _lib.ptr(g), ld, M, n,
                                      _lib.ptr(wt), ld, pq, q - pq, _lib.ptr(mb) if pq else None,
                                      _lib.ptr(dxo) if pq else None, q,
                                      _lib.ptr(dxo[:, pq:]) if q - pq else None, q, 0, st))
        t_w = timed(lambda: _lib.call("anr_nerf_linear_dw", _lib.ptr(g), ld, M, n, _lib.ptr(x),
                                      q, q, None, 0, 0, _lib.ptr(dw), _lib.ptr(db),
                                      _lib.ptr(ws), ws.numel() * 4, st))
        gg = g[:, :n]
        t_lf = timed(lambda: torch._addmm_activation(b, x, w.t()))
        t_lx = timed(lambda: gg @ w)
        t_lw = timed(lambda: gg.t() @ x)
        tf = lambda t: fl / (t * 1e-3) / 1e12
        print(f"q={q:4d} n={n:4d} | native fwd {t_f:.3f} ms {tf(t_f):6.1f} TF  dx {t_x:.3f} "
              f"{tf(t_x):6.1f}  dw {t_w:.3f} {tf(t_w):6.1f} | library fwd {t_lf:.3f} "
              f"{tf(t_lf):6.1f}  dx {t_lx:.3f} {tf(t_lx):6.1f}  dw {t_lw:.3f} {tf(t_lw):6.1f}",
              flush=True)
        del x, w, y, g, wt, dxo, ws


if __name__ == "__main__":
    main()
