"""Time the reference-numerics composite kernels (anr_composite_ref16_fwd / _bwd) at the
bench shape (profiling aid): 8,192 rays x 1,024 samples x 4 bands, atmospheric sigma,
f16 inputs as the field writes them, surface colour on. HIP-event averages of 10 warm
launches each.

    python tools/ref16_bench.py [--rays 8192] [--samples 1024]
"""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "atmospheric-neural-rendering_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from atmonr_amd import _lib  # noqa: E402
from atmonr_amd.graphics_utils import render_with_surface_ref16  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=8192)
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    B, N = a.rays, a.samples
    z = torch.sort(torch.rand(B, N, device=dev, generator=g), 1)[0] * 0.227
    color = torch.rand(B, N, 4, device=dev, generator=g).half().requires_grad_()
    sigma = (torch.rand(B, N, 1, device=dev, generator=g) * 2e-4).half().requires_grad_()
    cs = torch.rand(B, 4, device=dev, generator=g).half().requires_grad_()
    gcm = ((torch.rand(B, 4, device=dev, generator=g) - 0.5) * 2e-3).half()
    timer = _lib.KernelTimer()
    for it in range(a.iters + 2):
        if it == 2:
            timer.__enter__()
        out = render_with_surface_ref16(z, color, sigma, cs, z_scale=100.0)
        out[0].backward(gcm)
    timer.__exit__(None, None, None)
    torch.cuda.synchronize()
    for k, v in sorted(timer.summary().items()):
        print(f"{k}: avg {v['avg_ms']:.4f} ms ({v['launches']} calls)", flush=True)


if __name__ == "__main__":
    main()
