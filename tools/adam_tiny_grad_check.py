"""FusedAdam (f32, anr_adam_step_multi) against torch.optim.AdamW in f64 on gradients of
the sizes the reference-numerics hash grid sees (tcnn-quantised f16 / 128: 4.7e-10 up,
many exact zeros, sparse updates) with eps = 1e-15, where the update is ~lr * sign and
tiny arithmetic differences could matter. Prints the largest update difference in units
of lr, per step (diagnostic of the N = 1024 PSNR drift; needs the GPU).

    python tools/adam_tiny_grad_check.py [--n 1000000] [--steps 64]
"""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "atmospheric-neural-rendering_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=64)
    a = ap.parse_args()
    from atmonr_amd.optim import FusedAdam

    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    lr, wd = 1e-2, 0.0
    p0 = (torch.rand(a.n, generator=g, dtype=torch.float64) - 0.5) * 2e-4
    pf = torch.nn.Parameter(p0.float().to(dev))
    pr = torch.nn.Parameter(p0.float().double())
    of = FusedAdam([pf], lr=lr, betas=(0.9, 0.99), eps=1e-15, weight_decay=wd, decoupled=True)
    orf = torch.optim.AdamW([pr], lr=lr, betas=(0.9, 0.99), eps=1e-15, weight_decay=wd)
    worst = 0.0
    for t in range(a.steps):
        # log-uniform magnitudes 1e-10 .. 1e-2, random signs, 70 % exact zeros (untouched
        # entries), then tcnn's quantisation f16(f16(g * 128) / 128)
        mag = torch.exp(torch.empty(a.n, dtype=torch.float64).uniform_(-23, -4.6, generator=g))
        sgn = torch.randint(0, 2, (a.n,), generator=g).double() * 2 - 1
        keep = torch.rand(a.n, generator=g, dtype=torch.float64) > 0.7
        gr = (mag * sgn * keep).float()
        gr = ((gr * 128).half().float() / 128).half().float()
        before_f, before_r = pf.detach().double().cpu(), pr.detach().clone()
        pf.grad = gr.to(dev)
        pr.grad = gr.double()
        of.step()
        orf.step()
        # update difference in units of lr, from the same starting point per step
        du = ((pf.detach().double().cpu() - before_f) - (pr.detach() - before_r)).abs() / lr
        worst = max(worst, du.max().item())
        drift = (pf.detach().double().cpu() - pr.detach()).abs().max().item() / lr
        print(f"step {t + 1}: max |update_fused - update_ref| = {du.max().item():.3e} lr, "
              f"entries > 1e-3 lr: {int((du > 1e-3).sum())}, param drift {drift:.3e} lr",
              flush=True)
    print(f"worst {worst:.3e} lr")


if __name__ == "__main__":
    main()
