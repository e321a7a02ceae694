"""Side-by-side Instant-NGP training with PSNR checkpoints (helper of the PSNR tests and of
tools/ingp_oracle_spread.py; not collected by pytest).

A *runner* is an object with ``step(batch, u) -> float`` (forward, loss, backward, AdamW
step; returns the loss) and ``render(batch, u) -> (B, C) colour map`` (no grad). The
same batches (BatchLoader seed 3, batch 256) and stratified draws (generator seed 7)
feed every runner, so any difference between runners comes from their arithmetic.
PSNR is harp2.py:310-335's, of a midpoint (u = 0.5) render of every ray of the scene.
"""

from __future__ import annotations

import torch

BATCH, SEED_BATCH, SEED_U = 256, 3, 7
CHECKPOINTS = (0, 8, 16, 32, 64)


def render_psnr(render, scene, n_samples: int, chunk: int = 1024) -> float:
    n = len(scene)
    pix = torch.empty(n)
    with torch.no_grad():
        for s in range(0, n, chunk):
            idx = torch.arange(s, min(n, s + chunk), device=scene.device)
            b = scene.__getbatch__(idx)
            cm = render(b, torch.full((idx.numel(), n_samples), 0.5))
            pix[s:s + idx.numel()] = torch.take_along_dim(
                cm.double().cpu(), b["irgb_idx"].cpu()[:, None], 1)[:, 0].float()
    img = scene.scatter_image(pix.to(scene.device))
    return float(scene.get_image_metrics(img, scene.target_image())["PSNR_mean"])


def train_side_by_side(runners: dict, scene, n_samples: int, checkpoints=CHECKPOINTS,
                       batch: int = BATCH, progress=None) -> dict:
    """{name: [{"iteration", "loss", "psnr"}, ...]} at every checkpoint; ``progress(out)``
    is called after each checkpoint (the GPU tests write their JSON record there)."""
    from atmonr_amd.batch_loader import BatchLoader

    gen = torch.Generator().manual_seed(SEED_U)
    loader = BatchLoader(scene, batch, seed=SEED_BATCH)
    out = {k: [] for k in runners}
    loss = {k: float("nan") for k in runners}
    it = 0
    last = max(checkpoints)
    batches = iter(loader)
    while True:
        if it in checkpoints:
            for k, r in runners.items():
                # a runner with render_from > it skips this checkpoint's render (psnr None)
                skip = it < getattr(r, "render_from", 0)
                out[k].append({"iteration": it, "loss": loss[k],
                               "psnr": None if skip else render_psnr(r.render, scene, n_samples)})
            if progress is not None:
                progress(out)
        if it >= last:
            return out
        try:
            b = next(batches)
        except StopIteration:
            batches = iter(loader)
            b = next(batches)
        u = torch.rand(b["origin"].shape[0], n_samples, generator=gen)
        for k, r in runners.items():
            loss[k] = r.step(b, u, it)
        it += 1


class OracleRunner:
    """ref_ingp.RefInstantNGP + torch AdamW. ``perturb_ray=k``: at iteration 0 the
    loss gradient reaching the rendered colour of ray k (at its IRGB band), an f16 value,
    is moved by one f16 ulp: one rounding of the reference's f16 backward done the other
    way."""

    def __init__(self, oracle, opt_cfg, perturb_ray=None, perturb_dirs=None,
                 master: str = "f64", grad_noise=None):
        self.o = oracle
        self.opt = oracle.optimizer(opt_cfg)
        self.perturb_ray = perturb_ray
        # master="f32": parameters and AdamW moments rounded to f32 after every step, as
        # the reference keeps them (tinycudann's f32 params, torch AdamW in f32; the oracle
        # otherwise trains f64 masters)
        self.master = master
        # grad_noise=(eps, seed): every step, every parameter gradient times (1 + eps * n),
        # n standard normal per element -- per-step arithmetic noise of the size the GPU's
        # reference numerics differ from this oracle by (relative L2 ~3e-5, MFMA f32 vs
        # f64 accumulation and the f16 rounding flips it causes)
        self.grad_noise = grad_noise
        if grad_noise and len(grad_noise) > 2 and grad_noise[2] == "x":
            # the MLPs' input gradients (dL/d encoding) carry f32-dot-product noise before
            # tcnn's f16 rounding (oracle/ref_ingp.py _TcnnCall, spread experiments only)
            self.o.mlp_x_noise = (torch.Generator().manual_seed(int(grad_noise[1])),
                                  float(grad_noise[0]))
            self.grad_noise = None
        if grad_noise and len(grad_noise) > 2 and grad_noise[2] == "sum":
            # the hash grid's parameter gradient carries f32-summation-order noise instead
            # (oracle/ref_ingp.py _TcnnCall, spread experiments only)
            self.o.grid_sum_noise = (torch.Generator().manual_seed(int(grad_noise[1])),
                                     float(grad_noise[0]))
            self.grad_noise = None
        self._noise_gen = (torch.Generator().manual_seed(int(grad_noise[1]))
                           if grad_noise else None)
        # perturb_dirs=seed: every ray direction moved by one f32 ulp (sign per ray and
        # component from the seed) in training and rendering -- the size of the device-vs-
        # host f64 libm differences in scene construction
        self.perturb_dirs = perturb_dirs

    def _batch(self, b):
        from oracle import ref_ingp

        cb = ref_ingp.cpu_batch(b)
        if self.perturb_dirs is not None:
            sign = torch.Generator().manual_seed(int(self.perturb_dirs))
            table = torch.randint(0, 2, (1 << 20, 3), generator=sign).bool()
            up = table[cb["idx"] % (1 << 20)]
            d = cb["dir"]
            inf = torch.full_like(d, float("inf"))
            cb = dict(cb, dir=torch.where(up, torch.nextafter(d, inf), torch.nextafter(d, -inf)))
        return cb

    def step(self, b, u, it):
        cb = self._batch(b)
        res = self.o.forward(cb, u)
        self.last = res  # the step's forward results (tools/liveness_paired.py reads sigma)
        if it == 0 and self.perturb_ray is not None:
            k = self.perturb_ray
            c = int(cb["irgb_idx"][k])

            def bump(g):  # dL/dcolor_map of ray k, one f16 ulp up
                g = g.clone()
                v = g[k, c].half()
                g[k, c] = torch.nextafter(v, torch.tensor(float("inf"), dtype=v.dtype)).to(g.dtype)
                return g
            res["color_map_fine"].register_hook(bump)
        loss = self.o.loss(cb, res)
        self.opt.zero_grad()
        loss.backward()
        if self.grad_noise:
            with torch.no_grad():
                for g in self.opt.param_groups:
                    for p in g["params"]:
                        if p.grad is not None:
                            n = torch.randn(p.grad.shape, generator=self._noise_gen,
                                            dtype=p.grad.dtype)
                            p.grad.mul_(1 + self.grad_noise[0] * n)
        self.opt.step()
        if self.master == "f32":
            with torch.no_grad():
                for g in self.opt.param_groups:
                    for p in g["params"]:
                        p.copy_(p.float().double())
                        st = self.opt.state.get(p, {})
                        for k in ("exp_avg", "exp_avg_sq"):
                            if k in st:
                                st[k].copy_(st[k].float().double())
        return loss.item()

    def render(self, b, u):
        return self.o.forward(self._batch(b), u)["color_map_fine"]


class PipelineRunner:
    """An atmonr_amd InstantNGPPipeline on the GPU with its FusedAdam."""

    def __init__(self, pipe, opt_cfg, dev):
        self.p = pipe
        self.opt = pipe.get_optimizer(opt_cfg)
        self.dev = dev

    def step(self, b, u, it):
        loss = self.p.compute_loss(b, self.p.forward(b, u=u.to(self.dev)))
        self.opt.zero_grad()
        loss.backward()
        self.opt.step()
        return loss.item()

    def render(self, b, u):
        return self.p.forward(b, u=u.to(self.dev))["color_map_fine"]
