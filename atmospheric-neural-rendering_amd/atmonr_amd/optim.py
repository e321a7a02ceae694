"""FusedAdam — torch.optim.Optimizer on the K10 kernel (one HBM pass per tensor).

Drop-in for torch.optim.AdamW (instant_ngp.py:120-126; ``decoupled=True``) and
torch.optim.Adam (nerf.py:70; ``decoupled=False``): same param-group semantics, same
state keys (``step``, ``exp_avg``, ``exp_avg_sq``) so optimizer state dicts interchange
with torch's.
"""

from __future__ import annotations

import torch

from . import _lib
from ._lib import call, ptr


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 decoupled: bool = True, zero_grad_in_step: bool = False, **unused):
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.decoupled = decoupled
        # zero each gradient in the update pass (the next optimizer.zero_grad() is then a
        # no-op for buffers that stay allocated, e.g. a FlatGradBucket: see mark_zero)
        self.zero_grad_in_step = zero_grad_in_step
        self.zeroed_buckets: list = []  # FlatGradBucket.fuse_zero_into

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.dtype != torch.float32 or p.grad.dtype != torch.float32:
                    raise _lib.ANRError("FusedAdam needs float32 params and grads")
                st = self.state[p]
                if not st:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                if st["step"].device.type != "cpu":
                    # a checkpoint loaded with map_location=<gpu> puts 'step' on the device;
                    # keep it on the host so the step count never costs a device sync
                    st["step"] = st["step"].cpu()
                st["step"] += 1
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                # the f16 compute copy of the parameter (_lib.compute_copy), if a module
                # keeps one, is written in the same pass and stays current
                sh = getattr(p, "_anr_shadow", None)
                if sh is not None and (sh.dtype != torch.float16 or sh.shape != p.shape):
                    sh = None
                call("anr_adam_step", ptr(p), ptr(g), ptr(st["exp_avg"]),
                     ptr(st["exp_avg_sq"]), ptr(sh), p.numel(), float(group["lr"]),
                     float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]),
                     int(self.decoupled), int(st["step"].item()),
                     int(self.zero_grad_in_step), _lib.stream(p.device))
                if sh is not None:
                    p._anr_shadow_ver = p._version
        if self.zero_grad_in_step:
            for b in self.zeroed_buckets:
                b.mark_zero()
        return loss
