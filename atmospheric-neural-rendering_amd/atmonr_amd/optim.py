"""FusedAdam — torch.optim.Optimizer on the K10 kernel (one HBM pass per tensor).

Drop-in for torch.optim.AdamW (instant_ngp.py:120-126; ``decoupled=True``) and
torch.optim.Adam (nerf.py:70; ``decoupled=False``): same param-group semantics, same
state keys (``step``, ``exp_avg``, ``exp_avg_sq``) so optimizer state dicts interchange
with torch's.
"""

from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import call, ptr


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=None,
                 decoupled: bool = True, zero_grad_in_step: bool = False, **unused):
        if weight_decay is None:  # torch.optim.AdamW's default 1e-2, Adam's 0
            weight_decay = 1e-2 if decoupled else 0.0
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.decoupled = decoupled
        # zero each gradient in the update pass (the next optimizer.zero_grad() is then a
        # no-op for buffers that stay allocated, e.g. a FlatGradBucket: see mark_zero)
        self.zero_grad_in_step = zero_grad_in_step
        self.zeroed_buckets: list = []  # FlatGradBucket.fuse_zero_into
        self.multi_tensor = True  # one anr_adam_step_multi launch per step and device

    @torch.no_grad()
    def step(self, closure=None):
        """Every parameter of every group in one anr_adam_step_multi launch per device
        (``multi_tensor=False``: one anr_adam_step launch per parameter)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        # (device, beta1, beta2, eps) -> [anr_adam_tensor]: groups with their own betas /
        # eps get their own launch, as torch.optim.Adam(W) steps each group with its own
        batches: dict = {}
        for group in self.param_groups:
            b1, b2 = group["betas"]
            key_hp = (float(b1), float(b2), float(group["eps"]))
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
                if not p.grad.is_contiguous():
                    p.grad = p.grad.contiguous()
                # the f16 compute copy of the parameter (_lib.compute_copy), if a module
                # keeps one, is written in the same pass and stays current
                sh = getattr(p, "_anr_shadow", None)
                if sh is not None and (sh.dtype != torch.float16 or sh.shape != p.shape):
                    sh = None
                t = _lib.AdamTensor(ptr(p), ptr(p.grad), ptr(st["exp_avg"]),
                                    ptr(st["exp_avg_sq"]), ptr(sh), p.numel(),
                                    float(group["lr"]), float(group["weight_decay"]),
                                    int(st["step"].item()))
                batches.setdefault((p.device,) + key_hp, []).append(t)
                if sh is not None:
                    p._anr_shadow_ver = p._version
        for (dev, b1, b2, eps), ts in batches.items():
            if self.multi_tensor:
                arr = (_lib.AdamTensor * len(ts))(*ts)
                call("anr_adam_step_multi", ctypes.addressof(arr), len(ts), b1, b2, eps,
                     int(self.decoupled), int(self.zero_grad_in_step), _lib.stream(dev))
            else:
                for t in ts:
                    call("anr_adam_step", t.params, t.grad, t.exp_avg, t.exp_avg_sq,
                         t.params_f16, t.n, t.lr, b1, b2, eps, t.weight_decay,
                         int(self.decoupled), t.step, int(self.zero_grad_in_step),
                         _lib.stream(dev))
        if self.zero_grad_in_step:
            for b in self.zeroed_buckets:
                b.mark_zero()
        return loss

