"""FusedAdam — torch.optim.Optimizer on the K10 kernel (one HBM pass per tensor).

Drop-in for torch.optim.AdamW (instant_ngp.py:120-126; ``decoupled=True``) and
torch.optim.Adam (nerf.py:70; ``decoupled=False``): same param-group semantics, same
state keys (``step``, ``exp_avg``, ``exp_avg_sq``) so optimizer state dicts interchange
with torch's.

``capturable=True`` (as torch.optim.AdamW's flag of that name): the step count and the
learning rates live in device memory (anr_adam_step_multi_dev), so ``step()`` launches
the same kernels with the same arguments every time and can be captured in a hipGraph
(atmonr_amd.graph). The host copy of ``state["step"]`` is refreshed from the device by
``state_dict()``; learning-rate changes (schedulers write ``group["lr"]``) reach the
device in ``sync_hyper()``, which ``step()`` calls outside a capture and a graph replay
calls before launching.
"""

from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import call, ptr


def _grad_quant(p) -> float:
    """tinycudann's f16 gradient rounding deferred into this update (loss scale, or 0):
    set on a parameter by InstantNGPPipeline.defer_grad_quantize."""
    return float(getattr(p, "_anr_grad_quant", 0.0) or 0.0)


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=None,
                 decoupled: bool = True, zero_grad_in_step: bool = False,
                 capturable: bool = False, **unused):
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
        self.capturable = capturable
        self._devstate: dict = {}  # capturable: (device, b1, b2, eps) -> device step / lr
        # bumped whenever tensors a captured step points at (the device step / lr / scratch,
        # or exp_avg / exp_avg_sq storage) are replaced: GraphedTrainStep recaptures then
        self.generation = 0

    # ------------------------------------------------------------------ capturable mode
    def _entries(self):
        """(key, param, group) of every parameter with a gradient, launch order."""
        out = []
        for group in self.param_groups:
            b1, b2 = group["betas"]
            key_hp = (float(b1), float(b2), float(group["eps"]))
            for p in group["params"]:
                if p.grad is not None:
                    out.append(((p.device,) + key_hp, p, group))
        return out

    def _init_state(self, p):
        if p.dtype != torch.float32 or p.grad.dtype != torch.float32:
            raise _lib.ANRError("FusedAdam needs float32 params and grads")
        st = self.state[p]
        if not st:
            st["step"] = torch.tensor(0.0)
            st["exp_avg"] = torch.zeros_like(p)
            st["exp_avg_sq"] = torch.zeros_like(p)
        if st["step"].device.type != "cpu":
            st["step"] = st["step"].cpu()
        if not p.grad.is_contiguous():
            p.grad = p.grad.contiguous()
        return st

    def sync_hyper(self) -> None:
        """Write changed learning rates to the device (capturable mode; outside a capture)."""
        for ds in self._devstate.values():
            lrs = [float(g["lr"]) for g in ds["groups"]]
            if lrs != ds["lr_host"]:
                ds["lr"].copy_(torch.tensor(lrs, dtype=torch.float32))
                ds["lr_host"] = lrs

    def _signature(self):
        return tuple((k, id(p), id(g)) for k, p, g in self._entries())

    def _prepare(self):
        """Device step / lr buffers per launch key, built eagerly (never inside a capture:
        their initial values must not be part of the graph). The kernel reads tensor t's lr
        from d_lr[t] in launch order, so the state is rebuilt whenever the ordered list of
        (parameter, group) with gradients changes -- not only when the key set does (a
        parameter gaining / losing its grad, or moving between groups of equal betas).
        A rebuild first writes the device step counts back to the host state, and groups
        parameters by step count (a parameter that skipped steps keeps its own count, as
        torch's per-parameter ``step``)."""
        sig = self._signature()
        if sig != getattr(self, "_sig", None) or not self._devstate:
            if torch.cuda.is_current_stream_capturing():
                raise _lib.ANRError("FusedAdam(capturable=True): the parameters with gradients "
                                    "changed since the device step/lr state was built; run one "
                                    "step eagerly before capturing")
            self._sync_host_steps()
            self._devstate = {}
            self.generation += 1
            for key_hp, p, group in self._entries():
                st = self._init_state(p)
                key = key_hp + (int(st["step"].item()),)
                self._devstate.setdefault(key, {"params": [], "groups": []})
                self._devstate[key]["params"].append(p)
                self._devstate[key]["groups"].append(group)
            for key, ds in self._devstate.items():
                if len(ds["params"]) > _lib.ADAM_DEV_MAX_TENSORS:
                    raise _lib.ANRError(f"capturable FusedAdam: at most "
                                        f"{_lib.ADAM_DEV_MAX_TENSORS} tensors per launch")
                dev = key[0]
                lrs = [float(g["lr"]) for g in ds["groups"]]
                ds.update({"step": torch.tensor([key[4]], dtype=torch.int64, device=dev),
                           "lr": torch.tensor(lrs, device=dev), "lr_host": lrs,
                           "scratch": torch.zeros(3 * _lib.ADAM_DEV_MAX_TENSORS, device=dev)})
            self._sig = sig
        return {k: list(zip(ds["params"], ds["groups"])) for k, ds in self._devstate.items()}

    def _sync_host_steps(self) -> None:
        """Device step counts -> state[p]["step"] (host); synchronises."""
        for ds in self._devstate.values():
            n = float(ds["step"].item())
            for p in ds["params"]:
                self.state[p]["step"] = torch.tensor(n)

    def _step_capturable(self):
        batches = self._prepare()
        if not torch.cuda.is_current_stream_capturing():
            self.sync_hyper()
        for key, items in batches.items():
            dev, b1, b2, eps = key[:4]
            ds = self._devstate[key]
            ts = []
            for p, group in items:
                st = self._init_state(p)
                sh = getattr(p, "_anr_shadow", None)
                if sh is not None and (sh.dtype != torch.float16 or sh.shape != p.shape):
                    sh = None
                ts.append(_lib.AdamTensor(ptr(p), ptr(p.grad), ptr(st["exp_avg"]),
                                          ptr(st["exp_avg_sq"]), ptr(sh), p.numel(),
                                          float(group["lr"]), float(group["weight_decay"]), 0,
                                          _grad_quant(p)))
                if sh is not None:
                    p._anr_shadow_ver = p._version
            arr = (_lib.AdamTensor * len(ts))(*ts)
            call("anr_adam_step_multi_dev", ctypes.addressof(arr), len(ts), b1, b2, eps,
                 int(self.decoupled), int(self.zero_grad_in_step), ptr(ds["step"]),
                 ptr(ds["lr"]), ptr(ds["scratch"]), _lib.stream(dev), tag="adam")

    def device_step(self) -> int:
        """The step count held on the device (capturable mode; synchronises)."""
        return max((int(ds["step"].item()) for ds in self._devstate.values()), default=0)

    def state_dict(self):
        if self.capturable:
            self._sync_host_steps()
        return super().state_dict()

    def load_state_dict(self, state_dict):
        """torch's load replaces the state tensors and the param-group dicts. In capturable
        mode with device state built, the loaded values are copied INTO the existing
        exp_avg / exp_avg_sq / device step / lr storage instead, so a captured step
        (GraphedTrainStep) keeps pointing at live memory and replays from the loaded state.
        When that is impossible (new parameters, shapes, mixed steps, a different weight
        decay, which the captured launch holds by value) the device state is
        dropped and ``generation`` bumped: a graph built on it recaptures before replaying."""
        if not (self.capturable and self._devstate):
            super().load_state_dict(state_dict)
            self._devstate = {}  # rebuilt from the loaded host steps at the next step()
            self.generation += 1
            return
        old = {p: (st.get("exp_avg"), st.get("exp_avg_sq")) for p, st in self.state.items()}
        super().load_state_dict(state_dict)
        ok = True
        with torch.no_grad():
            for p, st in self.state.items():
                o = old.get(p)
                new_ = (st.get("exp_avg"), st.get("exp_avg_sq"))
                if (o is None or any(t is None for t in o + new_)
                        or any(a.shape != b.shape or a.dtype != b.dtype or a.device != b.device
                               for a, b in zip(o, new_))):
                    ok = False
                    break
                o[0].copy_(new_[0])
                o[1].copy_(new_[1])
                st["exp_avg"], st["exp_avg_sq"] = o
                if st["step"].device.type != "cpu":
                    st["step"] = st["step"].cpu()
            group_of = {id(p): g for g in self.param_groups for p in g["params"]}
            for ds in (self._devstate.values() if ok else ()):
                if any(id(p) not in group_of or p not in self.state for p in ds["params"]):
                    ok = False
                    break
                steps = {int(self.state[p]["step"].item()) for p in ds["params"]}
                if len(steps) != 1:
                    ok = False
                    break
                new_groups = [group_of[id(p)] for p in ds["params"]]
                # weight decay is captured by value in the launch descriptors: a loaded
                # value that differs needs a recapture, not an in-place reload
                if ([float(g["weight_decay"]) for g in ds["groups"]]
                        != [float(g["weight_decay"]) for g in new_groups]):
                    ok = False
                    break
                ds["step"].fill_(steps.pop())
                ds["groups"] = new_groups
                ds["lr_host"] = None  # sync_hyper rewrites the lr tensor in place
        if ok:
            # same parameters in the same launch order; only the group dicts are new
            old_sig = [(k, i) for k, i, _ in self._sig]
            ok = [(k, id(p)) for k, p, _ in self._entries()] == old_sig
        if ok:
            self._sig = self._signature()
            self.sync_hyper()
        else:
            self._devstate = {}
            self.generation += 1

    @torch.no_grad()
    def step(self, closure=None):
        """Every parameter of every group in one anr_adam_step_multi launch per device
        (``multi_tensor=False``: one anr_adam_step launch per parameter)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self.capturable:
            self._step_capturable()
            if self.zero_grad_in_step:
                for b in self.zeroed_buckets:
                    b.mark_zero()
            return loss
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
                                    int(st["step"].item()), _grad_quant(p))
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
                    if t.grad_quant:
                        raise _lib.ANRError("a deferred gradient quantisation needs "
                                            "FusedAdam(multi_tensor=True)")
                    call("anr_adam_step", t.params, t.grad, t.exp_avg, t.exp_avg_sq,
                         t.params_f16, t.n, t.lr, b1, b2, eps, t.weight_decay,
                         int(self.decoupled), t.step, int(self.zero_grad_in_step),
                         _lib.stream(dev))
        if self.zero_grad_in_step:
            for b in self.zeroed_buckets:
                b.mark_zero()
        return loss

