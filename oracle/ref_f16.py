"""ORACLE (test infrastructure only): the reference's f16 composite and loss, op by op.

In the reference's Instant-NGP path every tinycudann module returns f16, so
render_with_surface (src/atmonr/graphics_utils.py:6-77) and the loss
(src/atmonr/pipelines/instant_ngp.py:259-263, src/atmonr/losses.py:5-33) run as chains of
torch f16 ops, and autograd differentiates them with more f16 ops. This module restates
those chains explicitly (numpy, f32 arithmetic + round-to-nearest-even to f16 after every
op, as torch's f16 kernels compute in f32 "opmath" and store f16), forward AND backward,
so that the rounding points are written down rather than inherited from whichever torch
backend runs the oracle.

Why not just call torch on f16 CPU tensors: the reference requires CUDA (tinycudann), and
torch's CPU and CUDA f16 kernels differ where accumulation is involved (measured here on
the CPU; CUDA behaviour from torch's kernels, see below). ``acc`` selects the accumulation
semantics of the four accumulating ops:

================  ==========================================  =========================
op                acc="cuda" (default: the reference's)        acc="cpu" (torch on CPU)
================  ==========================================  =========================
cumprod (fwd)     sequential, accumulator stored f16 per step  f32 accumulator, each
                  (ATen cuda ScanUtils.cuh                     output rounded (verified
                  tensor_kernel_scan_outer_dim: scalar_t acc)  bit-exact against torch)
cumsum (cumprod   same as cumprod                              same as cumprod
backward's
reversed cumsum)
sum over samples  f32 accumulator, one rounding (reduce with   same (order: sequential)
                  opmath float)
prod over samples f32 accumulator, one rounding (prod_functor  not restated: torch CPU
                  <Half, float>)                               accumulates in f16 lanes
                                                              (~3 % low at 1,024 samples);
                                                              pass ``prod_override``
================  ==========================================  =========================

Autograd formulas (torch/csrc/autograd/FunctionsManual.cpp, derivatives.yaml): mul /
rsub / neg / exp elementwise; sum_to_size reductions in f32; prod_backward =
grad * (result / input) when the tensor holds no zero; cumprod_backward =
reversed_cumsum(output * grad) / input when no zero; alpha's three gradient
contributions accumulate in autograd's order ((1 - alpha) for the surface product first,
then alpha * T, then 1 - alpha + 1e-10) with an f16 rounding per addition. The zero-input
branches (alpha rounding to exactly 1 in f16, sigma * delta > ~9) are not restated:
``render_f16`` raises if one occurs.

The CPU-semantics form is pinned bit-exact against torch's own autograd of the
reference's render / render_with_surface (tests/test_oracle_f16.py); the CUDA form
differs from it only in the accumulation rows above.
"""

from __future__ import annotations

import numpy as np
import torch

F32 = np.float32


def h(x) -> np.ndarray:
    """Round to f16 (nearest even), keep as f32."""
    return np.asarray(x, dtype=F32).astype(np.float16).astype(F32)


def h64(x) -> np.ndarray:
    """f64 value rounded once to f16 (transcendentals: a correctly rounded f16 of exp/log)."""
    return np.asarray(x, dtype=np.float64).astype(np.float16).astype(F32)


def _scan(x: np.ndarray, op, acc: str, axis: int = 1) -> np.ndarray:
    """Inclusive scan along ``axis``: f16 accumulator (cuda) or f32 accumulator with each
    output rounded (cpu)."""
    x = np.moveaxis(x, axis, 0)
    out = np.empty_like(x)
    a = x[0].astype(F32)
    out[0] = h(a)
    for j in range(1, x.shape[0]):
        a = op(a, x[j]).astype(F32)
        if acc == "cuda":
            a = h(a)
        out[j] = h(a)
    return np.moveaxis(out, 0, axis)


def render_fwd(zk: np.ndarray, color: np.ndarray, sigma: np.ndarray, cs=None, acc="cuda",
               prod_override=None) -> dict:
    """graphics_utils.py:6-77 in f16. zk (B, N) f32 = z_vals * (scale / 1000) as the
    reference forms it (f32 tensor times a Python float); color (B, N, C), sigma (B, N, 1)
    and cs (B, C) hold f16 values (f32 arrays). Returns every intermediate the backward
    uses."""
    z = h(zk)                                              # z_vals.to(f16)       :28
    mid = h(h(z[:, :-1] + z[:, 1:]) * F32(0.5))            # (a + b) / 2          :31
    zm = np.concatenate([h(z[:, :1] * F32(0)), mid, z[:, -1:]], 1)   #            :33
    delta = h(zm[:, 1:] - zm[:, :-1])[..., None]           # diff                 :35
    x = h(-sigma * delta)                                  # -sigma * delta       :38
    e = h64(np.exp(x.astype(np.float64)))
    alpha = h(F32(1) - e)
    q2 = h(h(F32(1) - alpha) + F32(1e-10))                 # 1 - alpha + 1e-10    :45
    B, N = z.shape
    cpin = np.concatenate([np.ones((B, 1, 1), F32), q2], 1)
    cp = _scan(cpin, np.multiply, acc)                     # cumprod              :45
    T = cp[:, :-1]
    w = h(alpha * T)                                       # alpha * cumprod      :44
    atmo = h((h(color * w)).sum(1, dtype=np.float64).astype(F32)) if acc == "cpu" else \
        h(_seq_sum(h(color * w)))                          # sum(color * w)       :48
    r = {"z": z, "delta": delta, "x": x, "e": e, "alpha": alpha, "cpin": cpin, "cp": cp,
         "T": T, "w": w, "atmo": atmo, "color": color, "sigma": sigma, "cs": cs}
    if cs is None:
        r["color_map"] = atmo
        return r
    om = h(F32(1) - alpha)                                 # (1 - alpha)          :75
    pr = h(_seq_prod(om)) if prod_override is None else prod_override   # .prod(dim=1)
    surf = h(pr * cs)                                      # * color_surf
    r.update(om=om, pr=pr, surf=surf, color_map=h(atmo + surf))   #               :76
    return r


def _seq_sum(v: np.ndarray) -> np.ndarray:
    """f32 accumulation over axis 1, sequential."""
    a = np.zeros(v.shape[:1] + v.shape[2:], F32)
    for i in range(v.shape[1]):
        a = (a + v[:, i]).astype(F32)
    return a


def _seq_prod(v: np.ndarray) -> np.ndarray:
    a = np.ones(v.shape[:1] + v.shape[2:], F32)
    for i in range(v.shape[1]):
        a = (a * v[:, i]).astype(F32)
    return a


def render_bwd(r: dict, g_cm: np.ndarray, acc="cuda") -> dict:
    """Autograd of render_fwd for dL/dcolor_map (B, C) f16 values -> dL/d{color, sigma, cs}."""
    alpha, T, w, color = r["alpha"], r["T"], r["w"], r["color"]
    if (r["cpin"] == 0).any() or ("om" in r and (r["om"] == 0).any()):
        raise ValueError("alpha rounded to 1 in f16: torch's zero-input backward branch")
    out = {"color": h(g_cm[:, None, :] * w)}               # color * w -> color
    g_w = h(_sum_last(h(g_cm[:, None, :] * color)))        # -> w (sum_to_size)
    g_alpha_b = h(g_w * T)                                 # alpha * T -> alpha
    g_T = h(g_w * alpha)                                   # -> T
    B, N = T.shape[:2]
    g_cp = np.concatenate([g_T, np.zeros((B, 1, 1), F32)], 1)
    wcp = h(r["cp"] * g_cp)
    rc = np.flip(_scan(np.flip(wcp, 1), np.add, acc), 1)   # reversed cumsum
    g_cpin = h(rc / r["cpin"])
    g_alpha_c = -g_cpin[:, 1:]                             # 1 - alpha (+1e-10) -> alpha
    if r["cs"] is not None:
        cs, pr, om = r["cs"], r["pr"], r["om"]
        g_pr = h(_sum_last(h(g_cm * cs)))[:, None]         # pr * cs -> pr  (B, 1, 1)
        out["cs"] = h(g_cm * pr)                           # -> cs
        g_om = h(g_pr * h(pr[:, None] / om))               # prod backward
        g_alpha = h(h(-g_om + g_alpha_b) + g_alpha_c)      # autograd's accumulation order
    else:
        g_alpha = h(g_alpha_b + g_alpha_c)
    g_x = h(-g_alpha * r["e"])                             # 1 - e, exp
    out["sigma"] = -h(g_x * r["delta"])                    # -sigma * delta
    return out


def _sum_last(v: np.ndarray) -> np.ndarray:
    a = np.zeros(v.shape[:-1] + (1,), F32)
    for c in range(v.shape[-1]):
        a = (a + v[..., c:c + 1]).astype(F32)
    return a


class RenderF16(torch.autograd.Function):
    """render_with_surface (or render, cs=None) of f16 tensors with the restated forward and
    backward; z_km is the f32 tensor z_vals * (scale / 1000)."""

    @staticmethod
    def forward(ctx, z_km, color, sigma, cs, acc):
        r = render_fwd(z_km.detach().float().numpy(), color.detach().float().numpy(),
                       sigma.detach().float().numpy(),
                       None if cs is None else cs.detach().float().numpy(), acc=acc)
        ctx.r, ctx.acc, ctx.has_cs = r, acc, cs is not None
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).half()  # noqa: E731
        outs = (t(r["color_map"]), t(r["alpha"]), t(r["w"]), t(r["atmo"]))
        return outs + ((t(r["surf"]),) if cs is not None else ())

    @staticmethod
    def backward(ctx, g_cm, *_):
        g = render_bwd(ctx.r, g_cm.float().numpy(), ctx.acc)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).half()  # noqa: E731
        return (None, t(g["color"]), t(g["sigma"]), t(g["cs"]) if ctx.has_cs else None, None)


def render_with_surface(z_km, color, sigma, color_surf, acc="cuda"):
    """Same tuple as graphics_utils.render_with_surface: (color_map, alpha, weights, atmo,
    surf), f16; differentiable in color, sigma, color_surf (through dL/dcolor_map only)."""
    cm, alpha, w, atmo, surf = RenderF16.apply(z_km, color.half(), sigma.half(),
                                               color_surf.half(), acc)
    return cm, alpha, w, atmo, surf


# ------------------------------------------------------------------ loss (f16 ops)
def loss_f16(name: str, pred: np.ndarray, gt: np.ndarray, max_i: float, acc: str = "cuda"):
    """losses.py:5-33 on f16 pred (B,) and gt.to(f16) (B,), as torch's f16 ops compute it
    (elementwise ops in f32 then f16; x / scalar as x * (1 / scalar) in f32; mse_loss
    backward 2/numel * (a - b) * grad with f16 roundings between; means accumulate in
    f32). ``x + 1e-3 * max_i``: torch on CUDA adds the Python scalar in f32
    (``original_scalar_value``), torch on the CPU rounds it to f16 first (measured) --
    ``acc`` selects which. Returns (loss value, dL/dpred)."""
    p, g = h(pred), h(gt)
    n = p.shape[0]
    norm = h(F32(2.0 / n))
    inv = F32(1) / F32(max_i)
    eps = F32(1e-3 * max_i) if acc == "cuda" else h(1e-3 * max_i)

    def mse(a, b, gout):  # value, d/da
        d = h(a - b)
        val = h(_mean(h(d * d)))
        return val, h(h(norm * d) * gout)

    def l1(a, b, gout):
        d = h(a - b)
        val = h(_mean(np.abs(d)))
        return val, h(h(np.sign(d) * gout) * h(F32(1.0 / n)))

    def hdr(gout):  # F.mse_loss(log(gt + eps), log(pred + eps))
        xg = h(g + eps)
        xp = h(p + eps)
        la, lb = h64(np.log(xg.astype(np.float64))), h64(np.log(xp.astype(np.float64)))
        d = h(la - lb)
        val = h(_mean(h(d * d)))
        g_lb = h(h(norm * h(lb - la)) * gout)
        return val, h(g_lb / xp)

    def scaled(fn):  # fn(p/m, g/m)
        a, b = h(p * inv), h(g * inv)
        return a, b

    one = F32(1)
    c02 = h(F32(0.2))
    if name == "mse":
        a, b = scaled(None)
        v, ga = mse(a, b, one)
        return v, h(ga * inv)
    if name == "l1":
        a, b = scaled(None)
        v, ga = l1(a, b, one)
        return v, h(ga * inv)
    if name == "hdr":
        return hdr(one)
    if name in ("mse_plus_hdr", "l1_plus_hdr"):
        a, b = scaled(None)
        v1, ga = (mse if name == "mse_plus_hdr" else l1)(a, b, one)
        v2, gp2 = hdr(c02)
        val = h(v1 + h(v2 * F32(0.2)))
        return val, h(h(ga * inv) + gp2)
    if name == "dark":
        # (((p - g) / (p.detach() + eps)) ** 2).mean()
        den = h(p + eps)
        r = h(h(p - g) / den)
        val = h(_mean(h(r * r)))
        g_r = h(h(F32(2) * r) * h(F32(1.0 / n)))   # pow backward then mean backward
        return val, h(g_r / den)
    raise ValueError(name)


class LossF16(torch.autograd.Function):
    """loss_f16 as a differentiable function of the f16 prediction (B,)."""

    @staticmethod
    def forward(ctx, pred, gt, max_i, name, acc):
        v, g = loss_f16(name, pred.detach().float().numpy(), gt.detach().float().numpy(),
                        float(max_i), acc)
        ctx.g = torch.from_numpy(np.ascontiguousarray(g)).half()
        return torch.tensor(float(v), dtype=torch.float16)

    @staticmethod
    def backward(ctx, dl):
        return ctx.g * dl.half(), None, None, None, None


def _mean(v: np.ndarray) -> np.ndarray:
    return np.asarray(v, np.float64).sum().astype(F32) / F32(v.shape[0])
