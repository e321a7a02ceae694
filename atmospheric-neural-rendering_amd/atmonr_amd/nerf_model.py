"""AtmoNeRF — the NeRF MLP of src/atmonr/models/nerf.py:6-144 (same layers, init, skip
connection and noise), f32.

On the GPU the eleven layers run on hand-written f32 MFMA kernels (csrc/nerf_mlp.hip,
_AtmoNeRFFn). The forward carries the bias and ReLU epilogues and reads the fc6 skip and
fc10 direction concats in place. In the backward each input-gradient GEMM applies, in its
epilogue, the ReLU mask of the layer below. The weight and bias gradients accumulate
straight into the parameters' .grad, with a deterministic split over rows.
ANR_NERF_MLP=torch selects the earlier library-GEMM path (torch.nn.Linear through
hipBLASLt) for A/B. ``forward`` / ``forward_pos_only`` take an optional ``noise`` tensor
that replaces the training-mode ``torch.randn`` draw (parity tests).
"""

from __future__ import annotations

import os

import torch
import torch.nn.functional as F
from torch import nn


def _column_sum(g: torch.Tensor) -> torch.Tensor:
    """g.sum(0) for a tall (M, C) gradient in two stages: torch's one-pass column
    reduction runs a handful of blocks when C is not a multiple of 4 (fc9's 257 / 260
    outputs: 3.9 ms per step at 786 K rows); 512 row groups first spread it over the chip."""
    M, C = g.shape
    S = 512
    if M < 64 * S:
        return g.sum(0)
    r = M // S
    out = g[: S * r].view(S, r, C).sum(1).sum(0)
    if S * r < M:
        out = out + g[S * r:].sum(0)
    return out


_NATIVE = os.environ.get("ANR_NERF_MLP", "native") != "torch"


def _r4(n: int) -> int:
    return (n + 3) // 4 * 4


def _native_ok(x: torch.Tensor) -> bool:
    return (_NATIVE and x.is_cuda and x.dim() == 2 and x.dtype == torch.float32
            and x.stride(1) == 1 and x.stride(0) % 4 == 0 and x.data_ptr() % 16 == 0)


def _native_net_ok(net: "AtmoNeRF", x: torch.Tensor, with_dir: bool) -> bool:
    """The shapes csrc/nerf_mlp.hip's entry points accept (hidden width a multiple of 64,
    4-aligned channel segments) and a dense f32 input; otherwise the library path runs."""
    if not (_native_ok(x) and net.hidden_dim % 64 == 0 and net.pos_channels % 4 == 0):
        return False
    if with_dir:
        return (net.dir_channels % 4 == 0
                and x.shape[1] == net.pos_channels + net.dir_channels)
    return x.shape[1] == net.pos_channels


def _wt(layer: nn.Linear) -> tuple[torch.Tensor, int]:
    """(W^T as (in, round_up(out, 4)) with zero pad columns, its row stride)."""
    w = layer.weight.detach()
    n, k = w.shape
    ld = _r4(n)
    if ld == n:
        return w.t().contiguous(), n
    t = torch.zeros(k, ld, device=w.device, dtype=w.dtype)
    t[:, :n] = w.t()
    return t, ld


def _mlp_forward(net: "AtmoNeRF", x: torch.Tensor, pos_only: bool, masks: list | None = None):
    """The layer stack on csrc/nerf_mlp.hip; returns (y1..y8, y9 padded, y10, y11). With
    ``masks`` (a list) the ReLU layers also write their bitmasks there, by layer number."""
    from . import _lib

    M, dev = x.shape[0], x.device
    h, pc, dc = net.hidden_dim, net.pos_channels, net.dir_channels
    st, ldx = _lib.stream(dev), x.stride(0)
    x_dir = x[:, pc:] if not pos_only else None

    def lin(i, a1, lda1, q1, a2=None, lda2=0, q2=0, relu=1, ld=None):
        layer = getattr(net, f"fc{i}")
        n = layer.out_features
        ld = ld or _r4(n)
        y = torch.empty(M, ld, device=dev, dtype=torch.float32)
        bits = None
        if masks is not None and relu:
            bits = torch.empty(M, (n + 63) // 64, device=dev, dtype=torch.int64)
            masks[i] = bits
        _lib.call("anr_nerf_linear_fwd", _lib.ptr(a1), lda1, q1, _lib.ptr(a2), lda2, q2, M,
                  _lib.ptr(layer.weight), n, _lib.ptr(layer.bias), relu, _lib.ptr(y), ld,
                  _lib.ptr(bits), st, tag="nerf_linear_fwd")
        return y

    ys = [lin(1, x, ldx, pc)]
    for i in range(2, 6):
        ys.append(lin(i, ys[-1], h, h))
    ys.append(lin(6, ys[-1], h, h, x, ldx, pc))   # cat([x5, x_pos]) read in place
    for i in (7, 8):
        ys.append(lin(i, ys[-1], h, h))
    n9 = net.fc9.out_features
    y9 = lin(9, ys[-1], h, h, relu=0)   # its pad columns come out zero
    ys.append(y9)
    if pos_only:
        return ys
    ys.append(lin(10, y9, y9.shape[1], h, x_dir, ldx, dc))   # cat([x9[:, :h], d])
    ys.append(lin(11, ys[-1], ys[-1].shape[1], net.fc10.out_features, relu=0))
    return ys


class _AtmoNeRFFn(torch.autograd.Function):
    """AtmoNeRF.forward (models/nerf.py:48-93) on csrc/nerf_mlp.hip: (sigmoid colour,
    relu(sigma + noise)) from the (M, pos + dir) encoding. The backward is the chain of
    autograd's, layer by layer: the fc11 sigmoid backward as torch computes it, then per
    layer the weight / bias gradient (anr_nerf_linear_dw, accumulated into .grad) and the
    input gradient with the ReLU mask of the layer below (anr_nerf_linear_dx); the skip's
    two input gradients (fc1 and fc6) are summed into dL/dx."""

    @staticmethod
    def forward(ctx, x, noise, net, *params):
        from . import _lib

        _lib.grad_use(*params)
        masks = [None] * 12
        ys = _mlp_forward(net, x, pos_only=False, masks=masks)
        h, n9 = net.hidden_dim, net.fc9.out_features
        sig = ys[8][:, h:n9]
        if noise is not None:
            sig = sig + noise
        sigma = F.relu(sig)
        out = net.fc11.out_features
        color = torch.sigmoid(ys[10][:, :out])
        ctx.net = net
        ctx.save_for_backward(x, *ys[:10], color, sigma, *[masks[i] for i in range(1, 11)
                                                           if i != 9])
        return color, sigma

    @staticmethod
    def backward(ctx, dcolor, dsigma):
        from . import _lib

        net = ctx.net
        x, *rest = ctx.saved_tensors
        ys, (color, sigma), mb = rest[:10], rest[10:12], rest[12:]
        bits = dict(zip([i for i in range(1, 11) if i != 9], mb))   # layer -> ReLU bitmask
        M, dev = x.shape[0], x.device
        h, pc, dc = net.hidden_dim, net.pos_channels, net.dir_channels
        st, ldx = _lib.stream(dev), x.stride(0)
        layers = [getattr(net, f"fc{i}") for i in range(1, 12)]
        grads = {}
        ws_bytes = max(_lib.load().anr_nerf_linear_dw_workspace(
            M, L.out_features, L.in_features) for L in layers)
        ws = torch.empty(max(ws_bytes, 16) // 4 + 4, device=dev, dtype=torch.float32)

        def wgrad(i, g, a1, lda1, q1, a2=None, lda2=0, q2=0):
            L = layers[i - 1]
            dw, w_direct = _lib.grad_target(L.weight, dev)
            db, b_direct = _lib.grad_target(L.bias, dev)
            _lib.call("anr_nerf_linear_dw", _lib.ptr(g), g.stride(0), M, L.out_features,
                      _lib.ptr(a1), lda1, q1, _lib.ptr(a2), lda2, q2, _lib.ptr(dw),
                      _lib.ptr(db), _lib.ptr(ws), ws.numel() * 4, st, tag="nerf_linear_dw")
            grads[L.weight] = None if w_direct else dw
            grads[L.bias] = None if b_direct else db
            _lib.grad_done(*[p for p, d in ((L.weight, w_direct), (L.bias, b_direct)) if d])

        def dgrad(i, g, p1, mask=None, dx2=None, p2=0, acc2=0):
            """dL/d(input of layer i); ``mask`` = the layer whose ReLU output it is."""
            L = layers[i - 1]
            wt, ldwt = _wt(L)
            dx1 = torch.empty(M, max(p1, 1), device=dev, dtype=torch.float32) if p1 else None
            _lib.call("anr_nerf_linear_dx", _lib.ptr(g), g.stride(0), M, L.out_features,
                      _lib.ptr(wt), ldwt, p1, p2,
                      _lib.ptr(bits[mask]) if mask is not None else None, _lib.ptr(dx1),
                      dx1.stride(0) if dx1 is not None else 0, _lib.ptr(dx2),
                      dx2.stride(0) if dx2 is not None else 0, acc2, st,
                      tag="nerf_linear_dx")
            return dx1

        need_x = ctx.needs_input_grad[0]
        out = layers[10].out_features
        g11 = torch.zeros(M, _r4(out), device=dev, dtype=torch.float32)
        if dcolor is not None:   # torch's sigmoid_backward: g * (1 - y) * y
            g11[:, :out] = dcolor * (1 - color) * color
        y10 = ys[9]
        wgrad(11, g11, y10, y10.stride(0), y10.shape[1])
        g10 = dgrad(11, g11, layers[9].out_features, mask=10)
        y9 = ys[8]
        wgrad(10, g10, y9, y9.stride(0), h, x[:, pc:], ldx, dc)
        n9 = layers[8].out_features
        g9 = torch.empty(M, y9.shape[1], device=dev, dtype=torch.float32)
        dgrad(10, g10, 0, dx2=g9, p2=h)      # dL/dx9[:, :h] (fc9 has no activation)
        g9[:, h:n9] = (torch.where(sigma > 0, dsigma, torch.zeros_like(dsigma))
                       if dsigma is not None else 0.0)
        if n9 < g9.shape[1]:
            g9[:, n9:].zero_()
        wgrad(9, g9, ys[7], h, h)
        g = dgrad(9, g9, h, mask=8)       # G8
        for i in (8, 7):
            wgrad(i, g, ys[i - 2], h, h)
            g = dgrad(i, g, h, mask=i - 1)
        dx = torch.empty_like(x) if need_x else None
        wgrad(6, g, ys[4], h, h, x, ldx, pc)
        g = dgrad(6, g, h, mask=5, dx2=dx, p2=pc if need_x else 0)
        for i in (5, 4, 3, 2):
            wgrad(i, g, ys[i - 2], h, h)
            g = dgrad(i, g, h, mask=i - 1)
        wgrad(1, g, x, ldx, pc)
        if need_x:
            dgrad(1, g, 0, dx2=dx, p2=pc, acc2=1)
            dx[:, pc:].zero_()   # the directions are data
        pgrads = [grads[p] for L in layers for p in (L.weight, L.bias)]
        return (dx, None, None, *pgrads)


# split of the weight-gradient GEMMs (bench sweep, S = 1/8/16/32/64/128:
# 61.1/52.7/47.1/45.1/43.6/50.0 ms per NeRF step)
_SPLIT_K = int(os.environ.get("ANR_NERF_SPLITK", "64"))


def _weight_grad(g: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """g^T x for the tall (M rows) operands of a layer's weight gradient. As one GEMM the
    (out x in) result has only 32 tiles to spread over 256 CUs; split over the M rows into
    a batched GEMM of _SPLIT_K slices (bmm), then summed — same products, f32 partial sums
    added in a different order."""
    M = g.shape[0]
    S = _SPLIT_K
    if S <= 1 or M < S * 4096 or M % S:
        return g.t() @ x
    r = M // S
    return torch.bmm(g.view(S, r, g.shape[1]).transpose(1, 2), x.view(S, r, x.shape[1])).sum(0)


class _LinearFn(torch.autograd.Function):
    """F.linear with the same backward GEMMs as autograd's, but the bias gradient by
    _column_sum (summation order differs from autograd's by f32 rounding only)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, g):
        x, weight = ctx.saved_tensors
        g = g.contiguous()
        dx = g @ weight if ctx.needs_input_grad[0] else None
        dw = _weight_grad(g, x) if ctx.needs_input_grad[1] else None
        db = _column_sum(g) if ctx.needs_input_grad[2] else None
        return dx, dw, db


class _LinearReLUFn(torch.autograd.Function):
    """relu(F.linear(x, W, b)) as one library GEMM with a bias + ReLU epilogue
    (torch._addmm_activation, which has no autograd formula) and the matching backward:
    g' = g where y > 0 (relu's subgradient at 0 is 0, as torch's), then the GEMMs."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        y = torch._addmm_activation(bias, x, weight.t())
        ctx.save_for_backward(x, weight, y)
        return y

    @staticmethod
    def backward(ctx, g):
        x, weight, y = ctx.saved_tensors
        g = g.contiguous()
        M, C = g.shape
        if C % 4 == 0 and C <= 1024 and y.is_contiguous() and M >= 256:
            # one pass: mask + per-block column sums (anr_relu_bwd_colsum)
            from . import _lib

            parts = min(1024, M // 256)
            gm = torch.empty_like(g)
            partial = torch.empty(parts, C, device=g.device, dtype=torch.float32)
            _lib.call("anr_relu_bwd_colsum", _lib.ptr(g), _lib.ptr(y), M, C, _lib.ptr(gm),
                      _lib.ptr(partial), parts, _lib.stream(g.device))
            db = partial.sum(0) if ctx.needs_input_grad[2] else None
        else:
            gm = torch.ops.aten.threshold_backward(g, y, 0)
            db = _column_sum(gm) if ctx.needs_input_grad[2] else None
        dx = gm @ weight if ctx.needs_input_grad[0] else None
        dw = _weight_grad(gm, x) if ctx.needs_input_grad[1] else None
        return dx, dw, db


def _linear_relu(layer: nn.Linear, x: torch.Tensor) -> torch.Tensor:
    if x.is_cuda and x.dim() == 2 and x.dtype == torch.float32:
        if torch.is_grad_enabled():
            return _LinearReLUFn.apply(x, layer.weight, layer.bias)
        return torch._addmm_activation(layer.bias, x, layer.weight.t())
    return F.relu(layer(x))


class _Linear(nn.Linear):
    """nn.Linear (same parameters and state-dict keys) with _LinearFn's backward: split-K
    weight gradient, and a bias gradient that avoids torch's slow narrow-column reduction
    (out_features not a multiple of 4)."""

    def forward(self, x):
        if torch.is_grad_enabled() and x.is_cuda and x.dim() == 2:
            return _LinearFn.apply(x, self.weight, self.bias)
        return F.linear(x, self.weight, self.bias)


class AtmoNeRF(nn.Module):
    def __init__(self, pos_channels: int, dir_channels: int, out_channels: int,
                 volume_channels: int, hidden_dim: int = 256) -> None:
        super().__init__()
        self.pos_channels = pos_channels
        self.dir_channels = dir_channels
        self.out_channels = out_channels
        self.volume_channels = volume_channels
        self.hidden_dim = h = hidden_dim
        self.fc1 = nn.Linear(pos_channels, h)
        self.fc2 = nn.Linear(h, h)
        self.fc3 = nn.Linear(h, h)
        self.fc4 = nn.Linear(h, h)
        self.fc5 = nn.Linear(h, h)
        self.fc6 = nn.Linear(h + pos_channels, h)
        self.fc7 = nn.Linear(h, h)
        self.fc8 = nn.Linear(h, h)
        self.fc9 = _Linear(h, h + volume_channels)
        self.fc10 = nn.Linear(h + dir_channels, h // 2)
        self.fc11 = _Linear(h // 2, out_channels)
        for i in range(1, 12):  # models/nerf.py:45-46
            nn.init.kaiming_normal_(getattr(self, f"fc{i}").weight, mode="fan_out")

    def params_in_order(self) -> list[torch.nn.Parameter]:
        return [p for i in range(1, 12) for p in (getattr(self, f"fc{i}").weight,
                                                    getattr(self, f"fc{i}").bias)]

    def forward_pos_only(self, x_pos: torch.Tensor, noise: torch.Tensor | None = None):
        """models/nerf.py:48-71: returns (fc9 output, relu(sigma [+ noise if training]))."""
        if not torch.is_grad_enabled() and _native_net_ok(self, x_pos, with_dir=False):
            y9 = _mlp_forward(self, x_pos, pos_only=True)[8]
            x = y9[:, : self.fc9.out_features]
            sigma = x[:, self.hidden_dim:]
            if self.training:
                sigma = sigma + (noise if noise is not None
                                 else torch.randn(sigma.shape, device=sigma.device))
            return x, F.relu(sigma)
        x = _linear_relu(self.fc1, x_pos)
        x = _linear_relu(self.fc2, x)
        x = _linear_relu(self.fc3, x)
        x = _linear_relu(self.fc4, x)
        x = _linear_relu(self.fc5, x)
        x = torch.cat([x, x_pos], dim=1)  # skip connection
        x = _linear_relu(self.fc6, x)
        x = _linear_relu(self.fc7, x)
        x = _linear_relu(self.fc8, x)
        x = self.fc9(x)
        sigma = x[:, self.hidden_dim:]
        if self.training:
            sigma = sigma + (noise if noise is not None
                             else torch.randn(sigma.shape, device=sigma.device))
        return x, F.relu(sigma)

    def forward(self, x: torch.Tensor, noise: torch.Tensor | None = None):
        """models/nerf.py:73-93: (sigmoid color, sigma). fc9's hidden part feeds fc10
        without an activation, as in the reference."""
        if _native_net_ok(self, x, with_dir=True):
            if self.training and noise is None:
                noise = torch.randn(x.shape[0], self.volume_channels, device=x.device)
            return _AtmoNeRFFn.apply(x, noise if self.training else None, self,
                                     *self.params_in_order())
        x_pos, d = x[:, : self.pos_channels], x[:, self.pos_channels:]
        x, sigma = self.forward_pos_only(x_pos, noise)
        x = _linear_relu(self.fc10, torch.cat([x[:, : self.hidden_dim], d], dim=1))
        return torch.sigmoid(self.fc11(x)), sigma


def get_model(hidden_dim: int, N_lambda: int, L_x, L_d: int, include_height: bool
              ) -> tuple[AtmoNeRF, AtmoNeRF]:
    """models/nerf.py:96-144: coarse (1 density) and fine (N_lambda densities) models."""
    if isinstance(L_x, int):
        pos_channels = L_x * 6 + (L_x * 2 if include_height else 0)
    else:
        assert len(L_x) == (4 if include_height else 3)
        pos_channels = sum(L_x) * 2
    dir_channels = L_d * 6
    return (AtmoNeRF(pos_channels, dir_channels, N_lambda, 1, hidden_dim),
            AtmoNeRF(pos_channels, dir_channels, N_lambda, N_lambda, hidden_dim))
