"""Drop-in replacement for the ``tinycudann`` module API used by AtmoNR.

The reference does ``import tinycudann as tcnn`` (src/atmonr/pipelines/instant_ngp.py:4)
and builds six modules with it (:60-85): ``tcnn.Encoding(n_input_dims, config)`` and
``tcnn.Network(n_input_dims, n_output_dims, config)``. This module provides the same two
classes with the same constructor arguments, ``n_output_dims``, a single flat ``params``
Parameter per module (float32 master copy, as tcnn's torch bindings keep it) and
``forward(x) -> (M, n_output_dims)``. Compute runs in libanr_hip.so (HIP/gfx950):

* Encoding otypes: ``HashGrid`` (2-D / 3-D), ``SphericalHarmonics``, ``Identity`` and
  ``Composite`` of those.
* Network otypes: ``FullyFusedMLP`` (and ``CutlassMLP``, mapped to the same kernel),
  ReLU hidden activation, ``None`` / ``ReLU`` output activation, width 16/32/64/128.

``dtype`` follows tcnn: float16 by default (tables, weights and outputs in f16, f32
accumulation); pass ``dtype=torch.float32`` for the exact-f32 kernels used by the 1e-4
parity tests.
"""

from __future__ import annotations

import ctypes
import math
from typing import Any

import torch
from torch import nn

from . import _lib
from ._lib import ANRError, call, dtype_code, ptr


def _lower(d: dict) -> dict:
    return {k.lower() if isinstance(k, str) else k: v for k, v in d.items()}


# --------------------------------------------------------------------------- encodings
class _Sub:
    """One leaf encoding inside a (possibly composite) Encoding."""

    n_in: int
    n_out: int
    n_params: int = 0

    def fwd(self, x, params, out, col, stream):  # pragma: no cover - interface
        raise NotImplementedError

    def bwd(self, x, params, dout, col, dparams, dx, stream):  # pragma: no cover
        raise NotImplementedError


class _HashGrid(_Sub):
    def __init__(self, n_in: int, cfg: dict):
        if n_in not in (2, 3):
            raise ANRError(f"HashGrid supports 2 or 3 input dims, got {n_in}")
        self.n_in = n_in
        self.n_levels = int(cfg.get("n_levels", 16))
        self.n_features = int(cfg.get("n_features_per_level", 2))
        self.log2_T = int(cfg.get("log2_hashmap_size", 19))
        self.base_res = int(cfg.get("base_resolution", 16))
        self.pls = float(cfg.get("per_level_scale", 2.0))
        interp = cfg.get("interpolation", "Linear")
        if str(interp).lower() != "linear":
            raise ANRError(f"HashGrid interpolation {interp!r} not supported (Linear only)")
        self.desc = _lib.hashgrid_desc(n_in, self.n_levels, self.n_features, self.base_res,
                                       self.pls, self.log2_T)
        self.n_out = self.n_levels * self.n_features
        self.n_params = int(self.desc.n_params)

    def init_params(self, gen: torch.Generator) -> torch.Tensor:
        # tcnn GridEncoding: uniform(-1e-4, 1e-4)
        return torch.rand(self.n_params, generator=gen) * 2e-4 - 1e-4

    def fwd(self, x, params, out, col, stream):
        tdt = dtype_code(params.dtype)
        call("anr_hashgrid_fwd", ctypes.byref(self.desc), ptr(x), x.stride(0), x.shape[0],
             ptr(params), tdt, out.data_ptr() + col * out.element_size(),
             dtype_code(out.dtype), out.stride(0), stream)

    def bwd(self, x, params, dout, col, dparams, dx, stream):
        if dparams is None:
            return
        call("anr_hashgrid_bwd", ctypes.byref(self.desc), ptr(x), x.stride(0), x.shape[0],
             dout.data_ptr() + col * dout.element_size(), dtype_code(dout.dtype),
             dout.stride(0), ptr(dparams), stream)


class _SphericalHarmonics(_Sub):
    def __init__(self, n_in: int, cfg: dict):
        if n_in != 3:
            raise ANRError("SphericalHarmonics encodes exactly 3 dims")
        self.degree = int(cfg.get("degree", 4))
        if not 1 <= self.degree <= 4:
            raise ANRError(f"SphericalHarmonics degree {self.degree} not in [1, 4]")
        self.n_in = 3
        self.n_out = self.degree * self.degree

    def fwd(self, x, params, out, col, stream):
        call("anr_sh_fwd", self.degree, ptr(x), x.stride(0), x.shape[0],
             out.data_ptr() + col * out.element_size(), dtype_code(out.dtype), out.stride(0),
             stream)

    def bwd(self, x, params, dout, col, dparams, dx, stream):
        if dx is None:
            return
        call("anr_sh_bwd", self.degree, ptr(x), x.stride(0), x.shape[0],
             dout.data_ptr() + col * dout.element_size(), dtype_code(dout.dtype),
             dout.stride(0), ptr(dx), dx.stride(0), stream)


class _Identity(_Sub):
    def __init__(self, n_in: int, cfg: dict):
        self.n_in = n_in
        self.n_out = n_in

    def fwd(self, x, params, out, col, stream):
        call("anr_identity", ptr(x), dtype_code(x.dtype), x.stride(0), x.shape[0], self.n_in,
             out.data_ptr() + col * out.element_size(), dtype_code(out.dtype), out.stride(0),
             stream)

    def bwd(self, x, params, dout, col, dparams, dx, stream):
        if dx is None:
            return
        # dx is a column view (M, n_in) of the full input gradient
        call("anr_identity", dout.data_ptr() + col * dout.element_size(),
             dtype_code(dout.dtype), dout.stride(0), dout.shape[0], self.n_in, ptr(dx),
             dtype_code(dx.dtype), dx.stride(0), stream)


def _build(n_in: int, cfg: dict) -> list[tuple[int, _Sub]]:
    """Flatten a (Composite) encoding config into [(input column, leaf)]."""
    cfg = _lower(cfg)
    otype = str(cfg.get("otype", "")).lower()
    if otype == "composite":
        leaves: list[tuple[int, _Sub]] = []
        col = 0
        nested = cfg.get("nested", [])
        for i, sub in enumerate(nested):
            sub = _lower(sub)
            n = sub.get("n_dims_to_encode")
            if n is None:
                if i != len(nested) - 1:
                    raise ANRError("only the last Composite member may omit n_dims_to_encode")
                n = n_in - col
            for c, leaf in _build(int(n), sub):
                leaves.append((col + c, leaf))
            col += int(n)
        if col != n_in:
            raise ANRError(f"Composite encodes {col} dims but the input has {n_in}")
        return leaves
    if otype in ("hashgrid", "grid"):
        return [(0, _HashGrid(n_in, cfg))]
    if otype == "sphericalharmonics":
        return [(0, _SphericalHarmonics(n_in, cfg))]
    if otype == "identity":
        return [(0, _Identity(n_in, cfg))]
    raise ANRError(f"encoding otype {cfg.get('otype')!r} not supported")


class _EncodingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, params, enc: "Encoding"):
        M = x.shape[0]
        out = torch.empty(M, enc.n_output_dims, device=x.device, dtype=enc.output_dtype)
        p = _lib.compute_copy(params, enc.dtype) if params.numel() else params
        s = _lib.stream(x.device)
        col_out = 0
        for (col_in, leaf), poff in zip(enc._leaves, enc._param_offsets):
            xs = x[:, col_in:col_in + leaf.n_in]
            leaf.fwd(xs, p[poff:poff + leaf.n_params], out, col_out, s)
            col_out += leaf.n_out
        ctx.enc = enc
        ctx.save_for_backward(x, p)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, p = ctx.saved_tensors
        enc: Encoding = ctx.enc
        dout = dout.contiguous()
        s = _lib.stream(x.device)
        need_x = ctx.needs_input_grad[0]
        need_p = ctx.needs_input_grad[1]
        dx = torch.zeros(x.shape, device=x.device, dtype=torch.float32) if need_x else None
        # accumulate straight into an existing f32 .grad (e.g. a FlatGradBucket view) and
        # return no gradient for it: autograd's own accumulation, without the extra pass
        dparams, direct = ((_lib.grad_target(enc.params, x.device))
                           if need_p and enc.params.numel() else (None, False))
        col_out = 0
        for (col_in, leaf), poff in zip(enc._leaves, enc._param_offsets):
            xs = x[:, col_in:col_in + leaf.n_in]
            dxs = dx[:, col_in:col_in + leaf.n_in] if dx is not None else None
            dps = dparams[poff:poff + leaf.n_params] if dparams is not None else None
            leaf.bwd(xs, p[poff:poff + leaf.n_params], dout, col_out, dps, dxs, s)
            col_out += leaf.n_out
        if direct:
            _lib.grad_done(enc.params)
        if dx is not None:
            dx = dx.to(x.dtype)
        return dx, None if direct else dparams, None


class Encoding(nn.Module):
    """tinycudann.Encoding(n_input_dims, encoding_config, seed=1337, dtype=None)."""

    def __init__(self, n_input_dims: int, encoding_config: dict, seed: int = 1337,
                 dtype: torch.dtype | None = None, output_dtype: torch.dtype | None = None):
        super().__init__()
        self.n_input_dims = n_input_dims
        self.encoding_config = encoding_config
        self.dtype = torch.float16 if dtype is None else dtype
        # extension: outputs (and therefore their gradients) may be kept in f32
        self.output_dtype = self.dtype if output_dtype is None else output_dtype
        self._leaves = _build(n_input_dims, encoding_config)
        self.n_output_dims = sum(leaf.n_out for _, leaf in self._leaves)
        self._param_offsets = []
        off = 0
        gen = torch.Generator().manual_seed(seed)
        inits = []
        for _, leaf in self._leaves:
            self._param_offsets.append(off)
            off += leaf.n_params
            if leaf.n_params:
                inits.append(leaf.init_params(gen))
        init = torch.cat(inits) if inits else torch.zeros(0)
        self.params = nn.Parameter(init.float(), requires_grad=True)

    @property
    def hash_grids(self) -> list[_HashGrid]:
        return [leaf for _, leaf in self._leaves if isinstance(leaf, _HashGrid)]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.dim() != 2 or x.shape[1] != self.n_input_dims:
            raise ANRError(f"Encoding expects (M, {self.n_input_dims}) input, got {tuple(x.shape)}")
        x = x.to(torch.float32).contiguous()
        _lib.grad_use(self.params)
        return _EncodingFn.apply(x, self.params, self)

    def extra_repr(self) -> str:
        return f"n_input_dims={self.n_input_dims}, n_output_dims={self.n_output_dims}"


# --------------------------------------------------------------------------- network
class _NetworkFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, params, net: "Network"):
        M = x.shape[0]
        prec = _net_prec(net)
        p = _lib.compute_copy(params, net.dtype)
        out = torch.empty(M, net.n_output_dims, device=x.device, dtype=net.output_dtype)
        call("anr_mlp_fwd", ctypes.byref(net.desc), prec, ptr(p), ptr(x), dtype_code(x.dtype),
             x.stride(0), M, ptr(out), dtype_code(out.dtype), out.stride(0),
             _lib.stream(x.device))
        ctx.net = net
        ctx.save_for_backward(x, p)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, p = ctx.saved_tensors
        net: Network = ctx.net
        dout = dout.contiguous()
        prec = _net_prec(net)
        dparams, direct = _lib.grad_target(net.params, x.device)
        din = None
        if ctx.needs_input_grad[0]:
            din = torch.empty(x.shape, device=x.device, dtype=x.dtype)
        # small batches: per-wavefront dW rows + a fixed-order sum instead of atomics
        ws_bytes = net.bwd_workspace_bytes(x.shape[0])
        ws = (torch.empty(ws_bytes // 4, device=x.device, dtype=torch.float32)
              if ws_bytes else None)
        if net.loss_scale:  # tcnn's loss-scaled f16 backward (reference numerics)
            call("anr_mlp_bwd_ref16", ctypes.byref(net.desc), ptr(p), ptr(x),
                 dtype_code(x.dtype), x.stride(0), x.shape[0], ptr(dout),
                 dtype_code(dout.dtype), dout.stride(0), ptr(din), dtype_code(x.dtype),
                 x.stride(0) if din is not None else 0, ptr(dparams), ptr(ws), ws_bytes,
                 float(net.loss_scale), _lib.stream(x.device))
        else:
            call("anr_mlp_bwd_ws", ctypes.byref(net.desc), prec, ptr(p), ptr(x),
                 dtype_code(x.dtype), x.stride(0), x.shape[0], ptr(dout),
                 dtype_code(dout.dtype), dout.stride(0), ptr(din), dtype_code(x.dtype),
                 x.stride(0) if din is not None else 0, ptr(dparams), ptr(ws), ws_bytes,
                 _lib.stream(x.device))
        if direct:
            _lib.grad_done(net.params)
        return din, None if direct else dparams, None


def _net_prec(net) -> int:
    """Compute precision code of a standalone network kernel (anr_mlp_*): f16 or f32. bf16
    networks exist only inside the fused Instant-NGP field (anr_ingp_field_*)."""
    if net.dtype == torch.float16:
        return _lib.F16
    if net.dtype == torch.float32:
        return _lib.F32
    raise ANRError(f"Network dtype {net.dtype}: standalone MLP kernels run f16 or f32; bf16 "
                   "is the fused Instant-NGP field's MFMA precision only")


class Network(nn.Module):
    """tinycudann.Network(n_input_dims, n_output_dims, network_config, seed=1337)."""

    def __init__(self, n_input_dims: int, n_output_dims: int, network_config: dict,
                 seed: int = 1337, dtype: torch.dtype | None = None,
                 output_dtype: torch.dtype | None = None):
        super().__init__()
        cfg = _lower(network_config)
        otype = str(cfg.get("otype", "FullyFusedMLP")).lower()
        if otype not in ("fullyfusedmlp", "cutlassmlp"):
            raise ANRError(f"network otype {cfg.get('otype')!r} not supported")
        if str(cfg.get("activation", "ReLU")).lower() != "relu":
            raise ANRError("only ReLU hidden activation is supported")
        out_act = str(cfg.get("output_activation", "None")).lower()
        if out_act not in ("none", "relu"):
            raise ANRError(f"output_activation {out_act!r} not supported")
        self.n_input_dims = n_input_dims
        self.n_output_dims = n_output_dims
        self.network_config = network_config
        self.dtype = torch.float16 if dtype is None else dtype
        self.output_dtype = self.dtype if output_dtype is None else output_dtype
        # None: the kernels' own per-wavefront f16 gradient scaling; a number (tcnn: 128):
        # tinycudann's fixed loss scale and its f16 input gradient (reference numerics)
        self.loss_scale: float | None = None
        self.width = int(cfg.get("n_neurons", 64))
        self.n_hidden_layers = int(cfg.get("n_hidden_layers", 2))
        self.desc = _lib.mlp_desc(n_input_dims, n_output_dims, self.width, self.n_hidden_layers,
                                  out_act == "relu")
        self.layer_shapes = [(self.width, self.desc.n_input_padded)]
        self.layer_shapes += [(self.width, self.width)] * (self.n_hidden_layers - 1)
        self.layer_shapes += [(self.desc.n_output_padded, self.width)]
        gen = torch.Generator().manual_seed(seed)
        chunks = []
        for o, i in self.layer_shapes:  # tcnn: Xavier-uniform per layer
            bound = math.sqrt(6.0 / (o + i))
            chunks.append((torch.rand(o * i, generator=gen) * 2 - 1) * bound)
        self.params = nn.Parameter(torch.cat(chunks).float(), requires_grad=True)

    def bwd_workspace_bytes(self, M: int) -> int:
        """Scratch bytes the backward can use at batch M (anr_mlp_bwd_workspace_bytes)."""
        cache = self.__dict__.setdefault("_ws_bytes", {})
        if M not in cache:
            cache[M] = int(_lib.load().anr_mlp_bwd_workspace_bytes(ctypes.byref(self.desc), M))
        return cache[M]

    def layer(self, k: int) -> torch.Tensor:
        """View of layer k's (out, in) weight matrix inside the flat params."""
        off = sum(o * i for o, i in self.layer_shapes[:k])
        o, i = self.layer_shapes[k]
        return self.params[off:off + o * i].view(o, i)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.dim() != 2 or x.shape[1] != self.n_input_dims:
            raise ANRError(f"Network expects (M, {self.n_input_dims}) input, got {tuple(x.shape)}")
        if x.dtype not in (torch.float16, torch.float32):
            x = x.float()
        _lib.grad_use(self.params)
        return _NetworkFn.apply(x.contiguous(), self.params, self)

    def extra_repr(self) -> str:
        return (f"n_input_dims={self.n_input_dims}, n_output_dims={self.n_output_dims}, "
                f"width={self.width}, n_hidden_layers={self.n_hidden_layers}")


def free_temporary_memory() -> None:
    """tcnn API parity: the HIP library keeps no temporary device memory."""


def batch_size_granularity() -> int:
    """tcnn API parity: any batch size is accepted (no internal padding)."""
    return 1


__all__ = ["Encoding", "Network", "free_temporary_memory", "batch_size_granularity"]
_ = Any
