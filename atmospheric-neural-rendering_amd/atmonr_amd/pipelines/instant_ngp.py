"""InstantNGPPipeline — drop-in for src/atmonr/pipelines/instant_ngp.py on MI355X.

Same constructor ``(config, dataset)``, module names, optimizer contract (AdamW with
weight decay on the MLPs only, :107-127), ``forward`` result keys (:194-206),
``extract`` (:208-247), ``compute_loss`` (:249-263) and nested ``state_dict``
(:265-284). The six tinycudann modules (:60-85) are atmonr_amd.tcnn modules.

Two execution paths, identical semantics:

* ``fused=True`` (default, used by bench.py): K1+K2 sampler/preprocessor in one kernel,
  the per-sample field as one autograd node (atmonr_amd.field.IngpFieldFn) with f32
  gradients between kernels, the composite on K8 with z scaled in-kernel, the loss on K9.
* ``fused=False``: the reference's op-by-op graph (sample_uniform_bins, the point
  preprocessor, the (p+1)/2 remap, tcnn-style modules with f16 outputs) on the same
  kernels — used to check that the fused path changes nothing but speed.

Two numerics (``numerics=`` or the config key ``"numerics"``):

* ``"build"`` (default): f16 tables / weights / activations as tcnn, but the composite,
  the loss and every inter-kernel gradient in f32 (no f16 underflow in the backward).
* ``"reference"``: the reference's own f16 arithmetic wherever it differs — the composite
  and the loss as chains of f16 torch ops with torch's f16 autograd (graphics_utils.py:
  28-76, instant_ngp.py:259-263; csrc/ref16.hip), tinycudann's loss-scaled (x128) f16
  module backward with f16 gradients at the module boundaries, and tcnn's f16 parameter
  gradients (tinycudann/modules.py). Opt-in, for PSNR parity with the reference; f16
  networks, fused field, no occupancy culling.
"""

from __future__ import annotations

import os
from itertools import chain
from typing import Any, Mapping

import torch
import torch.nn.functional as F
from torch.optim import Optimizer

from .. import _lib
from ..field import IngpFieldFn, field_density, field_fused
from ..graphics_utils import render_with_surface, render_with_surface_ref16
from ..losses import LOSSES, indexed_loss, indexed_loss_ref16
from ..occupancy import OccupancyGrid, pipeline_density
from ..optim import FusedAdam
from ..samplers import preprocess_points, sample_and_preprocess, sample_uniform_bins
from ..tcnn import Encoding, Network
from .pipeline import Pipeline


class InstantNGPPipeline(Pipeline):
    module_names = ["pos_encoder", "pos_mlp", "dir_encoder", "dir_mlp", "surf_encoder",
                    "surf_mlp"]

    def __init__(self, config: dict, dataset: Any, dtype: torch.dtype = torch.float16,
                 fused: bool = True, seed: int = 1337, occupancy=None,
                 mlp_dtype: torch.dtype | None = None, numerics: str | None = None) -> None:
        """``dtype``: tcnn compute precision of every module (f16 as the reference, or f32).
        ``mlp_dtype=torch.bfloat16`` (BASELINE configs[4], beyond the reference): the
        per-sample pos / dir MLPs run bf16 MFMA over the f16 hash features (fused field
        only); the per-ray surface network keeps ``dtype``. ``numerics``: "build" or
        "reference" (module docstring)."""
        super().__init__(config, dataset)
        numerics = numerics or self.config.get("numerics", "build")
        if numerics not in ("build", "reference"):
            raise ValueError(f"numerics {numerics!r}: 'build' or 'reference'")
        self.numerics = numerics
        self.num_density_outputs = 1
        if self.config["multi_band_extinction"]:
            self.num_density_outputs = self.config["num_bands"]
        if self.config["include_height"]:
            raise NotImplementedError("include_height is disabled in both reference configs")
        if fused and self.num_density_outputs != 1:
            fused = False
        self.fused = fused
        self.dtype = dtype
        mlp_dtype = dtype if mlp_dtype is None else mlp_dtype
        if mlp_dtype == torch.bfloat16 and (dtype != torch.float16 or not fused):
            raise ValueError("bf16 field MLPs need f16 hash features and the fused path")
        self.mlp_dtype = mlp_dtype
        # tinycudann's loss scale for f16 modules (reference numerics only)
        self.loss_scale = 128.0 if numerics == "reference" else None
        if numerics == "reference" and not (fused and dtype == torch.float16 and
                                            mlp_dtype == torch.float16 and occupancy is None):
            raise ValueError("numerics='reference' runs the fused f16 field (f16 modules, "
                             "no occupancy culling)")
        # reference numerics: rays whose f16 alpha rounded to exactly 1 (their gradients are
        # zero, not torch's zero-input cumprod branch; ref16.hip), counted over the
        # pipeline's life (zero_rays_total; the Trainer warns when it grows)
        self._zero_rays = None
        self._defer_quant = False  # defer_grad_quantize
        self.surface_stream = os.environ.get("ANR_SURFACE_STREAM", "1") != "0"
        ingp = self.config["instant_ngp"]
        nb = self.config["num_bands"]
        # the fused path keeps activations / gradients in f32 (build numerics); tcnn's f16
        # outputs in reference numerics
        fdt = torch.float32 if fused and numerics == "build" else None
        self.pos_encoder = Encoding(3, ingp["encoding"], seed=seed, dtype=dtype)
        self.pos_mlp = Network(self.pos_encoder.n_output_dims, 16, ingp["network"],
                               seed=seed + 1, dtype=mlp_dtype)
        self.dir_encoder = Encoding(3 + 16 - self.num_density_outputs, ingp["dir_encoding"],
                                    seed=seed + 2, dtype=dtype)
        self.dir_mlp = Network(self.dir_encoder.n_output_dims, nb, ingp["rgb_network"],
                               seed=seed + 3, dtype=mlp_dtype)
        self.surf_encoder = Encoding(2 + 3, ingp["surface_encoding"], seed=seed + 4,
                                     dtype=dtype, output_dtype=fdt)
        self.surf_mlp = Network(self.surf_encoder.n_output_dims, nb, ingp["surface_network"],
                                seed=seed + 5, dtype=dtype, output_dtype=fdt)
        self.surf_mlp.loss_scale = self.loss_scale
        d = self.dir_mlp.desc
        self._dir_desc_relu = _lib.mlp_desc(d.n_input, d.n_output, d.width, d.n_hidden_layers,
                                            True)
        self.training = True
        self.max_i = dataset.max_i
        self.loss_name = self.config["loss"].lower()
        self.loss_fn = LOSSES[self.loss_name]
        self.alt_compress = float(self.config["alt_compress_factor"])
        if self.point_preprocessor is not None:
            self._prep_ngp = self.point_preprocessor.params(ngp_remap=True,
                                                            alt_compress=self.alt_compress)
        # occupancy-grid culling (beyond the reference, atmonr_amd.occupancy): off unless
        # passed in or configured; the uniform sampler stays the parity default
        occ_cfg = self.config.get("occupancy_grid")
        if occupancy is None and occ_cfg and numerics == "build":
            occupancy = OccupancyGrid.from_config(occ_cfg, self.alt_compress,
                                                  getattr(dataset, "device", None))
        self.occupancy = occupancy

    def defer_grad_quantize(self, optimizer) -> None:
        """Reference numerics: leave tinycudann's f16 rounding of the parameter gradients,
        f16(f16(g * 128) / 128), to ``optimizer`` -- a FusedAdam, which applies it as it
        reads each gradient (anr_adam_tensor.grad_quant) -- instead of a separate pass over
        every gradient at the end of backward (anr_grad_quantize_f16, ~0.03 ms per step at
        the bench shape). The update is the same; ``param.grad`` between backward and the
        step then holds the unrounded f32 sums, so code that reads or reduces gradients in
        between (all-reduce, clipping, parity tests) must not defer. No-op in build
        numerics."""
        from ..optim import FusedAdam

        if self.numerics != "reference":
            return
        if not isinstance(optimizer, FusedAdam) or not optimizer.multi_tensor:
            raise ValueError("defer_grad_quantize needs a FusedAdam(multi_tensor=True)")
        for m in self.modules():
            if m.params.numel():
                m.params._anr_grad_quant = float(self.loss_scale)
        self._defer_quant = True

    # ------------------------------------------------------------------ module plumbing
    def modules(self):
        return [getattr(self, n) for n in self.module_names]

    def send_tensors_to(self, device: int) -> None:
        self.device = device
        for m in self.modules():
            m.to(device)

    def get_optimizer(self, config: dict, fused: bool = True) -> Optimizer:
        """AdamW, weight decay on the MLPs only (instant_ngp.py:107-127)."""
        no_decay = chain(self.pos_encoder.parameters(), self.dir_encoder.parameters(),
                         self.surf_encoder.parameters())
        decay = chain(self.pos_mlp.parameters(), self.dir_mlp.parameters(),
                      self.surf_mlp.parameters())
        groups = [
            {"params": [p for p in no_decay if p.numel()], "weight_decay": 0},
            {"params": list(decay), "weight_decay": config["weight_decay"]},
        ]
        kw = dict(config)
        kw["betas"] = tuple(kw.get("betas", (0.9, 0.999)))
        if fused:
            return FusedAdam(groups, decoupled=True, **kw)
        return torch.optim.AdamW(groups, **kw)

    def parameters(self):
        return chain(*(m.parameters() for m in self.modules()))

    # ------------------------------------------------------------------ forward
    def forward(self, ray_batch: Mapping[str, torch.Tensor], u: torch.Tensor | None = None
                ) -> dict[str, torch.Tensor]:
        if self.fused:
            return self._forward_fused(ray_batch, u)
        return self._forward_reference(ray_batch, u)

    def _surface(self, ray_batch):
        # instant_ngp.py:143,150,173-174 (pts_surf in normalized Cartesian, then [0,1]);
        # surf_in = [pts_surf[:, :2] | dir] built by one kernel, rounded as torch rounds
        o, d, ln = (ray_batch[k].float().contiguous() for k in ("origin", "dir", "len"))
        surf_in = torch.empty(o.shape[0], 5, device=o.device, dtype=torch.float32)
        _lib.call("anr_ingp_surface_input", _lib.ptr(o), _lib.ptr(d), _lib.ptr(ln),
                  o.shape[0], _lib.ptr(surf_in), _lib.stream(o.device))
        return F.relu(self.surf_mlp(self.surf_encoder(surf_in)))

    def _surface_async(self, ray_batch):
        """Start the surface branch on the side stream; returns a callable giving its
        output on the current stream. ``surface_stream = False`` (or
        ANR_SURFACE_STREAM=0) keeps everything on one stream."""
        dev = ray_batch["origin"].device
        if not self.surface_stream or dev.type != "cuda":
            out = self._surface(ray_batch)
            return lambda: out
        main = torch.cuda.current_stream(dev)
        side = _lib.side_stream(dev)
        side.wait_stream(main)  # batch rows (gathered on main), f16 copies (AdamW on main)
        with torch.cuda.stream(side):
            out = self._surface(ray_batch)
            if out.requires_grad:
                out = _lib.JoinAtBackwardEnd.apply(out, main)

        def join():
            main.wait_stream(side)
            out.record_stream(main)
            return out
        return join

    def _forward_fused(self, ray_batch, u=None):
        B = ray_batch["origin"].shape[0]
        N = self.config["num_samples_per_ray"]
        # the per-ray surface branch (6 small kernels each way) is enqueued first, on its
        # own stream, so it runs beside the sampler / hash grid forward and, in backward,
        # beside the hash-grid backward
        surf_branch = self._surface_async(ray_batch)
        _, z_vals, coords = sample_and_preprocess(ray_batch, N, self._prep_ngp, u=u)
        occ = self.occupancy
        if occ is not None and self.training:
            occ.update(pipeline_density(self))
        params = (self.pos_encoder.params, self.pos_mlp.params, self.dir_mlp.params, self)
        _lib.grad_use(*params[:3])  # IngpFieldFn accumulates these three directly
        if occ is not None and occ.active:
            # only samples in occupied cells reach the hash grid and the MLPs; sigma and
            # color come back dense (B*N rows) with zeros at the culled samples
            rows, kept = occ.compact(coords.view(B * N, 3))
            sigma, color = IngpFieldFn.apply(kept, ray_batch["dir"].float(), N, *params, rows,
                                             B * N)
        else:
            sigma, color = IngpFieldFn.apply(coords.view(B * N, 3), ray_batch["dir"].float(), N,
                                             *params)
        color = color.view(B, N, -1)
        sigma = sigma.view(B, N, 1)
        color_surf = surf_branch()
        if self.numerics == "reference":
            if self._zero_rays is None:  # counts over the pipeline's life (no per-step op)
                self._zero_rays = torch.zeros(1, dtype=torch.int32, device=color.device)
            # the kernel also writes tcnn's f16 colour / density outputs for the results
            color_map, _, weights, atmo, surf, color, sigma = render_with_surface_ref16(
                z_vals, color, sigma, color_surf, z_scale=self.scale / 1000,
                zero_rays=self._zero_rays, inputs_f16=True)
            if color_map.requires_grad:
                color_map = _TcnnGradsAtBackwardEnd.apply(color_map, self)
        else:
            color_map, _, weights, atmo, surf = render_with_surface(
                z_vals, color, sigma, color_surf, z_scale=self.scale / 1000)
        return {
            "color_fine": color[:, :-1],
            "color_surf": color_surf,
            "color_map_surf": surf,
            "color_map_atmo": atmo,
            "sigma_fine": sigma[:, :-1],
            "color_map_fine": color_map,
            "weights_fine": weights,
            "z_vals_fine": z_vals,
        }

    def _forward_reference(self, ray_batch, u=None):
        # instant_ngp.py:137-206, op for op
        B_ = ray_batch["origin"].shape[0]
        N = self.config["num_samples_per_ray"]
        pts, z_vals = sample_uniform_bins(ray_batch, N, u=u)
        if self.point_preprocessor:
            pts = self.point_preprocessor(pts)
        pts = (pts + 1) / 2
        dirs = ray_batch["dir"][:, None].repeat(1, N, 1)
        pts[..., 2] = pts[..., 2] / self.config["alt_compress_factor"]
        pos_enc = self.pos_encoder(pts.view(B_ * N, -1))
        pos_out = self.pos_mlp(pos_enc)
        dir_enc = self.dir_encoder(
            torch.cat([dirs.view(B_ * N, 3), pos_out[:, self.num_density_outputs:]], dim=1))
        color = self.dir_mlp(dir_enc).view(B_, N, self.config["num_bands"])
        color_surf = self._surface(ray_batch)
        sigma = pos_out[..., : self.num_density_outputs].view(B_, N, -1)
        color = F.relu(color)
        sigma = F.relu(sigma)
        color_map, _, weights, atmo, surf = render_with_surface(
            z_vals * (self.scale / 1000), color, sigma, color_surf)
        return {
            "color_fine": color[:, :-1],
            "color_surf": color_surf,
            "color_map_surf": surf,
            "color_map_atmo": atmo,
            "sigma_fine": sigma[:, :-1],
            "color_map_fine": color_map,
            "weights_fine": weights,
            "z_vals_fine": z_vals,
        }

    @property
    def zero_rays_total(self) -> int:
        """Reference numerics: rays (over every training step so far) whose gradients were
        dropped because an f16 alpha rounded to exactly 1 (synchronises; 0 otherwise)."""
        if self._zero_rays is None:
            return 0
        return int(self._zero_rays.item())

    def extract(self, pts: torch.Tensor, run_length: int = 0) -> torch.Tensor:
        """Extinction at normalized scene points (P,3) (instant_ngp.py:208-247).
        ``run_length`` (optional, not in the reference's signature): the points come in
        runs of that many neighbours (an extract column), a hint for the hash-grid walker
        that does not change the values."""
        if self.point_preprocessor:
            pts = preprocess_points(pts, self._prep_ngp)
        else:
            pts = (pts + 1) / 2
            pts[..., 2] = pts[..., 2] / self.alt_compress
        if self.num_density_outputs == 1 and field_fused(self) and \
                self.pos_encoder.dtype == torch.float16:
            # the fused field's sigma output IS relu(pos_out[:, 0]) (f32 accumulator);
            # returned in tcnn's output precision, as the reference's clip of pos_out
            return field_density(self, pts, run_length).view(pts.shape[0], 1).to(
                self.pos_mlp.output_dtype)
        with torch.no_grad():
            pos_out = self.pos_mlp(self.pos_encoder(pts))
        return torch.clip(pos_out[..., : self.num_density_outputs].view(
            pts.shape[0], self.num_density_outputs), min=0)

    def compute_loss(self, ray_batch: Mapping[str, torch.Tensor],
                     results: dict[str, torch.Tensor]) -> torch.Tensor:
        """loss_fn(take_along_dim(color_map, irgb_idx), rad, max_i) (instant_ngp.py:249-263)."""
        if self.numerics == "reference":
            return indexed_loss_ref16(self.loss_name, results["color_map_fine"],
                                      ray_batch["irgb_idx"], ray_batch["rad"], self.max_i)
        return indexed_loss(self.loss_name, results["color_map_fine"], ray_batch["irgb_idx"],
                            ray_batch["rad"], self.max_i)

    # ------------------------------------------------------------------ state
    def state_dict(self) -> Mapping[str, Mapping[str, Any]]:
        return {n: getattr(self, n).state_dict() for n in self.module_names}

    def load_state_dict(self, state_dict: dict) -> None:
        for n in self.module_names:
            getattr(self, n).load_state_dict(state_dict[n])

    def train(self) -> None:
        self.training = True
        for m in self.modules():
            m.train()

    def eval(self) -> None:
        self.training = False
        for m in self.modules():
            m.eval()


class _TcnnGradsAtBackwardEnd(torch.autograd.Function):
    """Identity on the colour map (reference numerics). Its backward queues an
    end-of-backward callback that turns every module's accumulated f32 parameter gradient
    into the value tinycudann hands to torch: the module's f16 gradient at loss scale 128,
    divided by 128 in f16 (tinycudann/modules.py; anr_grad_quantize_f16). The callback
    runs once the whole backward has been enqueued; it first joins the surface branch's
    side stream, whose kernels write that branch's gradients."""

    @staticmethod
    def forward(ctx, x, pipe):
        ctx.pipe = pipe
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        pipe = ctx.pipe
        dev = g.device

        def quantize():
            main = torch.cuda.current_stream(dev)
            main.wait_stream(_lib.side_stream(dev))
            if pipe._defer_quant:
                return  # the optimizer rounds the gradients as it reads them
            grads = []
            for m in pipe.modules():
                p = m.params
                if p.numel() and p.grad is not None:
                    if p.grad.dtype != torch.float32 or not p.grad.is_contiguous():
                        raise _lib.ANRError("reference numerics: f32 contiguous grads only")
                    grads.append(p.grad)
            # gradients that tile one contiguous range (a FlatGradBucket's views) are
            # quantised in one launch (elementwise: the same values)
            grads.sort(key=lambda g: g.data_ptr())
            spans = []
            for g in grads:
                if spans and spans[-1][0] + 4 * spans[-1][1] == g.data_ptr():
                    spans[-1][1] += g.numel()
                else:
                    spans.append([g.data_ptr(), g.numel()])
            for base, n in spans:
                _lib.call("anr_grad_quantize_f16", base, n, float(pipe.loss_scale),
                          _lib.stream(dev), tag="grad_quantize")
        torch.autograd.Variable._execution_engine.queue_callback(quantize)
        return g, None
