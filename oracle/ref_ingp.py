"""ORACLE (test infrastructure only): the Instant-NGP train step on CPU, with autograd.

Restates src/atmonr/pipelines/instant_ngp.py:137-206 (forward) and :249-263
(compute_loss) in float64 torch on top of the other oracle pieces:

* sampler            samplers.py:8-47             -> ref_path.sample_uniform_bins
* point preprocessor harp2.py:357-388             -> ref_nerf.preprocess_torch
* remap              instant_ngp.py:143-160       -> (p + 1) / 2, z / alt_compress_factor
* tcnn HashGrid      instant_ngp.py:60-63,163     -> hashgrid() below, corners and weights
                                                     from ref_tcnn.hashgrid_corners
* tcnn FullyFusedMLP instant_ngp.py:64-77,164-171 -> ref_tcnn.mlp_fwd
* SH2 + Identity     instant_ngp.py:69-72,165-169 -> ref_tcnn.sh + the pos_out columns
* surface path       instant_ngp.py:78-85,173-174
* composite          graphics_utils.py:52-77      -> ref_path.render_with_surface
* loss               instant_ngp.py:249-263       -> ref_path.LOSSES
* AdamW groups       instant_ngp.py:107-127

``half=True`` rounds what the f16 GPU path rounds (hash table, encodings, MLP weights
and hidden activations, the f16 MLP outputs) so the oracle tracks the bench
configuration; the roundings act on values only, gradients pass through them in f64
(ref_tcnn.rounder; r02's plain ``.half().double()`` casts quantised the UNSCALED
gradients to f16 in autograd, so that oracle's "exact" f16-forward gradients carried
f16 underflow of their own). tcnn semantics are unpinned against real tinycudann (see
ref_tcnn).

``semantics="reference"`` (with ``half=True``) restates what the REFERENCE computes in
its f16 Instant-NGP path, as opposed to what this build computes:

* every tinycudann module returns an f16 tensor, and its backward follows tcnn's
  torch binding (tinycudann/modules.py, upstream; not in /root/reference): the incoming
  f16 gradient is multiplied by loss_scale = 128 in f16, the module's backward runs on
  f16 tiles (hidden-layer gradients rounded to f16 here), the parameter gradient comes
  back in f16 and is divided by 128, the input gradient likewise;
* the composite (graphics_utils.py:6-77) runs on those f16 tensors: z is cast to f16
  km (graphics_utils.py:28), alpha, the cumprod and the sums are f16 torch ops, and
  the f16 autograd of the composite rounds every gradient to f16 -- restated op by op
  in oracle/ref_f16.py with torch's CUDA accumulation (the reference needs CUDA: f16
  accumulator in cumprod and in its backward's cumsum, f32 in sum / prod), which
  differs from torch's CPU f16 kernels (``ref_acc="cpu"`` runs torch's CPU f16 ops
  instead, for comparison);
* the loss takes the f16 prediction and the target cast to f16 (instant_ngp.py:262),
  as f16 ops with their f16 autograd (ref_f16.loss_f16; the Python scalar
  ``1e-3 * max_i`` added in f32 as torch on CUDA does);
* a module's parameter gradient is f16(f16(g * 128) / 128): tcnn's f16 gradient at
  loss scale 128 divided by the loss scale in f16 (``params_grad / loss_scale``).
Approximations (tcnn absent): the MLP backward's rounding is applied per layer, not per
16x16 tile; the hash-grid gradient (tcnn: f16 half2 atomics) is summed in f64 and
rounded once.

``acc`` (reference semantics): the accumulation precision of the sums that feed each f16
rounding -- the MLP products (forward, dL/dx, dL/dW) and the hash grid's trilinear sums
and gradient scatter. tcnn's kernels accumulate in f32 (MMA / atomics) in an order of
their own, which no CPU restatement can reproduce; the arms are equally valid orders:
``"f64"`` (default) sums exactly enough that each f16 rounding sees the exact value;
``"f32"`` sums in f32 in torch-CPU's BLAS / index_add order (the GPU's precision, its
own order); ``"f32rev"`` sums in f32 with every reduction axis reversed (a third order).
Near f16's subnormal range a sum with cancellation rounds differently under f32 than
under f64, and AdamW with eps = 1e-15 turns a gradient that is 0 in one order and one
subnormal in another into a full lr step of a never-touched entry: the arms measure how
far the reference's own PSNR trajectory depends on its summation order.
"""

from __future__ import annotations

import numpy as np
import torch

from . import ref_f16, ref_nerf, ref_path, ref_tcnn

MODULES = ("pos_encoder", "pos_mlp", "dir_mlp", "surf_encoder", "surf_mlp")


def _grid_cfg(enc_cfg: dict, n_dims: int):
    return (n_dims, int(enc_cfg["n_levels"]), int(enc_cfg["base_resolution"]),
            float(enc_cfg["per_level_scale"]), int(enc_cfg["log2_hashmap_size"]))


def hashgrid(x: torch.Tensor, table: torch.Tensor, cfg, rnd, acc: str = "f64") -> torch.Tensor:
    """tcnn GridEncoding forward, differentiable in ``table``; x (M, D) float32. ``acc``
    "f32" / "f32rev": the corner sums and the gradient scatter in f32 (reversed sample
    order for the scatter with "f32rev")."""
    xn = x.detach().float().numpy()
    tab = rnd(table).view(-1, 2)
    if acc != "f64":
        tab = _Cast.apply(tab, torch.float32)
    outs = []
    for lvl in range(cfg[1]):
        idx, wt = ref_tcnn.hashgrid_corners(xn, cfg, lvl)
        wt_t = torch.from_numpy(wt).to(tab.dtype)
        idx_t = torch.from_numpy(idx)
        if acc == "f32rev":
            rev = torch.arange(idx_t.shape[0] - 1, -1, -1)
            g = _FlipGather.apply(tab, idx_t, rev)
        else:
            g = tab[idx_t]
        outs.append(torch.einsum("mc,mcf->mf", wt_t, g))
    return rnd(torch.cat(outs, dim=1).double())


class _Cast(torch.autograd.Function):
    """x -> x.to(dtype); the gradient comes back in x's dtype (value of the f32 sum)."""

    @staticmethod
    def forward(ctx, x, dtype):
        ctx.dt = x.dtype
        return x.to(dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(ctx.dt), None


class _FlipGather(torch.autograd.Function):
    """tab[idx] whose backward scatters the samples in reversed order (f32rev arm)."""

    @staticmethod
    def forward(ctx, tab, idx, rev):
        ctx.save_for_backward(idx, rev)
        ctx.n = tab.shape[0]
        return tab[idx]

    @staticmethod
    def backward(ctx, g):
        idx, rev = ctx.saved_tensors
        out = torch.zeros((ctx.n,) + tuple(g.shape[2:]), dtype=g.dtype)
        out.index_add_(0, idx[rev].reshape(-1), g[rev].reshape(-1, *g.shape[2:]))
        return out, None, None


class _MatmulAcc(torch.autograd.Function):
    """h @ W.t() with every sum of the forward and the backward in f32 (``rev``: each
    reduction axis reversed) -- the f32 / f32rev arms of RefInstantNGP(acc=...)."""

    @staticmethod
    def forward(ctx, h, W, rev):
        ctx.save_for_backward(h, W)
        ctx.rev = rev
        hf, Wf = h.float(), W.float()
        if rev:
            hf, Wf = hf.flip(1), Wf.flip(1)
        return (hf @ Wf.t()).double()

    @staticmethod
    def backward(ctx, g):
        h, W = ctx.saved_tensors
        gf, hf, Wf = g.float(), h.float(), W.float()
        if ctx.rev:
            dh = gf.flip(1) @ Wf.flip(0)
            dW = gf.flip(0).t() @ hf.flip(0)
        else:
            dh = gf @ Wf
            dW = gf.t() @ hf
        return dh.double(), dW.double(), None


LOSS_SCALE = 128.0  # tinycudann.modules default loss scale for f16 parameters


class _RoundBoth(torch.autograd.Function):
    """x -> f16(x) forward, g -> f16(g) backward (values and gradients on f16 tiles)."""

    @staticmethod
    def forward(ctx, x):
        return x.half().double()

    @staticmethod
    def backward(ctx, g):
        return g.half().double()


class _GradNoise(torch.autograd.Function):
    """SPREAD EXPERIMENT ONLY (tools/ingp_oracle_spread.py --perturb xnoise): identity
    forward; backward multiplies the incoming gradient by (1 + factor * 2^-24 * n), n
    standard normal -- an f32 accumulation's relative error, placed before the f16
    rounding of the hidden-layer gradient that follows in autograd's order."""

    @staticmethod
    def forward(ctx, x, noise):
        ctx.noise = noise
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        gen, factor = ctx.noise
        return g * (1 + torch.randn(g.shape, generator=gen, dtype=g.dtype) * factor
                    * 2.0 ** -24), None


class _TcnnCall(torch.autograd.Function):
    """One tinycudann module call in reference semantics: f16 output; backward with the
    f16 gradient scaled by LOSS_SCALE, the f64 module graph run on it, parameter and input
    gradients rounded to f16 and unscaled."""

    @staticmethod
    def forward(ctx, x, params, fn, sum_noise=None, x_noise=None):
        with torch.enable_grad():
            x64 = x.detach().double().requires_grad_(x.requires_grad)
            p64 = params.detach().double().requires_grad_(True)
            y = fn(x64, p64)
        ctx.graph = (x64, p64, y)
        ctx.x_dtype = x.dtype
        ctx.sum_noise = sum_noise
        ctx.x_noise = x_noise
        return y.detach().half()

    @staticmethod
    def backward(ctx, g):
        x64, p64, y = ctx.graph
        gs = (g.float() * LOSS_SCALE).half().double()
        ins = (x64, p64) if x64.requires_grad else (p64,)
        grads = torch.autograd.grad(y, ins, gs, allow_unused=True, retain_graph=True)
        gp = grads[-1]
        if gp is not None and ctx.sum_noise is not None:
            # SPREAD EXPERIMENT ONLY (tools/ingp_oracle_spread.py --perturb sumnoise): the
            # parameter gradient as an f32 sum in another order would carry, per entry, an
            # error of about u_f32 * sum|terms|; added here as seeded normal noise of that
            # size (sum|terms| = the same backward with |upstream gradient|)
            gen, factor = ctx.sum_noise
            (ga,) = torch.autograd.grad(y, (p64,), gs.abs(), allow_unused=True)
            if ga is not None:
                n = torch.randn(gp.shape, generator=gen, dtype=gp.dtype)
                gp = gp + n * factor * 2.0 ** -24 * ga
        gp = torch.zeros_like(p64) if gp is None else (gp.half() / LOSS_SCALE).double()
        gx = None
        if x64.requires_grad and grads[0] is not None:
            g0 = grads[0]
            if ctx.x_noise is not None:
                # SPREAD EXPERIMENT ONLY (--perturb xnoise): the input gradient as an f32
                # dot product would carry a relative error of about u_f32 * sqrt(K); as
                # seeded noise of that size before tcnn's f16 rounding
                gen, factor = ctx.x_noise
                g0 = g0 * (1 + torch.randn(g0.shape, generator=gen, dtype=g0.dtype)
                           * factor * 2.0 ** -24)
            gx = (g0.half().double() / LOSS_SCALE).to(ctx.x_dtype)
        return gx, gp, None, None, None


class RefInstantNGP:
    """Parameters (float64 leaf tensors, flat per module like tcnn) + forward / loss."""

    def __init__(self, config: dict, state: dict, prep: dict, scale: float, max_i: float,
                 half: bool = False, mlp_half=None, semantics: str = "build",
                 composite: str = "f32", ref_acc: str = "cuda", acc: str = "f64"):
        self.cfg = config
        self.ingp = config["instant_ngp"]
        self.N = int(config["num_samples_per_ray"])
        self.nb = int(config["num_bands"])
        self.alt = float(config["alt_compress_factor"])
        self.prep, self.scale, self.max_i = prep, float(scale), float(max_i)
        self.half = half
        # rounding of the per-sample pos / dir MLPs: as the rest (None) or "bf16" (the
        # build's bf16 MFMA field, BASELINE configs[4])
        self.mlp_half = half if mlp_half is None else mlp_half
        if semantics not in ("build", "reference") or (semantics == "reference" and half is not True):
            raise ValueError("semantics='reference' is the reference's f16 path (half=True)")
        self.semantics = semantics
        # "f32": the composite in f32 as the reference evaluates it; "f64": exact, to
        # measure how sensitive a gradient is to the composite's f32 rounding
        self.composite = composite
        # reference semantics: torch's CUDA ("cuda", ref_f16) or CPU ("cpu", torch ops)
        # f16 composite / loss kernels
        self.ref_acc = ref_acc
        if acc not in ("f64", "f32", "f32rev"):
            raise ValueError(f"acc={acc!r}: f64, f32 or f32rev")
        self.acc = acc  # reference semantics: accumulation arm (module docstring)
        self.params = {m: state[m]["params"].detach().cpu().double().clone().requires_grad_(True)
                       for m in MODULES}
        self.pos_grid = _grid_cfg(self.ingp["encoding"], 3)
        self.surf_grid = _grid_cfg(self.ingp["surface_encoding"]["nested"][0], 2)

    def _rnd(self, t):
        return ref_tcnn.rounder(self.half)(t)

    def _mlp(self, x, p, n_in, n_out, net_cfg, half=None):
        half = self.half if half is None else half
        y = ref_tcnn.mlp_fwd(x, p, n_in, n_out, int(net_cfg["n_neurons"]),
                             int(net_cfg["n_hidden_layers"]), half=half)
        return ref_tcnn.rounder(half)(y)

    def forward(self, b: dict, u: torch.Tensor | None) -> dict:
        """instant_ngp.py:137-206 on a CPU ray batch; u (B, N) or None (bin midpoints)."""
        if self.semantics == "reference":
            return self._forward_reference(b, u)
        P = self.params
        B, N = b["origin"].shape[0], self.N
        pts, z = ref_path.sample_uniform_bins(b["origin"], b["dir"], b["len"], u=u, n_bins=N)
        pts = ref_nerf.preprocess_torch(pts, **self.prep)
        pts = (pts + 1) / 2
        pts = torch.cat([pts[..., :2], pts[..., 2:] / self.alt], dim=-1)
        pos_enc = hashgrid(pts.reshape(B * N, 3), P["pos_encoder"], self.pos_grid, self._rnd)
        pos_out = self._mlp(pos_enc, P["pos_mlp"], 32, 16, self.ingp["network"],
                            self.mlp_half)
        dirs = b["dir"][:, None].expand(B, N, 3).reshape(B * N, 3)
        sh = torch.from_numpy(ref_tcnn.sh(dirs.numpy(), 2))
        dir_enc = torch.cat([self._rnd(sh), pos_out[:, 1:]], dim=1)  # SH2 | Identity (19)
        color = torch.relu(self._mlp(dir_enc, P["dir_mlp"], 19, self.nb,
                                     self.ingp["rgb_network"], self.mlp_half))
        sigma = torch.relu(pos_out[:, :1])
        # surface (instant_ngp.py:143,150,173-174): normalized Cartesian x, y
        ps = (b["origin"] + b["dir"] * b["len"][:, None] + 1) / 2
        surf_sh = self._rnd(torch.from_numpy(ref_tcnn.sh(b["dir"].numpy(), 2)))
        surf_enc = torch.cat([hashgrid(ps[:, :2], P["surf_encoder"], self.surf_grid,
                                       self._rnd), surf_sh], dim=1)
        color_surf = torch.relu(self._mlp(surf_enc, P["surf_mlp"], 36, self.nb,
                                          self.ingp["surface_network"]))
        # the composite in f32, as the reference evaluates graphics_utils.py in the network
        # output dtype (alpha = 1 - exp(-sigma * delta) cancels in that precision; the
        # GPU composite computes in f32 for every storage dtype)
        ct = torch.float64 if self.composite == "f64" else torch.float32
        cm, alpha, weights, atmo, surf = ref_path.render_with_surface(
            (z * (self.scale / 1000)).to(ct if ct == torch.float64 else z.dtype),
            color.view(B, N, -1).to(ct), sigma.view(B, N, 1).to(ct), color_surf.to(ct))
        return {"color_map_fine": cm.double(), "color_map_atmo": atmo.double(),
                "color_map_surf": surf.double(), "weights_fine": weights, "z_vals_fine": z,
                "color_fine": color.view(B, N, -1)[:, :-1],
                "sigma_fine": sigma.view(B, N, 1)[:, :-1], "color_surf": color_surf}

    # ------------------------------------------------------------ reference semantics
    def _mlp_ref(self, x, p, n_in, n_out, net_cfg):
        """FullyFusedMLP on f16 tiles: weights, activations and their gradients in f16."""
        shapes, nip, _ = ref_tcnn.mlp_layer_shapes(n_in, n_out, int(net_cfg["n_neurons"]),
                                                   int(net_cfg["n_hidden_layers"]))
        h = torch.cat([_RoundBoth.apply(x),
                       torch.ones(x.shape[0], nip - n_in, dtype=torch.float64)], dim=1)
        off = 0
        for k, (o, i) in enumerate(shapes):
            W = p[off:off + o * i].half().double().view(o, i)
            off += o * i
            h = h @ W.t() if self.acc == "f64" else _MatmulAcc.apply(h, W, self.acc == "f32rev")
            if k < len(shapes) - 1:
                # f16 tile: relu, rounded value and gradient, mask on the stored f16
                # activation (tcnn's ReLU backward)
                h = ref_tcnn.ReluRound.apply(h, torch.float16, True)
                xn = getattr(self, "mlp_x_noise", None)
                if xn is not None:
                    h = _GradNoise.apply(h, xn)
        return h[:, :n_out]

    def _grid_ref(self, cfg):
        def fn(x, p):
            return hashgrid(x, p, cfg, lambda t: t.half().double(), self.acc)
        return fn

    def _forward_reference(self, b: dict, u) -> dict:
        P = self.params
        B, N = b["origin"].shape[0], self.N
        pts, z = ref_path.sample_uniform_bins(b["origin"], b["dir"], b["len"], u=u, n_bins=N)
        pts = ref_nerf.preprocess_torch(pts, **self.prep)
        pts = (pts + 1) / 2
        pts = torch.cat([pts[..., :2], pts[..., 2:] / self.alt], dim=-1).float()
        ing = self.ingp
        pos_enc = _TcnnCall.apply(pts.reshape(B * N, 3), P["pos_encoder"],
                                  self._grid_ref(self.pos_grid),
                                  getattr(self, "grid_sum_noise", None))
        xn = getattr(self, "mlp_x_noise", None)
        pos_out = _TcnnCall.apply(pos_enc, P["pos_mlp"], lambda x, p: self._mlp_ref(
            x, p, 32, 16, ing["network"]), None, xn)
        dirs = b["dir"][:, None].expand(B, N, 3).reshape(B * N, 3).float()
        # dir_encoder(cat[dirs, pos_out[:, 1:]]): the cat promotes to f32 (instant_ngp.py:
        # 165-169); SH2 | Identity, f16 output; the identity part passes the gradient
        x_dir = torch.cat([dirs, pos_out[:, 1:]], dim=1)

        def dir_enc_fn(x, p):
            sh = _sh2(x[:, :3])
            return torch.cat([sh, x[:, 3:]], dim=1) + 0.0 * p.sum()
        dir_enc = _TcnnCall.apply(x_dir, torch.zeros(1, dtype=torch.float64), dir_enc_fn)
        color = _TcnnCall.apply(dir_enc, P["dir_mlp"], lambda x, p: self._mlp_ref(
            x, p, 19, self.nb, ing["rgb_network"]), None, xn)
        ps = ((b["origin"] + b["dir"] * b["len"][:, None] + 1) / 2).float()
        surf_in = torch.cat([ps[:, :2], b["dir"].float()], dim=1)
        surf_grid = self._grid_ref(self.surf_grid)

        def surf_enc_fn(x, p):
            return torch.cat([surf_grid(x[:, :2], p), _sh2(x[:, 2:5])], dim=1)
        surf_enc = _TcnnCall.apply(surf_in, P["surf_encoder"], surf_enc_fn)
        color_surf = _TcnnCall.apply(surf_enc, P["surf_mlp"], lambda x, p: self._mlp_ref(
            x, p, 36, self.nb, ing["surface_network"]), None, xn)
        color = torch.relu(color.view(B, N, -1))
        color_surf = torch.relu(color_surf)
        sigma = torch.relu(pos_out[:, :1]).view(B, N, 1)
        render = (ref_path.render_with_surface if self.ref_acc == "cpu" else
                  lambda *a: ref_f16.render_with_surface(*a, acc=self.ref_acc))
        cm, alpha, weights, atmo, surf = render(
            z * (self.scale / 1000), color, sigma, color_surf)  # f16 (z cast inside)
        return {"color_map_fine": cm, "color_map_atmo": atmo, "color_map_surf": surf,
                "weights_fine": weights, "z_vals_fine": z, "color_fine": color[:, :-1],
                "sigma_fine": sigma[:, :-1], "color_surf": color_surf}

    def loss(self, b: dict, res: dict, name: str = "mse_plus_hdr") -> torch.Tensor:
        """instant_ngp.py:249-263: loss_fn(take_along_dim(color_map, irgb), rad, max_i)
        (the target cast to the prediction's dtype, :262)."""
        pred = torch.take_along_dim(res["color_map_fine"], b["irgb_idx"][:, None], 1)[:, 0]
        gt = b["rad"].to(pred.dtype) if pred.dtype == torch.float16 else b["rad"].double()
        if self.semantics == "reference" and self.ref_acc != "cpu":
            return ref_f16.LossF16.apply(pred, gt, self.max_i, name, self.ref_acc)
        return ref_path.LOSSES[name](pred, gt, self.max_i)

    def optimizer(self, opt_cfg: dict) -> torch.optim.Optimizer:
        """AdamW, weight decay on the MLPs only (instant_ngp.py:107-127)."""
        groups = [{"params": [self.params[m] for m in ("pos_encoder", "surf_encoder")],
                   "weight_decay": 0.0},
                  {"params": [self.params[m] for m in ("pos_mlp", "dir_mlp", "surf_mlp")],
                   "weight_decay": opt_cfg["weight_decay"]}]
        return torch.optim.AdamW(groups, lr=opt_cfg["lr"], betas=tuple(opt_cfg["betas"]),
                                 eps=opt_cfg["eps"])


def _sh2(d: torch.Tensor) -> torch.Tensor:
    """tcnn SphericalHarmonics degree 2 on x in [0,1]^3 (remapped 2x-1), differentiable."""
    x = d * 2.0 - 1.0
    c1 = 0.48860251190291987
    return torch.stack([torch.full_like(x[:, 0], 0.28209479177387814), -c1 * x[:, 1],
                        c1 * x[:, 2], -c1 * x[:, 0]], dim=1)


def cpu_batch(b: dict) -> dict:
    return {k: v.detach().cpu() for k, v in b.items()}


def prep_kwargs(pp) -> dict:
    """Constants of a dataset's horizontal point preprocessor (harp2.py:357-370)."""
    return dict(scale=float(pp.scale),
                offset=torch.tensor(np.asarray(pp.offset, dtype=np.float64)),
                lat_min=pp.lat_min, lat_range=pp.lat_range, lon_min=pp.lon_min,
                lon_range=pp.lon_range, h0=pp.ray_origin_height, shift_lon=pp.shift_lon)
