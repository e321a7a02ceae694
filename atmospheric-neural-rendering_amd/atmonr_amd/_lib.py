"""ctypes binding of libanr_hip.so (the C ABI declared in include/anr.h).

This is the only place Python touches the native library. Every kernel call goes
through :func:`call`, which raises :class:`ANRError` with the library's message on a
non-zero status. There is no fallback: if the library is missing or a tensor is not on
a GPU, the call fails loudly.

torch is imported first so that its HIP runtime (libamdhip64.so.7) is already loaded;
libanr_hip.so then binds to that same runtime and can use torch's streams and memory.
"""

from __future__ import annotations

import ctypes
import os
from ctypes import (
    POINTER,
    Structure,
    c_double,
    c_float,
    c_int32,
    c_int64,
    c_uint32,
    c_void_p,
)

import torch  # noqa: F401  (must precede loading the HIP library)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ANR_HIP_LIB", os.path.join(_HERE, "_native", "libanr_hip.so"))

F32, F16, BF16 = 0, 1, 2
MAX_LEVELS = 32

LOSS_CODES = {
    "dark": 0,
    "hdr": 1,
    "l1": 2,
    "l1_plus_hdr": 3,
    "mse": 4,
    "mse_plus_hdr": 5,
}


class ANRError(RuntimeError):
    """A libanr_hip.so entry point returned an error status."""


class PrepParams(Structure):
    _fields_ = [
        ("mode", c_int32),
        ("shift_lon", c_int32),
        ("ngp_remap", c_int32),
        ("_pad", c_int32),
        ("scale", c_double),
        ("offset", c_double * 3),
        ("lat_min", c_double),
        ("lat_range", c_double),
        ("lon_min", c_double),
        ("lon_range", c_double),
        ("ray_origin_height", c_double),
        ("alt_compress", c_float),
        ("_pad2", c_float),
    ]


class HashGridDesc(Structure):
    _fields_ = [
        ("n_dims", c_int32),
        ("n_levels", c_int32),
        ("n_features", c_int32),
        ("base_resolution", c_int32),
        ("per_level_scale", c_float),
        ("log2_hashmap_size", c_int32),
        ("n_params", c_int64),
        ("offsets", c_uint32 * (MAX_LEVELS + 1)),
        ("resolutions", c_uint32 * MAX_LEVELS),
        ("scales", c_float * MAX_LEVELS),
    ]


class MlpDesc(Structure):
    _fields_ = [
        ("n_input", c_int32),
        ("n_input_padded", c_int32),
        ("n_output", c_int32),
        ("n_output_padded", c_int32),
        ("width", c_int32),
        ("n_hidden_layers", c_int32),
        ("activation", c_int32),
        ("output_activation", c_int32),
    ]


# name -> (restype, argtypes). Mirrors include/anr.h one to one.
class PosencDesc(Structure):
    """anr_posenc_desc (include/anr.h)."""

    _fields_ = [("n_dims", c_int32), ("interleaved", c_int32), ("L", c_int32 * 8)]


_P = c_void_p


class AdamTensor(Structure):
    """anr_adam_tensor (include/anr.h)."""
    _fields_ = [("params", c_void_p), ("grad", c_void_p), ("exp_avg", c_void_p),
                ("exp_avg_sq", c_void_p), ("params_f16", c_void_p), ("n", c_int64),
                ("lr", c_float), ("weight_decay", c_float), ("step", c_int64),
                ("grad_quant", c_float)]


ADAM_MAX_TENSORS = 16
ADAM_DEV_MAX_TENSORS = 64


class GatherCol(Structure):
    """anr_gather_col (include/anr.h)."""

    _fields_ = [("src", _P), ("dst", _P), ("row_bytes", c_int64)]


GATHER_MAX_COLS = 8

_SIGNATURES = {
    "anr_abi_version": (c_int32, []),
    "anr_last_error": (ctypes.c_char_p, []),
    "anr_gather_rows": (c_int32, [_P, c_int64, c_int32, POINTER(GatherCol), _P]),
    "anr_ingp_surface_input": (c_int32, [_P, _P, _P, c_int64, _P, _P]),
    "anr_sample_uniform_bins": (
        c_int32,
        [_P, _P, _P, _P, _P, c_int64, c_int32, _P, _P, POINTER(PrepParams), _P, _P],
    ),
    "anr_preprocess_points": (c_int32, [_P, c_int64, POINTER(PrepParams), _P, _P]),
    "anr_preprocess_points_f64": (c_int32, [_P, c_int64, POINTER(PrepParams), _P, _P]),
    "anr_preprocess_points_bwd": (c_int32, [_P, c_int64, POINTER(PrepParams), _P, _P, _P]),
    "anr_posenc_width": (c_int32, [POINTER(PosencDesc)]),
    "anr_posenc_fwd": (c_int32, [POINTER(PosencDesc), _P, c_int64, c_int64, _P, c_int64, _P]),
    "anr_posenc_bwd": (c_int32, [POINTER(PosencDesc), _P, c_int64, _P, c_int64, _P, _P]),
    "anr_relu_bwd_colsum": (c_int32, [_P, _P, c_int64, c_int32, _P, _P, c_int32, _P]),
    "anr_nerf_linear_fwd": (c_int32, [_P, c_int64, c_int32, _P, c_int64, c_int32, c_int64, _P,
                                      c_int32, _P, c_int32, _P, c_int64, _P, _P]),
    "anr_nerf_linear_dx": (c_int32, [_P, c_int64, c_int64, c_int32, _P, c_int64, c_int32,
                                     c_int32, _P, _P, c_int64, _P, c_int64, c_int32, _P]),
    "anr_nerf_linear_dw_workspace": (c_int64, [c_int64, c_int32, c_int32]),
    "anr_nerf_linear_dw": (c_int32, [_P, c_int64, c_int64, c_int32, _P, c_int64, c_int32, _P,
                                     c_int64, c_int32, _P, _P, _P, c_int64, _P]),
    "anr_sample_pdf_fwd": (
        c_int32,
        [_P, c_int64, c_int32, _P, _P, _P, _P, c_int64, c_int32, c_int32, _P, _P, _P, _P, _P,
         _P],
    ),
    "anr_sample_pdf_bwd": (
        c_int32,
        [_P, c_int64, c_int32, _P, _P, _P, _P, _P, _P, c_int64, c_int32, c_int32, _P, _P, _P,
         _P],
    ),
    "anr_hashgrid_init": (
        c_int32,
        [POINTER(HashGridDesc), c_int32, c_int32, c_int32, c_int32, c_float, c_int32],
    ),
    "anr_hashgrid_fwd": (
        c_int32,
        [POINTER(HashGridDesc), _P, c_int64, c_int64, _P, c_int32, _P, c_int32, c_int64, _P],
    ),
    "anr_hashgrid_fwd_runs": (
        c_int32,
        [POINTER(HashGridDesc), _P, c_int64, c_int64, c_int64, _P, c_int32, _P, c_int32,
         c_int64, _P],
    ),
    "anr_hashgrid_fwd_planes": (
        c_int32,
        [POINTER(HashGridDesc), _P, c_int64, c_int64, _P, c_int32, _P, c_int64, _P],
    ),
    "anr_hashgrid_bwd": (
        c_int32,
        [POINTER(HashGridDesc), _P, c_int64, c_int64, _P, c_int32, c_int64, _P, _P],
    ),
    "anr_hashgrid_bwd_tiles": (
        c_int32,
        [POINTER(HashGridDesc), _P, c_int64, c_int64, _P, c_int32, c_int64, _P, _P, _P],
    ),
    "anr_hashgrid_bwd_rows": (
        c_int32,
        [POINTER(HashGridDesc), _P, c_int64, c_int64, _P, c_int32, c_int64, _P, _P, _P],
    ),
    "anr_hashgrid_force_v1": (c_int32, [c_int32]),
    "anr_hashgrid_bwd_chunk": (c_int64, [c_int64]),
    "anr_hashgrid_bwd_count_requests": (
        c_int32,
        [POINTER(HashGridDesc), _P, c_int64, c_int64, _P, c_int32, c_int64, _P, _P, _P],
    ),
    "anr_sh_fwd": (c_int32, [c_int32, _P, c_int64, c_int64, _P, c_int32, c_int64, _P]),
    "anr_sh_bwd": (
        c_int32,
        [c_int32, _P, c_int64, c_int64, _P, c_int32, c_int64, _P, c_int64, _P],
    ),
    "anr_identity": (
        c_int32,
        [_P, c_int32, c_int64, c_int64, c_int32, _P, c_int32, c_int64, _P],
    ),
    "anr_fill_cols": (c_int32, [_P, c_int32, c_int64, c_int64, c_int32, c_float, _P]),
    "anr_mlp_n_params": (c_int64, [POINTER(MlpDesc)]),
    "anr_mlp_force_generic": (c_int32, [c_int32]),
    "anr_mlp_fwd": (
        c_int32,
        [POINTER(MlpDesc), c_int32, _P, _P, c_int32, c_int64, c_int64, _P, c_int32, c_int64, _P],
    ),
    "anr_mlp_bwd": (
        c_int32,
        [
            POINTER(MlpDesc), c_int32, _P, _P, c_int32, c_int64, c_int64, _P, c_int32,
            c_int64, _P, c_int32, c_int64, _P, _P,
        ],
    ),
    "anr_mlp_bwd_workspace_bytes": (c_int64, [POINTER(MlpDesc), c_int64]),
    "anr_mlp_bwd_ws": (
        c_int32,
        [
            POINTER(MlpDesc), c_int32, _P, _P, c_int32, c_int64, c_int64, _P, c_int32,
            c_int64, _P, c_int32, c_int64, _P, _P, c_int64, _P,
        ],
    ),
    "anr_ingp_dir_mlp_fwd": (
        c_int32,
        [POINTER(MlpDesc), c_int32, _P, _P, c_int64, _P, c_int64, c_int64, _P, c_int32,
         c_int64, _P],
    ),
    "anr_ingp_dir_mlp_bwd": (
        c_int32,
        [POINTER(MlpDesc), c_int32, _P, _P, c_int64, _P, c_int64, c_int64, _P, c_int64, _P,
         _P, c_int64, _P, _P],
    ),
    "anr_ingp_field_supported": (c_int32, [POINTER(MlpDesc), POINTER(MlpDesc)]),
    "anr_ingp_field_packed_size": (c_int64, [POINTER(MlpDesc), POINTER(MlpDesc)]),
    "anr_ingp_field_set_grad_scale": (c_int32, [c_int32]),
    "anr_ingp_field_force_fwd": (c_int32, [c_int32]),
    "anr_ingp_field_bwd_workspace_bytes": (
        c_int64, [POINTER(MlpDesc), POINTER(MlpDesc), c_int32, c_int64]),
    "anr_ingp_field_pack": (
        c_int32, [POINTER(MlpDesc), POINTER(MlpDesc), c_int32, _P, _P, _P, _P]),
    "anr_ingp_field_fwd": (
        c_int32,
        [POINTER(MlpDesc), POINTER(MlpDesc), c_int32, _P, _P, c_int64, _P, c_int64, c_int64,
         _P, _P, c_int64, _P],
    ),
    "anr_ingp_hash_field_fwd": (
        c_int32,
        [POINTER(HashGridDesc), _P, c_int64, _P, c_int32, _P, c_int64, POINTER(MlpDesc),
         POINTER(MlpDesc), c_int32, _P, _P, c_int64, _P, _P, c_int64, _P],
    ),
    "anr_ingp_field_density": (
        c_int32,
        [POINTER(MlpDesc), POINTER(MlpDesc), c_int32, _P, _P, c_int64, c_int64, _P, _P],
    ),
    "anr_ingp_field_bwd": (
        c_int32,
        [POINTER(MlpDesc), POINTER(MlpDesc), c_int32, _P, _P, c_int64, _P, c_int64, c_int64,
         _P, _P, c_int64, _P, c_int64, _P, _P, _P, c_int64, _P],
    ),
    "anr_ingp_field_fwd_rows": (
        c_int32,
        [POINTER(MlpDesc), POINTER(MlpDesc), c_int32, _P, _P, c_int64, _P, c_int64, c_int64,
         _P, _P, _P, c_int64, _P],
    ),
    "anr_ingp_field_bwd_rows": (
        c_int32,
        [POINTER(MlpDesc), POINTER(MlpDesc), c_int32, _P, _P, c_int64, _P, c_int64, c_int64,
         _P, _P, _P, c_int64, _P, c_int64, _P, _P, _P, c_int64, _P],
    ),
    "anr_occupancy_n_blocks": (c_int64, [c_int64]),
    "anr_occupancy_count": (
        c_int32, [_P, c_int64, _P, c_int32, c_int32, c_int32, c_float, _P, _P]),
    "anr_occupancy_compact": (
        c_int32, [_P, c_int64, _P, c_int32, c_int32, c_int32, c_float, _P, _P, _P, _P]),
    "anr_composite_force_generic": (c_int32, [c_int32]),
    "anr_composite_fwd": (
        c_int32,
        [_P, c_float, _P, _P, _P, c_int32, c_int64, c_int32, c_int32, c_int32,
         _P, _P, _P, _P, _P, _P],
    ),
    "anr_composite_bwd": (
        c_int32,
        [_P, c_float, _P, _P, _P, c_int32, c_int64, c_int32, c_int32, c_int32,
         _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    ),
    "anr_loss_workspace_bytes": (c_int64, [c_int64]),
    "anr_loss_fwd_bwd": (
        c_int32,
        [c_int32, _P, c_int32, c_int32, _P, _P, c_int64, c_float, c_float, _P, _P, _P, _P],
    ),
    "anr_composite_ref16_set_rays": (c_int32, [c_int32]),
    "anr_composite_ref16_fwd": (
        c_int32,
        [_P, c_float, _P, _P, _P, c_int32, c_int64, c_int32, c_int32, _P, _P, _P, _P, _P, _P,
         _P, _P],
    ),
    "anr_composite_ref16_bwd": (
        c_int32,
        [_P, c_float, _P, _P, _P, c_int32, c_int64, c_int32, c_int32, _P, _P, _P, _P, c_int32,
         _P, _P],
    ),
    "anr_loss_ref16_fwd_bwd": (
        c_int32, [c_int32, _P, c_int32, _P, _P, c_int64, c_float, _P, _P, _P, _P]),
    "anr_grad_quantize_f16": (c_int32, [_P, c_int64, c_float, _P]),
    "anr_ingp_field_bwd_ref16": (
        c_int32,
        [POINTER(MlpDesc), POINTER(MlpDesc), _P, _P, c_int64, _P, c_int64, c_int64, _P, _P,
         c_int64, _P, c_int64, _P, _P, c_float, _P],
    ),
    "anr_ingp_field_bwd_ref16_tiles": (
        c_int32,
        [POINTER(MlpDesc), POINTER(MlpDesc), _P, _P, c_int64, _P, c_int64, c_int64, _P, _P,
         c_int64, _P, c_int64, _P, _P, c_float, _P, _P],
    ),
    "anr_ingp_field_bwd_ref16_rows": (
        c_int32,
        [POINTER(MlpDesc), POINTER(MlpDesc), _P, _P, c_int64, _P, c_int64, c_int64, _P, _P,
         c_int64, _P, c_int64, _P, _P, c_float, _P, _P, c_int64, _P],
    ),
    "anr_ingp_field_bwd_ref16_rows_workspace_bytes": (c_int64, [c_int64]),
    "anr_mlp_bwd_ref16": (
        c_int32,
        [POINTER(MlpDesc), _P, _P, c_int32, c_int64, c_int64, _P, c_int32, c_int64, _P,
         c_int32, c_int64, _P, _P, c_int64, c_float, _P],
    ),
    "anr_adam_step": (
        c_int32,
        [_P, _P, _P, _P, _P, c_int64, c_float, c_float, c_float, c_float, c_float,
         c_int32, c_int64, c_int32, _P],
    ),
    "anr_adam_step_multi": (
        c_int32, [_P, c_int32, c_float, c_float, c_float, c_int32, c_int32, _P],
    ),
    "anr_adam_step_multi_dev": (
        c_int32, [_P, c_int32, c_float, c_float, c_float, c_int32, c_int32, _P, _P, _P, _P],
    ),
}

_lib = None
_timer = None  # optional KernelTimer: HIP events around every entry-point call


class KernelTimer:
    """Records a (start, end) torch.cuda.Event pair on the current stream around each
    libanr_hip call, keyed by entry-point name or tag (bench.py's per-kernel timing).
    ``only``: time just these names/tags (the other calls run without events).
    ``external``: events that a hipGraph capture records as event-record nodes (each
    replay re-records them), for timing a kernel inside a captured step."""

    def __init__(self, only: set[str] | None = None, external: bool = False):
        self.events: dict[str, list] = {}
        self.only = set(only) if only is not None else None
        self.external = external

    def __enter__(self):
        global _timer
        _timer = self
        return self

    def __exit__(self, *exc):
        global _timer
        _timer = None

    def summary(self) -> dict[str, dict]:
        """name -> {launches, total_ms, avg_ms}; synchronizes."""
        torch.cuda.synchronize()
        out = {}
        for name, evs in self.events.items():
            ts = [e[0].elapsed_time(e[1]) for e in evs]
            out[name] = {"launches": len(ts), "total_ms": sum(ts),
                         "avg_ms": sum(ts) / max(1, len(ts)),
                         # launches on a side stream (the surface branch, _surface_async):
                         # their event time runs beside the main chain and includes
                         # waiting for CU slots there, so it is not a step cost
                         "side_stream_launches": sum(1 for e in evs if e[2])}
        return out


def load() -> ctypes.CDLL:
    """Load libanr_hip.so (once) and declare every entry point's signature."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ANRError(
            f"libanr_hip.so not found at {LIB_PATH}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (or make -C csrc)"
        )
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def symbols() -> list[str]:
    return list(_SIGNATURES)


def call(name: str, *args, tag: str | None = None) -> int:
    """Call an entry point; raise ANRError on a non-zero status. ``tag`` names the call
    for the KernelTimer (defaults to the entry-point name)."""
    lib = load()
    if _timer is not None and (_timer.only is None or (tag or name) in _timer.only):
        kw = {"external": True} if _timer.external else {}
        a = torch.cuda.Event(enable_timing=True, **kw)
        b = torch.cuda.Event(enable_timing=True, **kw)
        a.record()
        rc = getattr(lib, name)(*args)
        b.record()
        cur = torch.cuda.current_stream()
        side = any(cur == st for st in _side_streams.values())
        _timer.events.setdefault(tag or name, []).append((a, b, side))
    else:
        rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.anr_last_error().decode(errors="replace")
        raise ANRError(f"{name} failed (status {rc}): {msg}")
    return rc


def dtype_code(dtype: torch.dtype) -> int:
    if dtype == torch.float32:
        return F32
    if dtype == torch.float16:
        return F16
    raise ANRError(f"unsupported dtype {dtype} (float32 / float16 only)")


def ptr(t: torch.Tensor | None) -> int | None:
    """Device pointer of a GPU tensor (None passes NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise ANRError("libanr_hip kernels need GPU tensors (got a CPU tensor)")
    return t.data_ptr()


def stream(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def gather_rows(idx: torch.Tensor, sources: list[torch.Tensor]) -> list[torch.Tensor]:
    """[src[idx] for src in sources] in one anr_gather_rows launch (contiguous sources on
    idx's device, rows of a 4-byte multiple)."""
    idx = idx.to(torch.int64).contiguous()
    B = idx.shape[0]
    outs = [torch.empty((B,) + tuple(s.shape[1:]), dtype=s.dtype, device=s.device)
            for s in sources]
    for k in range(0, len(sources), GATHER_MAX_COLS):
        part = list(zip(sources, outs))[k:k + GATHER_MAX_COLS]
        cols = (GatherCol * len(part))()
        for c, (s, o) in zip(cols, part):
            if not s.is_contiguous():
                raise ANRError("gather_rows: sources must be contiguous")
            c.src, c.dst = ptr(s), ptr(o)
            c.row_bytes = s[0].numel() * s.element_size() if s.dim() > 1 else s.element_size()
        call("anr_gather_rows", ptr(idx), B, len(part), cols, stream(idx.device))
    return outs


def grad_target(param: torch.nn.Parameter, dev) -> tuple[torch.Tensor, bool]:
    """Where a backward kernel should ACCUMULATE ``param``'s gradient: its existing f32
    ``.grad`` (direct=True: return None for it from autograd.Function.backward), else a
    fresh zero buffer for autograd to accumulate (direct=False)."""
    g = param.grad
    if g is not None and g.dtype == torch.float32 and g.is_contiguous() and g.device == dev:
        return g, True
    return torch.zeros(param.shape, device=dev, dtype=torch.float32), False


def grad_use(*params) -> None:
    """A forward that will accumulate these params' gradients directly (grad_target) is
    about to run with autograd recording: counted by an overlapping FlatGradBucket."""
    if not torch.is_grad_enabled():
        return
    for p in params:
        b = getattr(p, "_anr_bucket", None)
        if b is not None and p.requires_grad:
            b.grad_use(p)


def grad_done(*params) -> None:
    """The backward kernel that finishes these params' (direct) gradients for one use has
    been launched: an overlapping FlatGradBucket may issue the chunk's all-reduce."""
    for p in params:
        b = getattr(p, "_anr_bucket", None)
        if b is not None:
            b.grad_done(p)


_side_streams: dict = {}


def side_stream(device) -> "torch.cuda.Stream":
    """One extra HIP stream per device for work independent of the main per-sample chain
    (the per-ray surface branch of InstantNGPPipeline)."""
    key = torch.device(device).index
    st = _side_streams.get(key)
    if st is None:
        st = _side_streams[key] = torch.cuda.Stream(device=device)
    return st


class JoinAtBackwardEnd(torch.autograd.Function):
    """Identity on a tensor produced on a side stream. Its backward (which autograd runs
    on that side stream, as the forward) queues an end-of-backward callback making the
    caller's stream wait for the side stream: the branch's backward kernels write the
    parameter gradients directly (grad_target), so autograd's own leaf-stream sync does
    not cover them, and optimizer / gradient reads after ``backward()`` must see them."""

    @staticmethod
    def forward(ctx, x, main):
        ctx.main = main
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        side = torch.cuda.current_stream(g.device)
        g.record_stream(side)  # produced on the main stream, read here
        main = ctx.main
        torch.autograd.Variable._execution_engine.queue_callback(
            lambda: main.wait_stream(side))
        return g, None


def compute_copy(param: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """``param.detach().to(dtype)`` without a conversion pass per forward.

    The f16 copy a module computes with (tcnn keeps f16 weights next to the f32 master)
    is cached on the parameter. It is refreshed when torch has modified the parameter
    since (its ``_version`` moved: load_state_dict, copy_, torch optimizers); FusedAdam
    writes it in the same pass as the parameter update and marks it current.
    """
    if param.dtype == dtype:
        if getattr(param, "_anr_master_stale", False):
            raise ANRError("f32 compute from a parameter whose f32 master is stale "
                           "(ShardedAdam gather='f16' keeps only the f16 copies current: "
                           "use gather='f32' for f32 modules, or consolidate())")
        return param.detach()
    sh = getattr(param, "_anr_shadow", None)
    if sh is None or sh.dtype != dtype or sh.device != param.device or sh.shape != param.shape:
        sh = torch.empty(param.shape, dtype=dtype, device=param.device)
        param._anr_shadow = sh
        param._anr_shadow_ver = None
    if param._anr_shadow_ver != param._version:
        sh.copy_(param.detach())
        param._anr_shadow_ver = param._version
    return sh


def pack_source(param: torch.Tensor, mma_dtype: int) -> torch.Tensor:
    """The f32 values the fused field packs its MFMA weight fragments from: the f32 master,
    or -- when a ShardedAdam with gather='f16' left this rank's master slice stale -- the
    current f16 compute copy (identical after the pack's f16 rounding)."""
    if getattr(param, "_anr_master_stale", False):
        if mma_dtype != F16:
            raise ANRError("bf16 field weights need current f32 masters "
                           "(ShardedAdam gather='f32', or consolidate())")
        return compute_copy(param, torch.float16).float()
    return param.detach().float()


def hashgrid_desc(n_dims: int, n_levels: int, n_features: int, base_resolution: int,
                  per_level_scale: float, log2_hashmap_size: int) -> HashGridDesc:
    d = HashGridDesc()
    call("anr_hashgrid_init", ctypes.byref(d), n_dims, n_levels, n_features,
         base_resolution, per_level_scale, log2_hashmap_size)
    return d


def posenc_desc(L, n_dims: int = 3) -> PosencDesc:
    """encoders.py:4-28 frequency spec: int L (interleaved) or a per-coordinate list."""
    d = PosencDesc()
    if isinstance(L, int):
        d.n_dims, d.interleaved = n_dims, 1
        d.L[0] = L
    else:
        L = list(L)
        d.n_dims, d.interleaved = len(L), 0
        for i, v in enumerate(L):
            d.L[i] = int(v)
    if load().anr_posenc_width(ctypes.byref(d)) < 0:
        raise ANRError(f"unsupported positional-encoding spec {L!r}")
    return d


def mlp_desc(n_input: int, n_output: int, width: int, n_hidden_layers: int,
             output_relu: bool) -> MlpDesc:
    d = MlpDesc()
    d.n_input = n_input
    d.n_input_padded = (n_input + 15) // 16 * 16
    d.n_output = n_output
    d.n_output_padded = (n_output + 15) // 16 * 16
    d.width = width
    d.n_hidden_layers = n_hidden_layers
    d.activation = 1
    d.output_activation = 1 if output_relu else 0
    n = load().anr_mlp_n_params(ctypes.byref(d))
    if n < 0:
        raise ANRError(load().anr_last_error().decode())
    return d
