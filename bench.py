"""Train-step throughput of the AtmoNR Instant-NGP hot path on MI355X.

    python bench.py --gpus N --steps K --warmup W [--workload nerf]

Workload (BASELINE.json configs[2]): configs/instant_ngp.json with a 16-level T=2^19
hash grid and 2x64 fused MLPs, B = 8192 rays x N = 1024 samples per rank per step, on a
synthetic 90-view 512x512 HARP2-shaped scene (no L1B granule exists offline). One step =
batch gather -> fused sampler/preprocessor -> hash grid -> MLPs -> composite -> loss ->
backward -> [RCCL all-reduce of the flat gradient when N > 1] -> fused AdamW.
Data parallel over rays, one process per GPU, weak scaling (8192 rays per rank).

Numerics: the headline runs the reference's own f16 arithmetic (``--numerics reference``:
f16 composite and loss, tinycudann's x128 loss-scaled backward; the PSNR-parity path),
started from 10 build-numerics steps (``warm_start``: the reference's f16 gradients never
revive the density field that the first AdamW step kills on this scene, so a cold start
would time a dead field); the build numerics are timed in the same run (``alt_numerics``).
``d_enc_nonzero_frac`` reports how much of the step's dL/denc is nonzero (alive field).

``--workload extract`` measures scripts/extract.py's loop (32,768 columns x 81 altitudes
per batch, forward only) in points/s.

``--workload nerf`` measures BASELINE configs[1] instead (configs/nerf.json, batch 4096,
native f32 MFMA layers; see run_nerf). Rank 0 prints ONE JSON line.

``roofline`` is for the kernel that takes the most time per step, timed with HIP events on
the launch stream inside the timed region; its algorithmic bytes / FLOPs per launch
(kernel_models) are compulsory HBM traffic and dense MFMA work (the field
backward: dX + dW, the recomputed forward reported beside). ``peak`` / ``frac`` are against
the spec sheet (MI355X_MICROARCH.md: 8 TB/s, 2.5 PF/s f16); ``measured_ceiling`` gives the
fraction of the ceilings tools/ubench measures on the box in the same run. The bound is
whichever spec fraction is larger. ``roofline_targets`` lists north_star's two kernel
targets (hash encode >= 0.70 of HBM, fused MLP >= 0.50 of MFMA) for all four kernels.
``cpu_baseline`` times the oracle's CPU restatement of the configs/nerf.json train step
(rank 0, N = 1 only) on every core of the process's affinity mask.
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "atmospheric-neural-rendering_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# spec-sheet figures (MI355X_MICROARCH.md), used only with --spec-peaks; by default the
# peaks are MEASURED on the box in the untimed phase (tools/ubench: float4 copy, bare
# 16x16x32 MFMA loops on random operands, f32 atomic wave-instructions of the hash-grid
# backward's 16-B segment shape)
SPEC_PEAKS = {"hbm_copy_gbs": 8000.0, "mfma_f16_tfs": 2500.0, "mfma_bf16_tfs": 2500.0,
              "mfma_f32_tfs": 157.3, "atomic_seg16_greq_s": 20.3, "source": "spec"}


_T0 = time.time()


def say(msg: str) -> None:
    """Progress on stderr (rank 0's JSON line stays the only stdout line)."""
    print(f"[bench {time.time() - _T0:6.1f} s] {msg}", file=sys.stderr, flush=True)


def measured_peaks(dev, spec: bool) -> dict:
    if spec:
        return dict(SPEC_PEAKS)
    from tools.ubench import peaks as ub

    p = ub.measure(dev)
    p["source"] = "measured (tools/ubench/peaks.py, this box, this run)"
    return p


def pmc_entry(pmc: dict, tag: str, key_sfx: str):
    """(entry, stale) of profiles/pmc_traffic.json for a kernel tag: an entry measured on a
    different version of the kernel's source (sha1 stamped by tools/prof_summary.py) is
    stale and must not price this build's kernel."""
    ent = (pmc or {}).get(f"{tag}:{key_sfx}")
    if not ent:
        return None, False
    from tools.prof_summary import source_sha1

    if ent.get("kernel_source_sha1") != source_sha1(tag):
        return ent, True
    return ent, False


def kernel_models(pipe, M: int, pmc: dict | None = None, key_sfx: str = "",
                  requests: int | None = None, nz_rows: float | None = None,
                  dir_tiles: float | None = None) -> dict:
    """Algorithmic work per launch of each hot kernel.

    ``bytes`` = compulsory HBM traffic (every per-sample stream read or written once, the
    table / gradient array once per launch); ``flops`` = dense MFMA work at padded widths.
    ``survey_bytes`` = SURVEY §8(d)'s per-sample hash figures (forward 12 + 16x8x2x2 + 64 =
    588 B, backward 64 + 12 + 2 x 512 = 1,100 B), which count every corner access as HBM
    traffic; L2/MALL serve most of them, so that model reaches the HBM peak without
    discriminating and is reported beside the bound, not used for it. ``atomic_requests``
    (hash backward) = memory-side f32 atomic requests per launch, counted in the run
    (``requests``, count_hash_requests) or else from rocprofv3 PMC
    (profiles/pmc_traffic.json), priced against the measured request ceiling.

    Reference numerics with row bits (r06, field.py ``_ROW_BITS``): the field backward
    writes f16 dL/denc rows plus one bit per row, and the hash-grid backward reads the bits
    and only the rows with a nonzero value (``nz_rows``: their fraction, measured in the
    run). The field backward skips the dir network on 32-row tiles whose dL/dcolor is zero
    (``dir_tiles``: the fraction of tiles that still walk it, measured in the run), so its
    ``flops`` count the work it does (the pos network, plus the dir network on those
    tiles); ``flops_full`` is tinycudann's full backward beside it.
    """
    from atmonr_amd import field as _field

    ref_rows = (getattr(pipe, "numerics", None) == "reference" and _field._ROW_BITS
                and not _field._TILE_SKIP and pipe.pos_encoder.hash_grids[0].n_out == 32)
    grid = pipe.pos_encoder.hash_grids[0]
    n_table = grid.desc.n_params                # f16 table entries x features
    pos, dirm = pipe.pos_mlp.desc, pipe.dir_mlp.desc

    def mlp_flops(d):
        dims = [d.n_input_padded] + [d.width] * d.n_hidden_layers + [d.n_output_padded]
        return 2.0 * sum(a * b for a, b in zip(dims[:-1], dims[1:]))

    f_fwd = mlp_flops(pos) + mlp_flops(dirm)
    nb = dirm.n_output
    enc_b = 2 * grid.n_out                      # f16 features
    denc_b = 2 * grid.n_out if ref_rows else 4 * grid.n_out  # dL/denc row: f16 / f32
    bits_b = 1.0 / 8 if ref_rows else 0.0                     # row bits
    rows_read = nz_rows if (ref_rows and nz_rows is not None) else 1.0
    dir_frac = dir_tiles if (getattr(pipe, "numerics", None) == "reference"
                             and dir_tiles is not None) else 1.0
    f_bwd = 2 * (mlp_flops(pos) + dir_frac * mlp_flops(dirm))
    f_rec = mlp_flops(pos) + dir_frac * mlp_flops(dirm)
    out = {
        "hash_fwd": {"bytes": M * (12 + enc_b) + 2 * n_table, "flops": 0.0,
                     "survey_bytes": M * (12 + grid.n_levels * 8 * 2 * 2 + enc_b)},
        "hash_bwd": {"bytes": M * (bits_b + rows_read * (12 + denc_b)) + 8 * n_table,
                     "flops": 0.0,
                     "survey_bytes": M * (64 + 12 + 2 * grid.n_levels * 8 * 2 * 2)},
        # enc in, sigma + color out
        "field_fwd": {"bytes": M * (enc_b + 4 + 4 * nb), "flops": M * f_fwd},
        # the two in one kernel (anr_ingp_hash_field_fwd, r06): coordinates in, f16
        # features (planes, for the backward) + sigma + color out, the table once
        "hash_field_fwd": {"bytes": M * (12 + enc_b + 4 + 4 * nb) + 2 * n_table,
                           "flops": M * f_fwd,
                           "survey_bytes": M * (12 + grid.n_levels * 8 * 2 * 2 + enc_b + 4 + 4 * nb)},
        # enc in, sigma out; the pos MLP only (extract / occupancy)
        "field_density": {"bytes": M * (enc_b + 4), "flops": M * mlp_flops(pos)},
        # enc + dL/dcolor + dL/dsigma in, dL/denc (+ row bits) out; dX + dW (2x the forward)
        # is the algorithmic work, the forward the kernel recomputes is reported beside it
        "field_bwd": {"bytes": M * (enc_b + 4 * nb + 4 + denc_b + bits_b), "flops": M * f_bwd,
                      "flops_with_recompute": M * (f_bwd + f_rec)},
    }
    if dir_frac < 1.0:
        out["field_bwd"]["flops_full"] = 2 * M * f_fwd
        out["field_bwd"]["dir_tiles_frac"] = dir_frac
    if ref_rows:
        out["hash_bwd"]["rows_read_frac"] = rows_read
    ent, stale = pmc_entry(pmc, "hash_bwd", key_sfx)
    if requests is not None:
        out["hash_bwd"]["atomic_requests"] = float(requests)
        out["hash_bwd"]["atomic_requests_source"] = (
            "counted in this run: anr_hashgrid_bwd_count_requests replays the hash-grid "
            "backward of one benched step over its own inputs (coordinates, dL/denc, gradient "
            "buffer) and counts each flush instruction's distinct 64-B segments")
        if ent and ent.get("atomic_requests") and not stale:
            out["hash_bwd"]["atomic_requests_pmc"] = {
                "requests": float(ent["atomic_requests"]), "source":
                f"profiles/pmc_traffic.json [{ent.get('source')}], rocprofv3 --pmc "
                "TCC_EA0_ATOMIC_sum of this kernel source (sha1 match)"}
    elif ent and ent.get("atomic_requests") and not stale:
        out["hash_bwd"]["atomic_requests"] = float(ent["atomic_requests"])
        out["hash_bwd"]["atomic_requests_source"] = (
            f"profiles/pmc_traffic.json [{ent.get('source')}], rocprofv3 --pmc "
            "TCC_EA0_ATOMIC_sum of this kernel source (sha1 match)")
    elif ent and ent.get("atomic_requests"):
        out["hash_bwd"]["atomic_requests_stale"] = ent.get("source")
    return out


def count_hash_requests(job, n_samples: int) -> tuple[int, float, float, float] | None:
    """Memory-side atomic requests of the hash-grid backward in one benched step: one
    eager step of the job keeps the hash-grid backward's inputs (coordinates, dL/denc,
    gradient buffer), and the instrumented launch anr_hashgrid_bwd_count_requests replays
    that kernel over them, counting each flush instruction's distinct 64-B segments -- the
    zero-sum corners the kernel skips included, so the count follows the numerics (most
    f16 dL/denc underflow in reference numerics). Returns (requests, fraction of nonzero
    dL/denc in that step: is the field alive?, fraction of samples with any nonzero
    dL/denc, fraction of 32-row tiles with a nonzero dL/dcolor); None when the pipeline
    has no fused v2-eligible hash grid."""
    from atmonr_amd import _lib

    pipe = job.pipe
    grid = pipe.pos_encoder.hash_grids[0]
    if grid.desc.n_features != 2 or grid.desc.n_levels > 16 or grid.desc.n_dims != 3:
        return None
    pipe._keep_d_enc = True
    try:
        job.eager_step()
        coords, d_enc, g_hash = pipe._last_hash_bwd
    except AttributeError:
        return None
    finally:
        pipe._keep_d_enc = False
    cnt = torch.zeros(1, dtype=torch.int64, device=coords.device)
    _lib.call("anr_hashgrid_bwd_count_requests", ctypes.byref(grid.desc), coords.data_ptr(),
              3, coords.shape[0], d_enc.data_ptr(),
              _lib.F16 if d_enc.dtype == torch.float16 else _lib.F32, d_enc.stride(0),
              g_hash.data_ptr(), cnt.data_ptr(), _lib.stream(coords.device))
    torch.cuda.synchronize()
    if os.environ.get("ANR_BENCH_DEBUG"):
        ds_, dc_ = pipe._last_field_grads
        M_ = ds_.shape[0]
        up = (ds_.view(M_, -1) != 0).any(1) | (dc_.view(M_, -1) != 0).any(1)
        for T_ in (8, 32, 256, 1024):
            n_ = M_ // T_
            print(f"[count_hash_requests] upstream-nonzero {T_}-row tiles "
                  f"{up[:n_ * T_].view(n_, T_).any(1).float().mean().item():.4f} rows "
                  f"{up.float().mean().item():.4f}", file=sys.stderr, flush=True)
        dz_ = (d_enc != 0).any(1)
        for T_ in (8, 32, 256):
            n_ = M_ // T_
            print(f"[count_hash_requests] d_enc-nonzero {T_}-row tiles "
                  f"{dz_[:n_ * T_].view(n_, T_).any(1).float().mean().item():.4f}",
                  file=sys.stderr, flush=True)
        print(f"[count_hash_requests] M={coords.shape[0]} coords {tuple(coords.shape)} "
              f"{coords.stride()} d_enc {tuple(d_enc.shape)} {d_enc.stride()} nonzero "
              f"{(d_enc != 0).float().mean().item():.4f} g_hash {g_hash.numel()} "
              f"count {int(cnt.item())}", file=sys.stderr, flush=True)
    nz = (d_enc != 0).float().mean().item()
    # sample granularity (what the walker skips since r05): rows with any nonzero value
    nz_rows = (d_enc != 0).any(1).float().mean().item()
    # 32-row tiles with a nonzero dL/dcolor (the reference numerics' field backward walks
    # the dir network on those only)
    dc_ = pipe._last_field_grads[1]
    M_ = dc_.shape[0]
    dc_nz = (dc_.reshape(M_, -1) != 0).any(1)
    dc_nz = torch.nn.functional.pad(dc_nz, (0, -M_ % 32)).view(-1, 32).any(1)
    dir_tiles = dc_nz.float().mean().item()
    del pipe._last_hash_bwd, pipe._last_d_enc, pipe._last_field_grads
    return int(cnt.item()), nz, nz_rows, dir_tiles


def _roof(mdl: dict, avg_ms: float, peaks: dict, mfma_key: str) -> dict:
    """Achieved rates of one kernel and their fractions of peak. The ``*_frac`` fields are
    against the spec sheet (MI355X_MICROARCH.md: HBM3E 8 TB/s, dense f16/bf16 MFMA
    2.5 PF/s, the 'Global float atomics' 64-B request rate); ``*_frac_measured`` against
    the ceilings tools/ubench measured on this box in the same run. The bound is the
    larger spec fraction. ``flops`` is algorithmic work (for the field backward dX + dW,
    2x the forward); ``flops_with_recompute`` adds the forward the kernel recomputes."""
    sec = avg_ms * 1e-3
    gbs = mdl["bytes"] / sec / 1e9
    tfs = mdl["flops"] / sec / 1e12
    fb, ff = gbs / SPEC_PEAKS["hbm_copy_gbs"], tfs / SPEC_PEAKS[mfma_key]
    r = {"hbm_gbs": round(gbs, 1), "hbm_frac": round(fb, 4), "mfma_tfs": round(tfs, 2),
         "mfma_frac": round(ff, 4),
         "hbm_frac_measured": round(gbs / peaks["hbm_copy_gbs"], 4),
         "mfma_frac_measured": round(tfs / peaks[mfma_key], 4),
         "bound": "hbm" if fb >= ff else "mfma"}
    if mdl.get("flops_with_recompute"):
        tr = mdl["flops_with_recompute"] / sec / 1e12
        r["mfma_tfs_with_recompute"] = round(tr, 2)
        r["mfma_frac_with_recompute"] = round(tr / SPEC_PEAKS[mfma_key], 4)
        r["mfma_frac_with_recompute_measured"] = round(tr / peaks[mfma_key], 4)
    if "survey_bytes" in mdl:
        sg = mdl["survey_bytes"] / sec / 1e9
        r["survey_model_gbs"] = round(sg, 1)
        r["survey_model_frac"] = round(sg / SPEC_PEAKS["hbm_copy_gbs"], 4)
    if "atomic_requests" in mdl:
        rq = mdl["atomic_requests"] / sec / 1e9
        fa = rq / SPEC_PEAKS["atomic_seg16_greq_s"]
        r["atomic_greq_s"] = round(rq, 3)
        r["atomic_frac"] = round(fa, 4)
        r["atomic_frac_measured"] = round(rq / peaks["atomic_seg16_greq_s"], 4)
        if fa >= max(fb, ff):
            r["bound"] = "atomic"
    return r


def target_rooflines(kernels: dict, mfma_key: str, pmc: dict | None = None,
                     pmc_sfx: str = "") -> dict:
    """north_star's two kernel targets from the per-kernel table, against the spec peaks:
    the hash-encode kernels' compulsory-byte HBM fraction (target >= 0.70) and the fused
    MLP kernels' MFMA fraction (target >= 0.50); with the rocprofv3 PMC bytes per launch of
    the same kernel source (profiles/pmc_traffic.json) where they exist."""
    out = {}
    for name, key, tgt in (("hash_fwd", "hbm_frac", 0.70), ("hash_field_fwd", "hbm_frac", 0.70),
                           ("hash_bwd", "hbm_frac", 0.70), ("field_fwd", "mfma_frac", 0.50),
                           ("hash_field_fwd", "mfma_frac", 0.50),
                           ("field_bwd", "mfma_frac", 0.50)):
        k = kernels.get(name)
        if not k or key not in k:
            continue
        e = {"avg_ms": k["avg_ms"], "frac": k[key], "target": tgt,
             "achieved": k["hbm_gbs"] if key == "hbm_frac" else k["mfma_tfs"],
             "unit": "GB/s" if key == "hbm_frac" else "TFLOP/s",
             "peak": SPEC_PEAKS["hbm_copy_gbs"] if key == "hbm_frac" else SPEC_PEAKS[mfma_key]}
        for x in ("mfma_frac_with_recompute", "atomic_frac", "survey_model_frac",
                  "hbm_frac_measured", "mfma_frac_measured"):
            if x in k:
                e[x] = k[x]
        ent, stale = pmc_entry(pmc, name, pmc_sfx)
        if ent and not stale:
            e["traffic"] = ent["bytes"]
            e["traffic_gbs"] = round(ent["bytes"] / (k["avg_ms"] * 1e-3) / 1e9, 1)
            e["traffic_source"] = f"profiles/pmc_traffic.json [{ent.get('source')}]"
        out[name if name != "hash_field_fwd" else f"hash_field_fwd:{key[:4]}"] = e
    return out


def ingp_config(variant: str, n_samples: int) -> dict:
    import __graft_entry__ as ge

    cfg = ge._ingp_config(n_samples)
    ingp = cfg["instant_ngp"]
    if variant == "committed":  # configs/instant_ngp.json as committed: T=2^21, width 32
        ingp["encoding"]["log2_hashmap_size"] = 21
        for k in ("network", "rgb_network", "surface_network"):
            ingp[k]["n_neurons"] = 32
    return cfg


NERF_CFG = {  # configs/nerf.json "pipeline" (BASELINE configs[1])
    "type": "NeRF", "include_height": False, "point_preprocessor": "horizontal",
    "num_bands": 4, "ray_origin_height": 20000, "sampler": {"N_c": 64, "N_f": 128},
    "encoder": {"L_x": [14, 14, 10], "L_d": 4}, "mlp_hidden_dim": 256}


def nerf_mlp_flops(net, n_rows: int) -> float:
    """Dense forward FLOPs of one AtmoNeRF over n_rows samples (every nn.Linear)."""
    f = sum(2.0 * m.in_features * m.out_features for m in net.modules()
            if isinstance(m, torch.nn.Linear))
    return f * n_rows


def run_nerf(args, ds, dev, rank, world, t_scene):
    peaks = measured_peaks(dev, args.spec_peaks)
    """configs/nerf.json train step (nerf.py:179-240 + Adam, trainer.py:99-105): coarse
    64 stratified + fine 64+128 pdf samples per ray, two 8x256 AtmoNeRF MLPs (f32 library
    GEMMs), f32 composite, Adam. Batch 4096 rays per rank (nerf.json trainer.batch_size).
    The MLP FLOPs (forward + 2x backward) over the measured step time give the roofline
    line (f32 MFMA peak): the GEMMs are rocBLAS / hipBLASLt launches inside autograd, so
    the step time is their upper bound, not a per-kernel HIP-event average."""
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.parallel import FlatGradBucket
    from atmonr_amd.pipelines.factory import get_pipeline

    torch.manual_seed(0)
    if args.global_batch:
        if args.global_batch % world:
            sys.exit(f"--global-batch {args.global_batch} is not divisible by {world} ranks")
        batch_size = args.global_batch // world
    else:
        batch_size = args.batch if args.batch != 8192 else 4096
    pipe = get_pipeline(dict(NERF_CFG), ds)
    pipe.send_tensors_to(dev)
    opt = pipe.get_optimizer({"lr": 5e-4})
    bucket = FlatGradBucket([p for g in opt.param_groups for p in g["params"]], dev)
    if world > 1:
        bucket.broadcast_params(0)  # AtmoNeRF's nn.Linear init is unseeded per rank
    if not args.no_fused_zero:
        bucket.fuse_zero_into(opt)  # the Adam pass zeroes the bucket (no per-step fill)
    loader = BatchLoader(ds, batch_size, shuffle=True, rank=rank, world_size=world, seed=0)
    it = iter(loader)

    def step():
        nonlocal it
        try:
            batch = next(it)
        except StopIteration:
            it = iter(loader)
            batch = next(it)
        res = pipe.forward(batch)
        loss = pipe.compute_loss(batch, res)
        bucket.zero()
        loss.backward()
        bucket.all_reduce()
        opt.step()
        return loss

    for _ in range(args.warmup):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    final_loss = float(loss.item())
    ms = elapsed / args.steps * 1e3
    value = batch_size * world * args.steps / elapsed
    nc, nf = NERF_CFG["sampler"]["N_c"], NERF_CFG["sampler"]["N_f"]
    flops = 3.0 * (nerf_mlp_flops(pipe.nerf["coarse"], batch_size * nc)
                   + nerf_mlp_flops(pipe.nerf["fine"], batch_size * (nc + nf)))
    tfs = flops / (ms * 1e-3) / 1e12
    from atmonr_amd import _lib, nerf_model

    native = nerf_model._NATIVE
    roofline = {"kernel": ("nerf_linear_{fwd,dx,dw} (csrc/nerf_mlp.hip f32 MFMA GEMMs), "
                           "whole-step time" if native else
                           "nerf_mlp_gemms (library f32 GEMMs, whole-step time)"),
                "bound": "mfma", "achieved": round(tfs, 2), "peak": SPEC_PEAKS["mfma_f32_tfs"],
                "unit": "TFLOP/s", "frac": round(tfs / SPEC_PEAKS["mfma_f32_tfs"], 4),
                "ceiling": "f32 MFMA spec peak, MI355X_MICROARCH.md",
                "measured_ceiling": {"peak": peaks["mfma_f32_tfs"],
                                     "frac": round(tfs / peaks["mfma_f32_tfs"], 4)},
                "traffic": None,
                "algorithmic_flops": flops, "units_per_launch": batch_size,
                "flops_per_unit": flops / batch_size}
    kernels = None
    if native and not args.no_kernel_timer:
        # untimed profiling pass: HIP events around every dense-layer launch (same stream)
        tags = {"nerf_linear_fwd", "nerf_linear_dx", "nerf_linear_dw"}
        prof_steps = 3
        with _lib.KernelTimer(only=tags) as kt:
            for _ in range(prof_steps):
                step()
        summ = kt.summary()
        kernels = {k: {"ms_per_step": round(v["total_ms"] / prof_steps, 3),
                       "launches_per_step": v["launches"] // prof_steps}
                   for k, v in sorted(summ.items())}
        gemm_ms = sum(v["total_ms"] for v in summ.values()) / prof_steps
        if gemm_ms > 0:
            gtfs = flops / (gemm_ms * 1e-3) / 1e12
            roofline["gemm_kernels"] = {
                "ms_per_step": round(gemm_ms, 3), "achieved": round(gtfs, 2),
                "frac": round(gtfs / SPEC_PEAKS["mfma_f32_tfs"], 4),
                "frac_measured": round(gtfs / peaks["mfma_f32_tfs"], 4),
                "source": "HIP events around each nerf_linear_* launch, untimed pass of "
                          f"{prof_steps} steps; flops = the step's algorithmic MLP flops"}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import cpu_baseline

        cpu = cpu_baseline.run(budget_s=args.cpu_budget)
    if rank == 0:
        print(json.dumps({
            "metric": "train-step rays/sec", "value": round(value, 1), "unit": "rays/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "strong" if args.global_batch else "weak",
            "vs_baseline": None, "dtype": "f32",
            "data": f"synthetic ({args.views}-view {args.img_size}x{args.img_size} "
                    f"HARP2-shaped scene, {len(ds)} rays; random-init weights)",
            "config": {"workload": "nerf BASELINE configs[1]: configs/nerf.json (freq. "
                                   "positional enc + 8x256 MLP, 64 coarse + 192 fine "
                                   "samples/ray), full train step (fwd+loss+bwd+Adam)",
                       "global_batch": batch_size * world, "parallelism": f"dp{world}"},
            "roofline": roofline, "cpu_baseline": cpu, "peaks": peaks,
            "kernels": kernels, "mlp": "native" if native else "library",
            "final_loss": round(final_loss, 6),
            "scene_build_s": round(t_scene, 2)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_extract(args, ds, dev, rank, world, t_scene):
    """Extract throughput (scripts/extract.py:180-211 ->
    InstantNGPPipeline.extract, instant_ngp.py:208-247): the reference loop over an
    L1C-style grid of the scene's 512x512 columns x 81 altitudes (alt_step 250 m, 0 to
    20 km: harp2_extract.py's grid), batches of 32,768 columns x 81 = 2,654,208 points, unshuffled.
    One step = one batch: (xyz - offset) / scale in f64, the f64 preprocessor kernel, the
    hash-grid forward and the field's density, sigma[idx] = . / scale. Forward-only,
    random-init weights. Ranks take disjoint batches (no collective); `value` is points/s
    over all ranks."""
    from atmonr_amd import _lib
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.extract import GridExtractDataset
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline

    peaks = measured_peaks(dev, args.spec_peaks)
    cfg = ingp_config(args.variant, args.samples)
    pipe = InstantNGPPipeline(cfg, ds, dtype=torch.float16, fused=True, seed=1337)
    pipe.send_tensors_to(dev)
    pipe.eval()
    grid = GridExtractDataset(ds, alt_step=250.0)
    A = int(grid.sample_alt.shape[0])
    cols = args.extract_batch
    P = cols * A
    loader = BatchLoader(grid, batch_size=P, shuffle=False, rank=rank, world_size=world)
    sigma = torch.zeros((len(grid), 1), device=dev)
    offset = torch.as_tensor(ds.offset, dtype=torch.float64, device=dev)
    batches = [b for b in loader if b["idx"].shape[0] == P]  # full batches only
    k = [0]

    @torch.no_grad()
    def step():
        b = batches[k[0] % len(batches)]
        k[0] += 1
        pts = (b["xyz"] - offset) / ds.scale
        sigma[b["idx"]] = pipe.extract(pts, run_length=A).to(dtype=sigma.dtype) / ds.scale

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    prof = _lib.KernelTimer()
    with prof:
        for _ in range(args.profile_steps):
            step()
    kernels = {}
    models = kernel_models(pipe, P)
    models["field_fwd"] = dict(models["field_fwd"])
    for name, st in sorted(prof.summary().items(), key=lambda kv: -kv[1]["total_ms"]):
        e = {"avg_ms": round(st["avg_ms"], 4),
             "ms_per_step": round(st["total_ms"] / args.profile_steps, 4)}
        if name in models:
            e.update(_roof(models[name], st["avg_ms"], peaks, "mfma_f16_tfs"))
        kernels[name] = e
    dominant = next((n for n in kernels if "bound" in kernels[n]), None)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timer = _lib.KernelTimer(only={dominant}) if dominant else None
    t0 = time.perf_counter()
    with (timer or _NullCtx()):
        for _ in range(args.steps):
            step()
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    ms = elapsed / args.steps * 1e3
    value = P * world * args.steps / elapsed
    roofline = None
    if timer:
        st = timer.summary().get(dominant)
        mdl = models[dominant]
        r = _roof(mdl, st["avg_ms"], peaks, "mfma_f16_tfs")
        if r["bound"] == "hbm":
            ach, peak, frac, unit = r["hbm_gbs"], SPEC_PEAKS["hbm_copy_gbs"], r["hbm_frac"], "GB/s"
            mc = {"peak": peaks["hbm_copy_gbs"], "frac": r["hbm_frac_measured"]}
        else:
            ach, peak, frac, unit = (r["mfma_tfs"], SPEC_PEAKS["mfma_f16_tfs"], r["mfma_frac"],
                                     "TFLOP/s")
            mc = {"peak": peaks["mfma_f16_tfs"], "frac": r["mfma_frac_measured"]}
        roofline = {"kernel": dominant, "bound": r["bound"], "achieved": ach, "peak": peak,
                    "unit": unit, "frac": frac, "measured_ceiling": mc,
                    "traffic": None, "avg_ms": round(st["avg_ms"], 4),
                    "launches": st["launches"], "units_per_launch": P,
                    "algorithmic_bytes": mdl["bytes"], "algorithmic_flops": mdl["flops"],
                    "bytes_per_unit": mdl["bytes"] / P,
                    "ceiling": "HBM3E 8 TB/s, MI355X_MICROARCH.md" if r["bound"] == "hbm"
                    else "dense f16 MFMA spec peak, MI355X_MICROARCH.md"}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import cpu_baseline

        cpu = cpu_baseline.run_extract(budget_s=min(args.cpu_budget, 20.0))
    if rank == 0:
        print(json.dumps({
            "metric": "extract points/sec", "value": round(value, 1), "unit": "points/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms, 4), "host_ms_per_step": round(t_host / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f16",
            "data": f"synthetic ({args.views}-view {args.img_size}x{args.img_size} HARP2-shaped "
                    f"scene; extract grid {grid.shp[0]}x{grid.shp[1]} columns x {A} altitudes "
                    f"= {len(grid)} points; random-init weights)",
            "config": {"workload": f"extract (scripts/extract.py:180-211): batches of {cols} "
                                   f"columns x {A} altitudes = {P} points, f64 preprocessor + "
                                   f"hash grid + density MLP, forward only",
                       "points_per_batch": P, "parallelism": f"dp{world}"},
            "roofline": roofline, "cpu_baseline": cpu, "kernels": kernels,
            "kernels_source": f"untimed profiling pass of {args.profile_steps} batches",
            "peaks": peaks, "sigma_checksum": float(sigma.double().sum().item()),
            "scene_build_s": round(t_scene, 2)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def warm_start(job, args, cfg, ds, dev, rank, world, rank_batch, shard) -> dict | None:
    """Reference numerics start from a build-numerics warm-up. On the bench scene the first
    AdamW step (lr 1e-2) kills the density ReLU at ~all samples in both numerics; the build
    numerics' f32 gradients revive it by step ~8, the reference's f16 ones never do (40
    steps: sigma > 0 at 0 % of samples, dL/denc all zero; profiles/r04_liveness_*.log), so a
    reference-numerics step timed from a cold start would run a dead field whose backward
    does no work. Its parameters are therefore taken from ``max(10, warmup)`` build-numerics
    steps; from there the reference numerics keep the field alive (sigma > 0 at ~99 %,
    12-33 % of dL/denc nonzero, the rest the reference's f16 underflow) and train on."""
    if job.numerics != "reference":
        return None
    tmp = IngpJob(args, cfg, ds, dev, rank, world, rank_batch, "build", False, shard, None)
    n = max(10, args.warmup)
    for _ in range(n):
        tmp.step()
    with torch.no_grad():
        job.pipe.load_state_dict(tmp.pipe.state_dict())
    tmp.release()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return {"numerics": "build", "steps": n}


class IngpJob:
    """One Instant-NGP training job of the bench: pipeline, optimizer, flat gradient bucket
    and rank-sharded loader, stepped eagerly or through a captured hipGraph of the whole
    step (atmonr_amd.graph: one graph launch per step; the optimizer is in the graph on
    one rank, and runs eagerly after the replay with its collectives on more)."""

    def __init__(self, args, cfg, ds, dev, rank, world, rank_batch, numerics, graph, shard,
                 occ):
        from atmonr_amd.parallel import FlatGradBucket, ShardedAdam
        from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline

        self.args, self.ds, self.dev, self.rank, self.world = args, ds, dev, rank, world
        dtype = torch.float32 if args.dtype == "f32" else torch.float16
        mlp_dtype = torch.bfloat16 if args.dtype == "bf16" else dtype
        self.numerics = numerics
        pipe = InstantNGPPipeline(cfg, ds, dtype=dtype, fused=True, seed=1337, occupancy=occ,
                                  mlp_dtype=mlp_dtype, numerics=numerics)
        pipe.send_tensors_to(dev)
        opt_cfg = {"lr": 1e-2, "betas": [0.9, 0.99], "eps": 1e-15, "weight_decay": 1e-2}
        opt = pipe.get_optimizer(opt_cfg)
        self.sharded = shard != "off"
        self.grad_exchange = None
        self.shard = shard
        # the AdamW update joins the graph only without collectives after backward
        self.opt_in_graph = graph and not self.sharded and world == 1
        opt.capturable = self.opt_in_graph
        # one flat f32 gradient bucket; every param's .grad is a view into it, so backward
        # accumulates in place and DP needs exactly one all-reduce per step
        bucket = FlatGradBucket([p for g in opt.param_groups for p in g["params"]], dev,
                                pad_to=world)
        if world > 1:
            bucket.broadcast_params(0)  # replicas start from rank 0's weights
        if self.sharded:
            # reference numerics: every rank's gradients are tinycudann's f16 values, so the
            # reduce-scatter can move f16 (all-to-all + f32 sums on the owner: half the bytes)
            exch = args.grad_exchange
            if exch == "auto":
                exch = "f16" if numerics == "reference" and world > 1 else "f32"
            self.grad_exchange = exch
            opt = ShardedAdam(bucket, opt.param_groups, betas=opt_cfg["betas"],
                              eps=opt_cfg["eps"], gather=shard, exchange=exch)
        elif not args.no_fused_zero:
            bucket.fuse_zero_into(opt)  # the AdamW pass zeroes the bucket (no per-step fill)
        if not self.sharded and world == 1:
            # reference numerics: tcnn's f16 gradient rounding inside the AdamW pass (no-op
            # in build numerics; with more ranks the all-reduce reads the rounded values)
            pipe.defer_grad_quantize(opt)
        if not args.no_overlap and not self.sharded and not (graph and world > 1):
            # each chunk's all-reduce starts once its gradients are final: the surface and
            # MLP gradients reduce while the hash-grid backward runs
            bucket.enable_overlap()
        self.pipe, self.opt, self.bucket = pipe, opt, bucket
        self.set_batch(rank_batch, graph)

    def _after(self):
        if self.sharded:
            return self.opt.step  # reduce-scatter, sharded AdamW, all-gather
        bucket, opt = self.bucket, self.opt

        def after():
            bucket.all_reduce()
            opt.step()
        return after

    def _graph(self, bs):
        from atmonr_amd.graph import GraphedTrainStep

        return GraphedTrainStep(self.pipe, self.ds, bs, self.opt, self.bucket,
                                optimizer_in_graph=self.opt_in_graph,
                                after=None if self.opt_in_graph else self._after())

    def set_batch(self, bs: int, graph: bool) -> None:
        from atmonr_amd.batch_loader import BatchLoader

        if graph and self.world > 1 and self.bucket.overlap:
            graph = False  # the overlapped all-reduce issues collectives inside backward
        self.batch_size = bs
        self.loader = BatchLoader(self.ds, bs, shuffle=True, rank=self.rank,
                                  world_size=self.world, seed=0)
        self._it = self.loader.index_batches()
        self.graphed = graph
        self.gstep = self._graph(bs) if graph else None
        self._eager_left = 1 if graph else 0  # one eager step at the shape before capture

    def next_idx(self):
        try:
            return next(self._it)
        except StopIteration:
            self._it = self.loader.index_batches()
            return next(self._it)

    def eager_step(self, idx=None):
        idx = self.next_idx() if idx is None else idx
        batch = self.ds.__getbatch__(idx)
        res = self.pipe.forward(batch)
        loss = self.pipe.compute_loss(batch, res)
        self.bucket.zero()
        loss.backward()
        if not self.sharded:
            self.bucket.all_reduce()
        self.opt.step()  # ShardedAdam: reduce-scatter, sharded AdamW, all-gather
        return loss

    def step(self):
        if self.gstep is None or self._eager_left > 0:
            self._eager_left = max(0, self._eager_left - 1)
            return self.eager_step()
        return self.gstep(self.next_idx())

    def profile(self, n, models, peaks, mfma_key) -> dict:
        """Per-kernel table from ``n`` eager steps with events around every libanr call
        (a graphed job's replays run the same kernels with the same arguments)."""
        from atmonr_amd import _lib

        prof = _lib.KernelTimer()
        with prof:
            for _ in range(n):
                self.eager_step()
        out = {}
        for name, st in sorted(prof.summary().items(), key=lambda kv: -kv[1]["total_ms"]):
            entry = {"avg_ms": round(st["avg_ms"], 4), "ms_per_step": round(st["total_ms"] / n, 4)}
            if st.get("side_stream_launches"):
                # the per-ray surface branch runs on a side stream beside the per-sample
                # chain: its event span includes waiting for CU slots next to the field /
                # hash-grid backward, so it overlaps the step instead of adding to it
                entry["overlapped"] = True
                entry["side_stream_launches"] = st["side_stream_launches"]
            mdl = models.get(name)
            if mdl:
                entry.update(_roof(mdl, st["avg_ms"], peaks, mfma_key))
            out[name] = entry
        return out

    def time_dominant(self, name: str, n: int):
        """Duration of kernel ``name`` for a graphed job: HIP events around its launches in
        ``n`` eager steps of the same shape right after the timed replays (the graph runs
        the same kernels with the same arguments; ROCm's torch refuses the external events
        that would time a node inside a replay)."""
        from atmonr_amd import _lib

        timer = _lib.KernelTimer(only={name})
        with timer:
            for _ in range(n):
                self.eager_step()
        torch.cuda.synchronize()
        st = timer.summary().get(name)
        if st:
            st = dict(st, source=f"HIP events around the kernel in {n} eager steps of the "
                                 "graphed shape after the timed graph replays")
        return st

    def release(self) -> None:
        self.gstep = None
        self.pipe = self.opt = self.bucket = None


def _launch_ranks(n: int) -> int:
    """torch.distributed.run with N local ranks on this script (same arguments), as a
    child process: rendezvous on 127.0.0.1, one process per GPU."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10,
                    help="untimed steps first (the bench network's first AdamW steps kill its "
                         "densities; it is alive again from step ~7: tools/liveness.py)")
    ap.add_argument("--batch", type=int, default=8192,
                    help="rays per rank per step (weak scaling, the default)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="strong scaling: fixed rays per step over all ranks (SURVEY §8(e): "
                         "8192), each rank takes global/N")
    ap.add_argument("--no-strong", action="store_true",
                    help="N > 1 weak-scaling run: skip the extra strong-scaling segment at "
                         "a global batch of --batch rays")
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--views", type=int, default=90)
    ap.add_argument("--img-size", type=int, default=512)
    ap.add_argument("--workload", choices=["ingp", "nerf", "extract"], default="ingp",
                    help="ingp: BASELINE configs[2] (the headline line); nerf: configs[1]; "
                         "extract: the forward-only extract loop (SURVEY §8 f1), points/s")
    ap.add_argument("--extract-batch", type=int, default=32768,
                    help="extract: grid columns per batch (scripts/extract.py's batch_size; "
                         "x 81 altitudes points)")
    ap.add_argument("--variant", choices=["baseline", "committed"], default="baseline")
    ap.add_argument("--dtype", choices=["f16", "bf16", "f32"], default="f16",
                    help="f16: tcnn precision (the reference's); bf16: BASELINE configs[4], "
                         "f16 hash features + bf16 MFMA field MLP; f32: exact-f32 kernels")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--spec-peaks", action="store_true",
                    help="price the rooflines against spec-sheet peaks instead of measuring")
    ap.add_argument("--cpu-budget", type=float, default=150.0)
    ap.add_argument("--no-kernel-timer", action="store_true")
    ap.add_argument("--occupancy", action="store_true",
                    help="BASELINE configs[4]: occupancy-grid culling (beyond the reference); "
                         "use a long --warmup so the grid has learned the scene")
    ap.add_argument("--occ-warmup", type=int, default=100,
                    help="steps before the occupancy grid starts culling")
    ap.add_argument("--no-fused-zero", action="store_true",
                    help="zero the gradient bucket with a fill instead of in the AdamW pass")
    ap.add_argument("--no-overlap", action="store_true",
                    help="one all-reduce of the whole gradient bucket after backward")
    ap.add_argument("--shard-optimizer", choices=["auto", "off", "f16", "f32"],
                    default="auto",
                    help="ZeRO-1 (atmonr_amd.parallel.ShardedAdam): reduce-scatter of the "
                         "gradient, AdamW on 1/N of the parameters, all-gather of the f16 "
                         "compute copy (f16) or of the f32 parameters (f32), instead of "
                         "all-reduce + replicated AdamW; auto = f16 on more than one rank")
    ap.add_argument("--grad-exchange", choices=["auto", "f32", "f16"], default="auto",
                    help="sharded optimizer: gradient slices exchanged as f32 (reduce-scatter) "
                         "or f16 (all-to-all, f32 sums; exact for the reference numerics' f16 "
                         "gradients); auto = f16 under reference numerics on more than one rank")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="replay the whole train step as one captured hipGraph "
                         "(atmonr_amd.graph); auto = on for per-rank batches <= 2048 rays, "
                         "where issuing ~50 launches from Python is slower than running them")
    ap.add_argument("--numerics", choices=["build", "reference"], default="reference",
                    help="headline numerics of InstantNGPPipeline: reference (default: the "
                         "reference's f16 composite, loss and loss-scaled tcnn backward, the "
                         "path within 0.1 dB PSNR of the reference, BASELINE's metric) or "
                         "build (f32 composite / loss / inter-kernel gradients, a deliberate "
                         "deviation that trains differently, DESIGN.md §3.1); the other one "
                         "is timed after it unless --no-alt-numerics")
    ap.add_argument("--no-alt-numerics", action="store_true")
    ap.add_argument("--settle", type=int, default=150,
                    help="reference numerics: steps after the build-numerics warm start "
                         "before the --warmup / timed steps (the first --steps of them are "
                         "timed as transient_window); 0 = time right after the warm start")
    ap.add_argument("--cold-start", action="store_true",
                    help="reference numerics from the seed parameters: no build-numerics warm "
                         "start, no settle (ADVICE r04: the number beside the warm-started "
                         "headline; on the bench scene the field collapses, "
                         "profiles/r05_*liveness*)")
    ap.add_argument("--profile-steps", type=int, default=3,
                    help="untimed steps with every kernel timed (per-kernel breakdown)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            # `bench.py --gpus N` on its own: start N fresh rank processes (this process
            # has not touched HIP and never will) and exit with their status
            sys.exit(_launch_ranks(args.gpus))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}: "
                 "launch one rank per GPU with --nproc-per-node equal to --gpus")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the multi-rank path on a one-GPU box: ANR_DIST_BACKEND=gloo puts every
    # rank on the visible GPU(s) round-robin (the driver's N-GPU runs use RCCL, one GPU each)
    backend = os.environ.get("ANR_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from atmonr_amd import _lib
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline

    t0 = time.time()
    ds = SyntheticHARP2Dataset(n_views=args.views, img_size=args.img_size, device=dev, seed=0)
    torch.cuda.synchronize()
    t_scene = time.time() - t0
    say(f"scene built ({t_scene:.1f} s)")
    if args.workload == "nerf":
        return run_nerf(args, ds, dev, rank, world, t_scene)
    if args.workload == "extract":
        return run_extract(args, ds, dev, rank, world, t_scene)
    if args.global_batch:
        if args.global_batch % world:
            sys.exit(f"--global-batch {args.global_batch} is not divisible by {world} ranks")
        rank_batch, scaling = args.global_batch // world, "strong"
    else:
        rank_batch, scaling = args.batch, "weak"
    cfg = ingp_config(args.variant, args.samples)
    occ = None
    if args.occupancy:
        from atmonr_amd.occupancy import OccupancyGrid

        occ = OccupancyGrid((128, 128, 32), alt_compress=float(cfg["alt_compress_factor"]),
                            warmup=args.occ_warmup, update_every=16, device=dev)
    shard = args.shard_optimizer
    if shard == "auto":  # ZeRO-1 with the f16 all-gather on more than one rank
        shard = "f16" if world > 1 else "off"
    use_graph = {"on": True, "off": False}.get(args.graph, rank_batch <= 2048)
    if occ is not None:
        use_graph = False  # the occupancy grid's refresh and compaction sizes are dynamic
    # reference numerics are the reference's f16 step: f16 modules, no occupancy culling
    # (BASELINE configs[4]'s bf16 / occupancy variants and f32 run the build numerics)
    numerics = args.numerics if (args.dtype == "f16" and occ is None) else "build"
    job = IngpJob(args, cfg, ds, dev, rank, world, rank_batch, numerics, use_graph,
                  shard, occ)
    pipe, bucket, opt = job.pipe, job.bucket, job.opt
    sharded = job.sharded
    step = job.step
    say(f"job built ({numerics} numerics); warm start")
    warm = (None if args.cold_start else
            warm_start(job, args, cfg, ds, dev, rank, world, rank_batch, shard))
    say("warm start done; settling")
    transient = None
    if warm is not None and args.settle > 0:
        # The reference numerics' state right after the build-numerics warm start is a
        # transient: over the next ~100 steps the loss falls 0.07 -> 0.01 and the nonzero
        # share of dL/denc rows from ~0.65 to ~0.25 (profiles/r05_liveness_ref400.log),
        # then stays there for the rest of training. The timed steps run after
        # ``--settle`` reference-numerics steps; the first K of them are timed here too and
        # reported as ``transient_window`` (one rank).
        done = 0
        if world == 1:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            done = args.steps
            transient = {"steps_after_warm_start": [0, args.steps],
                         "value": round(rank_batch * args.steps / el, 1),
                         "ms_per_step": round(el / args.steps * 1e3, 3)}
        for _ in range(max(0, args.settle - done)):
            step()
        warm["settle_steps"] = args.settle
        warm["settle_numerics"] = numerics

    for _ in range(args.warmup):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    # Untimed profiling pass: HIP events around every libanr call give the per-kernel
    # breakdown and pick the dominant kernel; the timed region below then brackets only
    # that kernel's launches (events around every call would cost ~0.2 ms per step). A
    # graphed job profiles its eager form (the same kernels and arguments).
    M = rank_batch * args.samples
    say("warm-up done; measuring peaks")
    peaks = measured_peaks(dev, args.spec_peaks)
    mfma_key = {"f32": "mfma_f32_tfs", "bf16": "mfma_bf16_tfs"}.get(args.dtype, "mfma_f16_tfs")
    pmc = {}
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
        except (OSError, ValueError):
            pmc = {}
    pmc_sfx = (f"{args.variant}{'' if args.dtype == 'f16' else '-' + args.dtype}:"
               f"{rank_batch}x{args.samples}")
    req = count_hash_requests(job, args.samples) if occ is None else None
    nreq = None if req is None else req[0]
    models = kernel_models(pipe, M, pmc, pmc_sfx, requests=nreq,
                           nz_rows=None if req is None else req[2],
                           dir_tiles=None if req is None else req[3])
    kernels, dominant = {}, None
    if not args.no_kernel_timer:
        kernels = job.profile(args.profile_steps, models, peaks, mfma_key)
        dominant = next((n for n in kernels if "bound" in kernels[n]
                         and not kernels[n].get("overlapped")), None)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    # graphed steps cannot carry events per launch: their dominant kernel is timed by
    # job.time_dominant after the timed region (events recorded inside the graph)
    timer = _lib.KernelTimer(only={dominant}) if dominant and not job.graphed else None
    # two windows of the timed steps (GPU events at the start, after K // 2 steps and at
    # the end, on the compute stream): the reference numerics' field keeps learning
    # through the timed steps, so the step cost can drift between the halves
    win = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    half = args.steps // 2
    t_start = time.perf_counter()
    win[0].record()
    with (timer if timer else _NullCtx()):
        for k in range(args.steps):
            if k == half:
                win[1].record()
            loss = step()
    win[2].record()
    t_host = time.perf_counter() - t_start  # host time to issue the K steps (no waits)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    final_loss = float(loss.item())

    ms_per_step = elapsed / args.steps * 1e3
    windows = None
    if 0 < half < args.steps:
        windows = {"steps": [half, args.steps - half],
                   "ms_per_step": [round(win[0].elapsed_time(win[1]) / half, 4),
                                   round(win[1].elapsed_time(win[2]) / (args.steps - half), 4)],
                   "source": "HIP events on the compute stream around each half of the "
                             "timed steps (rank 0)"}
    rays_total = rank_batch * world * args.steps
    value = rays_total / elapsed
    dom_stats = None
    if timer:
        dom_stats = timer.summary().get(dominant)
    elif dominant and job.graphed:
        dom_stats = job.time_dominant(dominant, args.steps)
    if req is not None and "hash_bwd" in models and world == 1:
        # the field keeps learning through the timed steps (reference numerics: the
        # nonzero share of dL/denc, and with it the requests, drift): count once more
        # after them and price the roofline at the mean of the two counts
        req2 = count_hash_requests(job, args.samples)
        if req2 is not None:
            hb = models["hash_bwd"]
            hb["atomic_requests"] = 0.5 * (req[0] + req2[0])
            hb["atomic_requests_before_after"] = [req[0], req2[0]]
            hb["d_enc_nonzero_before_after"] = [round(req[1], 4), round(req2[1], 4)]
            hb["d_enc_nonzero_rows_before_after"] = [round(req[2], 4), round(req2[2], 4)]
            # the row-bit walker's bytes and the field backward's dir-network work follow
            # the same drift: price them at the mean of the two states as well
            m2 = kernel_models(pipe, M, nz_rows=0.5 * (req[2] + req2[2]),
                               dir_tiles=0.5 * (req[3] + req2[3]))
            for k in ("hash_bwd", "field_bwd"):
                for f in ("bytes", "flops", "flops_with_recompute", "rows_read_frac",
                          "dir_tiles_frac"):
                    if f in m2[k]:
                        models[k][f] = m2[k][f]
            models["field_bwd"]["d_color_nonzero_tiles_before_after"] = [
                round(req[3], 4), round(req2[3], 4)]

    strong = None
    if world > 1 and scaling == "weak" and not args.no_strong and args.batch % world == 0:
        # the same job at a fixed global batch of --batch rays (SURVEY §8(e)'s strong-
        # scaling target), timed the same way after a short warm-up at the new shape
        sb = args.batch // world
        job.set_batch(sb, {"on": True, "off": False}.get(args.graph, sb <= 2048)
                      and occ is None)
        for _ in range(max(2, args.warmup)):
            job.step()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            job.step()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t = torch.tensor([time.perf_counter() - t1], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
        strong = {"global_batch": args.batch, "per_rank_batch": sb, "graph": job.graphed,
                  "value": round(args.batch * args.steps / el, 1),
                  "ms_per_step": round(el / args.steps * 1e3, 3), "steps": args.steps}

    # the other numerics of the same workload, timed the same way (one rank): the
    # reference's f16 composite / loss / loss-scaled backward (numerics="reference", the
    # PSNR-parity path) beside the build numerics, or the other way round
    alt = None
    if world == 1 and not args.no_alt_numerics and occ is None and args.dtype == "f16":
        other = "reference" if numerics == "build" else "build"
        del step
        job.release()
        torch.cuda.empty_cache()
        say(f"timed region done; the {other} numerics")
        ajob = IngpJob(args, cfg, ds, dev, rank, world, rank_batch, other, use_graph, shard,
                       None)
        awarm = warm_start(ajob, args, cfg, ds, dev, rank, world, rank_batch, shard)
        for _ in range(args.warmup):
            ajob.step()
        areq = count_hash_requests(ajob, args.samples)
        akern = ajob.profile(args.profile_steps, kernel_models(ajob.pipe, M), peaks, mfma_key)
        torch.cuda.synchronize()
        ta = time.perf_counter()
        for _ in range(args.steps):
            aloss = ajob.step()
        torch.cuda.synchronize()
        ea = time.perf_counter() - ta
        alt = {"numerics": other, "value": round(rank_batch * args.steps / ea, 1),
               "ms_per_step": round(ea / args.steps * 1e3, 3), "graph": ajob.graphed,
               "warm_start": awarm,
               "d_enc_nonzero_frac": None if areq is None else round(areq[1], 4),
               "final_loss": round(float(aloss.item()), 6),
               "kernels": {k: {x: v[x] for x in ("avg_ms", "ms_per_step") if x in v}
                           for k, v in akern.items()}}
        ajob.release()

    roofline = None
    if dom_stats and "error" in dom_stats:
        roofline = {"kernel": dominant, "error": dom_stats["error"]}
    elif dom_stats:
        st = dom_stats
        if st:  # the dominant kernel, timed live over the timed region
            mdl = models[dominant]
            k = _roof(mdl, st["avg_ms"], peaks, mfma_key)
            bound = k["bound"]
            if bound == "atomic":
                # memory-side f32 atomic requests per second (each a 64-B request carrying
                # the kernel's 16-B segment), against the guide's request rate (1.3 TB/s of
                # 64-B requests = 20.3 G req/s) and the ceiling measured on the same shape
                ach, peak, frac, mpeak, mfrac = (
                    k["atomic_greq_s"], SPEC_PEAKS["atomic_seg16_greq_s"], k["atomic_frac"],
                    peaks["atomic_seg16_greq_s"], k["atomic_frac_measured"])
                unit = "Greq/s"
            elif bound == "hbm":
                ach, peak, frac, unit = k["hbm_gbs"], SPEC_PEAKS["hbm_copy_gbs"], k["hbm_frac"], "GB/s"
                mpeak, mfrac = peaks["hbm_copy_gbs"], k["hbm_frac_measured"]
            else:
                ach, peak, frac, unit = (k["mfma_tfs"], SPEC_PEAKS[mfma_key], k["mfma_frac"],
                                         "TFLOP/s")
                mpeak, mfrac = peaks[mfma_key], k["mfma_frac_measured"]
            roofline = {"kernel": dominant, "bound": bound,
                        "ceiling": ("memory-side f32 atomic requests, MI355X_MICROARCH.md "
                                    "'Global float atomics' (1.3 TB/s of 64-B requests)"
                                    if bound == "atomic" else
                                    "HBM3E 8 TB/s, MI355X_MICROARCH.md" if bound == "hbm" else
                                    "dense MFMA spec peak, MI355X_MICROARCH.md"),
                        "achieved": ach, "peak": peak, "unit": unit, "frac": frac,
                        "measured_ceiling": {
                            "peak": mpeak, "frac": mfrac,
                            "source": ("tools/ubench on this box in this run: " + (
                                "scattered no-return f32 atomics at 16-B segments"
                                if bound == "atomic" else "float4 copy" if bound == "hbm"
                                else "bare MFMA loop on random operands"))},
                        "traffic": None, "avg_ms": round(st["avg_ms"], 4),
                        "launches": st["launches"], "units_per_launch": M,
                        "algorithmic_bytes": mdl["bytes"], "algorithmic_flops": mdl["flops"],
                        "bytes_per_unit": mdl["bytes"] / M,
                        "fractions": {x: k[x] for x in (
                            "hbm_frac", "mfma_frac", "atomic_frac", "survey_model_frac",
                            "mfma_frac_with_recompute") if x in k}}
            if mdl.get("flops_with_recompute"):
                roofline["algorithmic_flops_with_recompute"] = mdl["flops_with_recompute"]
            for x in ("flops_full", "dir_tiles_frac", "d_color_nonzero_tiles_before_after",
                      "rows_read_frac"):
                if x in mdl:
                    roofline[x] = mdl[x]
            if st.get("source"):
                roofline["timing_source"] = st["source"]
            if "atomic_requests" in mdl:
                roofline["atomic_requests_per_launch"] = mdl["atomic_requests"]
                roofline["atomic_requests_per_sample"] = round(mdl["atomic_requests"] / M, 4)
                roofline["atomic_requests_source"] = mdl["atomic_requests_source"]
                for x in ("atomic_requests_before_after", "d_enc_nonzero_before_after",
                          "d_enc_nonzero_rows_before_after"):
                    if x in mdl:
                        roofline[x] = mdl[x]
                if "atomic_requests_pmc" in mdl:
                    roofline["atomic_requests_pmc"] = mdl["atomic_requests_pmc"]
            if "atomic_requests_stale" in mdl:
                roofline["atomic_requests_stale"] = (
                    f"PMC entry {mdl['atomic_requests_stale']} measured on another version of "
                    "the kernel source: not used (bound priced on bytes)")
            if "survey_bytes" in mdl:
                # SURVEY §8(d)'s per-sample model (every corner access as HBM bytes)
                roofline["survey_model"] = {
                    "bytes_per_unit": mdl["survey_bytes"] / M,
                    "achieved": k["survey_model_gbs"], "frac": k["survey_model_frac"]}
            ent, stale = pmc_entry(pmc, dominant, pmc_sfx)
            if ent and stale:
                roofline["traffic_stale"] = ent.get("source")
            elif ent:  # HBM bytes per launch from rocprofv3 PMC (tools/prof.sh)
                roofline["traffic"] = ent["bytes"]
                roofline["traffic_source"] = f"profiles/pmc_traffic.json [{ent.get('source')}]"
                roofline["traffic_frac_of_measured_hbm"] = round(
                    ent["bytes"] / (st["avg_ms"] * 1e-3) / 1e9 / peaks["hbm_copy_gbs"], 4)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import cpu_baseline

        say("CPU baseline (oracle, configs/nerf.json step)")
        cpu = cpu_baseline.run(budget_s=args.cpu_budget)

    if rank == 0:
        T = 2 ** cfg["instant_ngp"]["encoding"]["log2_hashmap_size"]
        width = cfg["instant_ngp"]["network"]["n_neurons"]
        line = {
            "metric": "train-step rays/sec",
            "value": round(value, 1),
            "unit": "rays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "host_ms_per_step": round(t_host / args.steps * 1e3, 3),
            "windows": windows,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": args.dtype,
            "numerics": numerics,
            "warm_start": warm,
            "start": "cold" if args.cold_start else ("warm" if warm else "seed"),
            "transient_window": transient,
            "d_enc_nonzero_frac": None if req is None else round(req[1], 4),
            "d_enc_nonzero_rows_frac": None if req is None else round(req[2], 4),
            "d_color_nonzero_tiles_frac": None if req is None else round(req[3], 4),
            "graph": job.graphed,
            "data": f"synthetic ({args.views}-view {args.img_size}x{args.img_size} "
                    f"HARP2-shaped scene, {len(ds)} rays; random-init weights)",
            "config": {
                "workload": (f"instant_ngp {'BASELINE configs[2]' if args.variant == 'baseline' else 'committed configs/instant_ngp.json'}"
                             f": 16-level T=2^{T.bit_length() - 1} hash grid, 2x{width} fused "
                             f"MLP, {args.samples} samples/ray, full train step "
                             f"(fwd+loss+bwd+AdamW)"
                             + (" + occupancy-grid culling (BASELINE configs[4], beyond the "
                                "reference)" if occ is not None else "")
                             + (", f16 hash features + bf16 MFMA field MLP (BASELINE "
                                "configs[4], beyond the reference)" if args.dtype == "bf16"
                                else "")),
                "global_batch": rank_batch * world,
                "per_rank_batch": rank_batch,
                "samples_per_ray": args.samples,
                "parallelism": f"dp{world}",
            },
            "roofline": roofline,
            "roofline_targets": target_rooflines(kernels, mfma_key, pmc, pmc_sfx),
            "cpu_baseline": cpu,
            "strong_scaling": strong,
            "alt_numerics": alt,
            "peaks": peaks,
            "kernels": kernels,
            "kernels_source": (f"untimed profiling pass of {args.profile_steps} steps; entries "
                               "marked overlapped ran on the side stream beside the per-sample "
                               "chain (event span, not step cost)"),
            "grad_all_reduce": None if sharded else {
                "bytes": 4 * bucket.numel, "overlap": bucket.overlap,
                "chunks": len(bucket._chunks) if bucket.overlap else 1,
                "issued_during_backward": bucket.early_issued if bucket.overlap else 0,
                "backend": dist.get_backend() if world > 1 else None},
            "sharded_optimizer": None if not sharded else {
                "grad_exchange": job.grad_exchange,
                "reduce_scatter_bytes": (2 if job.grad_exchange == "f16" else 4) * bucket.numel,
                "all_gather_bytes": (2 if shard == "f16" else 4) * bucket.numel,
                "state_floats_per_rank": opt.state_numel(), "gather": shard,
                "backend": dist.get_backend() if world > 1 else None},
            "occupancy": None if occ is None else {
                "grid": list(occ.res), "threshold": occ.threshold, "warmup": occ.warmup,
                "update_every": occ.update_every, "active": occ.active,
                "kept_fraction_last_step": round(occ.last_fraction, 4),
                "occupied_cells": round(occ.occupancy_fraction(), 4)},
            "final_loss": round(final_loss, 6),
            "scene_build_s": round(t_scene, 2),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
