"""Train-step throughput of the AtmoNR Instant-NGP hot path on MI355X.

    python bench.py --gpus N --steps K --warmup W [--workload nerf]

Workload (BASELINE.json configs[2]): configs/instant_ngp.json with a 16-level T=2^19
hash grid and 2x64 fused MLPs, B = 8192 rays x N = 1024 samples per rank per step, on a
synthetic 90-view 512x512 HARP2-shaped scene (no L1B granule exists offline). One step =
batch gather -> fused sampler/preprocessor -> hash grid -> MLPs -> composite -> loss ->
backward -> [RCCL all-reduce of the flat gradient when N > 1] -> fused AdamW.
Data parallel over rays, one process per GPU, weak scaling (8192 rays per rank).

``--workload nerf`` measures BASELINE configs[1] instead (configs/nerf.json, batch 4096,
f32 library GEMMs; see run_nerf). Rank 0 prints ONE JSON line. ``roofline`` is for the kernel that takes the most time per
step, timed with HIP events on the launch stream inside the timed region; its
algorithmic bytes / FLOPs per launch (kernel_models) are compulsory
HBM traffic and dense MFMA work, and the bound is whichever fraction of peak is larger. ``cpu_baseline`` times the
oracle's CPU restatement of the configs/nerf.json train step (rank 0, N = 1 only).
"""

from __future__ import annotations

import argparse
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


def kernel_models(pipe, M: int, pmc: dict | None = None, key_sfx: str = "") -> dict:
    """Algorithmic work per launch of each hot kernel.

    ``bytes`` = compulsory HBM traffic (every per-sample stream read or written once, the
    table / gradient array once per launch); ``flops`` = dense MFMA work at padded widths.
    ``survey_bytes`` = SURVEY §8(d)'s per-sample hash figures (forward 12 + 16x8x2x2 + 64 =
    588 B, backward 64 + 12 + 2 x 512 = 1,100 B), which count every corner access as HBM
    traffic; L2/MALL serve most of them, so that model reaches the HBM peak without
    discriminating and is reported beside the bound, not used for it. ``atomic_requests``
    (hash backward) = memory-side f32 atomic requests per launch from rocprofv3 PMC
    (profiles/pmc_traffic.json), priced against the measured request ceiling.
    """
    grid = pipe.pos_encoder.hash_grids[0]
    n_table = grid.desc.n_params                # f16 table entries x features
    pos, dirm = pipe.pos_mlp.desc, pipe.dir_mlp.desc

    def mlp_flops(d):
        dims = [d.n_input_padded] + [d.width] * d.n_hidden_layers + [d.n_output_padded]
        return 2.0 * sum(a * b for a, b in zip(dims[:-1], dims[1:]))

    f_fwd = mlp_flops(pos) + mlp_flops(dirm)
    nb = dirm.n_output
    enc_b = 2 * grid.n_out                      # f16 features
    out = {
        "hash_fwd": {"bytes": M * (12 + enc_b) + 2 * n_table, "flops": 0.0,
                     "survey_bytes": M * (12 + grid.n_levels * 8 * 2 * 2 + enc_b)},
        "hash_bwd": {"bytes": M * (12 + 4 * grid.n_out) + 8 * n_table, "flops": 0.0,
                     "survey_bytes": M * (64 + 12 + 2 * grid.n_levels * 8 * 2 * 2)},
        # enc in, sigma + color out
        "field_fwd": {"bytes": M * (enc_b + 4 + 4 * nb), "flops": M * f_fwd},
        # enc + dL/dcolor + dL/dsigma in, f32 dL/denc out; forward recompute + dX + dW
        "field_bwd": {"bytes": M * (enc_b + 4 * nb + 4 + 4 * grid.n_out), "flops": 3 * M * f_fwd},
    }
    ent, stale = pmc_entry(pmc, "hash_bwd", key_sfx)
    if ent and ent.get("atomic_requests") and not stale:
        out["hash_bwd"]["atomic_requests"] = float(ent["atomic_requests"])
        out["hash_bwd"]["atomic_requests_source"] = (
            f"profiles/pmc_traffic.json [{ent.get('source')}], rocprofv3 --pmc "
            "TCC_EA0_ATOMIC_sum of this kernel source (sha1 match)")
    elif ent and ent.get("atomic_requests"):
        out["hash_bwd"]["atomic_requests_stale"] = ent.get("source")
    return out


def _roof(mdl: dict, avg_ms: float, peaks: dict, mfma_key: str) -> dict:
    sec = avg_ms * 1e-3
    gbs = mdl["bytes"] / sec / 1e9
    tfs = mdl["flops"] / sec / 1e12
    fb, ff = gbs / peaks["hbm_copy_gbs"], tfs / peaks[mfma_key]
    r = {"hbm_gbs": round(gbs, 1), "hbm_frac": round(fb, 4), "mfma_tfs": round(tfs, 2),
         "mfma_frac": round(ff, 4), "bound": "hbm" if fb >= ff else "mfma"}
    if "survey_bytes" in mdl:
        sg = mdl["survey_bytes"] / sec / 1e9
        r["survey_model_gbs"] = round(sg, 1)
        r["survey_model_frac"] = round(sg / peaks["hbm_copy_gbs"], 4)
    if "atomic_requests" in mdl:
        rq = mdl["atomic_requests"] / sec / 1e9
        fa = rq / peaks["atomic_seg16_greq_s"]
        r["atomic_greq_s"] = round(rq, 3)
        r["atomic_frac"] = round(fa, 4)
        if fa >= max(fb, ff):
            r["bound"] = "atomic"
    return r


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
    roofline = {"kernel": "nerf_mlp_gemms (library f32 GEMMs, whole-step time)",
                "bound": "mfma", "achieved": round(tfs, 2), "peak": peaks["mfma_f32_tfs"],
                "unit": "TFLOP/s", "frac": round(tfs / peaks["mfma_f32_tfs"], 4), "traffic": None,
                "algorithmic_flops": flops, "units_per_launch": batch_size,
                "flops_per_unit": flops / batch_size}
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
            "final_loss": round(final_loss, 6),
            "scene_build_s": round(t_scene, 2)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


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
    ap.add_argument("--workload", choices=["ingp", "nerf"], default="ingp",
                    help="ingp: BASELINE configs[2] (the headline line); nerf: configs[1]")
    ap.add_argument("--variant", choices=["baseline", "committed"], default="baseline")
    ap.add_argument("--dtype", choices=["f16", "bf16", "f32"], default="f16",
                    help="f16: tcnn precision (the reference's); bf16: BASELINE configs[4], "
                         "f16 hash features + bf16 MFMA field MLP; f32: exact-f32 kernels")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--spec-peaks", action="store_true",
                    help="price the rooflines against spec-sheet peaks instead of measuring")
    ap.add_argument("--cpu-budget", type=float, default=40.0)
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
    ap.add_argument("--shard-optimizer", choices=["off", "f16", "f32"], default="off",
                    help="ZeRO-1 (atmonr_amd.parallel.ShardedAdam): reduce-scatter of the "
                         "gradient, AdamW on 1/N of the parameters, all-gather of the f16 "
                         "compute copy (f16) or of the f32 parameters (f32), instead of "
                         "all-reduce + replicated AdamW")
    ap.add_argument("--field-bwd", choices=["rt", "rt_lt", "lds"], default="rt",
                    help="fused field backward generation (anr_ingp_field_force_bwd): "
                         "register-transposed (default), the same with the dW operand "
                         "transposes through LDS, or LDS-staged tiles")
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

    _lib.load().anr_ingp_field_force_bwd({"lds": 0, "rt": 1, "rt_lt": 2}[args.field_bwd])
    t0 = time.time()
    ds = SyntheticHARP2Dataset(n_views=args.views, img_size=args.img_size, device=dev, seed=0)
    torch.cuda.synchronize()
    t_scene = time.time() - t0
    if args.workload == "nerf":
        return run_nerf(args, ds, dev, rank, world, t_scene)
    if args.global_batch:
        if args.global_batch % world:
            sys.exit(f"--global-batch {args.global_batch} is not divisible by {world} ranks")
        rank_batch, scaling = args.global_batch // world, "strong"
    else:
        rank_batch, scaling = args.batch, "weak"
    cfg = ingp_config(args.variant, args.samples)
    dtype = torch.float32 if args.dtype == "f32" else torch.float16
    mlp_dtype = torch.bfloat16 if args.dtype == "bf16" else dtype
    occ = None
    if args.occupancy:
        from atmonr_amd.occupancy import OccupancyGrid

        occ = OccupancyGrid((128, 128, 32), alt_compress=float(cfg["alt_compress_factor"]),
                            warmup=args.occ_warmup, update_every=16, device=dev)
    pipe = InstantNGPPipeline(cfg, ds, dtype=dtype, fused=True, seed=1337, occupancy=occ,
                              mlp_dtype=mlp_dtype)
    pipe.send_tensors_to(dev)
    opt_cfg = {"lr": 1e-2, "betas": [0.9, 0.99], "eps": 1e-15, "weight_decay": 1e-2}
    opt = pipe.get_optimizer(opt_cfg)

    # one flat f32 gradient bucket; every param's .grad is a view into it, so backward
    # accumulates in place and DP needs exactly one all-reduce per step
    from atmonr_amd.parallel import FlatGradBucket, ShardedAdam

    sharded = args.shard_optimizer != "off"
    bucket = FlatGradBucket([p for g in opt.param_groups for p in g["params"]], dev,
                            pad_to=world)
    if world > 1:
        bucket.broadcast_params(0)  # replicas start from rank 0's weights
    if sharded:
        opt = ShardedAdam(bucket, opt.param_groups, betas=opt_cfg["betas"], eps=opt_cfg["eps"],
                          gather=args.shard_optimizer)
    elif not args.no_fused_zero:
        bucket.fuse_zero_into(opt)  # the AdamW pass zeroes the bucket (no per-step fill)
    if not args.no_overlap and not sharded:
        # each chunk's all-reduce starts once its gradients are final: the surface and MLP
        # gradients reduce while the hash-grid backward runs
        bucket.enable_overlap()

    loader = BatchLoader(ds, rank_batch, shuffle=True, rank=rank, world_size=world, seed=0)
    it = iter(loader)

    def next_batch():
        nonlocal it
        try:
            return next(it)
        except StopIteration:
            it = iter(loader)
            return next(it)

    def step():
        batch = next_batch()
        res = pipe.forward(batch)
        loss = pipe.compute_loss(batch, res)
        bucket.zero()
        loss.backward()
        if not sharded:
            bucket.all_reduce()
        opt.step()  # ShardedAdam: reduce-scatter, sharded AdamW, all-gather
        return loss

    for _ in range(args.warmup):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    # Untimed profiling pass: HIP events around every libanr call give the per-kernel
    # breakdown and pick the dominant kernel; the timed region below then brackets only
    # that kernel's launches (events around every call would cost ~0.2 ms per step).
    M = rank_batch * args.samples
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
    models = kernel_models(pipe, M, pmc, pmc_sfx)
    kernels, dominant = {}, None
    if not args.no_kernel_timer:
        prof = _lib.KernelTimer()
        with prof:
            for _ in range(args.profile_steps):
                loss = step()
        summ = prof.summary()
        for name, st in sorted(summ.items(), key=lambda kv: -kv[1]["total_ms"]):
            entry = {"avg_ms": round(st["avg_ms"], 4),
                     "ms_per_step": round(st["total_ms"] / args.profile_steps, 4)}
            mdl = models.get(name)
            if mdl:
                entry.update(_roof(mdl, st["avg_ms"], peaks, mfma_key))
            kernels[name] = entry
        dominant = next((n for n in kernels if "bound" in kernels[n]), None)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    timer = _lib.KernelTimer(only={dominant}) if dominant else None
    t_start = time.perf_counter()
    if timer:
        with timer:
            for _ in range(args.steps):
                loss = step()
    else:
        for _ in range(args.steps):
            loss = step()
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
    rays_total = rank_batch * world * args.steps
    value = rays_total / elapsed

    strong = None
    if world > 1 and scaling == "weak" and not args.no_strong and args.batch % world == 0:
        # the same job at a fixed global batch of --batch rays (SURVEY §8(e)'s strong-
        # scaling target), timed the same way after a short warm-up at the new shape
        loader = BatchLoader(ds, args.batch // world, shuffle=True, rank=rank,
                             world_size=world, seed=0)
        it = iter(loader)
        for _ in range(max(2, args.warmup)):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t = torch.tensor([time.perf_counter() - t1], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
        strong = {"global_batch": args.batch, "per_rank_batch": args.batch // world,
                  "value": round(args.batch * args.steps / el, 1),
                  "ms_per_step": round(el / args.steps * 1e3, 3), "steps": args.steps}

    roofline = None
    if timer:
        st = timer.summary().get(dominant)
        if st:  # the dominant kernel, timed live over the timed region
            mdl = models[dominant]
            k = _roof(mdl, st["avg_ms"], peaks, mfma_key)
            bound = k["bound"]
            if bound == "atomic":
                # memory-side f32 atomic requests (16-B segments: the kernel's shape) per
                # launch, against the measured request ceiling of that shape; in GB/s of
                # the requests' segment bytes so the unit stays a bandwidth
                ach, peak, frac = (round(k["atomic_greq_s"] * 16, 1),
                                   round(peaks["atomic_seg16_greq_s"] * 16, 1), k["atomic_frac"])
                unit = "GB/s"
            elif bound == "hbm":
                ach, peak, frac, unit = k["hbm_gbs"], peaks["hbm_copy_gbs"], k["hbm_frac"], "GB/s"
            else:
                ach, peak, frac, unit = k["mfma_tfs"], peaks[mfma_key], k["mfma_frac"], "TFLOP/s"
            roofline = {"kernel": dominant, "bound": bound,
                        "ceiling": ("memory-side f32 atomic requests (MI355X_MICROARCH.md "
                                    "'Global float atomics'), measured at 16-B segments"
                                    if bound == "atomic" else
                                    "HBM float4 copy, measured" if bound == "hbm" else
                                    "dense MFMA loop on random operands, measured"),
                        "achieved": ach, "peak": peak, "unit": unit, "frac": frac,
                        "traffic": None, "avg_ms": round(st["avg_ms"], 4),
                        "launches": st["launches"], "units_per_launch": M,
                        "algorithmic_bytes": mdl["bytes"], "algorithmic_flops": mdl["flops"],
                        "bytes_per_unit": mdl["bytes"] / M,
                        "fractions": {x: k[x] for x in ("hbm_frac", "mfma_frac", "atomic_frac",
                                                        "survey_model_frac") if x in k}}
            if "atomic_requests" in mdl:
                roofline["atomic_requests_per_launch"] = mdl["atomic_requests"]
                roofline["atomic_requests_source"] = mdl["atomic_requests_source"]
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
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": args.dtype,
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
            "cpu_baseline": cpu,
            "strong_scaling": strong,
            "peaks": peaks,
            "kernels": kernels,
            "kernels_source": f"untimed profiling pass of {args.profile_steps} steps",
            "grad_all_reduce": None if sharded else {
                "bytes": 4 * bucket.numel, "overlap": bucket.overlap,
                "chunks": len(bucket._chunks) if bucket.overlap else 1,
                "issued_during_backward": bucket.early_issued if bucket.overlap else 0,
                "backend": dist.get_backend() if world > 1 else None},
            "sharded_optimizer": None if not sharded else {
                "reduce_scatter_bytes": 4 * bucket.numel,
                "all_gather_bytes": (2 if args.shard_optimizer == "f16" else 4) * bucket.numel,
                "state_floats_per_rank": opt.state_numel(), "gather": args.shard_optimizer,
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
