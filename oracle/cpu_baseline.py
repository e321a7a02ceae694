"""ORACLE (test infrastructure only): time the configs/nerf.json CPU train step.

bench.py's ``cpu_baseline`` leg: the reference's own CPU-runnable configuration
(BASELINE.json configs[0]: nerf.json's pipeline on an 8-view 64x64 synthetic scene), run
with oracle/ref_nerf.py at nerf.json's own batch of 4,096 rays, as BASELINE.md §3 plans it:
every core of the process's affinity mask, the median of five timed steps after two
warm-ups (r06; r05 took OMP_NUM_THREADS and 1 + 3 steps). The same step on the box's
per-GPU host share (OMP_NUM_THREADS = 16) is timed beside it, and the cgroup CPU quota is
reported, since threads beyond the quota only time-share.
"""

from __future__ import annotations

import os
import sys
import time

import torch


def host_threads(threads: int | None = None) -> tuple[int, str]:
    """The host cores the job may run on (the box's own host cores): the
    process's CPU affinity mask (else os.cpu_count()), capped at the cgroup CPU quota when
    one is set -- threads past the quota only time-share the same CPU time (on the GPU box
    the mask lists 256 CPUs and the quota grants 16: 256 spinning OpenMP threads there
    ran the step many times slower than 16)."""
    if threads is not None:
        return threads, "argument"
    try:
        n, src = len(os.sched_getaffinity(0)), "len(os.sched_getaffinity(0))"
    except (AttributeError, OSError):
        n, src = os.cpu_count() or 1, "os.cpu_count()"
    q = cpu_quota()
    if q is not None and q < n:
        return max(1, int(q + 0.999)), f"cgroup CPU quota ({src} = {n})"
    return n, src


def omp_share() -> int | None:
    """OMP_NUM_THREADS when set (the GPU box sets it to its per-GPU host share, 16)."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    return int(env) if env.isdigit() and int(env) > 0 else None


def _affinity() -> int | None:
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return None


def cpu_quota() -> float | None:
    """CPUs granted by the cgroup v2 CPU quota (cpu.max), None when unlimited / unknown:
    with an affinity mask wider than the quota, threads past it only time-share."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def cpu_model() -> str | None:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _nerf_setup(seed: int):
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from oracle.ref_nerf import RefNeRFPipeline

    torch.manual_seed(seed)
    ds = SyntheticHARP2Dataset(n_views=8, img_size=64, device="cpu", seed=seed)
    pp = ds._prep
    prep = dict(scale=pp.scale, offset=torch.tensor(pp.offset, dtype=torch.float64),
                lat_min=torch.tensor(pp.lat_min, dtype=torch.float32),
                lat_range=torch.tensor(pp.lat_range, dtype=torch.float32),
                lon_min=torch.tensor(pp.lon_min, dtype=torch.float32),
                lon_range=torch.tensor(pp.lon_range, dtype=torch.float32),
                h0=pp.ray_origin_height, shift_lon=pp.shift_lon)
    return ds, RefNeRFPipeline(prep, ds.scale)


def _progress(msg: str, threads: int, t_start: float) -> None:
    """One stderr line per CPU step (a long silent phase reads as a hang to a watchdog)."""
    print(f"[cpu_baseline] {threads} threads, {msg} ({time.perf_counter() - t_start:.0f} s)",
          file=sys.stderr, flush=True)


def _time_steps(threads, batch_size, seed, warmup, timed, budget_s):
    ds, pipe = _nerf_setup(seed)
    torch.set_num_threads(threads)
    perm = torch.randperm(len(ds))

    def batch(k):
        return ds.__getbatch__(perm[(k * batch_size) % len(ds):][:batch_size])

    t_start = time.perf_counter()
    for k in range(warmup):
        pipe.train_step(batch(k))
        _progress(f"warm-up step {k + 1}/{warmup}", threads, t_start)
    times = []
    k = warmup
    while True:
        t0 = time.perf_counter()
        pipe.train_step(batch(k))
        times.append(time.perf_counter() - t0)
        _progress(f"timed step {len(times)}/{timed}: {times[-1]:.2f} s", threads, t_start)
        k += 1
        if time.perf_counter() - t_start >= budget_s or len(times) >= timed:
            break
    times.sort()
    return batch_size / times[len(times) // 2], len(times)


def run(budget_s: float = 150.0, batch_size: int = 4096, threads: int | None = None,
        seed: int = 0, warmup: int = 2, timed: int = 5, share_budget_s: float = 75.0) -> dict:
    """median rays/s of ``timed`` train steps after ``warmup`` on every
    core of the affinity mask (stops early at ``budget_s``), and beside it the same step
    on the box's per-GPU host share (OMP_NUM_THREADS, when it differs)."""
    threads, source = host_threads(threads)
    prev = torch.get_num_threads()
    try:
        value, n = _time_steps(threads, batch_size, seed, warmup, timed, budget_s)
        share = omp_share()
        at_share = None
        if share and share != threads:
            v2, n2 = _time_steps(share, batch_size, seed, warmup, timed, share_budget_s)
            at_share = {"value": v2, "cores": share, "cores_source": "OMP_NUM_THREADS",
                        "timed_steps": n2}
    finally:
        torch.set_num_threads(prev)
    return {
        "value": value,
        "unit": "rays/s",
        "cores": threads,
        "cores_source": source,
        "affinity_cpus": _affinity(),
        "host_cpus": os.cpu_count(),
        "cgroup_cpu_quota": cpu_quota(),
        "cpu_model": cpu_model(),
        "at_host_share": at_share,
        "kind": "port",
        "sample": (f"configs/nerf.json train step (coarse 64 + fine 128 samples, 8x256 MLP, "
                   f"Adam) on an 8-view 64x64 synthetic HARP2 scene, batch {batch_size}; "
                   f"median of {n} timed steps after {warmup} warm-up, "
                   f"torch CPU {torch.__version__}, {threads} threads of "
                   f"{os.cpu_count()} host CPUs"),
    }


def run_extract(budget_s: float = 20.0, n_points: int = 131072, threads: int | None = None,
                seed: int = 0, timed: int = 3) -> dict:
    """Points/s of the extract loop body (scripts/extract.py:203-209 ->
    instant_ngp.py:208-247) restated on the CPU: (xyz - offset) / scale in f64, the
    horizontal preprocessor in f64 torch (ref_nerf.preprocess_torch), the INGP remap,
    the restated tcnn hash grid (numpy, f16 table) and the f16-rounded pos MLP
    (ref_tcnn), relu of output 0, / scale. Median of ``timed`` batches of ``n_points``
    random in-scene points (stops early at ``budget_s``)."""
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from oracle import ref_nerf, ref_tcnn

    threads, source = host_threads(threads)
    torch.set_num_threads(threads)
    gen = torch.Generator().manual_seed(seed)
    ds = SyntheticHARP2Dataset(n_views=8, img_size=64, device="cpu", seed=seed)
    pp = ds._prep
    offset = torch.tensor(pp.offset, dtype=torch.float64)
    cfg = (3, 16, 16, 1.3819, 19)
    n_table = int(ref_tcnn.grid_levels(3, 16, 16, 1.3819, 19)[4]) * 2
    table = ((torch.rand(n_table, generator=gen, dtype=torch.float64) * 2 - 1) * 1e-4
             ).half().double().numpy()
    w = (torch.rand(32 * 64 + 64 * 16, generator=gen, dtype=torch.float64) - 0.5) * 0.3
    pts_n = (torch.rand(n_points, 3, generator=gen, dtype=torch.float64) * 2 - 1) * torch.tensor(
        [0.9, 0.9, 0.2], dtype=torch.float64)
    xyz = pts_n * ds.scale + offset

    def body():
        pts = (xyz - offset) / ds.scale
        c = ref_nerf.preprocess_torch(pts, scale=float(pp.scale), offset=offset,
                                      lat_min=pp.lat_min, lat_range=pp.lat_range,
                                      lon_min=pp.lon_min, lon_range=pp.lon_range,
                                      h0=pp.ray_origin_height, shift_lon=pp.shift_lon)
        c = (c + 1) / 2
        c[..., 2] = c[..., 2] / 8.0
        enc = torch.from_numpy(ref_tcnn.hashgrid_fwd(c.float().double().numpy(), table, cfg))
        out = ref_tcnn.mlp_fwd(enc, w, 32, 16, 64, 1, half=True)
        return torch.clip(out[:, :1], min=0) / ds.scale

    times = []
    t_start = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        body()
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start >= budget_s or len(times) >= timed:
            break
    times.sort()
    med = times[len(times) // 2]
    return {
        "value": n_points / med, "unit": "points/s", "cores": threads,
        "cores_source": source, "affinity_cpus": _affinity(),
        "host_cpus": os.cpu_count(), "cgroup_cpu_quota": cpu_quota(), "kind": "port",
        "sample": (f"extract loop body (f64 preprocessor, tcnn hash grid T=2^19 and 2x64 "
                   f"pos MLP restated in numpy / torch CPU) on {n_points} random in-scene "
                   f"points, median of {len(times)} batches, {threads} threads of "
                   f"{os.cpu_count()} host CPUs"),
    }


if __name__ == "__main__":
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "atmospheric-neural-rendering_amd"))
    print(run())
