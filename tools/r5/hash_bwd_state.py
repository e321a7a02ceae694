"""Hash-grid backward on the benched step's own inputs (profiling aid, r05).

    python tools/r5/hash_bwd_state.py dump  [--numerics reference] [--out /tmp/hb_state.pt]
    python tools/r5/hash_bwd_state.py time  [--state /tmp/hb_state.pt] [--iters 20]

``dump`` builds bench.py's configs[2] job (90-view 512x512 scene, 8192 x 1024 samples),
warm-starts it as bench.py does, runs ``--steps`` steps and saves the hash-grid backward's
inputs of the next step (coordinates, dL/denc) plus zero statistics of dL/denc (elements,
rows, 8-sample batches) to ``--out``. ``time`` replays anr_hashgrid_bwd over them with HIP
events (the kernel generation / skip mode come from the ANR_HASH* environment, read once
per process), so variants can be compared on the exact state the bench times.
"""

from __future__ import annotations

import argparse
import ctypes
import os
import sys
import time
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "atmospheric-neural-rendering_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def dump(a):
    import bench
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    ds = SyntheticHARP2Dataset(n_views=90, img_size=512, device=dev, seed=0)
    args = SimpleNamespace(dtype="f16", no_fused_zero=False, no_overlap=False, warmup=10)
    cfg = bench.ingp_config("baseline", 1024)
    job = bench.IngpJob(args, cfg, ds, dev, 0, 1, 8192, a.numerics, False, "off", None)
    bench.warm_start(job, args, cfg, ds, dev, 0, 1, 8192, "off")
    for _ in range(a.steps):
        job.step()
    pipe = job.pipe
    pipe._keep_d_enc = True
    job.eager_step()
    pipe._keep_d_enc = False
    coords, d_enc, _ = pipe._last_hash_bwd
    M = coords.shape[0]
    nz = d_enc != 0
    rows = nz.any(1)
    st = {"elements_nonzero": nz.float().mean().item(), "rows_nonzero": rows.float().mean().item()}
    for T in (8, 64, 256, 1024):
        n = M // T
        st[f"batches{T}_nonzero"] = rows[: n * T].view(n, T).any(1).float().mean().item()
    # rows nonzero inside nonzero 8-batches (what the per-sample skip adds)
    b8 = rows[: (M // 8) * 8].view(-1, 8)
    live = b8.any(1)
    st["rows_nonzero_in_live_batches8"] = b8[live].float().mean().item()
    # field-backward tiles (32 samples) whose incoming gradients are all zero
    ds_, dc_ = pipe._last_field_grads
    zc = (dc_.reshape(M, -1) == 0).all(1)
    zs = (ds_.reshape(M) == 0)
    for T in (16, 32):
        n = M // T
        st[f"tiles{T}_color_grad_zero"] = zc[: n * T].view(n, T).all(1).float().mean().item()
        st[f"tiles{T}_all_grad_zero"] = (zc & zs)[: n * T].view(n, T).all(1).float().mean().item()
    print("state", a.numerics, "steps", a.steps, st, flush=True)
    torch.save({"coords": coords.contiguous(), "d_enc": d_enc.contiguous(), "stats": st,
                "numerics": a.numerics}, a.out)


def time_it(a):
    from atmonr_amd import _lib

    dev = torch.device("cuda:0")
    s = torch.load(a.state, map_location=dev, weights_only=True)
    coords, d_enc = s["coords"], s["d_enc"]
    M = coords.shape[0]
    desc = _lib.hashgrid_desc(3, 16, 2, 16, 1.3819, 19)
    grad = torch.zeros(desc.n_params, device=dev)
    stream = _lib.stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for it in range(a.iters + 2):
        grad.zero_()
        torch.cuda.synchronize()
        ev[0].record()
        _lib.call("anr_hashgrid_bwd", ctypes.byref(desc), coords.data_ptr(), 3, M,
                  d_enc.data_ptr(), _lib.F32, 32, grad.data_ptr(), stream)
        ev[1].record()
        torch.cuda.synchronize()
        if it >= 2:
            ts.append(ev[0].elapsed_time(ev[1]))
    ts.sort()
    env = {k: v for k, v in os.environ.items() if k.startswith("ANR_HASH")}
    print(f"hash_bwd {env} median {ts[len(ts) // 2]:.4f} ms min {ts[0]:.4f} "
          f"grad_l2 {grad.double().norm().item():.6e} state {s['stats']}", flush=True)
    if a.save_grad:
        torch.save(grad.cpu(), a.save_grad)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["dump", "time"])
    ap.add_argument("--numerics", default="reference")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--out", default="/tmp/hb_state.pt")
    ap.add_argument("--state", default="/tmp/hb_state.pt")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--save-grad", default="")
    a = ap.parse_args()
    t0 = time.time()
    dump(a) if a.mode == "dump" else time_it(a)
    print(f"[{a.mode} {time.time() - t0:.1f}s]", flush=True)


if __name__ == "__main__":
    main()
