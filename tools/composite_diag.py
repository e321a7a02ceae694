"""Diagnostic: per-sample dL/dcolor and dL/dsigma of the GPU composite (f32 pipeline,
1,024 samples per ray) against the oracle's f32 and f64 composites on the same inputs."""
import sys

import torch

sys.path.insert(0, "atmospheric-neural-rendering_amd")
sys.path.insert(0, ".")
import __graft_entry__ as ge  # noqa: E402
from oracle import ref_path  # noqa: E402
from atmonr_amd import graphics_utils  # noqa: E402
from atmonr_amd.batch_loader import BatchLoader  # noqa: E402
from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset  # noqa: E402
from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline  # noqa: E402

dev = torch.device("cuda:0")
ds = SyntheticHARP2Dataset(n_views=8, img_size=16, device=dev, seed=0)
for N, B in ((64, 200), (1024, 24)):
    cfg = ge._ingp_config(N)
    p = InstantNGPPipeline(cfg, ds, dtype=torch.float32, fused=True, seed=5)
    p.send_tensors_to(dev)
    cap = {}
    orig = graphics_utils.render_with_surface

    def hook(z, color, sigma, color_surf, z_scale=1.0):
        color.retain_grad(); sigma.retain_grad()
        cap.update(z=z.detach(), color=color, sigma=sigma, cs=color_surf.detach(), zs=z_scale)
        return orig(z, color, sigma, color_surf, z_scale)
    import atmonr_amd.pipelines.instant_ngp as ip
    ip.render_with_surface = hook
    batch = next(iter(BatchLoader(ds, B, seed=1)))
    u = torch.rand(B, N, generator=torch.Generator().manual_seed(2))
    res = p.forward(batch, u=u.to(dev))
    # a fixed upstream gradient on the colour map (loss-independent)
    gC = torch.randn(res["color_map_fine"].shape, generator=torch.Generator().manual_seed(4)).to(dev)
    (res["color_map_fine"] * gC).sum().backward()
    ip.render_with_surface = orig
    gpu_dc, gpu_ds = cap["color"].grad.double().cpu(), cap["sigma"].grad.double().cpu()
    z = (cap["z"] * cap["zs"]).cpu()
    out = {}
    for dt in (torch.float32, torch.float64):
        c = cap["color"].detach().cpu().to(dt).requires_grad_(True)
        s = cap["sigma"].detach().cpu().to(dt).requires_grad_(True)
        cm, *_ = ref_path.render_with_surface(z.to(dt) if dt == torch.float64 else z, c, s, cap["cs"].cpu().to(dt))
        (cm * gC.cpu().to(dt)).sum().backward()
        out[dt] = (c.grad.double(), s.grad.double())
    rel = lambda a, b: ((a - b).norm() / b.norm()).item()
    print(f"N={N}: dcolor gpu-vs-f32 {rel(gpu_dc, out[torch.float32][0]):.2e} gpu-vs-f64 {rel(gpu_dc, out[torch.float64][0]):.2e} "
          f"f32-vs-f64 {rel(out[torch.float32][0], out[torch.float64][0]):.2e} | dsigma gpu-vs-f32 {rel(gpu_ds, out[torch.float32][1]):.2e} "
          f"gpu-vs-f64 {rel(gpu_ds, out[torch.float64][1]):.2e} f32-vs-f64 {rel(out[torch.float32][1], out[torch.float64][1]):.2e}", flush=True)
    print("   z dtype", cap["z"].dtype, "scale", cap["zs"], "sigma max", cap["sigma"].max().item(), flush=True)
