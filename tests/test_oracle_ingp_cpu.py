"""The Instant-NGP oracle's two numerics modes on CPU (oracle/ref_ingp.py):
"build" (f64 with the build's f16 roundings, f32 composite) and "reference" (the
reference's f16 tcnn outputs, loss-scaled f16 module backward, f16 composite and loss).
At initialisation both render the same image within f16 resolution; the reference mode's
f16 autograd zeroes gradients the build keeps (the dir MLP's at step 0 on this scene)."""

import torch

import __graft_entry__ as ge
from oracle import ref_ingp


def _setup():
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline

    ds = SyntheticHARP2Dataset(n_views=8, img_size=16, device=torch.device("cpu"), seed=0)
    cfg = ge._ingp_config(32)
    p = InstantNGPPipeline(cfg, ds, dtype=torch.float16, fused=True, seed=5)
    pp = ds.get_point_preprocessor("horizontal")
    mk = lambda sem: ref_ingp.RefInstantNGP(cfg, p.state_dict(), ref_ingp.prep_kwargs(pp),
                                            p.scale, ds.max_i, half=True, semantics=sem)
    b = ref_ingp.cpu_batch(next(iter(BatchLoader(ds, 128, seed=3))))
    return mk("build"), mk("reference"), b


def test_reference_semantics_forward_and_underflow():
    ob, orf, b = _setup()
    u = torch.rand(128, 32, generator=torch.Generator().manual_seed(1))
    rb, rr = ob.forward(b, u), orf.forward(b, u)
    assert rr["color_map_fine"].dtype == torch.float16  # graphics_utils.py:28 in f16
    cb, cr = rb["color_map_fine"].detach(), rr["color_map_fine"].detach().double()
    assert ((cb - cr).abs().max() / cb.abs().max()).item() < 2e-2
    lb, lr = ob.loss(b, rb), orf.loss(b, rr)
    assert lr.dtype == torch.float16 and abs(lb.item() - lr.item()) / lb.item() < 2e-2
    lb.backward()
    lr.backward()
    gb, gr = ob.params["dir_mlp"].grad, orf.params["dir_mlp"].grad
    assert gb.abs().max().item() > 0
    assert gr.abs().max().item() == 0.0  # underflows in the reference's f16 autograd
    # gradients that survive agree in direction with the build's
    for m in ("pos_encoder", "surf_mlp"):
        a, c = ob.params[m].grad, orf.params[m].grad
        cos = (a * c).sum() / (a.norm() * c.norm())
        assert cos.item() > 0.9, (m, cos.item())
