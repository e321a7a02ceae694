"""Checkpoint layout compatibility on CPU: the Instant-NGP pipeline's
state dict has the reference's nested layout, {module_name: module.state_dict()} with
tcnn's one flat ``params`` tensor per module (instant_ngp.py:265-284, tinycudann
modules), at tcnn's parameter counts; it survives torch.save / torch.load(weights_only)
into a fresh pipeline. (tcnn's internal order of MLP weights inside ``params`` is
unpinned: tcnn is absent)"""

import torch

import __graft_entry__ as ge

REF_MODULES = ["pos_encoder", "pos_mlp", "dir_encoder", "dir_mlp", "surf_encoder", "surf_mlp"]


def _pipe(seed):
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline

    ds = SyntheticHARP2Dataset(n_views=4, img_size=8, device=torch.device("cpu"), seed=0)
    return InstantNGPPipeline(ge._ingp_config(16), ds, seed=seed)


def test_ingp_state_dict_reference_layout(tmp_path):
    p = _pipe(5)
    sd = p.state_dict()
    assert list(sd) == REF_MODULES  # instant_ngp.py:265-284 module order
    sizes = {m: [tuple(v.shape) for v in sd[m].values()] for m in sd}
    assert all(list(sd[m]) == ["params"] for m in sd), {m: list(sd[m]) for m in sd}
    # tcnn parameter counts: 16-level T=2^19 3-D grid, 2-D surface grid; MLPs at width
    # 64 with padded input / output widths (32->64->16; 32->64->64->16; 48->64->64->16)
    assert sizes == {"pos_encoder": [(12196240,)], "pos_mlp": [(32 * 64 + 64 * 16,)],
                     "dir_encoder": [(0,)],
                     "dir_mlp": [(32 * 64 + 64 * 64 + 64 * 16,)],
                     "surf_encoder": [(5522000,)],
                     "surf_mlp": [(48 * 64 + 64 * 64 + 64 * 16,)]}
    assert all(v.dtype == torch.float32 for m in sd for v in sd[m].values())
    path = tmp_path / "ckpt.pt"
    torch.save({"pipeline": sd}, path)
    loaded = torch.load(path, weights_only=True)["pipeline"]
    q = _pipe(6)
    assert not torch.equal(q.pos_mlp.params, p.pos_mlp.params)
    q.load_state_dict(loaded)
    for m in REF_MODULES:
        assert torch.equal(getattr(q, m).params, getattr(p, m).params)
