"""Cold-start liveness of the bench configuration, GPU vs the oracle.

From the seed-1337 parameters of BASELINE configs[2] (T = 2^19, 1,024 samples per ray,
AdamW lr 1e-2) on the bench scene (90-view 512x512 synthetic HARP2), the reference's f16
arithmetic kills the density field after the first AdamW step and revives it later. The
GPU pipeline in reference numerics and the reference-semantics oracle with f32 master
parameters (tinycudann's torch binding keeps f32 masters, as the GPU does) train side by
side on the same batches and draws (tools/liveness_paired.py); per step the fraction of
fine samples with sigma > 0 must agree within 0.02 and the loss within 1 % (measured:
5e-4 and 0.4 %: profiles/r06_liveness_paired_b128.log), and both must collapse at the same
step and revive within 2 steps of each other.
"""

import pytest

pytestmark = pytest.mark.gpu

BATCH, STEPS = 128, 24


@pytest.mark.timeout(600)
def test_cold_start_liveness_matches_f32_master_oracle(dev):
    from tools.liveness_paired import revival, run

    trace = run(BATCH, STEPS, 1024, "reference", ["oracle_f32_master"], threads=16,
                scene_img=512, views=90)
    gpu, orc = trace["gpu"], trace["oracle_f32_master"]
    for k, (a, b) in enumerate(zip(gpu, orc)):
        assert abs(a["sigma_pos"] - b["sigma_pos"]) <= 0.02, (k, gpu, orc)
        assert abs(a["loss"] - b["loss"]) <= 1e-2 * abs(b["loss"]), (k, gpu, orc)
    rg, ro = revival(gpu, 0.5), revival(orc, 0.5)
    assert rg["collapse_step"] is not None and rg["collapse_step"] == ro["collapse_step"], (rg, ro)
    assert ro["revival_step"] is not None and rg["revival_step"] is not None, (rg, ro)
    assert abs(rg["revival_step"] - ro["revival_step"]) <= 2, (rg, ro)
