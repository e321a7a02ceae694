"""atmonr_amd — MI355X-native volumetric renderer for AtmoNR's train/extract hot path.

Drop-in modules mirroring the reference package ``atmonr``:

* ``atmonr_amd.tcnn``            — tinycudann.Encoding / Network (HashGrid, SH, Identity,
                                   Composite, FullyFusedMLP) on HIP kernels
* ``atmonr_amd.samplers``        — sample_uniform_bins (+ fused HARP2 preprocessor)
* ``atmonr_amd.graphics_utils``  — render / render_with_surface
* ``atmonr_amd.losses``          — the six AtmoNR losses
* ``atmonr_amd.pipelines``       — Pipeline, InstantNGPPipeline, get_pipeline
* ``atmonr_amd.optim``           — FusedAdam (AdamW / Adam)
* ``atmonr_amd.batch_loader``    — device-side, rank-sharded BatchLoader
* ``atmonr_amd.datasets``        — HARP2-shaped synthetic scene

All compute goes through libanr_hip.so (include/anr.h); there is no CPU fallback.
"""

__version__ = "0.1.0"
