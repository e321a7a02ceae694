"""Trainer — src/atmonr/trainer.py:16-274 with the per-step host traffic taken out.

Same constructor, schedule, loop structure, epoch metrics and checkpoint contents as
the reference:

* ``num_epochs = ceil(num_iters / len(loader))`` (trainer.py:51);
* optimizer from ``pipeline.get_optimizer(config["optimizer"])`` (:52);
* ExponentialLR with ``type == "target_lr"`` (gamma = (final_lr / lr)^(1/num_epochs),
  stepped per epoch) or ``type == "fixed"`` (gamma, stepped every ``decay_interval``
  iterations once past ``decay_start``) (:54-67, :113-120, :179-181);
* step = forward -> compute_loss -> zero_grad -> backward -> step (:99-105);
* per-epoch image metrics via ``dataset.get_image_metrics`` and a checkpoint
  ``epoch_XXXX.pt`` with pipeline / optimizer / scheduler state and counters (:183-274).

MI355X-side differences (behaviour-preserving):

* The reference syncs the host at every step: ``loss.item()`` twice and three
  ``take_along_dim(...).cpu()`` copies into a numpy ProgressTracker (:108-140). Here the
  per-ray predictions are scattered into device buffers, the losses go into a device
  ring, and the host reads both only every ``print_frequency`` steps and at epoch end.
* Data parallel (one process per GPU): with torch.distributed initialised, each rank
  takes a disjoint ``batch_size / world_size`` share of every global batch
  (BatchLoader rank slicing), gradients live in one FlatGradBucket and are averaged by
  one all-reduce per step; the progress buffers are combined at epoch end.
* tensorboard is not installed: ``writer`` is any object with ``add_scalar`` (default:
  a JSON-lines scalar log next to the checkpoints). Checkpoints hold plain types only,
  so they load with ``torch.load(weights_only=True)`` (the reference stores a Path and
  needs weights_only=False, survey §0 bug 4).
"""

from __future__ import annotations

import json
from datetime import datetime
from pathlib import Path
from typing import Any

import torch
import torch.distributed as dist
from torch.optim.lr_scheduler import ExponentialLR

from .batch_loader import BatchLoader
from .parallel import FlatGradBucket

_PROGRESS_KEYS = ("color_map_fine", "color_map_surf", "color_map_atmo")


class ScalarLog:
    """Minimal SummaryWriter stand-in: one JSON line per scalar."""

    def __init__(self, path: Path | str) -> None:
        self.path = Path(path)
        self.path.parent.mkdir(parents=True, exist_ok=True)

    def add_scalar(self, tag: str, value: float, step: int) -> None:
        with open(self.path, "a") as f:
            f.write(json.dumps({"tag": tag, "value": float(value), "step": int(step)}) + "\n")


class Trainer:
    def __init__(self, config: dict, dataset: Any, pipeline: Any, exp_name: str = "run",
                 writer: Any = None, log_dir: Path | str | None = None, seed: int = 0,
                 verbose: bool = True) -> None:
        self.config = config
        self.dataset = dataset
        self.pipeline = pipeline
        self.verbose = verbose
        self.distributed = dist.is_available() and dist.is_initialized()
        self.rank = dist.get_rank() if self.distributed else 0
        self.world_size = dist.get_world_size() if self.distributed else 1
        bs = int(config["batch_size"])
        if bs % self.world_size:
            raise ValueError(f"batch_size {bs} is not divisible by world size {self.world_size}")
        # all_gpu / num_workers (trainer.py:35-47): the scene is device-resident here, so
        # both settings use the device BatchLoader
        # the shuffle seed must be the same on every rank (one shared permutation)
        self.dataloader = BatchLoader(dataset, batch_size=bs // self.world_size, shuffle=True,
                                      rank=self.rank, world_size=self.world_size,
                                      seed=int(config.get("seed", seed)))
        self.epoch_idx = 0
        self.iter_count = 0
        self.num_epochs = int(-(config["num_iters"] // -len(self.dataloader)))
        self.optimizer = pipeline.get_optimizer(config["optimizer"])
        sch = config["scheduler"]
        if sch["type"] == "target_lr":
            gamma = (sch["final_lr"] / config["optimizer"]["lr"]) ** (1 / self.num_epochs)
        elif sch["type"] == "fixed":
            gamma = sch["gamma"]
        else:
            raise NotImplementedError(f"Unknown scheduler type {sch['type']}")
        self.scheduler = ExponentialLR(optimizer=self.optimizer, gamma=gamma)
        self.bucket = FlatGradBucket(pipeline.parameters()) if self.distributed else None
        if self.bucket is not None:
            # replicas start from rank 0's weights: modules initialised from the global
            # torch RNG (nn.Linear in AtmoNeRF) differ per rank otherwise
            self.bucket.broadcast_params(0)
        now_str = datetime.now().strftime("%Y%m%d_%H%M%S")
        self.log_dir = Path(log_dir) if log_dir is not None else (
            Path("data") / "tensorboard" / f"{exp_name}_{now_str}")
        self.writer = writer if writer is not None else (
            ScalarLog(self.log_dir / "scalars.jsonl") if self.rank == 0 else None)
        self.history: list[dict] = []  # per-epoch metrics (rank 0)
        dev = dataset.ray_rad.device
        n = len(dataset)
        self.pred_pixels = {k: torch.zeros(n, device=dev) for k in _PROGRESS_KEYS}
        self._touched = torch.zeros(n, device=dev, dtype=torch.bool)

    # ------------------------------------------------------------------ one step
    def _step(self, batch: dict, loss_ring: torch.Tensor, slot: int) -> None:
        results = self.pipeline.forward(batch)
        loss = self.pipeline.compute_loss(batch, results)
        if self.bucket is not None:
            self.bucket.zero()
        else:
            self.optimizer.zero_grad()
        loss.backward()
        if self.bucket is not None:
            self.bucket.all_reduce()
        self.optimizer.step()
        loss_ring[slot] = loss.detach().float()
        idx, ii = batch["idx"], batch["irgb_idx"][:, None]
        with torch.no_grad():
            for k in _PROGRESS_KEYS:
                if k in results:
                    self.pred_pixels[k][idx] = torch.take_along_dim(
                        results[k], ii, dim=1)[:, 0].float()
            self._touched[idx] = True

    def _gather_progress(self) -> None:
        """Combine the ranks' progress buffers: each ray takes the value of the rank that
        processed it this epoch (every rank visits a disjoint slice)."""
        if not self.distributed or self.world_size == 1:
            self._touched.zero_()
            return
        mask = self._touched.float()
        cnt = mask.clone()
        dist.all_reduce(cnt)
        for k in _PROGRESS_KEYS:
            v = self.pred_pixels[k] * mask
            dist.all_reduce(v)
            self.pred_pixels[k] = torch.where(cnt > 0, v / cnt.clamp(min=1), self.pred_pixels[k])
        self._touched.zero_()

    # ------------------------------------------------------------------ loop
    def train(self, output_path: Path | str | None = None, profile: bool = False) -> None:
        """trainer.py:70-187."""
        output_path = Path(output_path) if output_path is not None else None
        if output_path is not None:
            output_path.mkdir(parents=True, exist_ok=True)
        prof = self.get_profiler() if profile else None
        if prof:
            prof.start()
        pf = int(self.config["print_frequency"])
        num_iters = int(self.config["num_iters"])
        sch = self.config["scheduler"]
        dev = self.dataset.ray_rad.device
        loss_ring = torch.zeros(pf, device=dev)
        running: list[float] = []
        ring_start = self.iter_count
        while self.iter_count < num_iters:
            for batch in self.dataloader:
                if prof:
                    prof.step()
                self._step(batch, loss_ring, (self.iter_count - ring_start) % pf)
                self.iter_count += 1
                if (sch["type"] == "fixed" and self.iter_count % sch["decay_interval"] == 0
                        and self.iter_count > sch["decay_start"]):
                    self.scheduler.step()
                done = self.iter_count >= num_iters
                if self.iter_count - ring_start == pf or done:
                    self._flush_losses(loss_ring, self.iter_count - ring_start, running)
                    ring_start = self.iter_count
                    if self.verbose and self.rank == 0 and not done:
                        mean_loss = sum(running) / len(running)
                        print(f"{self.iter_count}/{num_iters} | Loss: {mean_loss:.5f}", end="\r")
                if done:
                    break
            self.epoch_idx += 1
            if sch["type"] == "target_lr":
                self.scheduler.step()
            self._end_epoch(output_path)
            if prof:
                prof.stop()
                prof = None
        if self.verbose and self.rank == 0:
            print()

    def _flush_losses(self, ring: torch.Tensor, n: int, running: list[float]) -> None:
        vals = ring[:n].tolist()  # the one host sync per print_frequency steps
        start = self.iter_count - n
        if self.writer is not None:
            for i, v in enumerate(vals):
                self.writer.add_scalar("Loss", v, start + i)
        running.extend(vals)
        del running[: max(0, len(running) - int(self.config["print_frequency"]) - 1)]
        zr = getattr(self.pipeline, "zero_rays_total", 0)  # reference numerics only
        if zr and zr != getattr(self, "_zero_rays_seen", 0):
            self._zero_rays_seen = zr
            import warnings

            warnings.warn(f"numerics='reference': {zr} rays so far had an f16 alpha of exactly "
                          "1 and trained with zero gradients (torch's zero-input cumprod "
                          "backward is not reproduced)", RuntimeWarning)
            if self.writer is not None:
                self.writer.add_scalar("ZeroGradRays", zr, self.iter_count)

    def _end_epoch(self, output_path: Path | None) -> None:
        self._gather_progress()
        if self.rank == 0:
            pred_img = self.dataset.scatter_image(self.pred_pixels["color_map_fine"])
            target_img = self.dataset.target_image()
            metrics = self.dataset.get_image_metrics(pred_img, target_img)
            line = f"Epoch {self.epoch_idx}/{self.num_epochs}"
            for name, val in metrics.items():
                if isinstance(val, list):
                    continue
                line += f" | {name}: {val:.3f}"
                if self.writer is not None:
                    self.writer.add_scalar(name, val, self.epoch_idx)
            self.history.append({"epoch": self.epoch_idx, "iter": self.iter_count, **metrics})
            if self.verbose:
                print(line)
            if output_path is not None:
                self.save(output_path, self.epoch_idx)

    def get_profiler(self) -> torch.profiler.profile:
        """trainer.py:189-206."""
        return torch.profiler.profile(
            activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA],
            schedule=torch.profiler.schedule(wait=2, warmup=2, active=10, repeat=1),
            on_trace_ready=torch.profiler.tensorboard_trace_handler(str(self.log_dir)),
            record_shapes=True)

    # ------------------------------------------------------------------ checkpoints
    def save(self, output_path: Path | str, epoch: int) -> Path:
        """trainer.py:208-229 (the log dir is stored as a string)."""
        path = Path(output_path) / f"epoch_{epoch:04d}.pt"
        torch.save({
            "pipeline": self.pipeline.state_dict(),
            "optimizer": self.optimizer.state_dict(),
            "scheduler": self.scheduler.state_dict(),
            "tensorboard_dir": str(self.log_dir),
            "epoch_idx": self.epoch_idx,
            "iter_count": self.iter_count,
        }, path)
        return path

    def load(self, output_path: Path | str) -> None:
        """trainer.py:231-274: resume from the newest epoch_XXXX.pt (weights_only load)."""
        ckpts = list(Path(output_path).glob("epoch_*.pt"))
        if not ckpts:
            raise FileNotFoundError(f"no epoch_*.pt checkpoint in {output_path}")
        last = sorted(ckpts, key=lambda c: int(c.stem.split("_")[1]))[-1]
        ckpt = torch.load(last, weights_only=True, map_location=self.dataset.ray_rad.device)
        self.pipeline.load_state_dict(ckpt["pipeline"])
        self.optimizer.load_state_dict(ckpt["optimizer"])
        self.scheduler.load_state_dict(ckpt["scheduler"])
        self.log_dir = Path(ckpt["tensorboard_dir"])
        self.epoch_idx = int(ckpt["epoch_idx"])
        self.iter_count = int(ckpt["iter_count"])
        # continue the shuffle sequence where the checkpointed run left it
        self.dataloader.epoch = self.epoch_idx
        if self.bucket is not None:  # load_state_dict may have replaced .grad tensors
            self.bucket = FlatGradBucket(self.pipeline.parameters())
            self.bucket.broadcast_params(0)


def lr_at(config: dict, iters_per_epoch: int, iteration: int) -> float:
    """Closed-form learning rate the trainer's schedule gives at ``iteration`` (tests)."""
    lr0 = config["optimizer"]["lr"]
    sch = config["scheduler"]
    if sch["type"] == "fixed":
        k = sum(1 for i in range(1, iteration + 1)
                if i % sch["decay_interval"] == 0 and i > sch["decay_start"])
        return lr0 * sch["gamma"] ** k
    num_epochs = int(-(config["num_iters"] // -iters_per_epoch))
    gamma = (sch["final_lr"] / lr0) ** (1 / num_epochs)
    return lr0 * gamma ** (iteration // iters_per_epoch)


__all__ = ["Trainer", "ScalarLog", "lr_at"]
