"""GaussianTrainer (reference src/train/trainer.py:12-89, whose methods are
all `pass`).

One iteration: pick a training camera, render it (HIP path), fused L1 +
D-SSIM against its image, backward, [N > 1: one RCCL mean all-reduce of the
Gaussian gradients], learning-rate schedule, FusedAdam step, and density
control every densify_interval iterations inside [densify_from_iter,
densify_until_iter] (optimizer.py:34-141).  Nothing in a step reads a value
back to the host; losses are logged every log_interval iterations.

Data parallel: with torch.distributed initialised,
rank r renders camera perm[(i * world + r) mod n] at iteration i; every rank
applies the same averaged gradients and the same densification (the
gradients are identical after the all-reduce and the clone jitter is seeded
by the iteration), so the replicas stay bit-identical.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import numpy as np
import torch

from .config import TrainingConfig
from .dataset import CameraDataset, load_dataset
from .gaussian_model import GaussianModel
from .loss import photometric_loss
from .optim import GaussianOptimizer
from .renderer import GaussianRenderer, RenderSettings


class GaussianTrainer:
    def __init__(self, config: TrainingConfig, dataset: Optional[CameraDataset] = None):
        self.config = config
        self.dataset: Optional[CameraDataset] = dataset
        self.gaussians: Optional[GaussianModel] = None
        self.renderer = GaussianRenderer()
        self.optimizer: Optional[GaussianOptimizer] = None
        self.iteration = 0
        self.scene_extent = 0.0
        self.train_losses: List[float] = []
        self.val_losses: List[float] = []
        self._dist = None
        self._reducer = None
        self._reducer_n = -1
        self._perm: Optional[np.ndarray] = None

    # -- setup (trainer.py:32-44) ------------------------------------------
    def _device(self) -> torch.device:
        c = self.config
        return torch.device(c.device if c.device != "cuda" else f"cuda:{torch.cuda.current_device()}")

    def _setup_run(self) -> None:
        """Everything but the model: dataset, process group, scene extent and
        the camera order -- shared by setup() and load_checkpoint() (a resumed
        run needs them as much as a fresh one)."""
        c = self.config
        if self.dataset is None:
            self.dataset = load_dataset(c.data_path, device=self._device())
        if torch.distributed.is_available() and torch.distributed.is_initialized() and \
                torch.distributed.get_world_size() > 1:
            self._dist = torch.distributed
        self.scene_extent = self.get_scene_extent()
        n = len(self.dataset.get_train_cameras())
        self._perm = np.random.default_rng(c.seed).permutation(n)

    def setup(self) -> None:
        c = self.config
        dev = self._device()
        self._setup_run()
        g = GaussianModel(c)
        gen = torch.Generator().manual_seed(c.seed)
        if self.dataset.points is not None and len(self.dataset.points):
            g.create_from_points(torch.from_numpy(self.dataset.points).to(dev),
                                 torch.from_numpy(self.dataset.colors).to(dev) if self.dataset.colors is not None else None)
        else:
            # Blender scenes have no points: uniform in [-1.3, 1.3]^3 (the NeRF-synthetic object box)
            g.create_from_random(c.num_random_points, scene_extent=1.3, device=dev, generator=gen)
        self.gaussians = g
        self.optimizer = GaussianOptimizer(g, c)
        self.optimizer.setup_optimizer()

    def get_scene_extent(self) -> float:
        """trainer.py:87-89: camera-centre radius (get_scene_info)."""
        return float(self.dataset.get_scene_info()["radius"])

    def _settings(self, cam) -> RenderSettings:
        return RenderSettings(image_height=cam._height, image_width=cam._width, bg_color=torch.zeros(3))

    def _camera_for(self, it: int):
        cams = self.dataset.get_train_cameras()
        world = self._dist.get_world_size() if self._dist else 1
        rank = self._dist.get_rank() if self._dist else 0
        return cams[int(self._perm[(it * world + rank) % len(cams)])]

    # -- one step (trainer.py:65-69) ---------------------------------------
    def train_step(self, camera) -> Dict[str, torch.Tensor]:
        g, opt = self.gaussians, self.optimizer
        c = self.config
        if (c.sh_degree > g.active_sh_degree and c.sh_increase_interval > 0
                and self.iteration > 0 and self.iteration % c.sh_increase_interval == 0):
            g.max_sh_degree = max(g.max_sh_degree, c.sh_degree)
            g.oneup_sh_degree()
        opt.zero_grad()
        if self._dist is not None:
            # the bucket is attached before the render, so that its backward
            # writes the gradients into it and reduces them range by range
            params = g.grad_parameters()
            if self._reducer is None or self._reducer_n != g.get_num_points():
                from .distributed import GradAllReduce
                self._reducer = GradAllReduce(params, self._dist).attach(g)
                self._reducer_n = g.get_num_points()
            self._reducer.params = params
        out = self.renderer.render(camera, g, self._settings(camera))
        target = camera._image
        total, l1, dssim = photometric_loss(out["image"], target, self.config.lambda_dssim)
        total.backward()
        opt.update_learning_rate(self.iteration)
        if self._dist is not None:
            # mean all-reduce, then Adam; pipelined per Gaussian range when the
            # backward handed its rows over in ranges (GS_ALLREDUCE_CHUNKS)
            self._reducer.reduce_and_step(opt.optimizer)
        else:
            opt.step()
        info = opt.densify_and_prune(self.iteration, self.scene_extent)
        if info is not None:
            self._reducer = None
        return {"loss": total.detach(), "l1": l1, "dssim": dssim}

    def close(self) -> None:
        """Tear down the data-parallel transport: the native RCCL communicators
        go before the caller destroys the process group (every rank calls this
        at the same point, after its last step).  Also registered at exit by
        distributed._native_comm."""
        if self._dist is not None:
            from .distributed import close_native_comms
            close_native_comms()
        self._reducer = None

    # -- loop (trainer.py:46-63) -------------------------------------------
    def train(self, iterations: Optional[int] = None) -> None:
        if self.gaussians is None:
            self.setup()
        elif self._perm is None:
            self._setup_run()
        n = self.config.iterations if iterations is None else iterations
        for _ in range(n):
            self.iteration += 1
            st = self.train_step(self._camera_for(self.iteration))
            if self.iteration % self.config.log_interval == 0:
                self.train_losses.append(float(st["loss"]))

    @torch.no_grad()
    def validate(self) -> Dict[str, float]:
        """trainer.py:71-75: mean PSNR and loss over the test cameras (train if none)."""
        cams = self.dataset.get_test_cameras() or self.dataset.get_train_cameras()
        psnr, loss = [], []
        for cam in cams:
            img = self.renderer.render(cam, self.gaussians, self._settings(cam))["image"]
            mse = torch.mean((img - cam._image) ** 2)
            psnr.append(-10.0 * torch.log10(mse.clamp_min(1e-12)))
            loss.append(photometric_loss(img, cam._image, self.config.lambda_dssim)[0])
        out = {"psnr": float(torch.stack(psnr).mean()), "loss": float(torch.stack(loss).mean()),
               "num_gaussians": self.gaussians.get_num_points()}
        self.val_losses.append(out["loss"])
        return out

    # -- checkpoints (trainer.py:77-85): safetensors, no pickle --------------
    def _ckpt_path(self, iteration: int) -> str:
        return os.path.join(self.config.output_path, f"ckpt_{iteration:06d}.safetensors")

    def save_checkpoint(self, iteration: int) -> str:
        from safetensors.torch import save_file
        os.makedirs(self.config.output_path, exist_ok=True)
        names = ["xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity"]
        tensors = {}
        for name, p in zip(names, self.gaussians.parameter_list()):
            tensors[name] = p.detach().contiguous()
            st = self.optimizer.optimizer.state.get(p, {})
            if "exp_avg" in st:
                tensors[f"adam.{name}.m"] = st["exp_avg"].contiguous()
                tensors[f"adam.{name}.v"] = st["exp_avg_sq"].contiguous()
                tensors[f"adam.{name}.step"] = torch.tensor([st["step"]], dtype=torch.int64)
        path = self._ckpt_path(iteration)
        save_file({k: v.cpu() for k, v in tensors.items()}, path,
                  metadata={"iteration": str(iteration), "active_sh_degree": str(self.gaussians.active_sh_degree)})
        return path

    def load_checkpoint(self, iteration: int) -> None:
        from safetensors import safe_open
        path = self._ckpt_path(iteration)
        dev = self.gaussians._xyz.device if self.gaussians is not None else torch.device("cuda")
        with safe_open(path, framework="pt") as f:
            t = {k: f.get_tensor(k) for k in f.keys()}
            meta = f.metadata() or {}
        if self.gaussians is None:
            self.gaussians = GaussianModel(self.config)
        names = ["xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity"]
        self.gaussians._set(*[t[n].to(dev) for n in names])
        self.optimizer = GaussianOptimizer(self.gaussians, self.config)
        self.optimizer.setup_optimizer()
        for name, p in zip(names, self.gaussians.parameter_list()):
            if f"adam.{name}.m" in t:
                self.optimizer.optimizer.state[p] = {"step": int(t[f"adam.{name}.step"][0]),
                                                     "exp_avg": t[f"adam.{name}.m"].to(dev),
                                                     "exp_avg_sq": t[f"adam.{name}.v"].to(dev)}
        self.iteration = int(meta.get("iteration", iteration))
        self.gaussians.active_sh_degree = int(meta.get("active_sh_degree", 0))
        self._reducer = None
        if self._perm is None:
            self._setup_run()


__all__ = ["GaussianTrainer", "TrainingConfig"]
