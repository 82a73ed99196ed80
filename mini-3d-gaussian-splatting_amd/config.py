"""TrainingConfig (reference config/config.py:33-67), flat, no import-time
side effects (the reference prints on import, :97-98).  Fields and defaults
are the reference's; the few the trainer adds are marked."""
from __future__ import annotations

from dataclasses import asdict, dataclass, fields

import yaml


@dataclass
class TrainingConfig:
    data_path: str = "data/scene"
    output_path: str = "output"

    iterations: int = 30000
    learning_rate: float = 0.0025
    batch_size: int = 1

    position_lr_init: float = 0.00016
    position_lr_final: float = 0.0000016
    position_lr_delay_mult: float = 0.01
    position_lr_max_steps: int = 30000

    feature_lr: float = 0.0025
    opacity_lr: float = 0.05
    scaling_lr: float = 0.005
    rotation_lr: float = 0.001

    densify_from_iter: int = 500
    densify_until_iter: int = 15000
    densify_grad_threshold: float = 0.0002
    densify_interval: int = 100

    image_height: int = 800
    image_width: int = 800

    device: str = "cuda"

    # added by this trainer (not in the reference config)
    lambda_dssim: float = 0.2          # loss.py:42 default
    num_random_points: int = 100_000   # random init when the dataset has no points
    min_opacity: float = 0.01          # optimizer.py:64
    test_every: int = 8                # every k-th camera held out when a dataset has no test split
    log_interval: int = 100
    seed: int = 0
    sh_degree: int = 0                 # max SH degree of the colour (0 = the reference's DC-only render)
    sh_increase_interval: int = 1000   # active SH degree +1 every this many iterations, up to sh_degree


class ConfigManager:
    """config.py:69-95: YAML load / save of the flat config (unknown keys are
    rejected instead of silently ignored)."""

    @staticmethod
    def load(path: str) -> TrainingConfig:
        with open(path) as f:
            data = yaml.safe_load(f) or {}
        names = {f.name for f in fields(TrainingConfig)}
        unknown = sorted(set(data) - names)
        if unknown:
            raise KeyError(f"unknown config keys: {unknown}")
        return TrainingConfig(**data)

    @staticmethod
    def save(cfg: TrainingConfig, path: str) -> None:
        with open(path, "w") as f:
            yaml.safe_dump(asdict(cfg), f, sort_keys=False)
