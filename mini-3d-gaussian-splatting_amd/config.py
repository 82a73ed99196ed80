"""TrainingConfig (reference config/config.py:33-67), flat, no import-time
side effects (the reference prints on import, :97-98).  Fields and defaults
are the reference's; the few the trainer adds are marked."""
from __future__ import annotations

from dataclasses import asdict, dataclass, fields
from pathlib import Path

try:  # optional, as in the reference (config.py:1-8)
    import yaml
except ImportError:  # pragma: no cover
    yaml = None


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
    # after a densification the reference builds a fresh Adam (optimizer.py:133-137: moments and step
    # counts dropped); False keeps the kept Gaussians' moments (new ones start at zero)
    reset_adam_on_densify: bool = False


def _need_yaml():
    if yaml is None:
        raise ImportError("PyYAML is not installed")


class ConfigManager:
    """config.py:69-95: YAML load / save of the flat config (unknown keys are
    rejected instead of silently ignored).  The reference's names
    (load_from_yaml, save_to_yaml, get_default_config) and short aliases."""

    @staticmethod
    def load_from_yaml(config_path: str) -> TrainingConfig:
        _need_yaml()
        with open(config_path, encoding="utf-8") as f:
            data = yaml.safe_load(f) or {}
        names = {f.name for f in fields(TrainingConfig)}
        unknown = sorted(set(data) - names)
        if unknown:
            raise KeyError(f"unknown config keys: {unknown}")
        return TrainingConfig(**data)

    @staticmethod
    def save_to_yaml(config: TrainingConfig, config_path: str) -> None:
        _need_yaml()
        Path(config_path).parent.mkdir(parents=True, exist_ok=True)
        with open(config_path, "w", encoding="utf-8") as f:
            yaml.safe_dump(asdict(config), f, sort_keys=False, allow_unicode=True)

    @staticmethod
    def get_default_config() -> TrainingConfig:
        return TrainingConfig()

    load = load_from_yaml
    save = save_to_yaml
