"""MI355X-native differentiable Gaussian-splatting rasterizer.

Drop-in for the render path of Loveof1ife7/mini-3d-gaussian-splatting:
GaussianRenderer.render() (src/core/renderer.py) and the GaussianModel /
Camera interfaces it reads.  Compute runs only in the hand-written HIP
library libgsplat_mi355x.so (csrc/, C ABI in include/gsplat_mi355x.h).
"""
from .renderer import GaussianRenderer, RenderSettings, camera_params  # noqa: F401
from .gaussian_model import GaussianModel, build_rotation_matrix  # noqa: F401
from .camera import Camera, CameraUtils  # noqa: F401
from .rasterizer import CameraParams, rasterize  # noqa: F401
from .loss import SSIMLoss, GaussianLoss, photometric_loss  # noqa: F401
from .config import TrainingConfig, ConfigManager  # noqa: F401
from .dataset import CameraDataset, NeRFSyntheticDataset, COLMAPDataset, load_dataset  # noqa: F401
from .trainer import GaussianTrainer  # noqa: F401
from .graph_step import GraphedStep  # noqa: F401
from . import _native, synthetic, distributed, optim, loss, dataset, trainer, graph_step  # noqa: F401

__all__ = ["GaussianRenderer", "RenderSettings", "GaussianModel", "Camera", "CameraUtils",
           "CameraParams", "rasterize", "camera_params", "SSIMLoss", "GaussianLoss", "photometric_loss",
           "TrainingConfig", "ConfigManager", "CameraDataset", "NeRFSyntheticDataset", "COLMAPDataset",
           "load_dataset", "GaussianTrainer", "GraphedStep"]
