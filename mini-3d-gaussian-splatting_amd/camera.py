"""Camera record + W2C builder (reference src/core/camera.py:5-141).

The reference renderer calls `camera.world_view_transform()` (renderer.py:150)
while the reference Camera defines it as a (broken) property (camera.py:45-50).
Here it is a method returning the 4x4 W2C built by
CameraUtils.build_world_view_matrix (camera.py:80-141); the renderer accepts
either form.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch


class CameraUtils:
    @staticmethod
    def build_world_view_matrix(R_np, T_np, from_c2w: bool, device=None, dtype=None) -> torch.Tensor:
        """C2W (R_cw, C_w) -> [[R_cw^T, -R_cw^T C_w],[0,1]]; W2C passes through."""
        R = torch.as_tensor(np.asarray(R_np)).reshape(3, 3)
        T = torch.as_tensor(np.asarray(T_np)).reshape(3, 1)
        if dtype is not None:
            R, T = R.to(dtype), T.to(dtype)
        if device is not None:
            R, T = R.to(device), T.to(device)
        view = torch.eye(4, device=R.device, dtype=R.dtype)
        if from_c2w:
            Rwc = R.transpose(0, 1)
            t = -(Rwc @ T).flatten()
        else:
            Rwc, t = R, T.flatten()
        view[:3, :3] = Rwc
        view[:3, 3] = t
        return view


class Camera:
    def __init__(self, uid: int, R: np.ndarray, T: np.ndarray, FoVx: float, FoVy: float,
                 image: Optional[torch.Tensor], image_name: str, width: int, height: int,
                 from_c2w: bool = True):
        self._uid = uid
        self._R = torch.from_numpy(np.asarray(R, np.float32))
        self._T = torch.from_numpy(np.asarray(T, np.float32))
        self._FoVx, self._FoVy = float(FoVx), float(FoVy)
        self._image, self._image_name = image, image_name
        self._width, self._height = int(width), int(height)
        self._from_c2w = from_c2w
        self._wv: Optional[torch.Tensor] = None

    def world_view_transform(self) -> torch.Tensor:
        if self._wv is None:
            self._wv = CameraUtils.build_world_view_matrix(self._R.numpy(), self._T.numpy(), self._from_c2w)
        return self._wv

    @property
    def camera_center(self) -> torch.Tensor:
        wv = self.world_view_transform()
        return -(wv[:3, :3].T @ wv[:3, 3])
