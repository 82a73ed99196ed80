"""Camera datasets for training (reference src/data/dataset.py:6-61, whose
classes are stubs).

  NeRFSyntheticDataset: Blender-format scenes (transforms_{train,test}.json,
      camera_angle_x, OpenGL camera-to-world transform_matrix, RGBA PNGs).
  COLMAPDataset: COLMAP text models (sparse/0 or sparse/: cameras.txt,
      images.txt, points3D.txt) with the images they name.

Poses are converted to the renderer's camera frame (renderer.py:150-162:
X right, Y up, +Z forward, pixel y = -fy Y/Z + cy): OpenGL cameras look down
-Z (flip Z), COLMAP cameras have Y down (flip Y).  Images become [3,H,W]
fp32 tensors in [0,1]; RGBA is composited over the background colour.

Background: the reference blend adds bg twice (renderer.py:273 and :359), so
with a white background every pixel saturates at 1 and no gradient reaches
the Gaussians.  Training therefore composites on black by default.
"""
from __future__ import annotations

import json
import math
from pathlib import Path
from typing import Dict, List, Optional

import numpy as np
import torch

from .camera import Camera


def _load_image(path: Path, bg: np.ndarray) -> np.ndarray:
    from PIL import Image
    with Image.open(path) as im:
        a = np.asarray(im.convert("RGBA") if im.mode in ("RGBA", "LA", "P") else im.convert("RGB"), np.float32) / 255.0
    if a.shape[-1] == 4:
        a = a[..., :3] * a[..., 3:4] + bg[None, None, :] * (1.0 - a[..., 3:4])
    return np.ascontiguousarray(a.transpose(2, 0, 1))


def _fov(focal: float, pixels: int) -> float:
    return 2.0 * math.atan(pixels / (2.0 * focal))


class CameraDataset:
    """dataset.py:6-28"""

    def __init__(self, data_path: str, white_background: bool = False, device=None):
        self.data_path = Path(data_path)
        self.bg = np.ones(3, np.float32) if white_background else np.zeros(3, np.float32)
        self.device = torch.device(device) if device is not None else None
        self.cameras: List[Camera] = []
        self.train_cameras: List[Camera] = []
        self.test_cameras: List[Camera] = []
        self.points: Optional[np.ndarray] = None   # [P,3] initial point cloud, if the format has one
        self.colors: Optional[np.ndarray] = None   # [P,3] in [0,1]

    def load_cameras(self) -> None:
        raise NotImplementedError

    def _camera(self, uid, R, T, fovx, fovy, path: Path, w, h, from_c2w) -> Camera:
        img = torch.from_numpy(_load_image(path, self.bg))
        if self.device is not None:
            img = img.to(self.device)
        h_img, w_img = img.shape[1:]
        return Camera(uid, R, T, fovx, fovy, img, path.stem, w_img if w is None else w, h_img if h is None else h,
                      from_c2w=from_c2w)

    def split_train_test(self, split_ratio: float) -> None:
        """Every k-th camera (k = round(1 / split_ratio)) goes to test."""
        k = max(2, int(round(1.0 / split_ratio))) if split_ratio > 0 else 0
        self.train_cameras = [c for i, c in enumerate(self.cameras) if not k or i % k != 0]
        self.test_cameras = [c for i, c in enumerate(self.cameras) if k and i % k == 0]

    def get_train_cameras(self) -> List[Camera]:
        return self.train_cameras

    def get_test_cameras(self) -> List[Camera]:
        return self.test_cameras

    def get_scene_info(self) -> Dict[str, object]:
        """Camera-centre bounds (3DGS getNerfppNorm): centre, radius = 1.1 x max distance."""
        cams = self.train_cameras or self.cameras
        centers = np.stack([c.camera_center.numpy() for c in cams]) if cams else np.zeros((1, 3))
        center = centers.mean(0)
        radius = float(np.linalg.norm(centers - center, axis=1).max() * 1.1) if len(cams) > 1 else 1.0
        return {"center": center, "radius": max(radius, 1e-6), "num_train": len(self.train_cameras),
                "num_test": len(self.test_cameras)}


class NeRFSyntheticDataset(CameraDataset):
    """Blender scenes: transforms_{train,test}.json + PNGs."""

    def load_cameras(self) -> None:
        self.train_cameras = self._read("transforms_train.json", 0)
        self.test_cameras = self._read("transforms_test.json", len(self.train_cameras))
        self.cameras = self.train_cameras + self.test_cameras

    def _read(self, name: str, uid0: int) -> List[Camera]:
        path = self.data_path / name
        if not path.exists():
            return []
        meta = json.loads(path.read_text())
        fovx = float(meta["camera_angle_x"])
        out = []
        for i, fr in enumerate(meta["frames"]):
            img_path = self.data_path / (fr["file_path"] if Path(fr["file_path"]).suffix else fr["file_path"] + ".png")
            c2w = np.asarray(fr["transform_matrix"], np.float64).reshape(4, 4)
            R = c2w[:3, :3] @ np.diag([1.0, 1.0, -1.0])   # OpenGL -> +Z forward, Y up
            C = c2w[:3, 3]
            cam = self._camera(uid0 + i, R, C, fovx, fovx, img_path, None, None, True)
            cam._FoVy = 2.0 * math.atan(math.tan(fovx / 2) * cam._height / cam._width)
            out.append(cam)
        return out


def _qvec2rotmat(q):
    w, x, y, z = q
    return np.array([
        [1 - 2 * y * y - 2 * z * z, 2 * x * y - 2 * w * z, 2 * z * x + 2 * w * y],
        [2 * x * y + 2 * w * z, 1 - 2 * x * x - 2 * z * z, 2 * y * z - 2 * w * x],
        [2 * z * x - 2 * w * y, 2 * y * z + 2 * w * x, 1 - 2 * x * x - 2 * y * y]])


class COLMAPDataset(CameraDataset):
    """dataset.py:30-61: COLMAP text model + images (PINHOLE / SIMPLE_PINHOLE /
    SIMPLE_RADIAL / RADIAL / OPENCV read as pinhole; the renderer puts the
    principal point at the image centre, renderer.py:146-147)."""

    def __init__(self, data_path: str, white_background: bool = False, device=None, images_dir: str = "images",
                 test_every: int = 8):
        super().__init__(data_path, white_background, device)
        self.images_dir, self.test_every = images_dir, test_every

    def _sparse(self) -> Path:
        for cand in (self.data_path / "sparse" / "0", self.data_path / "sparse", self.data_path):
            if (cand / "cameras.txt").exists():
                return cand
        raise FileNotFoundError(f"no cameras.txt under {self.data_path}")

    def load_cameras(self) -> None:
        sp = self._sparse()
        intr = self._read_cameras_txt(sp / "cameras.txt")
        imgs = self._read_images_txt(sp / "images.txt")
        pts = sp / "points3D.txt"
        if pts.exists():
            self.points, self.colors = self._read_points3d_txt(pts)
        cams = []
        for uid, (q, t, cam_id, name) in enumerate(sorted(imgs.values(), key=lambda v: v[3])):
            w, h, fx, fy = intr[cam_id]
            R = np.diag([1.0, -1.0, 1.0]) @ _qvec2rotmat(q)   # W2C, COLMAP Y down -> Y up
            T = np.diag([1.0, -1.0, 1.0]) @ np.asarray(t)
            cams.append(self._camera(uid, R, T, _fov(fx, w), _fov(fy, h), self.data_path / self.images_dir / name,
                                     w, h, False))
        self.cameras = cams
        self.split_train_test(1.0 / self.test_every if self.test_every else 0.0)

    @staticmethod
    def _lines(path: Path):
        for line in path.read_text().splitlines():
            line = line.strip()
            if line and not line.startswith("#"):
                yield line

    def _read_cameras_txt(self, path: Path) -> Dict[int, tuple]:
        out = {}
        for line in self._lines(path):
            el = line.split()
            cid, model, w, h, p = int(el[0]), el[1], int(el[2]), int(el[3]), [float(v) for v in el[4:]]
            fx, fy = (p[0], p[0]) if model in ("SIMPLE_PINHOLE", "SIMPLE_RADIAL", "RADIAL") else (p[0], p[1])
            out[cid] = (w, h, fx, fy)
        return out

    def _read_images_txt(self, path: Path) -> Dict[int, tuple]:
        """Two lines per image (the second, its 2D points, may be empty)."""
        lines = [ln.strip() for ln in path.read_text().splitlines() if not ln.lstrip().startswith("#")]
        while lines and not lines[-1]:
            lines.pop()
        out = {}
        for i in range(0, len(lines), 2):
            el = lines[i].split()
            if len(el) < 10:
                continue
            out[int(el[0])] = ([float(v) for v in el[1:5]], [float(v) for v in el[5:8]], int(el[8]), " ".join(el[9:]))
        return out

    def _read_points3d_txt(self, path: Path):
        xyz, rgb = [], []
        for line in self._lines(path):
            el = line.split()
            xyz.append([float(v) for v in el[1:4]])
            rgb.append([int(v) / 255.0 for v in el[4:7]])
        return np.asarray(xyz, np.float32).reshape(-1, 3), np.asarray(rgb, np.float32).reshape(-1, 3)

    def get_point_cloud_path(self) -> str:
        return str(self._sparse() / "points3D.txt")


def load_point_cloud(path: str):
    """(points [N,3] f32, colours [N,3] f32 in [0,1] or None) from the formats
    the reference's IOUtils.load_point_cloud reads (io_utils.py:34-83): .npz
    (points / colors, no pickles), .npy ([N,3] or [N,>=6]), COLMAP
    points3D.txt, or text lines "x y z [r g b]"."""
    p = Path(path)
    suf = p.suffix.lower()
    if suf == ".npz":
        with np.load(str(p), allow_pickle=False) as z:
            pts = z["points"] if "points" in z.files else np.zeros((0, 3), np.float32)
            cols = z["colors"] if "colors" in z.files else None
        return pts.astype(np.float32).reshape(-1, 3), None if cols is None else cols.astype(np.float32).reshape(-1, 3)
    if suf == ".npy":
        arr = np.load(str(p), allow_pickle=False)
        if arr.ndim == 2 and arr.shape[1] >= 6:
            return arr[:, :3].astype(np.float32), arr[:, 3:6].astype(np.float32)
        return arr[:, :3].astype(np.float32), None
    pts, cols = [], []
    colmap = p.name == "points3D.txt"
    with open(p, encoding="utf-8", errors="ignore") as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            el = line.split()
            if colmap:
                if len(el) < 10:
                    continue
                pts.append([float(v) for v in el[1:4]])
                cols.append([float(v) / 255.0 for v in el[4:7]])
            else:
                try:
                    v = [float(x) for x in el]
                except ValueError:
                    continue
                if len(v) >= 3:
                    pts.append(v[:3])
                    if len(v) >= 6:
                        cols.append(v[3:6])
    P = np.asarray(pts, np.float32).reshape(-1, 3)
    Cc = np.asarray(cols, np.float32).reshape(-1, 3) if cols and len(cols) == len(pts) else None
    return P, Cc


def load_dataset(path: str, white_background: bool = False, device=None) -> CameraDataset:
    """NeRF-synthetic if transforms_train.json exists, else COLMAP."""
    p = Path(path)
    ds = NeRFSyntheticDataset(path, white_background, device) if (p / "transforms_train.json").exists() \
        else COLMAPDataset(path, white_background, device)
    ds.load_cameras()
    return ds


__all__ = ["CameraDataset", "NeRFSyntheticDataset", "COLMAPDataset", "load_dataset", "load_point_cloud"]
