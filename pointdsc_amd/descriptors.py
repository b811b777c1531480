"""Descriptor stage on the GPU: what demo_registration.py:
37-44 and misc/cal_fpfh.py:7-36 of AmnonDrory/PointDSC do through open3d --
read a PLY, estimate normals, voxel-downsample, compute FPFH -- on the gfx950
kernels of ``libpdsc.so`` (include/pdsc.h, f4).  open3d is not needed; its
algorithms are restated and the choices it leaves to its containers are fixed
(voxel order, tie order, normal sign: include/pdsc.h).

There is no CPU path: tensors must be HIP device tensors.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check
from .kernels import _dev, _p, _stream, _workspace

FPFH_DIM = 33


def read_ply(path: str) -> np.ndarray:
    """o3d.io.read_point_cloud(path).points as float32 [n,3] host memory (binary
    little-endian or ascii PLY, vertex x/y/z)."""
    L = _lib.load()
    n = ctypes.c_int64()
    check(L.pdsc_ply_read_xyz(str(path).encode(), None, 0, ctypes.byref(n)), "pdsc_ply_read_xyz")
    out = np.empty((n.value, 3), np.float32)
    check(L.pdsc_ply_read_xyz(str(path).encode(), out.ctypes.data_as(ctypes.c_void_p), n.value, ctypes.byref(n)),
          "pdsc_ply_read_xyz")
    return out


def radius_knn(points: torch.Tensor, radius: float, max_nn: int):
    """KDTreeSearchParamHybrid(radius, max_nn) for every point: (nbr int32 [n,K],
    dist2 fp64 [n,K], count int32 [n]); neighbours ascending by (d^2, index),
    the point itself first, -1 padded."""
    points = _dev(points, "points")
    n = points.shape[0]
    L = _lib.load()
    nb = L.pdsc_radius_knn_workspace_bytes(n)
    ws = _workspace(nb, points.device)
    nbr = torch.empty((n, max_nn), dtype=torch.int32, device=points.device)
    d2 = torch.empty((n, max_nn), dtype=torch.float64, device=points.device)
    cnt = torch.empty((n,), dtype=torch.int32, device=points.device)
    check(L.pdsc_radius_knn(_p(points), n, float(radius), int(max_nn), _p(nbr), _p(d2), _p(cnt), _p(ws), nb,
                            _stream(points.device)), "pdsc_radius_knn")
    return nbr, d2, cnt


ORIENT = {"open3d": 0, "viewpoint": 1, "centroid": 2}  # enum pdsc_normal_orientation


def estimate_normals(points: torch.Tensor, radius: float, max_nn: int = 30, viewpoint=None,
                     orient: str | None = None) -> torch.Tensor:
    """pcd.estimate_normals(KDTreeSearchParamHybrid(radius, max_nn)) (utils/pointcloud.py:20-21):
    unit normals [n,3] with open3d 0.9's sign (its FastEigen3x3: n_x >= 0) by
    default; orient='viewpoint' (or a `viewpoint` given) flips them towards
    `viewpoint` (3 floats), orient='centroid' towards the cloud's centroid."""
    points = _dev(points, "points")
    if orient is None:
        orient = "viewpoint" if viewpoint is not None else "open3d"
    if orient not in ORIENT:
        raise ValueError(f"orient must be one of {sorted(ORIENT)}, got {orient!r}")
    if orient == "viewpoint" and viewpoint is None:
        raise ValueError("orient='viewpoint' needs a viewpoint")
    n = points.shape[0]
    L = _lib.load()
    nb = L.pdsc_estimate_normals_workspace_bytes(n, int(max_nn))
    ws = _workspace(nb, points.device)
    vp = None
    if viewpoint is not None:
        vp = torch.as_tensor(np.asarray(viewpoint, np.float32).reshape(3), device=points.device)
    out = torch.empty_like(points)
    check(L.pdsc_estimate_normals(_p(points), n, float(radius), int(max_nn), ORIENT[orient], _p(vp), _p(out), _p(ws),
                                  nb, _stream(points.device)), "pdsc_estimate_normals")
    return out


def voxel_down_sample(points: torch.Tensor, voxel_size: float, normals: torch.Tensor | None = None):
    """pcd.voxel_down_sample(voxel_size): (points [m,3], normals [m,3] | None),
    voxels in ascending key order (open3d: its hash map's order)."""
    points = _dev(points, "points")
    n = points.shape[0]
    if normals is not None:
        normals = _dev(normals, "normals")
        if normals.shape != points.shape:
            raise ValueError(f"normals {tuple(normals.shape)} != points {tuple(points.shape)}")
    L = _lib.load()
    nb = L.pdsc_voxel_down_sample_workspace_bytes(n)
    ws = _workspace(nb, points.device)
    op = torch.empty_like(points)
    on = torch.empty_like(points) if normals is not None else None
    cnt = torch.empty((1,), dtype=torch.int32, device=points.device)
    check(L.pdsc_voxel_down_sample(_p(points), _p(normals), n, float(voxel_size), _p(op), _p(on), _p(cnt), _p(ws),
                                   nb, _stream(points.device)), "pdsc_voxel_down_sample")
    m = int(cnt.item())
    return op[:m], (on[:m] if on is not None else None)


def compute_fpfh(points: torch.Tensor, normals: torch.Tensor, radius: float, max_nn: int = 100):
    """o3d compute_fpfh_feature(pcd, KDTreeSearchParamHybrid(radius, max_nn)):
    (fpfh fp64 [n,33] = np.array(feature.data).T, the L2-normalised fp32 copy
    f / (||f|| + 1e-6) of demo_registration.py:42)."""
    points, normals = _dev(points, "points"), _dev(normals, "normals")
    if normals.shape != points.shape:
        raise ValueError(f"normals {tuple(normals.shape)} != points {tuple(points.shape)}")
    n = points.shape[0]
    L = _lib.load()
    nb = L.pdsc_compute_fpfh_workspace_bytes(n, int(max_nn))
    ws = _workspace(nb, points.device)
    f = torch.empty((n, FPFH_DIM), dtype=torch.float64, device=points.device)
    fn = torch.empty((n, FPFH_DIM), dtype=torch.float32, device=points.device)
    check(L.pdsc_compute_fpfh(_p(points), _p(normals), n, float(radius), int(max_nn), _p(f), _p(fn), _p(ws), nb,
                              _stream(points.device)), "pdsc_compute_fpfh")
    return f, fn


def extract_fpfh_features(pcd_path: str, downsample: float, device, orient: str = "open3d"):
    """demo_registration.py:37-44 on the GPU: normals on the raw cloud (radius
    2 v, 30 nearest; open3d 0.9's unoriented sign), voxel downsample (normals
    summed and normalised), FPFH (radius 5 v,
    100 nearest), L2-normalised.  Returns (raw points [n,3], downsampled
    points [m,3], features fp32 [m,33]) as device tensors."""
    raw = torch.from_numpy(read_ply(pcd_path)).to(device)
    nrm = estimate_normals(raw, radius=downsample * 2, max_nn=30, orient=orient)
    pts, pn = voxel_down_sample(raw, downsample, nrm)
    _, feats = compute_fpfh(pts, pn, radius=downsample * 5, max_nn=100)
    return raw, pts, feats
