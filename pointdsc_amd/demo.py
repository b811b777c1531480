"""demo_registration.py of AmnonDrory/PointDSC on the MI355X path (configs[0]):
two PLY clouds -> FPFH on the GPU (pointdsc_amd.descriptors) -> nearest-
neighbour matching (pointdsc_amd.correspondence, use_mutual=False as the demo's
argmin, :101-108) -> PointDSC testing forward (:111-117).

    python -m pointdsc_amd.demo --pcd1 cloud_bin_0.ply --pcd2 cloud_bin_1.ply \\
        [--weights model_best.pkl] [--config config.json] [--out result.npz]

Differences from the reference driver, all deliberate:
  * --descriptor fcgf is refused: FCGF needs MinkowskiEngine and its release
    checkpoint (misc/fcgf.py), outside this build's scope.
  * --use_gpu False is refused: this build has no CPU execution path (the
    product never falls back to the CPU or to the test oracle); the reference
    runs the same model on the CPU there.
  * the open3d windows (:120-123) are replaced by printing final_trans and an
    optional .npz of the result (points, correspondences, labels, pose).
  * without --weights the synthetic-trained weights of pointdsc_amd.synthetic
    are used (the release checkpoint is not distributed with the reference).
"""
from __future__ import annotations

import argparse
import json
import sys

import numpy as np
import torch

# snapshot/PointDSC_3DMatch_release/config.json (the demo's default snapshot)
RELEASE_3DMATCH = {"in_dim": 6, "num_layers": 12, "num_channels": 128, "num_iterations": 10, "ratio": 0.1,
                   "k": 40, "inlier_threshold": 0.1, "sigma_d": 0.1, "downsample": 0.05}


def build_model(config: dict, weights: str | None, device):
    """PointDSC(...) as demo_registration.py:78-88 builds it (nms_radius =
    inlier_threshold, the class default inlier_threshold)."""
    from .PointDSC import PointDSC
    from .synthetic import trained_state_dict
    model = PointDSC(in_dim=config["in_dim"], num_layers=config["num_layers"],
                     num_channels=config["num_channels"], num_iterations=config["num_iterations"],
                     ratio=config["ratio"], sigma_d=config["sigma_d"], k=config["k"],
                     nms_radius=config["inlier_threshold"])
    if weights:
        sd = torch.load(weights, map_location="cpu", weights_only=True)
    else:
        sd = {k: torch.from_numpy(v) for k, v in trained_state_dict("3dmatch", config["num_layers"]).items()}
    model.load_state_dict(sd, strict=False)
    return model.to(device).eval()


def register(model, pcd1, pcd2, downsample: float, device, orient: str = "open3d"):
    """The demo's pipeline for two clouds (paths or [n,3] arrays): returns a dict
    with final_trans [4,4], final_labels [n], the correspondence inputs and the
    downsampled points / features of both clouds.  orient: the normals' sign
    (descriptors.estimate_normals; 'open3d' = the reference's)."""
    from . import descriptors as D
    from .correspondence import build_correspondences

    def feats(pcd):
        if isinstance(pcd, str):
            return D.extract_fpfh_features(pcd, downsample, device, orient)
        raw = torch.as_tensor(np.asarray(pcd, np.float32)).to(device)
        nrm = D.estimate_normals(raw, radius=downsample * 2, max_nn=30, orient=orient)
        pts, pn = D.voxel_down_sample(raw, downsample, nrm)
        return raw, pts, D.compute_fpfh(pts, pn, radius=downsample * 5, max_nn=100)[1]

    _, src_pts, src_f = feats(pcd1)
    _, tgt_pts, tgt_f = feats(pcd2)
    c = build_correspondences(src_pts, tgt_pts, src_f, tgt_f, use_mutual=False)
    with torch.no_grad():
        res = model({"corr_pos": c["corr_pos"][None], "src_keypts": c["src_keypts"][None],
                     "tgt_keypts": c["tgt_keypts"][None], "testing": True})
    return {"final_trans": res["final_trans"][0], "final_labels": res["final_labels"][0], "corr": c["corr"],
            "src_keypts": c["src_keypts"], "tgt_keypts": c["tgt_keypts"], "src_pts": src_pts, "tgt_pts": tgt_pts,
            "src_features": src_f, "tgt_features": tgt_f}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--pcd1", default="demo_data/cloud_bin_0.ply")
    ap.add_argument("--pcd2", default="demo_data/cloud_bin_1.ply")
    ap.add_argument("--descriptor", default="fpfh", choices=["fcgf", "fpfh"])
    ap.add_argument("--use_gpu", default="True")
    ap.add_argument("--config", default=None, help="a snapshot config.json (default: the 3DMatch release values)")
    ap.add_argument("--weights", default=None, help="state dict (torch.load weights_only=True)")
    ap.add_argument("--out", default=None, help="write the result arrays to this .npz")
    ap.add_argument("--normals", default="open3d", choices=["open3d", "centroid"],
                    help="normal sign: open3d 0.9's (the reference's) or towards the cloud's centroid")
    a = ap.parse_args(argv)
    if a.descriptor != "fpfh":
        sys.exit("descriptor 'fcgf' needs MinkowskiEngine and the FCGF checkpoint: out of scope (use --descriptor fpfh)")
    if a.use_gpu.lower() in ("false", "0", "no", "n", "f"):
        sys.exit("--use_gpu False: this build has no CPU execution path (see DESIGN.md)")
    config = dict(RELEASE_3DMATCH)
    if a.config:
        with open(a.config) as f:
            config.update({k: v for k, v in json.load(f).items() if k in RELEASE_3DMATCH})
    device = torch.device("cuda")
    model = build_model(config, a.weights, device)
    res = register(model, a.pcd1, a.pcd2, config["downsample"], device, a.normals)
    T = res["final_trans"].cpu().numpy()
    print(f"{len(res['corr'])} correspondences, {int((res['final_labels'] > 0).sum())} inliers")
    print("final_trans =\n" + np.array2string(T, precision=6, suppress_small=True))
    if a.out:
        np.savez(a.out, **{k: v.cpu().numpy() for k, v in res.items()})
    return T


if __name__ == "__main__":
    main()
