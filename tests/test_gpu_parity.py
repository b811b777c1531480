"""HIP path vs the reference's golden vectors, an exact-arithmetic (fp64) yardstick
and the CPU oracle (run with -m gpu).

Bars (north_star):
  * index / mask work bit-exact: M, is_local_max, NMS, kNN selection, fitness,
    final_labels -- up to the near-ties fp32 re-ordering is free to decide
    either way, which every such check names explicitly;
  * poses within 1e-4;
  * encoder features / confidences: within ENVELOPE x the reference's OWN
    distance from exact arithmetic (conftest.py): the reference itself sits up to
    4e-4 (logits) from exact math on these goldens, so a literal 1e-4 against it
    is below fp32's resolution for this network.
Both precision modes are held to the same bars.  Every call goes through the C
ABI (libpdsc.so) via pointdsc_amd.kernels."""
import numpy as np
import pytest
import torch

from conftest import (BULK, ENVELOPE, FEAT_FLOOR, LOGIT_FLOOR, RMS_FLOOR, assert_knn_equivalent, assert_poses_close,
                      assert_rigid,
                      assert_seeds_equivalent,
                      assert_seeds_near_ties, fp32_envelope, golden_hparams, golden_names, golden_state_dict,
                      load_golden, rms, seed_H_rank)

pytestmark = pytest.mark.gpu

NAMES = golden_names()
PRECISIONS = ["h3", "f32"]
POSE_ATOL = 1e-4
_FP64 = {}


def _t(x, dev, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev, dtype)


def _model(g, dev, precision="h3"):
    from pointdsc_amd.PointDSC import PointDSC
    hp = golden_hparams(g)
    m = PointDSC(in_dim=hp["in_dim"], num_layers=hp["num_layers"], num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=hp["inlier_threshold"], sigma_d=float(g["sigma_d"]), k=40,
                 nms_radius=hp["nms_radius"], precision=precision)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in golden_state_dict(g).items()})
    return m.to(dev).eval()


def _inputs(g, dev):
    return (_t(g["corr_pos"][None], dev), _t(g["src_keypts"][None], dev), _t(g["tgt_keypts"][None], dev))


def _bulk(name, g, dev):
    """(fp32 bulk feature noise / max|f|, fp32 bulk logit noise): the RMS distances, cached."""
    key = name + "#bulk"
    if key not in _FP64:
        e_f, e_c, f64, c64, mx, r_f, r_c = fp32_envelope(g, golden_state_dict(g), dev, bulk=True)
        _FP64[name] = (e_f, e_c, f64, c64, mx)
        _FP64[key] = (r_f, r_c)
    return _FP64[key]


def _envelope(name, g, dev):
    """(fp32 feature noise / max|f|, fp32 logit noise, f64, c64, max|f|): conftest.fp32_envelope, cached."""
    if name not in _FP64:
        _FP64[name] = fp32_envelope(g, golden_state_dict(g), dev)
    return _FP64[name]


@pytest.mark.parametrize("name", NAMES)
def test_compat(name, gpu_device):
    from pointdsc_amd import kernels
    g = load_golden(name)
    _, src, tgt = _inputs(g, gpu_device)
    sd = torch.tensor([float(g["sigma_d"])], dtype=torch.float32, device=gpu_device)
    M = kernels.compat(src, tgt, sd)[0]
    if "M" in g:
        assert np.array_equal(M.cpu().numpy(), g["M"])  # bit-exact
    # the forward's packed layout holds the same bits
    assert torch.equal(kernels.compat_packed(src, tgt, sd)[0], M)
    assert np.array_equal(torch.diagonal(M).cpu().numpy(), g["M_diag"])
    assert torch.equal(M, M.T)
    np.testing.assert_allclose(M.double().sum(-1).cpu().numpy(), g["M_row_sums"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("name", NAMES)
def test_encoder_and_classifier(name, precision, gpu_device):
    """a2-a4: features, normed features and logits within ENVELOPE x the reference's
    own distance from exact arithmetic (plus an fp32-resolution floor), and in
    bulk (RMS) within BULK x the fp32 realisations'."""
    from pointdsc_amd import kernels
    g = load_golden(name)
    m = _model(g, gpu_device, precision)
    corr, src, tgt = _inputs(g, gpu_device)
    M = kernels.compat(src, tgt, m.sigma_spat)
    feat, normed, conf = kernels.encoder(m.pdsc_config(), m.packed_weights(), corr, M)
    r_f, r_c = _bulk(name, g, gpu_device)
    e_f, e_c, f64, c64, mx = _envelope(name, g, gpu_device)
    ours_c = np.abs(conf[0].double().cpu().numpy() - c64).max()
    assert ours_c <= ENVELOPE * e_c + LOGIT_FLOOR, (ours_c, e_c)
    f = feat[0].double().cpu().numpy()
    ours_f = np.abs(f - f64).max() / mx
    assert ours_f <= ENVELOPE * e_f + FEAT_FLOOR, (ours_f, e_f)
    # in bulk too (conftest.BULK): RMS distance from exact arithmetic vs the fp32 realisations'
    rms_f, rms_c = rms(f - f64) / mx, rms(conf[0].double().cpu().numpy() - c64)
    assert rms_f <= BULK * r_f + RMS_FLOOR, (rms_f, r_f)
    assert rms_c <= BULK * r_c + RMS_FLOOR, (rms_c, r_c)
    # normed rows are unit vectors: their error is the feature error relative to the row norm
    n64 = f64 / np.maximum(np.linalg.norm(f64, axis=1, keepdims=True), 1e-12)
    rel_row = (np.abs(f - f64).max(1) / np.maximum(np.linalg.norm(f64, axis=1), 1e-12)).max()
    assert np.abs(normed[0].double().cpu().numpy() - n64).max() <= 2 * rel_row + 1e-6


@pytest.mark.parametrize("name", ["wide9_1k", "wide70_1k"])
@pytest.mark.parametrize("B", [1, 40])  # pw_first (LDS-tiled) and pw2_first (register-chained) layer0
def test_wide_layer0_inputs(name, B, gpu_device):
    """in_dim = 70 (corr_pos + both 32-d descriptors, datasets/ThreeDMatch.py:311-315)
    and 9 (:308-309): layer0 wider than the 16 inputs held in registers, against
    the REFERENCE's own outputs for these widths (tools/gen_goldens.py runs
    models/PointDSC.py with in_dim 9 / 70).  Single pairs and a 40-pair batch of
    the same pair (the batched layer-0 kernel): features / logits in the fp32
    envelope, labels and seeds as the reference, poses 1e-4."""
    from pointdsc_amd import kernels
    g = load_golden(name)
    assert int(g["in_dim"]) == g["corr_pos"].shape[1]
    m = _model(g, gpu_device)
    e_f, e_c, f64, c64, mx = _envelope(name, g, gpu_device)
    rep = lambda a: _t(np.repeat(a[None], B, 0), gpu_device)
    corr, src, tgt = rep(g["corr_pos"]), rep(g["src_keypts"]), rep(g["tgt_keypts"])
    M = kernels.compat(src, tgt, m.sigma_spat)
    feat, _, conf = kernels.encoder(m.pdsc_config(), m.packed_weights(), corr, M)
    for b in (0, B - 1):
        ours_f = np.abs(feat[b].double().cpu().numpy() - f64).max() / mx
        ours_c = np.abs(conf[b].double().cpu().numpy() - c64).max()
        assert ours_f <= ENVELOPE * e_f + FEAT_FLOOR, (b, ours_f, e_f)
        assert ours_c <= ENVELOPE * e_c + LOGIT_FLOOR, (b, ours_c, e_c)
    # the whole testing forward against the reference's outputs
    T, L = m.forward_batched(corr, src, tgt)
    for b in (0, B - 1):
        assert np.array_equal(L[b].cpu().numpy(), g["final_labels"]), b
        np.testing.assert_allclose(T[b].cpu().numpy(), g["final_trans"], atol=POSE_ATOL)


@pytest.mark.parametrize("name", ["degen_1k", "rel_1k", "rel_1k_kitti"])
def test_long_key_chain_encoder(name, gpu_device):
    """40 copies of a 1000-point golden: the batched plan's attention runs every
    query's 32 key tiles as ONE online-softmax chain (fused, one split), where a
    single pair gets many short splits.  Same bars as test_encoder_and_classifier
    (max and bulk).  r03's V-tile scale (max|v'| up to 2^14) failed this at up to
    5x the fp32 envelope: the p of keys far below the row max fell under fp16's
    2^-24 (attention_h3.hpp, h3_vexp)."""
    import ctypes
    from pointdsc_amd import _lib, kernels
    B = 40
    g = load_golden(name)
    N = len(g["corr_pos"])
    fused, npad, nsplit = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    _lib.check(_lib.load().pdsc_encoder_plan(B, N, 0, ctypes.byref(fused)), "encoder_plan")
    _lib.check(_lib.load().pdsc_attention_layout(B, N, 0, ctypes.byref(npad), ctypes.byref(nsplit)), "layout")
    assert fused.value == 1 and nsplit.value == 1
    m = _model(g, gpu_device)
    rep = lambda a: _t(np.repeat(a[None], B, 0), gpu_device)
    corr, src, tgt = rep(g["corr_pos"]), rep(g["src_keypts"]), rep(g["tgt_keypts"])
    feat, _, conf = kernels.encoder(m.pdsc_config(), m.packed_weights(), corr, M=kernels.compat(src, tgt, m.sigma_spat))
    r_f, r_c = _bulk(name, g, gpu_device)
    e_f, e_c, f64, c64, mx = _envelope(name, g, gpu_device)
    for b in (0, B - 1):
        f, c = feat[b].double().cpu().numpy(), conf[b].double().cpu().numpy()
        assert np.abs(f - f64).max() / mx <= ENVELOPE * e_f + FEAT_FLOOR, (b, np.abs(f - f64).max() / mx, e_f)
        assert np.abs(c - c64).max() <= ENVELOPE * e_c + LOGIT_FLOOR, (b, np.abs(c - c64).max(), e_c)
        assert rms(f - f64) / mx <= BULK * r_f + RMS_FLOOR, (b, rms(f - f64) / mx, r_f)
        assert rms(c - c64) <= BULK * r_c + RMS_FLOOR, (b, rms(c - c64), r_c)


@pytest.mark.parametrize("name", NAMES)
def test_h3_matches_exact_fp32(name, gpu_device):
    """The 3xfp16 contractions against the exact-fp32 MFMA mode on the same inputs:
    features and logits within the same envelope, identical labels, poses 1e-4."""
    from pointdsc_amd import kernels
    g = load_golden(name)
    corr, src, tgt = _inputs(g, gpu_device)
    out = {}
    for p in PRECISIONS:
        m = _model(g, gpu_device, p)
        M = kernels.compat(src, tgt, m.sigma_spat)
        feat, _, conf = kernels.encoder(m.pdsc_config(), m.packed_weights(), corr, M)
        T, L = kernels.forward_testing(m.pdsc_config(), m.packed_weights(), corr, src, tgt)
        out[p] = (feat[0].double().cpu().numpy(), conf[0].double().cpu().numpy(), T[0].cpu().numpy(),
                  L[0].cpu().numpy())
    e_f, e_c, f64, c64, mx = _envelope(name, g, gpu_device)
    (fh, ch, Th, Lh), (ff, cf, Tf, Lf) = out["h3"], out["f32"]
    assert np.abs(fh - ff).max() / mx <= 2 * ENVELOPE * e_f + FEAT_FLOOR  # each within ENVELOPE of exact
    assert np.abs(ch - cf).max() <= 2 * ENVELOPE * e_c + LOGIT_FLOOR
    assert np.array_equal(Lh, Lf)
    np.testing.assert_allclose(Th, Tf, atol=POSE_ATOL)


@pytest.mark.parametrize("name", NAMES)
def test_pick_seeds_exact(name, gpu_device):
    from pointdsc_amd import kernels
    g = load_golden(name)
    _, src, _ = _inputs(g, gpu_device)
    conf = _t(g["confidence"][None], gpu_device)
    S = len(g["seeds"])
    seeds, lm = kernels.pick_seeds(src, conf, float(g["nms_radius"]), S)
    assert np.array_equal(lm[0].cpu().numpy(), g["is_local_max"])
    assert_seeds_equivalent(seeds[0].cpu().numpy(), g["seeds"], g["confidence"] * g["is_local_max"])


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("name", NAMES)
def test_nsm_chain(name, precision, gpu_device):
    """a6-a11, each stage fed with the reference's inputs for that stage.  Seeds
    whose covariance H has rank < 2 (collinear / duplicated neighbourhoods: the
    rotation is LAPACK's arbitrary choice in a one-parameter family) are held to
    the rigid-transform properties instead of the reference's pose."""
    from pointdsc_amd import kernels
    g = load_golden(name)
    sd = golden_state_dict(g)
    _, src, tgt = _inputs(g, gpu_device)
    if len(g["corr_features"]):
        f = g["corr_features"]
        nrm = f / np.maximum(np.linalg.norm(f, axis=1, keepdims=True), 1e-12)
        normed = _t(nrm, gpu_device)[None]
        seeds = _t(g["seeds"][None], gpu_device, torch.int32)
        k = g["knn_idx"].shape[1]
        knn = kernels.seed_knn(normed, seeds, k, precision=precision)
        assert_knn_equivalent(knn[0].cpu().numpy(), g["knn_idx"], nrm, g["seeds"])
        ref_knn = _t(g["knn_idx"][None], gpu_device, torch.int32)
        w, iters = kernels.nsm_weights(normed, src, tgt, ref_knn, 10, _t(sd["sigma"], gpu_device),
                                       _t(sd["sigma_spat"], gpu_device), precision=precision)
        v = g["leading_eig"]
        np.testing.assert_allclose(w[0].cpu().numpy(), v / (v.sum(-1, keepdims=True) + 1e-6), atol=2e-5)
    v = g["leading_eig"]
    w_ref = (v / (v.sum(-1, keepdims=True) + np.float32(1e-6))).astype(np.float32)
    ref_knn = _t(g["knn_idx"][None], gpu_device, torch.int32)
    seed_trans, fit, best, trans, labels = kernels.seed_hypotheses(src, tgt, ref_knn, _t(w_ref[None], gpu_device),
                                                                   float(g["inlier_threshold"]))
    st = seed_trans[0].cpu().numpy()
    ok = seed_H_rank(g) > 1e-5
    kn = g["knn_idx"][ok]
    assert_poses_close(st[ok], g["seed_trans"][ok], g["src_keypts"][kn], g["tgt_keypts"][kn], w_ref[ok], POSE_ATOL)
    for s in np.nonzero(~ok)[0]:
        assert_rigid(st[s], g["src_keypts"][g["knn_idx"][s]], g["tgt_keypts"][g["knn_idx"][s]], w_ref[s])
    assert np.array_equal(fit[0].cpu().numpy()[ok], g["seed_fitness"][ok])
    np.testing.assert_allclose(trans[0].cpu().numpy(), g["trans_pre_refine"], atol=POSE_ATOL)
    assert np.array_equal(labels[0].cpu().numpy(), g["final_labels"])
    thr = 0.10 if float(g["inlier_threshold"]) == 0.10 else 1.2
    ref = kernels.post_refine(_t(g["trans_pre_refine"][None], gpu_device), src, tgt, thr)
    np.testing.assert_allclose(ref[0].cpu().numpy(), g["final_trans"], atol=POSE_ATOL)


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("name", NAMES)
def test_module_forward_end_to_end(name, precision, gpu_device):
    """PointDSC.forward(data) with 'testing' -- the drop-in contract: labels
    bit-exact, pose within 1e-4."""
    g = load_golden(name)
    m = _model(g, gpu_device, precision)
    corr, src, tgt = _inputs(g, gpu_device)
    with torch.no_grad():
        res = m({"corr_pos": corr, "src_keypts": src, "tgt_keypts": tgt, "testing": True})
    assert res["M"] is None
    assert res["final_trans"].shape == (1, 4, 4) and res["final_labels"].shape == (1, len(g["src_keypts"]))
    assert np.array_equal(res["final_labels"][0].cpu().numpy(), g["final_labels"])
    np.testing.assert_allclose(res["final_trans"][0].cpu().numpy(), g["final_trans"], atol=POSE_ATOL)


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("name", NAMES)
def test_forward_seeds_near_ties(name, precision, gpu_device):
    """The seeds the full forward picks (a5 on our own confidences) equal the
    reference's except where a local-max decision or a ranking swap involves two
    reference confidences closer than twice our measured logit error."""
    from pointdsc_amd import kernels
    g = load_golden(name)
    m = _model(g, gpu_device, precision)
    corr, src, tgt = _inputs(g, gpu_device)
    trans, labels, conf, seeds = kernels.forward_testing(m.pdsc_config(), m.packed_weights(), corr, src, tgt,
                                                         debug=True)
    conf = conf[0].cpu().numpy()
    tol = float(np.abs(conf - g["confidence"]).max())
    _, e_c, _, _, _ = _envelope(name, g, gpu_device)
    assert tol <= (ENVELOPE + 1) * e_c + LOGIT_FLOOR  # |ours - ref| <= |ours - exact| + |ref - exact|
    flips, moved = assert_seeds_near_ties(seeds[0].cpu().numpy(), conf, g, tol)
    assert moved <= 4 * flips + 0.1 * len(g["seeds"])


def test_kabsch_degenerate_goldens(gpu_device):
    """rigid_transform_3d on the reference's own degenerate cases
    (tests/golden/kabsch_degenerate.npz): zero / negative weights (H = 0 -> the
    reference's R = I), three points and coplanar points (rank-2 H: unique R) are
    pinned at 1e-4; rank-1 H (collinear, duplicated points) by the properties."""
    from pointdsc_amd import kernels
    from conftest import GOLDEN
    import os
    z = np.load(os.path.join(GOLDEN, "kabsch_degenerate.npz"))
    names = sorted({k.split("__")[0] for k in z.files})
    for n in names:
        A, B, w, T = z[n + "__A"], z[n + "__B"], z[n + "__w"], z[n + "__T"]
        ours = kernels.rigid_transform_3d(_t(A[None], gpu_device), _t(B[None], gpu_device),
                                          _t(w[None], gpu_device))[0].cpu().numpy()
        if bool(z[n + "__pinned"]):
            np.testing.assert_allclose(ours, T, atol=POSE_ATOL, err_msg=n)
        else:
            assert_rigid(ours, A.astype(np.float64), B.astype(np.float64), w)


@pytest.mark.parametrize("B", [6, 24, 64])
def test_batched_equals_single(B, gpu_device):
    """B pairs in one call == B single-pair calls: labels bitwise, poses within
    twice the north-star tolerance (the batched launches take other kernel
    variants: B = 24 the 4-wave seed kernels (B*ceil(S/4) >= 512), B = 64 also
    the register-chained pointwise kernels; fp32 sums in another order)."""
    from pointdsc_amd.synthetic import synthetic_batch
    g = load_golden("rel_1k")
    m = _model(g, gpu_device)
    b = synthetic_batch(B, 1000, seed=5)
    corr, src, tgt = (_t(b[k], gpu_device) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    T, Lb = m.forward_batched(corr, src, tgt)
    for i in range(B):
        r = m({"corr_pos": corr[i:i + 1], "src_keypts": src[i:i + 1], "tgt_keypts": tgt[i:i + 1],
               "testing": True})
        assert torch.equal(r["final_labels"][0], Lb[i]), i
        np.testing.assert_allclose(r["final_trans"][0].cpu().numpy(), T[i].cpu().numpy(), atol=2 * POSE_ATOL)


def _fusion_outputs(dev, B=64, N=1000):
    """Encoder (dense M) and forward (packed M) outputs at a shape the encoder
    plan fuses (attention + pointwise chain per launch)."""
    from pointdsc_amd import kernels
    from pointdsc_amd.synthetic import synthetic_batch
    g = load_golden("rel_1k")
    m = _model(g, dev)
    cfg, packed = m.pdsc_config(), m.packed_weights()
    b = synthetic_batch(B, N, seed=21)
    corr, src, tgt = (_t(b[k], dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    M = kernels.compat(src, tgt, torch.tensor([float(g["sigma_d"])], device=dev))
    feat, normed, conf = kernels.encoder(cfg, packed, corr, M)
    T, L, fconf, seeds = kernels.forward_testing(cfg, packed, corr, src, tgt, debug=True)
    return {k: v.cpu().numpy() for k, v in dict(feat=feat, normed=normed, conf=conf, T=T, L=L, fconf=fconf,
                                                  seeds=seeds).items()}


def _dump_fusion_outputs(path, B=64, N=1000):  # child process entry (A/B knobs set by the parent)
    np.savez(path, **_fusion_outputs(torch.device("cuda:0"), B, N))


def test_fused_encoder_bit_identical(gpu_device, tmp_path):
    """attn_pw2_kernel (attention_l + the pointwise chain_l in one launch, partials
    kept in registers) gives exactly the bits of the separate attention_h3 +
    pw2_mid launches (run in a child process with the PDSC_FUSE=0 knob): encoder
    features / confidences with dense M, and the whole forward with packed M; a
    two-round headline-like batch and a 1.25-round one (320 workgroups).  The
    unfused child keeps the split grid (PDSC_W64_SK=0): its one key split per
    query block is the fused kernel's arithmetic, where stream-K's segments
    (40 x 1000: 3 per block) would combine in another fp32 order."""
    import ctypes
    import os
    import subprocess
    import sys
    from pointdsc_amd import _lib
    here = os.path.dirname(os.path.abspath(__file__))
    for B, N in ((64, 1000), (40, 1000)):
        fused = ctypes.c_int32()
        _lib.check(_lib.load().pdsc_encoder_plan(B, N, 0, ctypes.byref(fused)), "encoder_plan")
        assert fused.value == 1, (B, N)
        ours = _fusion_outputs(gpu_device, B, N)
        out = tmp_path / f"unfused_{B}_{N}.npz"
        env = dict(os.environ, PDSC_FUSE="0", PDSC_W64_SK="0")
        code = f"import sys; sys.path[:0] = [{here!r}, {os.path.dirname(here)!r}]; " \
               f"import test_gpu_parity as t; t._dump_fusion_outputs({str(out)!r}, {B}, {N})"
        subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=240)
        ref = np.load(out)
        for k, v in ours.items():
            assert np.array_equal(v, ref[k]), (B, N, k)


def test_precombine_bit_identical(gpu_device, tmp_path):
    """Small batches combine the split-K attention partials in their own launch
    (combine_rows_kernel, one split handed to pw_mid / pw_last) instead of in
    the pointwise kernel's prologue: the same bits as the in-kernel combine (a
    child process with PDSC_PRECOMBINE=0), encoder and forward: a single pair
    (16 key splits) and a ragged-tail N."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for B, N in ((1, 1000), (1, 1500)):
        ours = _fusion_outputs(gpu_device, B, N)
        out = tmp_path / f"inkernel_{B}_{N}.npz"
        env = dict(os.environ, PDSC_PRECOMBINE="0")
        code = f"import sys; sys.path[:0] = [{here!r}, {os.path.dirname(here)!r}]; " \
               f"import test_gpu_parity as t; t._dump_fusion_outputs({str(out)!r}, {B}, {N})"
        subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=240)
        ref = np.load(out)
        for k, v in ours.items():
            assert np.array_equal(v, ref[k]), (B, N, k)


def test_pw_waves8_bit_identical(gpu_device, tmp_path):
    """Tiny batches run pw_mid with 8-wave workgroups (the chain's output tiles
    over twice the waves): the same bits as the 4-wave kernel (a child process
    with PDSC_PW_WAVES=4), encoder and forward: a single pair and a 5-pair batch
    with a padded tail."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for B, N in ((1, 1000), (5, 777)):
        ours = _fusion_outputs(gpu_device, B, N)
        out = tmp_path / f"w4_{B}_{N}.npz"
        env = dict(os.environ, PDSC_PW_WAVES="4")
        code = f"import sys; sys.path[:0] = [{here!r}, {os.path.dirname(here)!r}]; " \
               f"import test_gpu_parity as t; t._dump_fusion_outputs({str(out)!r}, {B}, {N})"
        subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=240)
        ref = np.load(out)
        for k, v in ours.items():
            assert np.array_equal(v, ref[k]), (B, N, k)


def test_pw_qkv_split_bit_identical(gpu_device, tmp_path):
    """Single pairs and 2-pair batches run the 8-wave pw_mid as three workgroups
    per point tile, one per Q / K / V projection (pcn_qkv8's `only`): the same
    bits as one workgroup writing all three (a child process with
    PDSC_PW_QKV_SPLIT=0), encoder and forward, including a padded tail."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for B, N in ((1, 1000), (2, 777), (1, 2500)):
        ours = _fusion_outputs(gpu_device, B, N)
        out = tmp_path / f"qkv1_{B}_{N}.npz"
        env = dict(os.environ, PDSC_PW_QKV_SPLIT="0")
        code = f"import sys; sys.path[:0] = [{here!r}, {os.path.dirname(here)!r}]; " \
               f"import test_gpu_parity as t; t._dump_fusion_outputs({str(out)!r}, {B}, {N})"
        subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=240)
        ref = np.load(out)
        for k, v in ours.items():
            assert np.array_equal(v, ref[k]), (B, N, k)


def test_pw_qkv_split_delayed_readers(gpu_device, monkeypatch):
    """The split pw_mid's K and V workgroups read the layer's residual rows that
    the Q workgroup replaces with the new PointCN rows: the rows ping-pong
    between two feat buffers, so delaying the K / V workgroups until the Q one
    has stored (pdsc_diag_qkv_delay: s_sleep loops before their first load) must
    leave every output bit unchanged.  Before the ping-pong this read the new
    rows as the residual (wrong K / V)."""
    for B, N in ((1, 1000), (2, 777)):
        ref = _fusion_outputs(gpu_device, B, N)
        from pointdsc_amd import _lib
        _lib.check(_lib.load().pdsc_diag_qkv_delay(24), "pdsc_diag_qkv_delay")  # ~100 us: longer than pw_mid
        try:
            late = _fusion_outputs(gpu_device, B, N)
        finally:
            _lib.load().pdsc_diag_qkv_delay(0)
        for k, v in ref.items():
            assert np.array_equal(v, late[k]), (B, N, k)


def test_kabsch_fused_bit_identical(gpu_device, tmp_path):
    """Batches of <= 1024 seeds finish each seed's Kabsch solve in the wave that
    summed it (kabsch_sums_kernel<true>): the same bits as the separate solve
    kernel (a child process with PDSC_KABSCH_FUSED=0), a single pair and a
    4-pair batch."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for B, N in ((1, 1000), (4, 2000)):
        ours = _fusion_outputs(gpu_device, B, N)
        out = tmp_path / f"kabsch2_{B}_{N}.npz"
        env = dict(os.environ, PDSC_KABSCH_FUSED="0")
        code = f"import sys; sys.path[:0] = [{here!r}, {os.path.dirname(here)!r}]; " \
               f"import test_gpu_parity as t; t._dump_fusion_outputs({str(out)!r}, {B}, {N})"
        subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=240)
        ref = np.load(out)
        for k, v in ours.items():
            assert np.array_equal(v, ref[k]), (B, N, k)


def test_graph_replay_equals_eager(gpu_device):
    """ForwardPlan.capture(): a HIP-graph replay of the forward gives the eager
    result bitwise, and picks up new contents of the same input buffers; the
    stage-timing hook records 8 events per forward."""
    import ctypes
    from pointdsc_amd import _lib, kernels
    from pointdsc_amd.synthetic import synthetic_batch
    g = load_golden("rel_1k")
    m = _model(g, gpu_device)
    cfg, packed = m.pdsc_config(), m.packed_weights()
    b1, b2 = synthetic_batch(2, 1000, seed=11), synthetic_batch(2, 1000, seed=12)
    corr, src, tgt = (_t(b1[k], gpu_device) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    eager = kernels.ForwardPlan(cfg, packed, 2, 1000, gpu_device)
    T1, L1 = (x.clone() for x in eager.run(corr, src, tgt))
    graph = kernels.ForwardPlan(cfg, packed, 2, 1000, gpu_device).capture(corr, src, tgt)
    Tg, Lg = graph.run(corr, src, tgt)
    assert torch.equal(T1, Tg) and torch.equal(L1, Lg)
    for x, k in zip((corr, src, tgt), ("corr_pos", "src_keypts", "tgt_keypts")):
        x.copy_(_t(b2[k], gpu_device))
    T2, L2 = (x.clone() for x in eager.run(corr, src, tgt))
    Tg, Lg = graph.run(corr, src, tgt)
    assert torch.equal(T2, Tg) and torch.equal(L2, Lg) and not torch.equal(T1, T2)
    # stage timing hook
    hip = ctypes.CDLL("libamdhip64.so")
    ev = (ctypes.c_void_p * 16)()
    for i in range(16):
        e = ctypes.c_void_p()
        assert hip.hipEventCreate(ctypes.byref(e)) == 0
        ev[i] = e.value
    cnt = ctypes.c_int32(0)
    L = _lib.load()
    _lib.check(L.pdsc_forward_timing(ev, 16, ctypes.byref(cnt)), "pdsc_forward_timing")
    for _ in range(3):
        eager.run(corr, src, tgt)
    L.pdsc_forward_timing(None, 0, None)
    torch.cuda.synchronize(gpu_device)
    assert cnt.value == 16  # the third call did not fit
    ms = ctypes.c_float()
    for i in range(7):
        assert hip.hipEventElapsedTime(ctypes.byref(ms), ctypes.c_void_p(ev[i]), ctypes.c_void_p(ev[i + 1])) == 0
        assert ms.value >= 0
    for i in range(16):
        hip.hipEventDestroy(ctypes.c_void_p(ev[i]))


def _attention_fp64(q, k, v, M):
    return torch.softmax(M.double() * (q.double() @ k.double().transpose(1, 2)) / 128 ** 0.5, -1) @ v.double()


@pytest.mark.parametrize("precision", PRECISIONS)
def test_attention_vs_torch_fp64(precision, gpu_device):
    """The attention core (:36-42) against a plain PyTorch fp64 evaluation."""
    from pointdsc_amd import kernels
    torch.manual_seed(0)
    for B, N in [(1, 1000), (2, 333), (1, 4096)]:
        q, k, v = (torch.randn(B, N, 128, device=gpu_device) for _ in range(3))
        src = torch.rand(B, N, 3, device=gpu_device) * 3
        tgt = src + 0.05 * torch.randn(B, N, 3, device=gpu_device)
        M = kernels.compat(src, tgt, torch.tensor([0.1], device=gpu_device))
        out = kernels.attention(q, k, v, M, precision=precision).double()
        ref = _attention_fp64(q, k, v, M)
        assert (out - ref).abs().max().item() <= 1e-6 * v.abs().max().item()


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("sv", [1e-3, 1.0, 1e2])
@pytest.mark.parametrize("sqk", [(1e-3, 1e-3), (7.0, 1.0), (1e2, 1e-1)])
@pytest.mark.parametrize("B,N", [(2, 700), (48, 1024)])  # many short key splits; one 32-tile chain per query
def test_attention_adversarial_magnitudes(B, N, sqk, sv, precision, gpu_device):
    """Operand magnitudes far from the encoder's O(1): Q, K scaled so the logits are
    ~1e-6 or spread over ~+-20 (softmax weights over > 2^50, i.e. > 30 log2
    units), V scaled by 1e-3 .. 1e2.  Error bound relative to max|V| (the output's
    scale); the 3xfp16 path keeps small V exact through its per-tile exponent.
    48 x 1024: the standalone plan runs one key split (a 1024-key online softmax
    per query), where weights far below the running max must not fall off fp16."""
    from pointdsc_amd import kernels
    torch.manual_seed(1)
    sq, sk = sqk
    q = torch.randn(B, N, 128, device=gpu_device) * sq
    k = torch.randn(B, N, 128, device=gpu_device) * sk
    v = torch.randn(B, N, 128, device=gpu_device) * sv
    v[:, ::7] *= 1e-3  # rows of very different magnitude inside one 32-key tile
    src = torch.rand(B, N, 3, device=gpu_device) * 3
    tgt = src + 0.02 * torch.randn(B, N, 3, device=gpu_device)
    M = kernels.compat(src, tgt, torch.tensor([0.1], device=gpu_device))
    lg = M.double() * (q.double() @ k.double().transpose(1, 2)) / 128 ** 0.5
    spread = (lg.max(-1).values - lg.min(-1).values).max().item()
    if sq * sk > 1:
        assert spread > 30 * np.log(2)
    out = kernels.attention(q, k, v, M, precision=precision).double()
    ref = _attention_fp64(q, k, v, M)
    # logits of magnitude L carry fp32 rounding ~2^-24 L in both the reference and here,
    # and the softmax turns an absolute logit error into that relative weight error
    tol = 2e-6 + 4 * 2.0 ** -24 * max(1.0, lg.abs().max().item())
    assert (out - ref).abs().max().item() <= tol * v.abs().max().item()


def test_rigid_transform_vs_oracle(gpu_device):
    from oracle import pdsc_oracle as O
    from pointdsc_amd import kernels
    from pointdsc_amd.synthetic import random_rotation
    rng = np.random.RandomState(1)
    for n in (3, 40, 777, 5000):
        A = rng.rand(3, n, 3).astype(np.float32) * 2
        R = np.stack([random_rotation(rng) for _ in range(3)]).astype(np.float32)
        Bp = (np.einsum("bij,bnj->bni", R, A) + rng.rand(3, 1, 3) + 0.01 * rng.randn(3, n, 3)).astype(np.float32)
        w = rng.rand(3, n).astype(np.float32)
        T = kernels.rigid_transform_3d(_t(A, gpu_device), _t(Bp, gpu_device), _t(w, gpu_device)).cpu().numpy()
        np.testing.assert_allclose(T, O.rigid_transform_3d(A, Bp, w), atol=2e-5)


@pytest.mark.parametrize("preset,N,B", [("3dmatch", 5000, 4), ("kitti", 5000, 4), ("kitti", 12000, 1)])
def test_full_size_registration_properties(preset, N, B, gpu_device):
    """BASELINE sizes and the KITTI driver's largest (num_node=12000,
    evaluation/test_KITTI.py:151): the recovered pose matches ground truth and
    every label is 0/1 with most inliers found."""
    from pointdsc_amd.synthetic import PRESETS, synthetic_batch, trained_state_dict
    from pointdsc_amd.PointDSC import PointDSC
    p = PRESETS[preset]
    m = PointDSC(num_layers=12, inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"],
                 nms_radius=p["nms_radius"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict(preset).items()})
    m = m.to(gpu_device).eval()
    b = synthetic_batch(B, N, seed=77, preset=preset)
    corr, src, tgt = (_t(b[k], gpu_device) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    T, labels = m.forward_batched(corr, src, tgt)
    T, labels = T.cpu().numpy(), labels.cpu().numpy()
    for i in range(B):
        gt = b["gt_trans"][i]
        cosang = (np.trace(T[i, :3, :3].T @ gt[:3, :3]) - 1) / 2
        re = np.degrees(np.arccos(np.clip(cosang, -1, 1)))
        te = np.linalg.norm(T[i, :3, 3] - gt[:3, 3])
        assert re < 1.0 and te < 0.2 * p["inlier_threshold"] * 10, (re, te)
        assert labels[i].sum() >= 0.9 * b["gt_labels"][i].sum()
        assert set(np.unique(labels[i])) <= {0.0, 1.0}


@pytest.mark.parametrize("precision", PRECISIONS)
def test_recall_parity_synthetic(precision, gpu_device):
    """Registration-recall parity proxy (the 3DMatch recall claim needs data and
    weights absent here): on 64 FPFH-like pairs (6 % inliers, N = 1000) the HIP
    path and the CPU oracle succeed (RE < 15 deg, TE < 30 cm, libs/loss.py:44-51)
    on exactly the same pairs."""
    from oracle import pdsc_oracle as O
    from pointdsc_amd.evaluate import pair_stats
    from pointdsc_amd.synthetic import synthetic_batch, trained_state_dict
    g = load_golden("rel_1k")
    m = _model(g, gpu_device, precision)
    b = synthetic_batch(64, 1000, seed=606, inlier_ratio=0.06)
    corr, src, tgt = (_t(b[k], gpu_device) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    T, L = m.forward_batched(corr, src, tgt)
    ours = pair_stats(T.cpu(), torch.from_numpy(b["gt_trans"]), L.cpu(), torch.from_numpy(b["gt_labels"]))
    sd = golden_state_dict(g)
    hp = golden_hparams(g)
    ref_T, ref_L = [], []
    for i in range(64):
        o = O.forward_testing(b["corr_pos"][i], b["src_keypts"][i], b["tgt_keypts"][i], sd, **hp)
        ref_T.append(o["final_trans"])
        ref_L.append(o["final_labels"])
    ref = pair_stats(torch.from_numpy(np.stack(ref_T)), torch.from_numpy(b["gt_trans"]),
                     torch.from_numpy(np.stack(ref_L)), torch.from_numpy(b["gt_labels"]))
    assert torch.equal(ours[:, 0], ref[:, 0]), (ours[:, 0].sum().item(), ref[:, 0].sum().item())
    assert 0 < ours[:, 0].sum().item() < 64  # a regime where success is not trivial


@pytest.mark.parametrize("scale,sigma", [(1e-3, 1e-4), (3.0, 0.1), (60.0, 1.2), (5e3, 37.0)])
def test_compat_bit_exact_random_scales(scale, sigma, gpu_device):
    """a1 against the oracle's bit-exact C restatement (oracle/exact.c) on random
    clouds over six decades of coordinate scale, duplicate points included:
    the kernel's fast sqrt/division path and its library fallback must both
    reproduce the reference's correctly rounded sqrtf and '/'."""
    from oracle import pdsc_oracle as O
    from pointdsc_amd import kernels
    rng = np.random.RandomState(int(scale * 7) % 1000)
    B, N = 3, 517
    src = (rng.rand(B, N, 3) * scale).astype(np.float32)
    tgt = (src + rng.randn(B, N, 3).astype(np.float32) * np.float32(sigma)).astype(np.float32)
    src[:, 5] = src[:, 9]  # duplicate points: squared distance exactly 0
    tgt[:, 7] = tgt[:, 8]
    src[:, 11] = src[:, 12] + np.float32(1e-20)  # a tiny positive squared distance -> library path
    src[:, 20] = np.float32(4e3 * scale)  # far points: past compat4's sqrt-free zero test guard
    sd = torch.tensor([sigma], dtype=torch.float32, device=gpu_device)
    M = kernels.compat(_t(src, gpu_device), _t(tgt, gpu_device), sd).cpu().numpy()
    Mp = kernels.compat_packed(_t(src, gpu_device), _t(tgt, gpu_device), sd).cpu().numpy()
    for b in range(B):
        ref = O.compat(src[b], tgt[b], float(np.float32(sigma)))
        assert np.array_equal(M[b], ref), b
        assert np.array_equal(Mp[b], ref), b


@pytest.mark.parametrize("radius", [0.05, 0.1, 0.6])
def test_local_max_bit_exact_random(radius, gpu_device):
    """a5's NMS (squared-distance threshold form) against the oracle's sqrtf form."""
    from oracle import pdsc_oracle as O
    from pointdsc_amd import kernels
    rng = np.random.RandomState(3)
    B, N = 2, 1500
    src = (rng.rand(B, N, 3) * 1.5).astype(np.float32)
    conf = rng.randn(B, N).astype(np.float32)
    conf[:, 10:20] = conf[:, 0:1]  # ties
    seeds, lm = kernels.pick_seeds(_t(src, gpu_device), _t(conf, gpu_device), radius, 150)
    lm = lm.cpu().numpy()
    for b in range(B):
        assert np.array_equal(lm[b], O.local_max(src[b], conf[b], radius)), b


@pytest.mark.parametrize("B,N,S,zeros", [(3, 1000, 100, 0.0), (2, 5000, 500, 0.97), (1, 777, 77, 1.0),
                                          (2, 9000, 900, 0.5), (1, 3000, 2999, 0.3)])
def test_seed_ranking_ties(B, N, S, zeros, gpu_device):
    """a5's ranking = argsort(score, descending) with ties by ascending index, on
    scores with a fraction of exact zeros (non-maxima, +0 and -0), duplicates
    and negatives.  radius 0: every point a local maximum, so the scores are the
    confidences themselves."""
    from pointdsc_amd import kernels
    rng = np.random.RandomState(N + S)
    src = rng.rand(B, N, 3).astype(np.float32)
    conf = np.round(rng.randn(B, N), 2).astype(np.float32)  # many duplicates
    z = rng.rand(B, N) < zeros
    conf[z] = np.where(rng.rand(int(z.sum())) < 0.5, 0.0, -0.0).astype(np.float32)
    seeds, lm = kernels.pick_seeds(_t(src, gpu_device), _t(conf, gpu_device), 0.0, S)
    seeds = seeds.cpu().numpy()
    assert lm.cpu().numpy().min() == 1.0
    for b in range(B):
        order = sorted(range(N), key=lambda i: (-float(conf[b, i]), i))[:S]
        assert np.array_equal(seeds[b], np.array(order, np.int32)), b


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("N", [300, 2000, 5000, 9000])  # 9000: rows past the register variants (R = 0)
def test_seed_knn_random(N, precision, gpu_device):
    """a6 (seed-row distances + register radix select) against the oracle's fp32
    restatement, up to near-ties (assert_knn_equivalent); duplicate rows make
    exact distance ties that must resolve by ascending index."""
    from oracle import pdsc_oracle as O
    from pointdsc_amd import kernels
    rng = np.random.RandomState(N)
    f = rng.randn(1, N, 128).astype(np.float32)
    f[0, 50:60] = f[0, 40]  # exact ties
    f /= np.linalg.norm(f, axis=-1, keepdims=True)
    S = N // 10
    seeds = rng.choice(N, S, replace=False).astype(np.int32)
    seeds[0] = 40
    k = 40
    knn = kernels.seed_knn(_t(f, gpu_device), _t(seeds[None], gpu_device, torch.int32), k,
                           precision=precision)[0].cpu().numpy()
    ref = O.knn_seed_rows(f[0], seeds.astype(np.int64), k)
    assert_knn_equivalent(knn, ref, f[0], seeds)
    # the tie group of seed 40 (rows 40, 50..59 identical): ascending index after the dropped first
    assert list(knn[0][:10]) == list(ref[0][:10])


@pytest.mark.parametrize("k,dups", [(40, 0), (63, 0), (63, 300), (40, 300), (8, 2)])
def test_seed_knn_select_paths(k, dups, gpu_device):
    """knn_select's lane-minimum threshold fast path (want = k+1 <= 64, <= 128
    qualifying keys) and its radix fallback (`dups` copies of a seed's
    row giving > 128 keys tied at the threshold) pick the same (key, index)-ordered
    neighbours as the oracle."""
    from oracle import pdsc_oracle as O
    from pointdsc_amd import kernels
    N = 3000
    rng = np.random.RandomState(7 + k + dups)
    f = rng.randn(1, N, 128).astype(np.float32)
    if dups:
        f[0, 1000:1000 + dups] = f[0, 5]
    f /= np.linalg.norm(f, axis=-1, keepdims=True)
    seeds = rng.choice(N, 200, replace=False).astype(np.int32)
    seeds[0] = 5
    seeds[1] = 1000
    knn = kernels.seed_knn(_t(f, gpu_device), _t(seeds[None], gpu_device, torch.int32), k)[0].cpu().numpy()
    ref = O.knn_seed_rows(f[0], seeds.astype(np.int64), k)
    assert_knn_equivalent(knn, ref, f[0], seeds)
    if dups:
        assert list(knn[0]) == list(ref[0])  # the tie group resolves by ascending index


@pytest.mark.parametrize("name,B,N,S,k,dups", [("b16_1k", 16, 1000, 100, 40, 0), ("b2_5k", 2, 5000, 500, 40, 0),
                                                ("odd_777", 3, 777, 77, 63, 0), ("ties_3k", 1, 3000, 200, 40, 300)])
def test_seed_knn_batched_cases(name, B, N, S, k, dups, gpu_device):
    """The seed kNN (knn_dist + knn_select) on batches vs the oracle row by row: a
    batch, N % 32 != 0 with k = 63, and a 300-point tie group (exact duplicate
    features) that resolves by ascending index."""
    from oracle import pdsc_oracle as O
    from pointdsc_amd import kernels
    rng = np.random.RandomState(N + B)
    f = rng.randn(B, N, 128).astype(np.float32)
    if dups:
        f[:, 1000:1000 + dups] = f[:, 5:6]
    f /= np.linalg.norm(f, axis=-1, keepdims=True)
    seeds = np.stack([rng.choice(N, S, replace=False) for _ in range(B)]).astype(np.int32)
    if dups:
        seeds[:, 0], seeds[:, 1] = 5, 1000
    knn = kernels.seed_knn(_t(f, gpu_device), _t(seeds, gpu_device, torch.int32), k).cpu().numpy()
    for b in range(B):
        ref = O.knn_seed_rows(f[b], seeds[b].astype(np.int64), k)
        assert_knn_equivalent(knn[b], ref, f[b], seeds[b])
        if dups:
            assert list(knn[b][0]) == list(ref[0]) and list(knn[b][1]) == list(ref[1])
