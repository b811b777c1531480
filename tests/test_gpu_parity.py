"""HIP path vs the reference's golden vectors and the CPU oracle (run with -m gpu).

Tolerances (north_star): inlier masks / seeds / kNN / fitness bit-exact;
confidences and poses within 1e-4 (fp32).  Every call goes through the C ABI
(libpdsc.so) via pointdsc_amd.kernels."""
import numpy as np
import pytest
import torch

from conftest import (assert_close_scaled, assert_knn_equivalent, assert_seeds_equivalent, golden_hparams, golden_names,
                      golden_state_dict, load_golden)

pytestmark = pytest.mark.gpu

NAMES = golden_names()
POSE_ATOL = 1e-4


def _t(x, dev, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev, dtype)


def _model(g, dev):
    from pointdsc_amd.PointDSC import PointDSC
    hp = golden_hparams(g)
    m = PointDSC(in_dim=6, num_layers=hp["num_layers"], num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=hp["inlier_threshold"], sigma_d=float(g["sigma_d"]), k=40,
                 nms_radius=hp["nms_radius"])
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in golden_state_dict(g).items()})
    return m.to(dev).eval()


def _inputs(g, dev):
    return (_t(g["corr_pos"][None], dev), _t(g["src_keypts"][None], dev), _t(g["tgt_keypts"][None], dev))


@pytest.mark.parametrize("name", NAMES)
def test_compat(name, gpu_device):
    from pointdsc_amd import kernels
    g = load_golden(name)
    _, src, tgt = _inputs(g, gpu_device)
    sd = torch.tensor([float(g["sigma_d"])], dtype=torch.float32, device=gpu_device)
    M = kernels.compat(src, tgt, sd)[0].cpu().numpy()
    if "M" in g:
        assert np.array_equal(M, g["M"])  # bit-exact
    assert np.array_equal(np.diagonal(M), g["M_diag"])
    assert np.array_equal(M, M.T)
    np.testing.assert_allclose(M.astype(np.float64).sum(-1), g["M_row_sums"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("name", NAMES)
def test_encoder_and_classifier(name, gpu_device):
    from pointdsc_amd import kernels
    g = load_golden(name)
    m = _model(g, gpu_device)
    corr, src, tgt = _inputs(g, gpu_device)
    M = kernels.compat(src, tgt, m.sigma_spat)
    feat, normed, conf = kernels.encoder(m.pdsc_config(), m.packed_weights(), corr, M)
    assert_close_scaled(feat[0].cpu().numpy(), g["corr_features"])
    np.testing.assert_allclose(conf[0].cpu().numpy(), g["confidence"], rtol=1e-5, atol=1e-3)
    ref_n = g["corr_features"] / np.maximum(np.linalg.norm(g["corr_features"], axis=1, keepdims=True), 1e-12)
    np.testing.assert_allclose(normed[0].cpu().numpy(), ref_n, atol=1e-4)  # unit vectors


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


@pytest.mark.parametrize("name", NAMES)
def test_nsm_chain(name, gpu_device):
    """a6-a11, each stage fed with the reference's inputs for that stage."""
    from pointdsc_amd import kernels
    g = load_golden(name)
    sd = golden_state_dict(g)
    _, src, tgt = _inputs(g, gpu_device)
    f = g["corr_features"]
    nrm = f / np.maximum(np.linalg.norm(f, axis=1, keepdims=True), 1e-12)
    normed = _t(nrm, gpu_device)[None]
    seeds = _t(g["seeds"][None], gpu_device, torch.int32)
    k = g["knn_idx"].shape[1]
    knn = kernels.seed_knn(normed, seeds, k)
    assert_knn_equivalent(knn[0].cpu().numpy(), g["knn_idx"], nrm, g["seeds"])
    ref_knn = _t(g["knn_idx"][None], gpu_device, torch.int32)
    sigma = _t(sd["sigma"], gpu_device)
    sigma_d = _t(sd["sigma_spat"], gpu_device)
    w, iters = kernels.nsm_weights(normed, src, tgt, ref_knn, 10, sigma, sigma_d)
    v = g["leading_eig"]
    np.testing.assert_allclose(w[0].cpu().numpy(), v / (v.sum(-1, keepdims=True) + 1e-6), atol=2e-5)
    w_ref = _t((v / (v.sum(-1, keepdims=True) + np.float32(1e-6)))[None], gpu_device)
    seed_trans, fit, best, trans, labels = kernels.seed_hypotheses(src, tgt, ref_knn, w_ref,
                                                                   float(g["inlier_threshold"]))
    np.testing.assert_allclose(seed_trans[0].cpu().numpy(), g["seed_trans"], atol=POSE_ATOL)
    assert np.array_equal(fit[0].cpu().numpy(), g["seed_fitness"])
    np.testing.assert_allclose(trans[0].cpu().numpy(), g["trans_pre_refine"], atol=POSE_ATOL)
    assert np.array_equal(labels[0].cpu().numpy(), g["final_labels"])
    thr = 0.10 if float(g["inlier_threshold"]) == 0.10 else 1.2
    ref = kernels.post_refine(_t(g["trans_pre_refine"][None], gpu_device), src, tgt, thr)
    np.testing.assert_allclose(ref[0].cpu().numpy(), g["final_trans"], atol=POSE_ATOL)


@pytest.mark.parametrize("name", NAMES)
def test_module_forward_end_to_end(name, gpu_device):
    """PointDSC.forward(data) with 'testing' -- the drop-in contract."""
    g = load_golden(name)
    m = _model(g, gpu_device)
    corr, src, tgt = _inputs(g, gpu_device)
    with torch.no_grad():
        res = m({"corr_pos": corr, "src_keypts": src, "tgt_keypts": tgt, "testing": True})
    assert res["M"] is None
    assert res["final_trans"].shape == (1, 4, 4) and res["final_labels"].shape == (1, len(g["src_keypts"]))
    assert np.array_equal(res["final_labels"][0].cpu().numpy(), g["final_labels"])
    np.testing.assert_allclose(res["final_trans"][0].cpu().numpy(), g["final_trans"], atol=POSE_ATOL)


@pytest.mark.parametrize("name", ["rel_1k", "rel_1k_kitti"])
def test_debug_outputs_match_reference(name, gpu_device):
    from pointdsc_amd import kernels
    g = load_golden(name)
    m = _model(g, gpu_device)
    corr, src, tgt = _inputs(g, gpu_device)
    trans, labels, conf, seeds = kernels.forward_testing(m.pdsc_config(), m.packed_weights(), corr, src, tgt,
                                                         debug=True)
    np.testing.assert_allclose(conf[0].cpu().numpy(), g["confidence"], rtol=1e-5, atol=1e-3)
    ours = set(seeds[0].cpu().numpy().tolist())
    assert len(ours & set(g["seeds"].tolist())) >= 0.98 * len(g["seeds"])


def test_batched_equals_single(gpu_device):
    """B pairs in one call == B single-pair calls (labels bitwise; poses within
    the north-star pose tolerance: the attention's split-K over keys depends on
    B, so the softmax partials combine in a different fp32 order)."""
    from pointdsc_amd.synthetic import synthetic_batch
    g = load_golden("rel_1k")
    m = _model(g, gpu_device)
    b = synthetic_batch(6, 1000, seed=5)
    corr, src, tgt = (_t(b[k], gpu_device) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    T, Lb = m.forward_batched(corr, src, tgt)
    for i in range(6):
        r = m({"corr_pos": corr[i:i + 1], "src_keypts": src[i:i + 1], "tgt_keypts": tgt[i:i + 1],
               "testing": True})
        assert torch.equal(r["final_labels"][0], Lb[i])
        # two fp32 evaluation orders of the same pair (split-K differs with B), each
        # within POSE_ATOL of the reference on the goldens: allow twice that between them
        np.testing.assert_allclose(r["final_trans"][0].cpu().numpy(), T[i].cpu().numpy(), atol=2 * POSE_ATOL)


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


def test_attention_vs_torch_fp32(gpu_device):
    """The attention kernel against a plain PyTorch fp32 reference of :36-42."""
    from pointdsc_amd import kernels
    torch.manual_seed(0)
    for B, N in [(1, 1000), (2, 333), (1, 4096)]:
        q, k, v = (torch.randn(B, N, 128, device=gpu_device) for _ in range(3))
        src = torch.rand(B, N, 3, device=gpu_device) * 3
        tgt = src + 0.05 * torch.randn(B, N, 3, device=gpu_device)
        M = kernels.compat(src, tgt, torch.tensor([0.1], device=gpu_device))
        out = kernels.attention(q, k, v, M)
        ref = torch.softmax(M.double() * (q.double() @ k.double().transpose(1, 2)) / 128 ** 0.5, -1) @ v.double()
        np.testing.assert_allclose(out.cpu().numpy(), ref.float().cpu().numpy(), rtol=1e-4, atol=2e-5)


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


@pytest.mark.parametrize("preset", ["3dmatch", "kitti"])
def test_full_size_registration_properties(preset, gpu_device):
    """N=5000, B=4 (BASELINE sizes): the recovered pose matches ground truth and
    every label set is the inlier set of the returned pre-refinement pose."""
    from pointdsc_amd.synthetic import PRESETS, synthetic_batch, trained_state_dict
    from pointdsc_amd.PointDSC import PointDSC
    p = PRESETS[preset]
    m = PointDSC(num_layers=12, inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"],
                 nms_radius=p["nms_radius"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict(preset).items()})
    m = m.to(gpu_device).eval()
    b = synthetic_batch(4, 5000, seed=77, preset=preset)
    corr, src, tgt = (_t(b[k], gpu_device) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    T, labels = m.forward_batched(corr, src, tgt)
    T, labels = T.cpu().numpy(), labels.cpu().numpy()
    for i in range(4):
        gt = b["gt_trans"][i]
        cosang = (np.trace(T[i, :3, :3].T @ gt[:3, :3]) - 1) / 2
        re = np.degrees(np.arccos(np.clip(cosang, -1, 1)))
        te = np.linalg.norm(T[i, :3, 3] - gt[:3, 3])
        assert re < 1.0 and te < 0.2 * p["inlier_threshold"] * 10, (re, te)
        assert labels[i].sum() >= 0.9 * b["gt_labels"][i].sum()
        assert set(np.unique(labels[i])) <= {0.0, 1.0}


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


@pytest.mark.parametrize("N", [300, 2000, 5000, 9000])  # 9000: rows past the register variants (R = 0)
def test_seed_knn_random(N, gpu_device):
    """a6 (split-fp16 distances + register radix select) against the oracle's
    fp32 restatement, up to near-ties (assert_knn_equivalent); duplicate rows
    make exact distance ties that must resolve by ascending index."""
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
    knn = kernels.seed_knn(_t(f, gpu_device), _t(seeds[None], gpu_device, torch.int32), k)[0].cpu().numpy()
    ref = O.knn_seed_rows(f[0], seeds.astype(np.int64), k)
    assert_knn_equivalent(knn, ref, f[0], seeds)
    # the tie group of seed 40 (rows 40, 50..59 identical): ascending index after the dropped first
    assert list(knn[0][:10]) == list(ref[0][:10])


@pytest.mark.gpu
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
