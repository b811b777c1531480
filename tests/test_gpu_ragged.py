"""Ragged batches (pdsc_forward_testing_ragged, PointDSC.forward_list): pairs of
different N in one call -- the evaluation loop's shape (datasets/ThreeDMatch.py:
268-290 keeps every keypoint of a fragment, so N differs per pair;
evaluation/test_3DMatch.py:33-53 feeds them one by one at bs = 1).  Run with -m gpu.

  * against the oracle (the reference's algorithm, pinned to its goldens), pair
    by pair: labels bit-exact and poses within 1e-4 -- or, where fp32 rounding
    decided a seed / kNN near-tie the other way, the oracle run on OUR seeds and
    kNN rows within 1e-4 (tests/test_gpu_bench_parity.py);
  * no cross-pair leakage: a pair's outputs are bitwise those of the same pair in
    a batch of the same shape (B, N: the same kernel plan) made of copies of it;
  * against per-pair ``forward`` calls (other launch plans, other fp32 summation
    orders): labels bitwise, poses within north_star's 1e-4 -- or, where the two
    fp32 orders decided a seed / kNN near-tie differently, BOTH results held to
    the oracle by the near-tie rules (conftest.assert_held_to_oracle);
  * counts all equal to the padded N: bitwise the uniform entry (the same
    attention form, Ragged::eq), at every plan (fused 64 / 128 pairs, the
    64-query-wave stream-K plan at 65)."""
import numpy as np
import pytest
import torch

from conftest import assert_held_to_oracle, assert_knn_equivalent

pytestmark = pytest.mark.gpu

SIZES = [777, 1000, 5000, 12000]


def _model(dev, precision="h3"):
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, trained_state_dict
    p = PRESETS["3dmatch"]
    m = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"],
                 precision=precision)
    sd = trained_state_dict("3dmatch", 12, *BENCH_CLS)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return m.to(dev).eval(), sd


def _pairs(sizes, seed=77):
    from pointdsc_amd.synthetic import synthetic_pair
    return [synthetic_pair(n, seed * 1000 + i) for i, n in enumerate(sizes)]


def _datas(ps, dev):
    return [{k: torch.from_numpy(q[k])[None].to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts")} for q in ps]


def _ragged_stages(m, ds):
    """forward_list's call with every stage's output: (T, L, stage dict on host, counts)."""
    from pointdsc_amd import kernels
    corr, counts = kernels.pad_pairs([d["corr_pos"] for d in ds])
    src, _ = kernels.pad_pairs([d["src_keypts"] for d in ds])
    tgt, _ = kernels.pad_pairs([d["tgt_keypts"] for d in ds])
    T, L, st = kernels.forward_ragged(m.pdsc_config(), m.packed_weights(), corr, src, tgt, counts, debug=True)
    return T, L, {k: v.cpu().numpy() for k, v in st.items()}, counts


def _vs_single(m, sd, q, d, Tb, Lb, stb, n, what):
    """Pair b of a batched call against its own bs = 1 forward: labels bitwise;
    poses within 1e-4, or both held to the oracle by the near-tie rules."""
    from pointdsc_amd import kernels
    r = m(dict(d, testing=True))
    assert torch.equal(r["final_labels"][0], Lb[:n]), what
    dT = float((r["final_trans"][0] - Tb).abs().max())
    if dT <= 1e-4:
        return "equal"
    one = kernels.forward_stages(m.pdsc_config(), m.packed_weights(), d["corr_pos"], d["src_keypts"], d["tgt_keypts"])
    one = {k: v[0].cpu().numpy() for k, v in one.items()}
    S = int(n * 0.1)
    for name, (lab, tr, conf, seeds, knn) in {
            "single": (one["final_labels"], one["final_trans"], one["conf"], one["seeds"], one["knn"]),
            "batched": (Lb[:n].cpu().numpy(), Tb.cpu().numpy(), stb["conf"][:n], stb["seeds"][:S], stb["knn"][:S])}.items():
        assert_held_to_oracle(q, lab, tr, conf, seeds, knn, sd, f"{what} {name} (dT {dT:.3g})", num_layers=12)
    return "near-tie"


@pytest.mark.parametrize("precision", ["h3", "f32"])
def test_ragged_vs_oracle(precision, gpu_device):
    from oracle import pdsc_oracle as O
    from pointdsc_amd import kernels
    m, sd = _model(gpu_device, precision)
    ps = _pairs(SIZES)
    ds = _datas(ps, gpu_device)
    res = m.forward_list(ds)
    corr, counts = kernels.pad_pairs([d["corr_pos"] for d in ds])
    src, _ = kernels.pad_pairs([d["src_keypts"] for d in ds])
    tgt, _ = kernels.pad_pairs([d["tgt_keypts"] for d in ds])
    T, L, st = kernels.forward_ragged(m.pdsc_config(), m.packed_weights(), corr, src, tgt, counts, debug=True)
    assert all(torch.equal(r["final_trans"][0], T[b]) for b, r in enumerate(res))
    assert float(L[0, counts[0]:].abs().sum()) == 0.0  # rows past a pair's count are 0
    st = {k: v.cpu().numpy() for k, v in st.items()}
    for b, (q, n) in enumerate(zip(ps, counts)):
        lab, tr = res[b]["final_labels"][0].cpu().numpy(), res[b]["final_trans"][0].cpu().numpy()
        assert lab.shape == (n,)
        S = int(n * 0.1)
        seeds, knn = st["seeds"][b, :S], st["knn"][b, :S]
        r = O.forward_testing(q["corr_pos"], q["src_keypts"], q["tgt_keypts"], sd, num_layers=12, record=True)
        if np.abs(tr - r["final_trans"]).max() <= 1e-4 and np.array_equal(lab, r["final_labels"]):
            continue
        # a near-tie decided the other way: the stages after it pinned on our decisions
        assert np.abs(st["conf"][b, :n] - r["confidence"]).max() <= 1e-3 * max(1.0, np.abs(r["confidence"]).max())
        r2 = O.forward_testing(q["corr_pos"], q["src_keypts"], q["tgt_keypts"], sd, num_layers=12, seeds=seeds,
                               record=True)
        assert_knn_equivalent(knn, r2["knn_idx"], r2["normed"], seeds)
        r3 = O.forward_testing(q["corr_pos"], q["src_keypts"], q["tgt_keypts"], sd, num_layers=12, seeds=seeds,
                               knn_idx=knn)
        assert np.array_equal(lab, r3["final_labels"]), f"pair {b} (N={n})"
        np.testing.assert_allclose(tr, r3["final_trans"], atol=1e-4, err_msg=f"pair {b} (N={n})")


def test_ragged_no_cross_pair_leakage(gpu_device):
    """Pair b of a mixed batch == pair b in a batch of B copies of it (same B and
    padded N, so the same kernel plan), bitwise: nothing of the other pairs (their
    rows, keys, seeds or padding) reaches it."""
    from pointdsc_amd import kernels
    m, _ = _model(gpu_device)
    sizes = [777, 1000, 3000, 2111, 5000]
    ds = _datas(_pairs(sizes, seed=78), gpu_device)
    N = max(sizes)
    corr, counts = kernels.pad_pairs([d["corr_pos"] for d in ds], N)
    src, _ = kernels.pad_pairs([d["src_keypts"] for d in ds], N)
    tgt, _ = kernels.pad_pairs([d["tgt_keypts"] for d in ds], N)
    T, L = kernels.forward_ragged(m.pdsc_config(), m.packed_weights(), corr, src, tgt, counts)
    for b in (0, 2, 3):
        B = len(sizes)
        rep = lambda x: x[b:b + 1].expand(B, -1, -1).contiguous()  # noqa: E731
        T1, L1 = kernels.forward_ragged(m.pdsc_config(), m.packed_weights(), rep(corr), rep(src), rep(tgt),
                                        [counts[b]] * B)
        assert torch.equal(T1[0], T[b]) and torch.equal(L1[0], L[b]), b


def test_ragged_uniform_equals_batched(gpu_device):
    """Counts all equal to N: bitwise the uniform batched forward."""
    from pointdsc_amd import kernels
    from pointdsc_amd.synthetic import synthetic_batch
    m, _ = _model(gpu_device)
    d = synthetic_batch(24, 1000, seed=79)
    corr, src, tgt = (torch.from_numpy(d[k]).to(gpu_device) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    T, L = m.forward_batched(corr, src, tgt)
    T2, L2 = kernels.forward_ragged(m.pdsc_config(), m.packed_weights(), corr, src, tgt, [1000] * 24)
    assert torch.equal(T, T2) and torch.equal(L, L2)


@pytest.mark.parametrize("B", [64, 65, 128])
def test_ragged_halves_equal_uniform(B, gpu_device):
    """From 32 pairs on the fused plan a ragged batch runs the encoder as two half
    batches on two streams (api.hip: run_encoder_fwd), each keeping the whole
    batch's plan (at 64 pairs a half of 32 alone would take the unfused chains);
    with every count N it is bitwise the uniform forward, which stays on one
    stream.  (Odd splits: test_ragged_vs_single_forwards[130] and the other
    ragged tests, which all run with the halves.)  65 pairs leave the fused plan
    for the 64-query-wave split plan (pdsc_encoder_plan 2, two key splits), where
    the uniform entry runs the stream-K attention: a ragged call whose counts
    all equal N takes it too (Ragged::eq), so it is bitwise the uniform call --
    round 5 measured conf 8.6e-5 / poses 2.1e-4 apart when the ragged call ran
    the split grid, another key partition (profiles/r05_ragged_halves_eq.log)."""
    import ctypes
    from pointdsc_amd import _lib, kernels
    plan = ctypes.c_int32()
    _lib.check(_lib.load().pdsc_encoder_plan(B, 1000, 0, ctypes.byref(plan)), "encoder_plan")
    assert plan.value == (2 if B == 65 else 1), (B, plan.value)
    from pointdsc_amd.synthetic import synthetic_batch
    m, _ = _model(gpu_device)
    d = synthetic_batch(B, 1000, seed=83)
    corr, src, tgt = (torch.from_numpy(d[k]).to(gpu_device) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    T, L = m.forward_batched(corr, src, tgt)
    T2, L2 = kernels.forward_ragged(m.pdsc_config(), m.packed_weights(), corr, src, tgt, [1000] * B)
    assert torch.equal(T, T2) and torch.equal(L, L2)


def test_ragged_halves_graph_capture(gpu_device):
    """The halves' event fork / join onto the side stream records into a HIP
    graph: a captured ragged forward (128 pairs, N in [700, 1300]: the fused
    plan, bench.py's ragged leg) replays to bitwise the eager results."""
    from pointdsc_amd import kernels
    m, _ = _model(gpu_device)
    rng = np.random.RandomState(5)
    sizes = rng.randint(700, 1301, size=128).tolist()
    ds = _datas(_pairs(sizes, seed=84), gpu_device)
    corr, counts = kernels.pad_pairs([d["corr_pos"] for d in ds])
    src, _ = kernels.pad_pairs([d["src_keypts"] for d in ds])
    tgt, _ = kernels.pad_pairs([d["tgt_keypts"] for d in ds])
    cfg, pk = m.pdsc_config(), m.packed_weights()
    T, L = kernels.forward_ragged(cfg, pk, corr, src, tgt, counts, check_range=False)  # eager (and warm)
    torch.cuda.synchronize(gpu_device)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        Tg, Lg = kernels.forward_ragged(cfg, pk, corr, src, tgt, counts, check_range=False)
    g.replay()
    torch.cuda.synchronize(gpu_device)
    assert torch.equal(T, Tg) and torch.equal(L, Lg)


@pytest.mark.parametrize("B", [8, 130])
def test_ragged_vs_single_forwards(B, gpu_device):
    """forward_list over B pairs of N in [600, 1400] (B = 130: the fused
    attention + pointwise launches) against B separate ``forward`` calls."""
    m, sd = _model(gpu_device)
    rng = np.random.RandomState(B)
    sizes = rng.randint(600, 1401, size=B).tolist()
    ps = _pairs(sizes, seed=80 + B)
    ds = _datas(ps, gpu_device)
    res = m.forward_list(ds)
    T, L, st, counts = _ragged_stages(m, ds)
    for b in range(0, B, max(1, B // 16)):
        assert torch.equal(T[b], res[b]["final_trans"][0])
        stb = {k: v[b] for k, v in st.items()}
        _vs_single(m, sd, ps[b], ds[b], T[b], L[b], stb, counts[b], f"pair {b} (N={counts[b]})")


@pytest.mark.parametrize("sizes", [[777, 1000, 3000, 2111, 5000],  # key-split plan
                                   [1000 - 7 * i for i in range(40)],  # fused attention + chain
                                   [5000 - 13 * i for i in range(8)]])  # 64-query-wave split plan
def test_ragged_padding_content_ignored(sizes, gpu_device):
    """Rows past counts[b] are ignored whatever they hold (include/pdsc.h): NaN
    corr_pos and 1e30 coordinates there give bitwise the zero-padded call's poses,
    labels and the pairs' own logits -- and no range-guard mark."""
    from pointdsc_amd import kernels
    m, _ = _model(gpu_device)
    ds = _datas(_pairs(sizes, seed=81), gpu_device)
    N = max(sizes)
    corr, counts = kernels.pad_pairs([d["corr_pos"] for d in ds], N)
    src, _ = kernels.pad_pairs([d["src_keypts"] for d in ds], N)
    tgt, _ = kernels.pad_pairs([d["tgt_keypts"] for d in ds], N)
    T, L, st = kernels.forward_ragged(m.pdsc_config(), m.packed_weights(), corr, src, tgt, counts, debug=True)
    c2, s2, t2 = corr.clone(), src.clone(), tgt.clone()
    for b, n in enumerate(counts):
        c2[b, n:] = float("nan")
        s2[b, n:] = 1e30
        t2[b, n:] = -1e30
    T2, L2, st2 = kernels.forward_ragged(m.pdsc_config(), m.packed_weights(), c2, s2, t2, counts, debug=True)
    assert torch.equal(T, T2) and torch.equal(L, L2)
    for b, n in enumerate(counts):
        assert torch.equal(st["conf"][b, :n], st2["conf"][b, :n]), b


def test_forward_list_small_pairs(gpu_device):
    """Pairs with count <= k (their forward clips k to count - 1, :250) in a list
    with larger ones: forward_list runs them alone (bitwise their own forward),
    the rest as one ragged batch; every pair matches its own forward."""
    m, sd = _model(gpu_device)
    sizes = [30, 1000, 41, 800, 12]
    ps = _pairs(sizes, seed=82)
    ds = _datas(ps, gpu_device)
    res = m.forward_list(ds)
    big = [b for b, n in enumerate(sizes) if n > 40]
    T, L, st, _ = _ragged_stages(m, [ds[b] for b in big])
    for b, n in enumerate(sizes):
        r = m(dict(ds[b], testing=True))
        assert res[b]["final_labels"].shape == (1, n)
        assert torch.equal(r["final_labels"], res[b]["final_labels"]), b
        if n <= 40:
            assert torch.equal(r["final_trans"], res[b]["final_trans"]), b
            continue
        j = big.index(b)
        assert torch.equal(T[j], res[b]["final_trans"][0])
        _vs_single(m, sd, ps[b], ds[b], T[j], L[j], {k: v[j] for k, v in st.items()}, n, f"pair {b} (N={n})")


def test_ragged_w64_extra_split_slots(gpu_device):
    """24 pairs up to N = 1500 take the 64-query-wave split plan with 3 partial
    slots per query block (the stream-K count a uniform batch of this shape
    would use); a ragged batch runs the split grid, whose one key split leaves
    slots 1 and 2 as empty splits (m = -inf, skipped by the combine).  Against
    per-pair ``forward`` calls: labels bitwise, poses within 1e-4 or both held
    to the oracle (near-tie rules)."""
    import ctypes
    from pointdsc_amd import _lib
    m, sd = _model(gpu_device)
    sizes = [1500 - 17 * i for i in range(24)]
    plan, npad, ns = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    _lib.check(_lib.load().pdsc_encoder_plan(24, 1500, 0, ctypes.byref(plan)), "encoder_plan")
    _lib.check(_lib.load().pdsc_attention_layout(24, 1500, 0, ctypes.byref(npad), ctypes.byref(ns)), "layout")
    assert plan.value == 2 and ns.value == 3, (plan.value, ns.value)
    ps = _pairs(sizes, seed=91)
    ds = _datas(ps, gpu_device)
    res = m.forward_list(ds)
    T, L, st, counts = _ragged_stages(m, ds)
    for b in range(0, 24, 3):
        assert torch.equal(T[b], res[b]["final_trans"][0])
        _vs_single(m, sd, ps[b], ds[b], T[b], L[b], {k: v[b] for k, v in st.items()}, counts[b], f"pair {b}")
