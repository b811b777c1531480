"""The fp16 range guard (include/pdsc.h, PDSC_ERR_RANGE; run with -m gpu).

A pair whose coordinates are scaled by 1e5 drives the encoder's activations far
past fp16's 65504, where the 3xfp16 split cannot represent them.  The bar: no
call ever hands back that pair's NaN pose as a success --
  * the testing forward marks it (pdsc_range_status -> PDSC_ERR_RANGE, the
    kernels wrappers raise RangeError), poisons its pose (NaN) and labels (0),
    and leaves every other pair of the batch bitwise as without it;
  * the module (PointDSC.forward_batched / forward / forward_list) reruns the
    marked pair with exact fp32 contractions: its result is bitwise the 'f32'
    model's, the other pairs' the 'h3' model's;
  * the exact-fp32 mode itself takes the scaled pair without a mark;
  * a normal batch has no marks (PDSC_OK)."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SCALE = 1e5


def _model(dev, precision):
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, trained_state_dict
    p = PRESETS["3dmatch"]
    m = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"],
                 precision=precision)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict("3dmatch", 12, *BENCH_CLS).items()})
    return m.to(dev).eval()


def _batch(dev, B=4, N=1000, bad=(2,)):
    from pointdsc_amd.synthetic import synthetic_pair
    ps = [synthetic_pair(N, 4242 + i) for i in range(B)]
    corr = np.stack([q["corr_pos"] for q in ps])
    for b in bad:
        corr[b] = corr[b] * SCALE
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return t(corr), t(np.stack([q["src_keypts"] for q in ps])), t(np.stack([q["tgt_keypts"] for q in ps]))


def test_range_marks_and_poisons(gpu_device):
    from pointdsc_amd import kernels
    m = _model(gpu_device, "h3")
    corr, src, tgt = _batch(gpu_device)
    with pytest.raises(kernels.RangeError) as ei:
        kernels.forward_testing(m.pdsc_config(), m.packed_weights(), corr, src, tgt)
    assert ei.value.pairs == [2]
    T, L = ei.value.outputs
    assert torch.isnan(T[2]).all() and float(L[2].abs().sum()) == 0.0
    # the other pairs: bitwise as in the same batch without the scaled pair
    corr0, _, _ = _batch(gpu_device, bad=())
    T0, L0 = kernels.forward_testing(m.pdsc_config(), m.packed_weights(), corr0, src, tgt)
    for b in (0, 1, 3):
        assert torch.equal(T[b], T0[b]) and torch.equal(L[b], L0[b]), b
        assert torch.isfinite(T[b]).all()
    # the C ABI: PDSC_ERR_RANGE with the flags; PDSC_OK on the normal batch
    from pointdsc_amd import _lib
    L_ = _lib.load()
    plan = kernels.ForwardPlan(m.pdsc_config(), m.packed_weights(), 4, 1000, gpu_device)
    plan.run(corr, src, tgt)
    flags = (ctypes.c_int32 * 4)()
    assert L_.pdsc_range_status(kernels._p(plan.ws), 4, flags, kernels._stream(gpu_device)) == kernels.PDSC_ERR_RANGE
    assert list(flags) == [0, 0, 1, 0]
    # pdsc_range_poll: the same answer through the host word, repeatedly (the sequence advances)
    for _ in range(3):
        assert L_.pdsc_range_poll(kernels._p(plan.ws), 4, kernels._stream(gpu_device)) == kernels.PDSC_ERR_RANGE
    assert L_.pdsc_range_poll(kernels._p(plan.ws), 2, kernels._stream(gpu_device)) == 0  # pairs 0-1 unmarked
    plan.run(corr0, src, tgt)
    assert L_.pdsc_range_poll(kernels._p(plan.ws), 4, kernels._stream(gpu_device)) == 0
    assert L_.pdsc_range_status(kernels._p(plan.ws), 4, flags, kernels._stream(gpu_device)) == 0
    assert list(flags) == [0, 0, 0, 0]
    # the poll returns once the stream's earlier work has run: the outputs are final
    plan.run(corr, src, tgt)
    assert L_.pdsc_range_poll(kernels._p(plan.ws), 4, kernels._stream(gpu_device)) == kernels.PDSC_ERR_RANGE
    assert torch.isnan(plan.trans[2]).all() and torch.isfinite(plan.trans[0]).all()


def test_range_poll_behind_a_long_queue(gpu_device):
    """pdsc_range_poll when the stream holds more than its 20 ms spin (a GPU
    sleep enqueued ahead of the forward): it falls back to hipStreamSynchronize
    and still returns the forward's own answer, with the outputs final."""
    from pointdsc_amd import _lib, kernels
    m = _model(gpu_device, "h3")
    corr, src, tgt = _batch(gpu_device)
    corr0, _, _ = _batch(gpu_device, bad=())
    L_ = _lib.load()
    plan = kernels.ForwardPlan(m.pdsc_config(), m.packed_weights(), 4, 1000, gpu_device)
    s = kernels._stream(gpu_device)
    import time
    plan.run(corr0, src, tgt)
    torch.cuda.synchronize()
    t_sleep = time.perf_counter()
    torch.cuda._sleep(int(1e8))  # >= 50 ms of GPU spin (1e8 clocks) ahead of the forward
    torch.cuda.synchronize()
    t_sleep = time.perf_counter() - t_sleep
    assert t_sleep > 0.03, t_sleep  # (else the case would not reach the fallback)
    for c, want in ((corr, kernels.PDSC_ERR_RANGE), (corr0, 0)):
        t0 = time.perf_counter()
        torch.cuda._sleep(int(1e8))
        plan.run(c, src, tgt)
        assert L_.pdsc_range_poll(kernels._p(plan.ws), 4, s) == want
        assert time.perf_counter() - t0 >= 0.9 * t_sleep  # it waited for the queue
    assert torch.isfinite(plan.trans).all()


def test_range_poll_two_threads(gpu_device):
    """pdsc_range_poll's host word is per host thread: two threads, each on its
    own stream and plan (one batch marked, one not), polling concurrently, each
    get their own forward's answer every time."""
    import threading
    from pointdsc_amd import _lib, kernels
    m = _model(gpu_device, "h3")
    corr, src, tgt = _batch(gpu_device)
    corr0, _, _ = _batch(gpu_device, bad=())
    L_ = _lib.load()
    cfg, pk = m.pdsc_config(), m.packed_weights()
    errors = []

    def worker(c, want):
        try:
            st = torch.cuda.Stream(gpu_device)
            with torch.cuda.stream(st):
                plan = kernels.ForwardPlan(cfg, pk, 4, 1000, gpu_device)
                for _ in range(8):
                    plan.run(c, src, tgt)
                    rc = L_.pdsc_range_poll(kernels._p(plan.ws), 4, ctypes.c_void_p(st.cuda_stream))
                    if rc != want:
                        errors.append((want, rc))
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    torch.cuda.synchronize()
    ts = [threading.Thread(target=worker, args=(corr, kernels.PDSC_ERR_RANGE)),
          threading.Thread(target=worker, args=(corr0, 0))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts)
    assert errors == []


def test_module_reruns_marked_pairs_in_f32(gpu_device):
    m, m32 = _model(gpu_device, "h3"), _model(gpu_device, "f32")
    corr, src, tgt = _batch(gpu_device)
    with pytest.warns(RuntimeWarning, match="fp16"):
        T, L = m.forward_batched(corr, src, tgt)
    assert torch.isfinite(T).all()
    # the scaled pair: the exact-fp32 model's result on it alone; the rest: the h3 batch's
    T32, L32 = m32.forward_batched(corr[2:3], src[2:3], tgt[2:3])
    assert torch.equal(T[2], T32[0]) and torch.equal(L[2], L32[0])
    corr0, _, _ = _batch(gpu_device, bad=())
    T0, L0 = m.forward_batched(corr0, src, tgt)
    for b in (0, 1, 3):
        assert torch.equal(T[b], T0[b]) and torch.equal(L[b], L0[b])
    # bs = 1 forward and the ragged list take the same route
    with pytest.warns(RuntimeWarning):
        r = m({"corr_pos": corr[2:3], "src_keypts": src[2:3], "tgt_keypts": tgt[2:3], "testing": True})
    assert torch.equal(r["final_trans"], T32) and torch.equal(r["final_labels"], L32)
    ds = [{"corr_pos": corr[b:b + 1, :n], "src_keypts": src[b:b + 1, :n], "tgt_keypts": tgt[b:b + 1, :n]}
          for b, n in zip(range(4), (1000, 900, 950, 1000))]
    with pytest.warns(RuntimeWarning):
        res = m.forward_list(ds)
    assert all(torch.isfinite(x["final_trans"]).all() for x in res)


def test_f32_mode_takes_the_scaled_pair(gpu_device):
    from pointdsc_amd import kernels
    m32 = _model(gpu_device, "f32")
    corr, src, tgt = _batch(gpu_device)
    T, L = kernels.forward_testing(m32.pdsc_config(), m32.packed_weights(), corr, src, tgt)  # no RangeError
    assert torch.isfinite(T).all()


def test_training_forward_range_guard(gpu_device):
    from pointdsc_amd import kernels
    m = _model(gpu_device, "h3")
    corr, src, tgt = _batch(gpu_device)
    with pytest.raises(kernels.RangeError) as ei:
        kernels.forward_training(m.pdsc_config(), m.packed_weights(), corr, src, tgt, want_M=False)
    assert ei.value.pairs == [2]
    assert torch.isnan(ei.value.outputs[0][2]).all()
    with pytest.warns(RuntimeWarning):
        r = m({"corr_pos": corr, "src_keypts": src, "tgt_keypts": tgt})
    assert torch.isfinite(r["final_trans"]).all()


def _plan2_child(path, sk):  # child process entry: the split-grid (PDSC_W64_SK=0) arm
    import os
    os.environ["PDSC_W64_SK"] = sk
    from pointdsc_amd import kernels
    dev = torch.device("cuda:0")
    m = _model(dev, "h3")
    corr, src, tgt = _batch(dev, B=8, N=5000)
    try:
        kernels.forward_testing(m.pdsc_config(), m.packed_weights(), corr, src, tgt)
        pairs, T, L = [], None, None
    except kernels.RangeError as e:
        pairs, (T, L) = e.pairs, e.outputs
    np.savez(path, pairs=np.array(pairs), T=T.cpu().numpy(), L=L.cpu().numpy())


def test_range_guard_on_the_split_plan(gpu_device, tmp_path):
    """The key-split plan (pdsc_encoder_plan 2: attention_w64 on the packed
    M, stream-K by default and the split grid with PDSC_W64_SK=0), whose combine
    skips a split whose running max stayed -inf (fmaxf ignores NaN): a scaled
    pair among 8 x 5000 is still marked, its pose NaN and labels 0, every other
    pair bitwise as without it, and the module splices the exact-fp32 rerun."""
    import os
    import subprocess
    import sys
    from pointdsc_amd import _lib, kernels
    plan = ctypes.c_int32()
    _lib.check(_lib.load().pdsc_encoder_plan(8, 5000, 0, ctypes.byref(plan)), "encoder_plan")
    assert plan.value == 2
    m = _model(gpu_device, "h3")
    corr, src, tgt = _batch(gpu_device, B=8, N=5000)
    corr0, _, _ = _batch(gpu_device, B=8, N=5000, bad=())
    T0, L0 = kernels.forward_testing(m.pdsc_config(), m.packed_weights(), corr0, src, tgt)
    here = os.path.dirname(os.path.abspath(__file__))
    arms = {}
    for sk in ("1", "0"):
        out = tmp_path / f"plan2_sk{sk}.npz"
        code = f"import sys; sys.path[:0] = [{here!r}, {os.path.dirname(here)!r}]; " \
               f"import test_gpu_range as t; t._plan2_child({str(out)!r}, {sk!r})"
        subprocess.run([sys.executable, "-c", code], check=True, timeout=240)
        arms[sk] = np.load(out)
    for sk, r in arms.items():
        assert list(r["pairs"]) == [2], sk
        assert np.isnan(r["T"][2]).all() and float(np.abs(r["L"][2]).sum()) == 0.0, sk
    with pytest.raises(kernels.RangeError) as ei:
        kernels.forward_testing(m.pdsc_config(), m.packed_weights(), corr, src, tgt)
    T, L = ei.value.outputs
    for b in (0, 1, 3, 4, 5, 6, 7):
        assert torch.equal(T[b], T0[b]) and torch.equal(L[b], L0[b]), b
    with pytest.warns(RuntimeWarning, match="fp16"):
        Tm, Lm = m.forward_batched(corr, src, tgt)
    assert torch.isfinite(Tm).all()
    m32 = _model(gpu_device, "f32")
    T32, L32 = m32.forward_batched(corr[2:3], src[2:3], tgt[2:3])
    assert torch.equal(Tm[2], T32[0]) and torch.equal(Lm[2], L32[0])


def test_nonfinite_input_keeps_other_pairs(gpu_device):
    """A pair with a NaN coordinate is marked in both precisions: the module
    returns every other pair's result (bitwise the clean batch's) and that
    pair's NaN pose / zero labels with a warning, instead of raising."""
    m = _model(gpu_device, "h3")
    corr, src, tgt = _batch(gpu_device, bad=())
    T0, L0 = m.forward_batched(corr, src, tgt)
    corr[1, 5, 0] = float("nan")
    with pytest.warns(RuntimeWarning, match="non-finite"):
        T, L = m.forward_batched(corr, src, tgt)
    assert torch.isnan(T[1]).all() and float(L[1].abs().sum()) == 0.0
    for b in (0, 2, 3):
        assert torch.equal(T[b], T0[b]) and torch.equal(L[b], L0[b]), b
