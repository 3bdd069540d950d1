"""bf16 mode (WK_PREC_BF16): bf16 convolutions
(bf16 MFMA, K = 32 per step, fp32 accumulation) inside the fused kernel, fp32
front-end and classifier.  Tolerance vs the fp32 reference path: 0.05 in logit
(bf16 keeps 8 mantissa bits; observed ~1e-2), identical decisions on the
reference WAVs."""
import os

import numpy as np
import pytest

from oracle import wk_oracle as O

pytestmark = pytest.mark.gpu
BF16_LOGIT_ATOL = 0.05


@pytest.fixture(scope="module")
def m16(gpu, golden_dir):
    import wakeword
    return wakeword.load_onnx(os.path.join(golden_dir, "xiaoa.onnx"), precision="bf16")


def test_bf16_golden_wavs(m16, golden_dir):
    w = np.load(os.path.join(golden_dir, "wavs.npz"))
    got = m16.detect(w["x_noise"]).reshape(-1).cpu().numpy()
    ref = w["logit_noise"].reshape(-1)
    assert np.abs(got - ref).max() <= BF16_LOGIT_ATOL
    assert ((got > 0) == (ref > 0)).all()


@pytest.mark.parametrize("n", [1, 5, 300])
def test_bf16_synth_vs_oracle_and_batch_invariance(m16, xiaoa_sd, n):
    x = O.synth_clips(31, 0, n, 16000)
    got = m16.detect(x).reshape(-1).cpu().numpy()
    ref = O.detect_mode_b(x[: min(n, 32)].astype(np.float64), xiaoa_sd)
    assert np.abs(got[: ref.size] - ref).max() <= BF16_LOGIT_ATOL
    one = m16.detect(x[:1]).reshape(-1).cpu().numpy()
    np.testing.assert_array_equal(one, got[:1])      # per-clip results do not depend on the batch


@pytest.mark.parametrize("prec,atol", [("bf16", BF16_LOGIT_ATOL), ("bf16x3", 1e-3)])
def test_cnn_only_entry_all_precisions(gpu, golden_dir, xiaoa_sd, prec, atol):
    """wk_cnn (LightweightKWS.forward on given features) runs the fused
    kernel's CNN role fed from HBM in every precision: the reference module's
    golden logits on the golden features, and the fused path's logits for the
    same clips (ragged batch: 37 clips, two CNN roles per workgroup)."""
    import wakeword
    m = wakeword.load_onnx(os.path.join(golden_dir, "xiaoa.onnx"), precision=prec)
    g = np.load(os.path.join(golden_dir, "synth.npz"))
    got = m(g["feats"]).reshape(-1).cpu().numpy()
    assert np.abs(got - g["logits"].reshape(-1)).max() <= atol
    x = O.synth_clips(51, 0, 37, 16000)
    logit_fused, feats = m.detect(x, return_features=True)
    np.testing.assert_allclose(m(feats).reshape(-1).cpu().numpy(), logit_fused.cpu().numpy(), atol=1e-5)


# ---- WK_PREC_BF16X3: split-bf16 convolutions held to the fp32 logit tolerance.
X3_LOGIT_ATOL = 1e-3   # the same bound as the fp32 path (tests/test_gpu_parity.py)


@pytest.fixture(scope="module")
def m3(gpu, golden_dir):
    import wakeword
    return wakeword.load_onnx(os.path.join(golden_dir, "xiaoa.onnx"), precision="bf16x3")


def test_bf16x3_golden_wavs(m3, golden_dir):
    w = np.load(os.path.join(golden_dir, "wavs.npz"))
    got = m3.detect(w["x_noise"]).reshape(-1).cpu().numpy()
    ref = w["logit_noise"].reshape(-1)
    assert np.abs(got - ref).max() <= X3_LOGIT_ATOL


@pytest.mark.parametrize("n", [1, 5, 300])
def test_bf16x3_synth_vs_oracle(m3, xiaoa_sd, n):
    x = O.synth_clips(41, 0, n, 16000)
    got = m3.detect(x).reshape(-1).cpu().numpy()
    ref = O.detect_mode_b(x[: min(n, 32)].astype(np.float64), xiaoa_sd)
    assert np.abs(got[: ref.size] - ref).max() <= X3_LOGIT_ATOL
    one = m3.detect(x[:1]).reshape(-1).cpu().numpy()
    np.testing.assert_array_equal(one, got[:1])


def test_bf16x3_tracks_fp32_at_scale(m3, golden_dir):
    """65,536 device-generated clips: split-bf16 against the fp32-MFMA path, clip for clip."""
    import torch
    import wakeword
    m32 = wakeword.load_onnx(os.path.join(golden_dir, "xiaoa.onnx"))
    x = wakeword.synth_clips(1234, 0, 65536, device=0)
    a = m3.detect(x).reshape(-1)
    b = m32.detect(x).reshape(-1)
    d = (a - b).abs().max().item()
    assert d <= X3_LOGIT_ATOL, d
    assert bool(torch.isfinite(a).all())


def test_bf16x3_int16_matches_float(m3):
    x = O.synth_clips(43, 0, 7, 16000)
    q = np.round(x * 32767).astype(np.int16)
    a = m3.detect(q).reshape(-1).cpu().numpy()
    b = m3.detect(q.astype(np.float32) / 32768.0).reshape(-1).cpu().numpy()
    np.testing.assert_allclose(a, b, atol=1e-5)


@pytest.mark.parametrize("precision", ["fp32", "bf16", "bf16x3"])
def test_fused_repeatable_at_scale(gpu, golden_dir, precision):
    """Four full-size launches (65,536 clips) give bit-identical logits: the
    fused kernel's role hand-offs and MFMA chains have no timing dependence."""
    import wakeword
    m = wakeword.load_onnx(os.path.join(golden_dir, "xiaoa.onnx"), precision=precision)
    x = wakeword.synth_clips(777, 0, 65536, device=0)
    ref = m.detect(x).reshape(-1)
    for _ in range(4):
        got = m.detect(x).reshape(-1)
        assert int((got != ref).sum()) == 0
    m.check_device_errors()


@pytest.mark.parametrize("prec,atol,rtol", [("bf16", BF16_LOGIT_ATOL, 0.02), ("bf16x3", 1e-3, 1e-5)])
def test_cnn_only_bf16_family_full_size_repeatable(gpu, golden_dir, prec, atol, rtol):
    """wk_cnn_fused_kernel in the bf16 family at 65,536 clips (config 2's
    size; four K = 32 waves per SIMD, two CNN roles per workgroup): two
    launches are bit-identical and every logit is within the precision's
    tolerance of the fp32 CNN on the same features (the K = 32 rule,
    DESIGN 5.1 / tests/test_isa_rules.py, checked at run time).  The
    features are N(0, 1) draws (CMVN'd features are unit-variance per
    coefficient), so logits run larger than on speech: the bound is
    atol + rtol |fp32 logit|."""
    import wakeword
    torch = gpu
    g = torch.Generator(device="cuda:0").manual_seed(6)
    x = torch.randn((65536, 13, 63), generator=g, device="cuda:0", dtype=torch.float32)
    m = wakeword.load_onnx(os.path.join(golden_dir, "xiaoa.onnx"), precision=prec)
    m32 = wakeword.load_onnx(os.path.join(golden_dir, "xiaoa.onnx"), precision="fp32")
    a = m(x).reshape(-1)
    b = m(x).reshape(-1)
    ref = m32(x).reshape(-1)
    torch.cuda.synchronize()
    assert torch.isfinite(a).all()
    assert torch.equal(a, b), int((a != b).sum())
    excess = (a - ref).abs() - (atol + rtol * ref.abs())
    assert float(excess.max()) <= 0.0, float((a - ref).abs().max())
