"""int8 mode (WK_PREC_INT8): the device's esp-dl int8
network on the GPU, bit-exact against oracle.kws_forward_int8, and the
reference's int8 known-answer test (xiaoa.info: -40 at exp -3)."""
import os

import numpy as np
import pytest

from oracle import wk_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def m8(gpu, golden_dir):
    import wakeword
    return wakeword.load_onnx(os.path.join(golden_dir, "xiaoa.onnx"), precision="int8")


def test_int8_kat_exact(m8, golden_dir):
    k = np.load(os.path.join(golden_dir, "kat.npz"))
    feats = (k["kat_in_int8"][0].T[None].astype(np.float32) / 16.0)     # exp -4 -> exactly representable
    out = m8(feats).reshape(-1).cpu().numpy()
    assert out[0] == -40 * 0.125


def test_int8_bit_exact_vs_oracle(m8, xiaoa_sd):
    import wakeword
    x = O.synth_clips(99, 0, 300, 16000)
    feats = wakeword.mfcc(x).cpu().numpy()                          # identical inputs for both sides
    got = m8(feats).reshape(-1).cpu().numpy()
    want = O.kws_forward_int8(O.quantize_input(feats), O.quantize_int8(xiaoa_sd)) * 0.125
    np.testing.assert_array_equal(got, want.astype(np.float32))
    det = m8.detect(x).reshape(-1).cpu().numpy()                    # audio -> fp32 front-end -> int8 CNN
    np.testing.assert_array_equal(det, got)


def test_int8_mfma_bit_exact_at_scale(m8, xiaoa_sd):
    """The int8 matrix-core kernel (one wave per clip, grid-stride) over 4,100
    clips of wide-range features (input saturation, every requantisation
    clamp): bit for bit the oracle's integer network."""
    feats = (4.0 * np.random.default_rng(5).standard_normal((4100, 13, 63))).astype(np.float32)
    got = m8(feats).reshape(-1).cpu().numpy()
    want = O.kws_forward_int8(O.quantize_input(feats), O.quantize_int8(xiaoa_sd)) * 0.125
    np.testing.assert_array_equal(got, want.astype(np.float32))


def test_int8_mfma_repeatable_at_scale(m8, xiaoa_sd):
    """65,536 clips of wide-range features through the int8 matrix-core kernel,
    three launches, bit for bit; and a strided sample of 512 clips equal to
    the oracle's integer network.  v_mfma_i32_16x16x64_i8 is one of the forms
    that change co-resident packed-fp32 VALU results (DESIGN 5.1, K = 32):
    this kernel's own VALU work is integer requantisation, and this test is
    the at-scale check that it stays exact."""
    import torch
    g = torch.Generator().manual_seed(11)
    feats = (4.0 * torch.randn((65536, 13, 63), generator=g)).cuda()
    ref = m8(feats).reshape(-1).clone()
    for _ in range(2):
        assert torch.equal(m8(feats).reshape(-1), ref)
    idx = np.arange(0, 65536, 128)
    f_s = feats[torch.from_numpy(idx).cuda()].cpu().numpy()
    want = O.kws_forward_int8(O.quantize_input(f_s), O.quantize_int8(xiaoa_sd)) * 0.125
    np.testing.assert_array_equal(ref.cpu().numpy()[idx], want.astype(np.float32))
