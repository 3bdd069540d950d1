"""GPU tests of front-end mode A (main/esp_mfcc/mfcc.c:431-527) through the C
ABI: wk_mfcc(mode=ESP_MFCC) and the mfcc.h compatibility shims, against the C
restatement oracle/esp_mfcc_oracle.c.  PARITY STATUS: mode A is "parity
unpinned" (mfcc.c needs ESP-IDF + esp-dsp and cannot be built here; no
reference fixture holds its values) -- these tests pin the HIP kernel to the
restatement, which tests/test_oracle.py cross-checks against a second,
independent numpy restatement."""
import numpy as np
import pytest

from oracle import build_oracle as B
from oracle import wk_oracle as O

pytestmark = pytest.mark.gpu


def _tol(ref):
    # Raw (un-normalised) MFCCs reach |40|; the HIP path runs a float32 FFT
    # where the oracle takes an exact DFT: 2e-5 of the row scale + 2e-4.
    return 2e-5 * np.abs(ref).max() + 2e-4


@pytest.mark.parametrize("pack", [True, False])
def test_mode_a_matches_c_oracle(gpu, pack):
    import wakeword
    x = O.synth_clips(77, 0, 12, 16000)
    got = wakeword.mfcc(x, mode="esp", esp_dsp_packing=pack).cpu().numpy()
    assert got.shape == (12, 62, 13)
    for i in range(12):
        ref = B.esp_mfcc(x[i], pack)
        assert np.abs(got[i] - ref).max() <= _tol(ref), i


@pytest.mark.parametrize("L", [320, 575, 16192, 32000, 48123])
def test_mode_a_lengths(gpu, L):
    """1 frame, a ragged tail, the firmware's 63-frame length, and multi-chunk signals."""
    import wakeword
    x = O.synth_clips(5, 0, 3, L)
    got = wakeword.mfcc(x, mode="esp").cpu().numpy()
    nf = (L - 320) // 256 + 1
    assert got.shape == (3, nf, 13)
    for i in range(3):
        ref = B.esp_mfcc(x[i])
        assert np.abs(got[i] - ref).max() <= _tol(ref), (L, i)


def test_mode_a_int16_input(gpu):
    import wakeword
    x = (O.synth_clips(9, 0, 4, 16000) * 32767).astype(np.int16)
    got = wakeword.mfcc(x, mode="esp").cpu().numpy()
    for i in range(4):
        ref = B.esp_mfcc(x[i].astype(np.float32) / 32768.0)
        assert np.abs(got[i] - ref).max() <= _tol(ref)


def test_extract_mfcc_shim_matches_oracle(gpu):
    """mfcc.h:10-17 signature and ownership: host in, malloc'd host out, freed by free_mfcc."""
    import wakeword
    x = O.synth_clips(11, 0, 1, 16192)[0]
    got = wakeword.extract_mfcc(x, 16192, 16000, 320, 256, 512, 40, 13)
    ref = B.esp_mfcc(x)
    assert got.shape == (63, 13)
    assert np.abs(got - ref).max() <= _tol(ref)
    # Same NULL-on-bad-arguments behaviour as the reference (mfcc.c:434-437).
    assert wakeword.extract_mfcc(x[:100], 100) is None
    # Parameters outside the reference configuration are refused (NULL), not approximated.
    assert wakeword.extract_mfcc(x, 16192, 16000, 400, 160, 512, 40, 13) is None


def test_single_frame_shim_matches_oracle(gpu):
    """mfcc.c:297-427 flow_extract_mfcc_single_frame: no pre-emphasis, one frame."""
    import ctypes as C
    from wakeword import _lib
    L = _lib.lib()
    fp = C.POINTER(C.c_float)
    for seed in (1, 2, 3):
        frame = O.synth_clips(seed, 0, 1, 320)[0]
        p = L.flow_extract_mfcc_single_frame(frame.ctypes.data_as(fp), 320, 16000, 512, 40, 13)
        assert p
        got = np.ctypeslib.as_array(p, shape=(13,)).copy()
        L.free_mfcc(p)
        ref = B.esp_mfcc(frame, pre=0.0)[0]
        assert np.abs(got - ref).max() <= _tol(ref)
        p5 = L.flow_extract_mfcc_single_frame(frame.ctypes.data_as(fp), 320, 16000, 512, 40, 5)
        np.testing.assert_array_equal(np.ctypeslib.as_array(p5, shape=(5,)), got[:5])
        L.free_mfcc(p5)
    assert not L.flow_extract_mfcc_single_frame(None, 320, 16000, 512, 40, 13)            # mfcc.c:300-303
    assert not L.flow_extract_mfcc_single_frame(frame.ctypes.data_as(fp), 600, 16000, 512, 40, 13)
