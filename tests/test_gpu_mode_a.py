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


# (sampling_rate, frame, hop, n_fft, n_filters, n_mfcc): mfcc.c's general
# parameter set -- an 8 kHz narrow band, the CTC head's 25 ms / 10 ms framing,
# a 22.05 kHz 1024-point FFT, a frame longer than n_fft (mfcc.c:252 keeps its
# first n_fft samples), more coefficients than filters (the extras stay 0),
# the 4096-point maximum, and a bank crowded past its bins (degenerate
# triangles: 0/0 weights, mfcc.c:224, whose NaN energies fmaxf turns into 1e-12).
GENERAL = [(8000, 200, 80, 256, 26, 12), (16000, 400, 160, 512, 40, 13), (22050, 1024, 512, 1024, 64, 20),
           (16000, 512, 128, 256, 30, 13), (16000, 320, 256, 512, 40, 45), (44100, 2048, 441, 4096, 128, 40),
           (4000, 100, 50, 128, 64, 13)]


@pytest.mark.parametrize("cfg", GENERAL)
def test_extract_mfcc_general_parameters(gpu, cfg):
    """extract_mfcc at parameter sets other than the reference's (wk_esp_mfcc
    behind the shim) against the C restatement run at the same parameters."""
    import wakeword
    sr, frame, hop, n_fft, nfil, nmfcc = cfg
    L = sr + 777
    x = O.synth_clips(13, 0, 1, L)[0]
    got = wakeword.extract_mfcc(x, L, sr, frame, hop, n_fft, nfil, nmfcc)
    ref = B.esp_mfcc(x, True, sr, frame, hop, n_fft, nfil, nmfcc)
    assert got is not None and got.shape == ref.shape == ((L - frame) // hop + 1, nmfcc)
    assert np.isfinite(got).all()
    assert np.abs(got - ref).max() <= _tol(ref), np.abs(got - ref).max()
    if nmfcc > nfil:
        assert not got[:, nfil:].any()


def test_extract_mfcc_general_refusals(gpu):
    """NULL outside mfcc.c's domain: a non-power-of-2 n_fft (esp-dsp's FFT
    refuses it), n_fft past 4096, hop 0 (mfcc.c:447 divides by it), no
    filters or coefficients, and the reference's own signal checks."""
    import wakeword
    x = O.synth_clips(14, 0, 1, 16000)[0]
    assert wakeword.extract_mfcc(x, 16000, 16000, 400, 160, 500, 40, 13) is None
    assert wakeword.extract_mfcc(x, 16000, 16000, 400, 160, 8192, 40, 13) is None
    assert wakeword.extract_mfcc(x, 16000, 16000, 400, 0, 512, 40, 13) is None
    assert wakeword.extract_mfcc(x, 16000, 16000, 400, 160, 512, 0, 13) is None
    assert wakeword.extract_mfcc(x, 16000, 16000, 400, 160, 512, 40, 0) is None
    assert wakeword.extract_mfcc(x[:300], 300, 16000, 400, 160, 512, 40, 13) is None
    assert wakeword.extract_mfcc(x, 16000, 16000, 0, 160, 512, 40, 13) is None


@pytest.mark.parametrize("cfg", [(8000, 200, 256, 26, 12), (16000, 400, 512, 40, 20), (16000, 512, 512, 64, 13)])
def test_single_frame_general_parameters(gpu, cfg):
    import ctypes as C
    from wakeword import _lib
    L = _lib.lib()
    fp = C.POINTER(C.c_float)
    sr, frame_size, n_fft, nfil, nmfcc = cfg
    frame = O.synth_clips(15, 0, 1, frame_size)[0]
    p = L.flow_extract_mfcc_single_frame(frame.ctypes.data_as(fp), frame_size, sr, n_fft, nfil, nmfcc)
    assert p
    got = np.ctypeslib.as_array(p, shape=(nmfcc,)).copy()
    L.free_mfcc(p)
    ref = B.esp_mfcc(frame, True, sr, frame_size, frame_size, n_fft, nfil, nmfcc, pre=0.0)[0]
    assert np.abs(got - ref).max() <= _tol(ref)


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


def test_esp_mfcc_object_batched(gpu):
    """wakeword.EspMfcc (wk_esp_mfcc_create / run): a batch of 5 signals at a
    general parameter set, each against the C restatement."""
    import wakeword
    sr, frame, hop, n_fft, nfil, nmfcc = 8000, 200, 80, 256, 26, 12
    x = O.synth_clips(16, 0, 5, 4000)
    m = wakeword.EspMfcc(sr, frame, n_fft, nfil, nmfcc)
    got = m(x, hop).cpu().numpy()
    assert got.shape == (5, (4000 - frame) // hop + 1, nmfcc)
    for i in range(5):
        ref = B.esp_mfcc(x[i], True, sr, frame, hop, n_fft, nfil, nmfcc)
        assert np.abs(got[i] - ref).max() <= _tol(ref)
    with pytest.raises(wakeword.WakewordError):
        wakeword.EspMfcc(sr, frame, 500, nfil, nmfcc)
