"""Cross-check of the mode-B oracle against an independent restatement of the
torchaudio front-end (CPU).

torchaudio itself is absent from the image, so the mode-B oracle
(oracle/wk_oracle.py, B1-B6) is our own restatement of the call site
ml_models/src/extract_mfcc.py:137-175 (T.MFCC with n_fft 512, win 320, hop 256,
40 HTK mels, 13 coefficients, log-mels, then CMVN).  This test pins that
restatement against a second one written by other people:
transformers.audio_utils (installed wheel), whose `spectrogram`,
`window_function` and `mel_filter_bank` are documented as adapted from
torchaudio (mel_filter_bank docstring: "adapted from *torchaudio* and
*librosa* ... torchaudio's `melscale_fbanks` implement the "htk" filters").
The DCT comes from scipy.fft.dct(type=2, norm="ortho"), which is torchaudio's
create_dct(norm="ortho"); pre-emphasis (torchaudio.functional.preemphasis,
extract_mfcc.py:171) and CMVN (normalize_mfcc, extract_mfcc.py:73-80) are
restated inline.  Agreement is checked on the committed golden fixtures, so
the GPU parity tests that compare against those fixtures inherit the pin.
"""
import os

import numpy as np
import pytest

from oracle import wk_oracle as O

audio_utils = pytest.importorskip("transformers.audio_utils")
sfft = pytest.importorskip("scipy.fft")

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _features_third_party(x: np.ndarray) -> np.ndarray:
    """(16000,) waveform -> CMVN'd (13, 63) through transformers + scipy."""
    x = np.asarray(x, np.float64)
    y = x.copy()
    y[1:] -= 0.97 * x[:-1]                                       # preemphasis(coeff=0.97)
    win = audio_utils.window_function(320, "hamming", periodic=True, frame_length=512, center=True)
    fb = audio_utils.mel_filter_bank(257, 40, 0.0, 8000.0, 16000, norm=None, mel_scale="htk")
    mel = audio_utils.spectrogram(y, win, frame_length=512, hop_length=256, fft_length=512, power=2.0,
                                  center=True, pad_mode="reflect", mel_filters=fb, mel_floor=0.0,
                                  dtype=np.float64)              # (40, 63)
    mf = sfft.dct(np.log(mel + 1e-6), type=2, norm="ortho", axis=0)[:13]   # (13, 63)
    mean = mf.mean(axis=1, keepdims=True)
    std = mf.std(axis=1, ddof=1, keepdims=True)
    std = np.where(std == 0, 1.0, std)
    return (mf - mean) / (std + 1e-8)


def test_fbank_matches_third_party():
    fb = audio_utils.mel_filter_bank(257, 40, 0.0, 8000.0, 16000, norm=None, mel_scale="htk")
    ours = O.melscale_fbanks()
    assert fb.shape == ours.shape == (257, 40)
    assert int((fb != 0).sum()) == int((ours != 0).sum())
    np.testing.assert_allclose(ours, fb, rtol=0, atol=1e-12)


def test_window_matches_third_party():
    win = audio_utils.window_function(320, "hamming", periodic=True, frame_length=512, center=True)
    ours = np.zeros(512)
    ours[96:416] = O.hamming_periodic(320)
    np.testing.assert_allclose(ours, win, rtol=0, atol=1e-15)


def test_dct_matches_scipy():
    eye = np.eye(40)
    np.testing.assert_allclose(O.create_dct(), sfft.dct(eye, type=2, norm="ortho", axis=0)[:13].T, atol=1e-14)


@pytest.mark.parametrize("which", ["synth", "wavs"])
def test_golden_features_match_third_party(which):
    d = np.load(os.path.join(GOLDEN, f"{which}.npz"))
    if which == "synth":
        x = O.synth_clips(int(d["seed"]), int(d["first"]), int(d["count"]))
        golden = d["feats"]
    else:
        x, golden = d["x_noise"], d["feat_noise"]
    tp = np.stack([_features_third_party(c) for c in x])
    assert tp.shape == golden.shape
    # transformers stores the STFT in complex64 (float32 rounding, ~1e-7 in the
    # features); everything else is float64.  Far below the 5e-4 feature
    # tolerance of the GPU tests.
    np.testing.assert_allclose(golden, tp, rtol=0, atol=1e-6)
    np.testing.assert_allclose(O.features_mode_b(x), tp, rtol=0, atol=1e-6)


def test_ctc_logmel_matches_third_party():
    """The CTC head's front-end (X1, ctc.py:82-107: torchaudio MelSpectrogram
    n_fft 400, hop 160, 80 HTK mels, periodic Hann, centre/reflect, power 2;
    ln(mel + 1e-8); one global z-score) against the same third-party restatement."""
    torch = pytest.importorskip("torch")
    from oracle import wk_ctc_oracle as CO
    fb = audio_utils.mel_filter_bank(201, 80, 0.0, 8000.0, 16000, norm=None, mel_scale="htk")
    # (torchaudio, like the oracle, builds the filterbank in float32)
    np.testing.assert_allclose(CO.mel_fbanks().double().numpy(), fb, rtol=0, atol=1e-5)
    win = audio_utils.window_function(400, "hann", periodic=True)
    x = O.synth_clips(77, 0, 3, 48000)
    ours = CO.features(torch.from_numpy(x).float()).double().numpy()   # (3, T, 80)
    for u in range(x.shape[0]):
        mel = audio_utils.spectrogram(x[u].astype(np.float64), win, frame_length=400, hop_length=160,
                                      fft_length=400, power=2.0, center=True, pad_mode="reflect",
                                      mel_filters=fb, mel_floor=0.0, dtype=np.float64)   # (80, T)
        lm = np.log(mel + 1e-8).T
        lm = (lm - lm.mean()) / lm.std(ddof=1)
        assert lm.shape == ours[u].shape == (301, 80)
        # the oracle runs torch.stft in fp32: ~1e-6 typical on unit-scale
        # z-scores, up to ~3e-4 where a mel band is near the 1e-8 floor
        err = np.abs(ours[u] - lm)
        assert np.median(err) < 1e-5 and err.max() < 1e-3, (np.median(err), err.max())
