"""The timed mode-A CPU baseline (oracle/esp_mfcc_oracle.c, FFT batch path on
host threads) computes what the exact-DFT restatement computes, to float
rounding: the two C paths against each other, packing on and off (host only)."""
import numpy as np
import pytest

from oracle import build_oracle as EO


@pytest.mark.parametrize("esp_pack", [True, False])
def test_fft_batch_path_matches_dft_path(esp_pack):
    rng = np.random.default_rng(3)
    x = (0.1 * rng.standard_normal((5, 16000))).astype(np.float32)
    x[2] += (0.2 * np.sin(2 * np.pi * 440 * np.arange(16000) / 16000)).astype(np.float32)
    x[4] = 0.0
    ref = np.stack([EO.esp_mfcc(c, esp_pack=esp_pack) for c in x])
    got = EO.esp_mfcc_batch(x, esp_pack=esp_pack, n_threads=3)
    assert got.shape == ref.shape == (5, 62, 13)
    assert np.abs(got - ref).max() <= 1e-4 * max(1.0, float(np.abs(ref).max()))


def test_fft_batch_path_thread_count_invariant():
    x = (0.1 * np.random.default_rng(4).standard_normal((7, 4000))).astype(np.float32)
    a = EO.esp_mfcc_batch(x, n_threads=1)
    b = EO.esp_mfcc_batch(x, n_threads=4)
    assert np.array_equal(a, b)
