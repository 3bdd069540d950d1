"""WAV ingest and augmentation: the native host loader
against Python's wave module, torch's F.interpolate, and the reference's own
WAV files (tests/golden/wav).  CPU only."""
import os
import struct
import wave

import numpy as np
import pytest

WAV_DIR = os.path.join(os.path.dirname(__file__), "golden", "wav")


def _files():
    return sorted(os.path.join(WAV_DIR, f) for f in os.listdir(WAV_DIR) if f.endswith(".wav"))


def _py_read(path):
    with wave.open(path) as w:
        raw = np.frombuffer(w.readframes(w.getnframes()), "<i2")
        return raw.reshape(-1, w.getnchannels())[:, 0], w.getframerate()


def _write(path, samples, chunks_before_data=(), bits=16, fmt_extra=b""):
    data = np.asarray(samples, "<i2").tobytes() if bits == 16 else np.asarray(samples, "u1").tobytes()
    fmt = struct.pack("<HHIIHH", 1, 1, 16000, 16000 * bits // 8, bits // 8, bits) + fmt_extra
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt
    for tag, payload in chunks_before_data:
        body += tag + struct.pack("<I", len(payload)) + payload + (b"\0" if len(payload) & 1 else b"")
    body += b"data" + struct.pack("<I", len(data)) + data
    with open(path, "wb") as fh:
        fh.write(b"RIFF" + struct.pack("<I", len(body)) + body)


def test_reads_reference_wavs_like_wave_module():
    from wakeword import wav
    files = _files()
    assert len(files) >= 4
    for f in files:
        ref, sr = _py_read(f)
        got, info = wav.read_wav(f, max_samples=1 << 20)
        assert info["sample_rate"] == sr and info["bits_per_sample"] == 16
        np.testing.assert_array_equal(got, ref)
        t, _ = wav.read_wav(f)                        # the reference's 16000-sample truncation
        np.testing.assert_array_equal(t, ref[:16000])


def test_skips_unknown_chunks_and_odd_padding(tmp_path):
    from wakeword import wav
    x = (np.arange(3000) % 200 - 100).astype(np.int16)
    p = str(tmp_path / "list.wav")
    _write(p, x, chunks_before_data=[(b"LIST", b"INFOISFT" + b"abc"), (b"junk", b"\1" * 7)], fmt_extra=b"\0\0")
    got, info = wav.read_wav(p)
    np.testing.assert_array_equal(got, x)
    assert info["data_samples"] == 3000


def test_rejects_bad_files(tmp_path):
    from wakeword import wav, WakewordError
    p8 = str(tmp_path / "u8.wav")
    _write(p8, np.zeros(100, np.uint8), bits=8)
    with pytest.raises(WakewordError, match="UNSUPPORTED"):
        wav.read_wav(p8)
    bad = tmp_path / "bad.wav"
    bad.write_bytes(b"RIFX" + b"\0" * 40)
    with pytest.raises(WakewordError, match="INVALID_ARG"):
        wav.read_wav(str(bad))
    with pytest.raises(WakewordError):
        wav.read_wav(str(tmp_path / "missing.wav"))


def test_load_batch_scaling_and_padding():
    from wakeword import wav
    files = _files()[:4]
    z, n_read = wav.load_batch(files, pad_to=16000, noise_level=0.0)
    for i, f in enumerate(files):
        ref, _ = _py_read(f)
        k = min(ref.size, 16000)
        assert n_read[i] == k
        np.testing.assert_array_equal(z[i, :k], ref[:k].astype(np.float32) / 32768.0)   # torchaudio.load
        assert not z[i, k:].any()
    a, _ = wav.load_batch(files, noise_level=0.005, seed=3)
    b, _ = wav.load_batch(files, noise_level=0.005, seed=3)
    np.testing.assert_array_equal(a, b)                                                 # seeded, thread-count independent
    pad = np.concatenate([a[i, n_read[i]:] for i in range(len(files)) if n_read[i] < 16000])
    if pad.size > 2000:
        assert abs(pad.std() - 0.005) < 0.0005 and abs(pad.mean()) < 0.0005            # N(0, 0.005^2)


def test_augment_matches_torch_interpolate():
    import torch
    from wakeword import wav
    x = (np.random.RandomState(0).randn(11200) * 0.2).astype(np.float32)
    for speed in (0.8, 1.2):
        m = int(x.size * speed)
        ref = torch.nn.functional.interpolate(torch.from_numpy(x)[None, None], size=m, mode="linear",
                                              align_corners=False)[0, 0].numpy()
        got = wav.augment(x, speed=speed, out_len=16000)
        k = min(m, 16000)
        np.testing.assert_allclose(got[:k], ref[:k], rtol=0, atol=1e-7)
        assert not got[k:].any()
    v = wav.augment(x * 4, volume=1.3, out_len=x.size)
    np.testing.assert_array_equal(v, np.clip(x * 4 * np.float32(1.3), -1, 1))
    assert len(wav.augment_variants(x)) == 5


def test_cli_prepare_zero_pad_matches_wave_module(golden_dir):
    """The config-1 CLI's host side: native WAV read + zero pad (no GPU)."""
    import wave as _wave
    from wakeword import test as cli
    p = os.path.join(golden_dir, "wav", "xiaoa_095.wav")
    x = cli.prepare([p], "zero")
    with _wave.open(p) as w:
        raw = np.frombuffer(w.readframes(w.getnframes()), "<i2")[:16000].astype(np.float32) / 32768.0
    assert x.shape == (1, 16000) and x.dtype == np.float32
    np.testing.assert_array_equal(x[0, :raw.size], raw)
    assert not x[0, raw.size:].any()
    xn = cli.prepare([p], "noise", seed=3)
    np.testing.assert_array_equal(xn[0, :raw.size], raw)
    assert 0.002 < xn[0, raw.size:].std() < 0.008
    assert cli.prepare([], "zero").shape == (0, 16000)
