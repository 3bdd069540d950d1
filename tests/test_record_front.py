"""The firmware record task's front (SURVEY 8(f) item 1,
esp_wake_word_detector.cpp:102-131): 4-channel TDM int16 mix, [1, 2, 1] >> 2
decimation 48 -> 16 kHz, and the lroundf / saturate int8 frame quantisation.
Integer work: the device results are compared bit for bit with the oracle's
transcription of the C loops (oracle/wk_oracle.py: record_front, pinned here to
a statement-by-statement loop version and to hand-computed values).  No
reference fixture holds these values (the firmware reads a live I2S TDM
stream), so the transcription is the pin.  The esp-dl MFCC between the two
stages is third-party and absent: callers supply the frames."""
import os

import numpy as np
import pytest

from oracle import wk_oracle as O


def _tdm(rng, n_frames):
    x = rng.integers(-32768, 32768, size=(n_frames, 960, 4), dtype=np.int32).astype(np.int16)
    x[0, :8] = 32767                 # the mix overflows int16: (int16_t) keeps the low 16 bits
    x[0, 8:16] = -32768
    x[0, 16:24, :3] = (-1, 0, 0)     # arithmetic >> of small negatives
    return x


def test_oracle_hand_values():
    f = np.zeros((3, 4), np.int16)
    f[:, :3] = 32767                 # weighted 5,242,720 >> 7 = 40,958 -> int16 -24,578
    assert O.record_front(f).tolist() == [-24578]
    f[:, :3] = -32768                # -5,242,880 >> 7 = -40,960 -> int16 24,576
    assert O.record_front(f).tolist() == [24576]
    f[:] = 0
    f[:, 0] = -1                     # -64 >> 7 = -1 each; (-1 - 2 - 1) >> 2 = -1
    assert O.record_front(f).tolist() == [-1]
    f[:] = 0
    f[1, 2] = 200                    # mono [0, 100, 0] -> 200 >> 2 = 50
    assert O.record_front(f).tolist() == [50]
    f[1, 3] = 12345                  # CH3 is not mixed
    assert O.record_front(f).tolist() == [50]


def test_oracle_vectorised_equals_loop_transcription():
    rng = np.random.default_rng(0)
    x = _tdm(rng, 2)
    for fr in x:
        np.testing.assert_array_equal(O.record_front(fr), O.record_front_loop(fr))


def test_quantize_oracle_half_away_from_zero():
    v = np.array([0.5, -0.5, 1.5, -1.5, 2.4999, 126.5, 127.5, -128.5, 1e9, -1e9, 0.0], np.float32)
    assert O.device_quantize_frames(v).tolist() == [1, -1, 2, -2, 2, 127, 127, -128, 127, -128, 0]


@pytest.mark.gpu
def test_record_front_bit_exact(gpu):
    import torch
    import wakeword
    rng = np.random.default_rng(1)
    x = _tdm(rng, 1500)                                   # 30 s of TDM audio, 480,000 output samples
    out, f = wakeword.record_front(x, float_out=True)
    ref = O.record_front(x)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    np.testing.assert_array_equal(f.cpu().numpy(), ref.astype(np.float32) / 32768.0)
    # odd sample counts (the kernel's single-sample tail) and tiny inputs
    for n_tdm in (3, 9, 15, 2883):
        xs = x.reshape(-1, 4)[:n_tdm]
        np.testing.assert_array_equal(wakeword.record_front(xs).cpu().numpy(), O.record_front(xs))
    assert wakeword.record_front(np.zeros((0, 4), np.int16)).numel() == 0
    with pytest.raises(ValueError):
        wakeword.record_front(np.zeros((4, 4), np.int16))      # not whole groups of 3
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_record_front_feeds_the_sliding_window_path(gpu, golden_dir, xiaoa_sd):
    """TDM -> record_front -> int16 16 kHz samples -> wk_forward (WK_DTYPE_I16,
    1 s windows at a 30 ms hop): equals the same windows of the oracle's samples
    as floats, and a sample of windows matches the oracle end to end."""
    import ctypes as C
    import torch
    import wakeword
    from wakeword import _lib
    rng = np.random.default_rng(2)
    x = (rng.standard_normal((150, 960, 4)) * 3000).astype(np.int16)   # 3 s of speech-level TDM audio
    pcm = wakeword.record_front(x)
    ref = O.record_front(x)
    model = wakeword.load_onnx(os.path.join(golden_dir, "xiaoa.onnx"))
    hop, W = 480, 16000
    n = (pcm.numel() - W) // hop + 1
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    a = torch.empty(n, device="cuda")
    _lib.check(_lib.lib().wk_forward(model._h.h, C.c_void_p(pcm.data_ptr()), _lib.WK_DTYPE_I16, n, W, hop,
                                     C.c_void_p(a.data_ptr()), None, st), "wk_forward")
    xf = torch.from_numpy(ref.astype(np.float32) / 32768.0).cuda()
    b = torch.empty(n, device="cuda")
    _lib.check(_lib.lib().wk_forward(model._h.h, C.c_void_p(xf.data_ptr()), _lib.WK_DTYPE_F32, n, W, hop,
                                     C.c_void_p(b.data_ptr()), None, st), "wk_forward")
    np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), atol=1e-5)
    idx = np.linspace(0, n - 1, 4).astype(int)
    clips = np.stack([ref[k * hop:k * hop + W] for k in idx]).astype(np.float64) / 32768.0
    assert np.abs(a.cpu().numpy()[idx] - O.detect_mode_b(clips, xiaoa_sd)).max() < 1e-3


@pytest.mark.gpu
def test_quantize_frames_and_cmvn_chain(gpu):
    """float MFCC frames -> wk_quantize_frames -> int8 -> wk_device_cmvn equals
    wk_device_cmvn on the float frames (which quantises them itself) and the
    oracle, bit for bit."""
    import wakeword
    rng = np.random.default_rng(3)
    mf = (rng.standard_normal((400, 13)) * 40).astype(np.float32)
    mf[0, :6] = [0.5, -0.5, 1.5, -1.5, 300.0, -300.0]
    q = wakeword.quantize_frames(mf)
    np.testing.assert_array_equal(q.cpu().numpy(), O.device_quantize_frames(mf))
    q8, f8 = wakeword.device_cmvn(q)
    qf, ff = wakeword.device_cmvn(mf)
    np.testing.assert_array_equal(q8.cpu().numpy(), qf.cpu().numpy())
    np.testing.assert_array_equal(q8.cpu().numpy(), O.device_cmvn(O.device_quantize_frames(mf)))
