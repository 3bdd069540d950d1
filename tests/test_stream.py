"""Streaming mode: the device sample ring behind
wk_stream_push, sliding windows (clip_stride < win_len), and the firmware's
decision rule (esp_wake_word_detector.cpp:241-257)."""
import os

import numpy as np
import pytest

from oracle import wk_oracle as O
from wakeword.stream import DecisionRule, WIN


def _logit(p):
    return float(np.log(p / (1 - p)))


def test_decision_rule_threshold_and_refractory():
    r = DecisionRule(threshold=0.8, refractory_samples=80000)
    assert not r(16000, _logit(0.79)).detected
    w = r(16480, _logit(0.81))
    assert w.detected and abs(w.prob - 0.81) < 1e-9
    # deaf for 5 s: windows must START at or after 16480 + 80000
    assert not r(16480 + 80000 + WIN - 480, _logit(0.99)).detected
    assert r(16480 + 80000 + WIN, _logit(0.99)).detected


def test_decision_rule_probability_is_sigmoid():
    r = DecisionRule()
    assert abs(r(WIN, 0.0).prob - 0.5) < 1e-12


@pytest.fixture(scope="module")
def model(golden_dir):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    import wakeword
    return wakeword.load_onnx(os.path.join(golden_dir, "xiaoa.onnx"))


def _stream_audio(seconds):
    clips = O.synth_clips(4321, 0, seconds)
    return clips.reshape(-1)


def _batch_logits(model, audio, hop):
    """All windows of `audio` at `hop` through one strided wk_forward (sliding windows)."""
    import torch
    import ctypes as C
    from wakeword import _lib
    d = torch.from_numpy(audio).cuda()
    n = (audio.size - WIN) // hop + 1
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream()
    _lib.check(_lib.lib().wk_forward(model._h.h, C.c_void_p(d.data_ptr()), _lib.WK_DTYPE_F32, n, WIN, hop,
                                     C.c_void_p(out.data_ptr()), None, C.c_void_p(st.cuda_stream)), "wk_forward")
    return out.cpu().numpy()


@pytest.mark.gpu
def test_sliding_windows_equal_copied_clips(model):
    import torch
    audio = _stream_audio(3)
    hop = 480
    got = _batch_logits(model, audio, hop)
    idx = np.arange(0, got.size, 7)
    clips = np.stack([audio[i * hop:i * hop + WIN] for i in idx])
    ref = model.detect(torch.from_numpy(clips)).reshape(-1).cpu().numpy()
    np.testing.assert_array_equal(got[idx], ref)      # same kernel, same samples: bit-identical
    want = O.detect_mode_b(clips[:4].astype(np.float64), O_W())
    assert np.abs(got[idx[:4]] - want).max() < 1e-3


def O_W():
    from wakeword.onnx_reader import read_onnx, xiaoa_state_dict
    inits, _, _ = read_onnx(os.path.join(os.path.dirname(__file__), "golden", "xiaoa.onnx"))
    return xiaoa_state_dict(inits)


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [480, 1000, 7919, 20000])
def test_stream_push_matches_batch(model, chunk):
    import wakeword
    audio = _stream_audio(4)
    hop = 480
    ref = _batch_logits(model, audio, hop)
    det = wakeword.StreamingDetector(model, hop=hop, capacity=1 << 16)
    ends, logits = [], []
    for p in range(0, audio.size, chunk):
        for w in det.push(audio[p:p + chunk]):
            ends.append(w.end)
            logits.append(w.logit)
    det.close()
    assert ends == [WIN + k * hop for k in range(ref.size)]
    np.testing.assert_array_equal(np.asarray(logits, np.float32), ref)


@pytest.mark.gpu
def test_stream_overwrite_oldest_and_reset(model):
    import wakeword
    hop, cap = 480, WIN + 4 * 480
    audio = _stream_audio(3)
    ref = _batch_logits(model, audio, hop)
    det = wakeword.StreamingDetector(model, hop=hop, capacity=cap)
    # One push of 3 s into a 1.12 s ring: only the windows still fully in the ring are scored.
    out = det.push(audio)
    total = audio.size
    oldest = -(-(total - cap) // hop)
    last = (total - WIN) // hop
    assert [w.end for w in out] == [WIN + k * hop for k in range(oldest, last + 1)]
    np.testing.assert_array_equal(np.asarray([w.logit for w in out], np.float32), ref[oldest:last + 1])
    # Wrap-around inside the mirrored ring, hop-sized pushes.
    det.reset()
    got = []
    for p in range(0, audio.size, hop):
        got += [w.logit for w in det.push(audio[p:p + hop])]
    np.testing.assert_array_equal(np.asarray(got, np.float32), ref)
    det.close()


@pytest.mark.gpu
def test_stream_deferred_ingest(model):
    """Pushes that score nothing (max_out = 0) launch nothing, so their samples
    reach the device ring at the next push that scores windows: across more
    than a ring's worth of such pushes, that push's windows equal the batch
    path's bit for bit."""
    import ctypes as C
    import wakeword
    from wakeword import _lib
    hop, cap = 480, WIN + 6 * 480
    audio = _stream_audio(4)
    ref = _batch_logits(model, audio, hop)
    det = wakeword.StreamingDetector(model, hop=hop, capacity=cap)
    L = _lib.lib()
    logits, ends = np.zeros(64, np.float32), np.zeros(64, np.int64)
    n = C.c_int32(0)
    split = audio.size - 3 * 480   # silent pushes up to here (> cap samples), then one scoring push
    for p in range(0, split, 1000):
        x = np.ascontiguousarray(audio[p:min(p + 1000, split)])
        _lib.check(L.wk_stream_push(det._s, x.ctypes.data_as(C.POINTER(C.c_float)), x.size,
                                    logits.ctypes.data_as(C.POINTER(C.c_float)),
                                    ends.ctypes.data_as(C.POINTER(C.c_int64)), 0, C.byref(n)), "wk_stream_push")
        assert n.value == 0
    assert split > cap
    out = det.push(audio[split:])   # scores the windows this push completes
    first, last = (split - WIN) // hop + 1, (audio.size - WIN) // hop
    assert last - first + 1 == 3
    assert [w.end for w in out] == [WIN + k * hop for k in range(first, last + 1)]
    np.testing.assert_array_equal(np.asarray([w.logit for w in out], np.float32), ref[first:last + 1])
    det.close()
