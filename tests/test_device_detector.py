"""The firmware's detector over an MFCC frame stream (SURVEY 8(f) item 1;
esp_wake_word_detector.cpp): int8 frame quantisation (record_task :128-131),
the 63-frame ring (:21-48), the per-window CMVN with population std
(detect_task :179-211) on the GPU (wk_device_cmvn), the int8 network, and the
80 % threshold + 5 s sleep + ring reset decision loop (:245-257).

Parity: the CMVN is bit-exact against oracle.device_cmvn, which is pinned here
to a scalar transcription of the firmware's C loops.  No reference fixture
holds device CMVN values (the firmware's MFCC frames come from esp-dl, absent
here), so the frame streams are synthetic or derived from the reference's WAVs
through the mode-A front-end: parity unpinned against the physical device."""
import math
import os
import wave

import numpy as np
import pytest

from oracle import wk_oracle as O
from wakeword.stream import FrameDecisionLoop


def _c_loop_cmvn(win):
    """detect_task :179-211 transcribed statement by statement (np.float32 scalars)."""
    f32 = np.float32
    out = np.zeros((63, 13), np.int8)
    mean = [f32(0)] * 13
    sd = [f32(0)] * 13
    for dim in range(13):
        s = f32(0)
        for fr in range(63):
            s = f32(s + f32(win[fr, dim]))
        mean[dim] = f32(s / f32(63.0))
    for dim in range(13):
        v = f32(0)
        for fr in range(63):
            d = f32(f32(win[fr, dim]) - mean[dim])
            v = f32(v + f32(d * d))
        sd[dim] = f32(np.sqrt(f32(v / f32(63.0))))
    for i in range(13 * 63):
        fr, dim = divmod(i, 13)
        nrm = f32(f32(f32(win[fr, dim]) - mean[dim]) / f32(sd[dim] + f32(1e-8)))
        q = int(math.floor(abs(float(nrm)) + 0.5)) * (1 if nrm >= 0 else -1)   # lroundf
        out[fr, dim] = max(-128, min(127, q))
    return out


def _frames(seed, n):
    r = np.random.default_rng(seed)
    f = np.round(r.normal(0, 20, (n, 13))).clip(-128, 127).astype(np.int8)
    f[100:180] = 7                                        # constant stretch: std 0 -> all zeros
    f[300:310] = np.where(np.arange(13) % 2, 127, -128)   # saturated frames
    return f


def _wav_frames():
    """Reference WAVs -> 20 ms frames (hop 320, as record_task feeds them) through
    the mode-A front-end, quantised like record_task (a stand-in for esp-dl's MFCC)."""
    d = os.path.join(os.path.dirname(__file__), "golden", "wav")
    out = []
    for name in sorted(os.listdir(d))[:4]:
        with wave.open(os.path.join(d, name)) as w:
            x = np.frombuffer(w.readframes(w.getnframes()), "<i2").astype(np.float32)
        xs = np.concatenate([np.zeros(4000, np.float32), x, np.zeros(4000, np.float32)])
        out.append(O.mfcc_esp(xs, frame=320, hop=320).astype(np.float32))
    return np.concatenate(out)


def test_quantize_frames_is_lroundf_saturated():
    v = np.array([0.5, -0.5, 1.49999, 2.5, -2.5, 127.6, -130.0, 0.49999997], np.float32)
    np.testing.assert_array_equal(O.device_quantize_frames(v), [1, -1, 1, 3, -3, 127, -128, 0])


def test_oracle_cmvn_matches_firmware_loops():
    f = _frames(1, 420)
    got = O.device_cmvn(f)
    assert got.shape == (420 - 62, 63, 13) and got.dtype == np.int8
    for w in (0, 40, 60, 100, 150, 250, 300, 357):
        np.testing.assert_array_equal(got[w], _c_loop_cmvn(f[w:w + 63].astype(np.float32)), err_msg=f"window {w}")
    assert not got[110].any()                             # inside the constant stretch
    assert O.device_cmvn(f[:62]).shape == (0, 63, 13)


def test_decision_loop_matches_oracle():
    r = np.random.default_rng(3)
    n = 3000
    logits = r.normal(-4, 1, n - 62).astype(np.float32)
    logits[[100, 101, 400, 700, 701, 2900]] = 3.0
    want = O.device_decisions(n, logits)
    loop, got = FrameDecisionLoop(), []
    for e in range(62, n):
        if loop.scored(e):
            w = loop(e, float(logits[e - 62]))
            got.append((w.end, w.detected))
    assert got == want
    fired = [e for e, d in want if d]
    assert fired[0] == 162 and 100 + 62 + 251 + 63 <= fired[1]   # deaf 250 frames, then 64 new frames
    assert want[0][0] == 63                                      # the 64th frame completes the first window


def _walk(loop, n, logits, zero_logit):
    """DeviceDetector's order of events on precomputed window logits (host only)."""
    got = []
    for e in range(62, n):
        while loop.pending is not None and loop.pending < e:
            w = loop(loop.pending, zero_logit, cleared=True)
            got.append((w.end, w.detected))
        if loop.scored(e):
            w = loop(e, float(logits[e - 62]))
            got.append((w.end, w.detected))
    while loop.pending is not None and loop.pending < n:
        w = loop(loop.pending, zero_logit, cleared=True)
        got.append((w.end, w.detected))
    return got


@pytest.mark.parametrize("zero_logit", [-4.0, 3.0])
def test_post_sleep_inference_on_the_cleared_ring(zero_logit):
    """After each 5 s sleep the firmware scores the just-cleared (all-zero)
    ring once (pending notification, :141-143,172,248-257): one extra window
    at the wake frame; if it fires, another sleep and another extra window."""
    r = np.random.default_rng(4)
    n = 3000
    logits = r.normal(-4, 1, n - 62).astype(np.float32)
    logits[[100, 101, 400, 700, 701, 2900]] = 3.0
    want = O.device_decisions(n, logits, cleared_logit=zero_logit)
    assert _walk(FrameDecisionLoop(), n, logits, zero_logit) == want
    fired = [e for e, d in want if d]
    assert (162 + 250, zero_logit > 0) in want                 # the wake frame's extra window
    if zero_logit > 0:                                           # fires again every 250 frames to the end
        assert fired == list(range(162, n, 250))
    else:
        assert fired[0] == 162 and (412, False) in want and fired[1] >= 412 + 1 + 63
    assert _walk(FrameDecisionLoop(cleared_inference=False), n, logits, zero_logit) == O.device_decisions(n, logits)


def test_decision_threshold_is_sigmoid_percent():
    loop = FrameDecisionLoop()
    w = loop(63, math.log(4.0) - 1e-4)       # sigmoid = 0.8 - eps
    assert not w.detected and abs(w.pct - 80.0) < 1e-2
    assert loop(64, 1.5).detected             # int8 output 12 * 2^-3


def test_device_cmvn_rejects_bad_args():
    from wakeword import _lib
    L = _lib.lib()
    assert L.wk_device_cmvn(None, 7, 100, None, None, None) == 1
    assert L.wk_device_cmvn(None, 2, 100, None, None, None) == 1   # no output
    assert L.wk_device_cmvn(None, 2, -1, None, None, None) == 1


# ---------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("src", ["int8", "float"])
def test_gpu_device_cmvn_bit_exact(gpu, src):
    import wakeword
    if src == "int8":
        f = _frames(7, 2500)
        ref = O.device_cmvn(f)
    else:
        f = _wav_frames()
        f[5, :4] = [0.5, -0.5, 2.5, 300.0]       # halves away from zero, saturation
        ref = O.device_cmvn(O.device_quantize_frames(f))
    q, feats = wakeword.device_cmvn(f)
    np.testing.assert_array_equal(q.cpu().numpy(), ref)
    np.testing.assert_array_equal(feats.cpu().numpy(), ref.transpose(0, 2, 1).astype(np.float32))


@pytest.mark.gpu
def test_gpu_device_pipeline_int8_logits(gpu, golden_dir, xiaoa_sd):
    """frames -> device CMVN -> the device's int8 network, bit-exact in int8 logits."""
    import wakeword
    m8 = wakeword.load_onnx(os.path.join(golden_dir, "xiaoa.onnx"), precision="int8")
    f = np.concatenate([O.device_quantize_frames(_wav_frames()), _frames(9, 400)])
    det = wakeword.DeviceDetector(m8)
    got = []
    for p in range(0, f.shape[0], 37):
        got += det.push(f[p:p + 37])
    c = O.device_cmvn(f)
    want = O.kws_forward_int8(O.quantize_input(c.transpose(0, 2, 1).astype(np.float64)), O.quantize_int8(xiaoa_sd))
    want = (want * 0.125).astype(np.float32)
    zero = float(O.kws_forward_int8(O.quantize_input(np.zeros((1, 13, 63))), O.quantize_int8(xiaoa_sd))[0] * 0.125)
    assert det.cleared_logit() == zero                    # the int8 net on the cleared ring
    dec = O.device_decisions(f.shape[0], want, cleared_logit=zero)
    assert [(w.end, w.detected) for w in got] == dec
    np.testing.assert_array_equal(np.asarray([w.logit for w in got if not w.cleared], np.float32),
                                  want[[w.end - 62 for w in got if not w.cleared]])


class _StubModel:
    """Logit per window = a fixed function of the device CMVN features (so the
    decision walk sees firing windows; the int8 model never fires on these streams)."""
    device = 0

    def __call__(self, feats):
        return (feats[:, 0, :].amax(dim=1) / 2.0 - 1.0).reshape(-1, 1)


@pytest.mark.gpu
def test_gpu_device_detector_decisions(gpu):
    import wakeword
    r = np.random.default_rng(11)
    f = np.round(r.normal(0, 10, (4000, 13))).astype(np.int8)
    f[::97, 0] = 120                    # sparse spikes in coefficient 0 -> occasional high scores
    det = wakeword.DeviceDetector(_StubModel())
    got = []
    for p in range(0, f.shape[0], 500):
        got += det.push(f[p:p + 500])
    c = O.device_cmvn(f)
    logits = (c[:, :, 0].astype(np.float32).max(axis=1) / np.float32(2.0) - np.float32(1.0)).astype(np.float32)
    want = O.device_decisions(f.shape[0], logits, cleared_logit=-1.0)   # the stub on the all-zero ring
    assert any(d for _, d in want) and [(w.end, w.detected) for w in got] == want
    assert any(w.cleared for w in got)
