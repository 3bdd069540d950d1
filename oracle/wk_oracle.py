"""CPU ORACLE for the wake-word hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the timed CPU baseline.
The product path (``esp32-wake-word_amd/wakeword`` + ``libwakeword.so``) never
imports or calls anything in ``oracle/``.

What it restates (float64 numpy, citations are to /root/reference):

* Front-end mode B, the training front-end the xiaoa CNN was fit to:
  ``ml_models/src/extract_mfcc.py:137-175`` -> torchaudio
  ``functional.preemphasis`` (:171) + ``transforms.MFCC`` (:137-148) +
  ``normalize_mfcc(method='cmvn')`` (:73-80).  torchaudio is a third-party
  dependency that is absent from this image (unpinned version, torchaudio 2.x
  semantics restated: Spectrogram(center=True, pad_mode='reflect', periodic
  window zero-padded to n_fft centred), MelScale(htk, norm=None),
  AmplitudeToDB is NOT used because log_mels=True -> ln(mel + 1e-6),
  create_dct(norm='ortho')).
  PARITY STATUS: no reference test or fixture holds torchaudio MFCC values, so
  the front-end restatement is "parity unpinned" at the torchaudio boundary;
  it is pinned indirectly (KAT statistics, detections on the reference WAVs)
  and cross-checked against torch.stft in tests/golden/make_golden.py.

* The xiaoa CNN ``LightweightKWS`` (``ml_models/src/wakeModel.py:4-34``) with
  the ``ml_models/xiaoa.onnx`` weights.  PINNED: golden logits in
  tests/golden were produced by importing the reference's own class.

* The GRU-CTC head (``ml_models/ctc.py:82-152,453-471``) lives in
  ``oracle/wk_ctc_oracle.py``; front-end mode A (``main/esp_mfcc/mfcc.c``) is
  the C restatement ``oracle/esp_mfcc_oracle.c``.
"""
from __future__ import annotations

import numpy as np

SAMPLE_RATE = 16000
WIN_SAMPLES = 16000
N_FFT = 512
WIN_LENGTH = 320
HOP = 256
N_MELS = 40
N_MFCC = 13
N_FRAMES = 1 + WIN_SAMPLES // HOP  # 63 with center=True


# --------------------------------------------------------------------------
# B0: pad / trim (extract_mfcc.py:7-23)
# --------------------------------------------------------------------------
def pad_audio(audio: np.ndarray, target_length: int = WIN_SAMPLES, noise: np.ndarray | None = None) -> np.ndarray:
    """extract_mfcc.py:7-23.  ``noise`` is the pre-drawn N(0,1)*0.005 pad (the
    reference draws it with torch.randn); None -> zero pad (add_noise_to_pad=False)."""
    audio = np.asarray(audio, dtype=np.float32)
    n = audio.shape[-1]
    if n > target_length:
        return audio[..., :target_length].copy()
    if n < target_length:
        pad = np.zeros(target_length - n, np.float32) if noise is None else np.asarray(noise, np.float32)
        return np.concatenate([audio, pad], axis=-1)
    return audio.copy()


# --------------------------------------------------------------------------
# B1: preemphasis (torchaudio.functional.preemphasis, extract_mfcc.py:171)
# --------------------------------------------------------------------------
def preemphasis(x: np.ndarray, coeff: float = 0.97) -> np.ndarray:
    x = np.asarray(x, np.float64)
    y = x.copy()
    y[..., 1:] -= coeff * x[..., :-1]
    return y


# --------------------------------------------------------------------------
# B2: Spectrogram (power=2, center/reflect, periodic hamming(320) in 512)
# --------------------------------------------------------------------------
def hamming_periodic(n: int) -> np.ndarray:
    k = np.arange(n, dtype=np.float64)
    return 0.54 - 0.46 * np.cos(2.0 * np.pi * k / n)


def power_spectrogram(y: np.ndarray) -> np.ndarray:
    """(..., L) -> (..., T, 257) power |X|^2, torch.stft(center=True, reflect)."""
    y = np.asarray(y, np.float64)
    pad = N_FFT // 2
    yp = np.pad(y, [(0, 0)] * (y.ndim - 1) + [(pad, pad)], mode="reflect")
    n_frames = 1 + (yp.shape[-1] - N_FFT) // HOP
    win = np.zeros(N_FFT)
    left = (N_FFT - WIN_LENGTH) // 2
    win[left:left + WIN_LENGTH] = hamming_periodic(WIN_LENGTH)
    idx = np.arange(n_frames)[:, None] * HOP + np.arange(N_FFT)[None, :]
    frames = yp[..., idx] * win
    spec = np.fft.rfft(frames, n=N_FFT, axis=-1)
    return spec.real ** 2 + spec.imag ** 2


# --------------------------------------------------------------------------
# B3: MelScale fbanks (htk, norm=None)
# --------------------------------------------------------------------------
def _hz_to_mel_htk(f):
    return 2595.0 * np.log10(1.0 + np.asarray(f, np.float64) / 700.0)


def _mel_to_hz_htk(m):
    return 700.0 * (10.0 ** (np.asarray(m, np.float64) / 2595.0) - 1.0)


def melscale_fbanks(n_freqs: int = N_FFT // 2 + 1, f_min: float = 0.0, f_max: float = SAMPLE_RATE / 2,
                    n_mels: int = N_MELS, sample_rate: int = SAMPLE_RATE) -> np.ndarray:
    """(n_freqs, n_mels) triangular HTK filterbank, no area normalisation."""
    all_freqs = np.linspace(0, sample_rate // 2, n_freqs)
    m_pts = np.linspace(_hz_to_mel_htk(f_min), _hz_to_mel_htk(f_max), n_mels + 2)
    f_pts = _mel_to_hz_htk(m_pts)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts[None, :] - all_freqs[:, None]
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return np.maximum(0.0, np.minimum(down, up))


# --------------------------------------------------------------------------
# B5: DCT-II ortho (create_dct)
# --------------------------------------------------------------------------
def create_dct(n_mfcc: int = N_MFCC, n_mels: int = N_MELS) -> np.ndarray:
    """(n_mels, n_mfcc) DCT-II matrix, norm='ortho'."""
    n = np.arange(n_mels, dtype=np.float64)
    k = np.arange(n_mfcc, dtype=np.float64)[:, None]
    dct = np.cos(np.pi / n_mels * (n + 0.5) * k)
    dct[0] *= 1.0 / np.sqrt(2.0)
    dct *= np.sqrt(2.0 / n_mels)
    return dct.T


def mfcc_torchaudio(x: np.ndarray) -> np.ndarray:
    """B1..B5: (..., 16000) waveform -> (..., 13, 63) MFCC (coefficient-major)."""
    p = power_spectrogram(preemphasis(x))               # (..., T, 257)
    mel = p @ melscale_fbanks()                          # (..., T, 40)
    logmel = np.log(mel + 1e-6)
    mf = logmel @ create_dct()                           # (..., T, 13)
    return np.swapaxes(mf, -1, -2)


# --------------------------------------------------------------------------
# B6: normalize_mfcc (extract_mfcc.py:47-88)
# --------------------------------------------------------------------------
def normalize_mfcc(m: np.ndarray, method: str = "cmvn") -> np.ndarray:
    m = np.asarray(m, np.float64)
    if method in ("standardization", "cmvn"):
        mean = m.mean(axis=-1, keepdims=True)
        std = m.std(axis=-1, ddof=1, keepdims=True)
        std = np.where(std == 0, 1.0, std)
        return (m - mean) / (std + 1e-8)
    if method == "minmax":
        mn = m.min(axis=-1, keepdims=True)
        mx = m.max(axis=-1, keepdims=True)
        return (m - mn) / (mx - mn + 1e-8)
    return m


def features_mode_b(x: np.ndarray) -> np.ndarray:
    """Full mode-B front-end: waveform (..., 16000) -> CMVN'd (..., 13, 63)."""
    return normalize_mfcc(mfcc_torchaudio(x), "cmvn")


# --------------------------------------------------------------------------
# CNN: LightweightKWS (wakeModel.py:4-34), NCW layout
# --------------------------------------------------------------------------
def _conv1d_k3p1(x: np.ndarray, w: np.ndarray) -> np.ndarray:
    """x (B, Cin, T), w (Cout, Cin, 3) -> (B, Cout, T); padding=1, no bias."""
    xp = np.pad(x, ((0, 0), (0, 0), (1, 1)))
    T = x.shape[-1]
    out = np.zeros((x.shape[0], w.shape[0], T))
    for k in range(3):
        out += np.einsum("oc,bct->bot", w[:, :, k], xp[:, :, k:k + T])
    return out


def _maxpool2(x: np.ndarray) -> np.ndarray:
    T = x.shape[-1] // 2
    return np.maximum(x[..., 0:2 * T:2], x[..., 1:2 * T:2])


def kws_forward(feats: np.ndarray, w: dict) -> np.ndarray:
    """feats (B, 13, 63) -> logits (B, 1).  ``w`` keys follow the reference
    state dict: conv_layers.{0,3,6}.weight, classifier.{0,2}.weight."""
    x = np.asarray(feats, np.float64)
    for key in ("conv_layers.0.weight", "conv_layers.3.weight", "conv_layers.6.weight"):
        x = _maxpool2(np.maximum(_conv1d_k3p1(x, np.asarray(w[key], np.float64)), 0.0))
    g = x.mean(axis=-1)                                               # (B, 128)
    h = np.maximum(g @ np.asarray(w["classifier.0.weight"], np.float64).T, 0.0)
    return h @ np.asarray(w["classifier.2.weight"], np.float64).T      # (B, 1)


def detect_mode_b(x: np.ndarray, w: dict) -> np.ndarray:
    """Waveform (B, 16000) -> logits (B,)."""
    return kws_forward(features_mode_b(x), w)[:, 0]


# --------------------------------------------------------------------------
# Synthetic clip generator -- host restatement of the
# device generator in csrc/wk_synth.hip (same counter-based hash).
# --------------------------------------------------------------------------
def _mix32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(16)
    return x


def synth_clips(seed: int, first: int, count: int, n: int = WIN_SAMPLES) -> np.ndarray:
    """clamp(0.1*N(0,1), -1, 1) (+ 0.1*sin(2*pi*440*t/16000) on odd clips).

    N(0,1) from Box-Muller over two 24-bit uniforms drawn from a counter hash
    keyed on (seed, global clip index, sample index).  float32 output."""
    clip = np.arange(first, first + count, dtype=np.uint64)[:, None]
    s = np.arange(n, dtype=np.uint64)[None, :]
    key = _mix32(np.uint64(seed) ^ (clip * np.uint64(0x9E3779B9)))
    h1 = _mix32(key ^ (s * np.uint64(2) + np.uint64(0x68E31DA4)))
    h2 = _mix32(h1 ^ np.uint64(0xB5297A4D))
    u1 = ((h1 >> np.uint64(8)).astype(np.float32) + np.float32(1.0)) * np.float32(1.0 / 16777216.0)
    u2 = (h2 >> np.uint64(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    r = np.sqrt(np.float32(-2.0) * np.log(u1))
    g = (r * np.cos(np.float32(2.0 * np.pi) * u2)).astype(np.float32)
    x = np.clip(np.float32(0.1) * g, -1.0, 1.0).astype(np.float32)
    odd = (clip % np.uint64(2)) == 1
    phase = ((s * np.uint64(440)) % np.uint64(16000)).astype(np.float32) * np.float32(1.0 / 16000.0)
    sine = (np.float32(0.1) * np.sin(np.float32(2.0 * np.pi) * phase)).astype(np.float32)
    return np.where(odd, x + sine, x).astype(np.float32)


# --------------------------------------------------------------------------
# Front-end mode A: main/esp_mfcc/mfcc.c:431-527 (numpy restatement; the C
# restatement is oracle/esp_mfcc_oracle.c -- the two cross-check each other,
# no reference fixture pins mode-A values: "parity unpinned").
# --------------------------------------------------------------------------
def fbank_mode_a(sr: int = SAMPLE_RATE, n_filters: int = N_MELS, n_fft: int = N_FFT) -> np.ndarray:
    """(n_fft/2+1, n_filters) integer-bin triangles (mfcc.c:133-234), float32
    arithmetic as in the C code (hz_to_mel 1127 ln(1+f/700), f=0 -> 1; the
    inverse uses 700 (10^(m/2595) - 1), the reference's mixed definitions)."""
    f32 = np.float32
    nb = n_fft // 2 + 1

    def h2m(f):
        f = f32(1.0) if f == 0 else f32(f)
        return f32(1127.0) * np.log1p(f32(f / f32(700.0)), dtype=np.float32)

    lo, hi = h2m(0.0), h2m(sr // 2)
    bw = f32(sr) / f32(n_fft)
    bins = []
    for i in range(n_filters + 2):
        m = f32(lo + f32(i) * (hi - lo) / f32(n_filters + 1))
        hz = f32(700.0) * (np.power(f32(10.0), f32(m / f32(2595.0)), dtype=np.float32) - f32(1.0))
        bins.append(int(np.floor(f32(hz / bw))))
    fb = np.zeros((n_filters, nb), np.float32)
    for i in range(n_filters):
        l, c, r = (min(max(b, 0), nb - 1) for b in bins[i:i + 3])
        if l >= c:
            c = l + 1
        if c >= r:
            r = c + 1
        if r >= nb:
            r = nb - 1
        for j in range(l, c + 1):
            fb[i, j] = f32(j - l) / f32(c - l)
        for j in range(c, r + 1):
            fb[i, j] = f32(r - j) / f32(r - c)
    return fb.T


def mfcc_esp(x: np.ndarray, esp_pack: bool = True, frame: int = 320, hop: int = 256, n_fft: int = N_FFT,
             n_filters: int = N_MELS, n_mfcc: int = N_MFCC) -> np.ndarray:
    """Mode-A MFCC of one signal (L,) -> (n_frames, n_mfcc), frame-major.
    float64 DFT (exact) in place of esp-dsp's float radix-2 FFT."""
    x = np.asarray(x, np.float32)
    L = x.shape[0]
    nf = (L - frame) // hop + 1
    y = np.empty_like(x)
    y[0] = x[0]
    y[1:] = x[1:] - np.float32(0.97) * x[:-1]
    i = np.arange(frame)
    win = (np.float32(0.53836) - np.float32(1.0 - 0.53836) *
           np.cos(2.0 * np.pi * i / (frame - 1)).astype(np.float32)).astype(np.float32)
    idx = np.arange(nf)[:, None] * hop + i[None, :]
    fr = (y[idx] * win).astype(np.float64)
    X = np.fft.rfft(fr, n=n_fft, axis=-1)
    re, im = X.real.astype(np.float32), X.imag.astype(np.float32)
    if esp_pack:
        re[:, 1:-1] *= 2.0
        im[:, 1:-1] *= 2.0
        re[:, -1] = 0.0
        im[:, -1] = 0.0
    pw = (re * re + im * im) / np.float32(n_fft) + np.float32(1e-12)
    mel = np.log(np.maximum(pw.astype(np.float64) @ fbank_mode_a(n_filters=n_filters, n_fft=n_fft), 1e-12))
    k = np.arange(n_mfcc)[:, None]
    n = np.arange(n_filters)[None, :]
    D = np.cos(np.pi * k * (2 * n + 1) / (2.0 * n_filters))
    scale = np.where(np.arange(n_mfcc) == 0, np.sqrt(1.0 / n_filters), np.sqrt(2.0 / n_filters))
    return (mel @ D.T) * scale[None, :]


# --------------------------------------------------------------------------
# int8 CNN in the device's esp-dl arithmetic:
# power-of-2 per-tensor exponents of ml_models/xiaoa.info:3139-3150,
# weights rne(w * 2^-e) (pinned: equal to xiaoa.info's int8 weights), requant
# round-half-even (pinned only by the xiaoa.info KAT: test input -> -40).
# --------------------------------------------------------------------------
INT8_W_EXP = {"conv_layers.0.weight": -8, "conv_layers.3.weight": -9, "conv_layers.6.weight": -9,
              "classifier.0.weight": -9, "classifier.2.weight": -9}


def quantize_int8(w: dict) -> dict:
    return {k: np.clip(np.round(np.asarray(w[k], np.float64) * 2.0 ** (-e)), -128, 127).astype(np.int64)
            for k, e in INT8_W_EXP.items()}


def _rne_shift(acc: np.ndarray, s: int) -> np.ndarray:
    return np.clip(np.round(acc / float(1 << s)), -128, 127).astype(np.int64)   # exact in float64 (|acc| < 2^31)


def kws_forward_int8(q_in: np.ndarray, qw: dict) -> np.ndarray:
    """q_in (B, 13, 63) int8 at exp -4 -> int8 logits (B,) at exp -3."""
    x = np.asarray(q_in, np.int64)

    def conv(a, W):   # a (B, Cin, T), W (Cout, Cin, 3)
        T = a.shape[-1]
        ap = np.pad(a, ((0, 0), (0, 0), (1, 1)))
        return sum(np.einsum("oc,bct->bot", W[:, :, k], ap[:, :, k:k + T]) for k in range(3))

    for key, s in (("conv_layers.0.weight", 7), ("conv_layers.3.weight", 9), ("conv_layers.6.weight", 10)):
        x = np.maximum(_rne_shift(conv(x, qw[key]), s), 0)
        T = x.shape[-1] // 2
        x = np.maximum(x[..., 0:2 * T:2], x[..., 1:2 * T:2])
    g = np.clip(np.round(x.sum(-1) * 2.0 / 7.0), -128, 127).astype(np.int64)   # GAP, exp -4 -> -5
    h = np.maximum(_rne_shift(g @ qw["classifier.0.weight"].T, 10), 0)
    return _rne_shift(h @ qw["classifier.2.weight"].T, 10)[:, 0]


def quantize_input(feats: np.ndarray) -> np.ndarray:
    """TensorBase::assign float -> int8 at exp -4 (round half away from zero, saturate)."""
    v = np.asarray(feats, np.float64) * 16.0
    return np.clip(np.sign(v) * np.floor(np.abs(v) + 0.5), -128, 127).astype(np.int64)


# --------------------------------------------------------------------------
# The firmware's detector over an MFCC frame stream:
# main/esp_wake_word_detector/src/esp_wake_word_detector.cpp.  fp32 numpy ops
# are each IEEE-rounded, in the firmware's loop order, so the int8 results are
# the C loops' results bit for bit.
# --------------------------------------------------------------------------
def record_front(tdm: np.ndarray) -> np.ndarray:
    """record_task's sample path, esp_wake_word_detector.cpp:102-121, in int32
    like the C: tdm int16 [..., 4] 48 kHz TDM samples (CH0 MIC-L, CH1 AEC ref,
    CH2 MIC-R, CH3 unused), a multiple of 3 of them -> int16 16 kHz samples.
      :106-111  weighted = (L<<6) + (AEC<<5) + (R<<6);  mono = (int16_t)(weighted >> 7)
      :114-121  out = (int16_t)((mono[3i] + 2 mono[3i+1] + mono[3i+2]) >> 2)
    The int16 casts keep the low 16 bits (numpy's int32 -> int16 cast wraps the
    same way); >> on int32 is arithmetic in both."""
    q = np.asarray(tdm, np.int16).reshape(-1, 4).astype(np.int32)
    assert q.shape[0] % 3 == 0, "whole groups of 3 TDM samples"
    weighted = (q[:, 0] << 6) + (q[:, 1] << 5) + (q[:, 2] << 6)
    mono = (weighted >> 7).astype(np.int16).astype(np.int32)
    m = mono.reshape(-1, 3)
    return ((m[:, 0] * 1 + m[:, 1] * 2 + m[:, 2] * 1) >> 2).astype(np.int16)


def record_front_loop(tdm_frame: np.ndarray) -> np.ndarray:
    """The same for one 20 ms frame (3840 int16), statement by statement as the
    C loops run (small inputs only; pins record_front)."""
    def i16(v):
        return ((int(v) + 32768) % 65536) - 32768
    x = [int(v) for v in np.asarray(tdm_frame, np.int16).reshape(-1)]
    mono = []
    for i in range(len(x) // 4):
        weighted = x[i * 4] * 64 + x[i * 4 + 1] * 32 + x[i * 4 + 2] * 64    # (int32)v << k == v * 2^k
        mono.append(i16(weighted >> 7))                                     # Python >> is arithmetic
    return np.array([i16((mono[3 * i] + 2 * mono[3 * i + 1] + mono[3 * i + 2]) >> 2) for i in range(len(mono) // 3)],
                    np.int16)


def device_quantize_frames(mfcc: np.ndarray) -> np.ndarray:
    """record_task :128-131: (int32_t)lroundf(v), saturated to int8."""
    v = np.asarray(mfcc, np.float32).astype(np.float64)
    return np.clip(np.sign(v) * np.floor(np.abs(v) + 0.5), -128, 127).astype(np.int8)


def device_cmvn(frames: np.ndarray) -> np.ndarray:
    """detect_task :179-211 for every 63-frame window of an int8 frame stream
    [n][13] (window w = frames w..w+62, read_whole_mfcc_buffer order :21-29):
    mean, population std (/63), (v - mean) / (std + 1e-8), lroundf, saturate.
    Returns int8 [n-62][63][13] (the firmware's mfcc_cmvn_buffer)."""
    f = np.asarray(frames, np.int8).astype(np.float32)
    n = f.shape[0]
    if n < 63:
        return np.zeros((0, 63, 13), np.int8)
    win = np.lib.stride_tricks.sliding_window_view(f, (63, 13))[:, 0]   # (W, 63, 13)
    s = np.zeros((win.shape[0], 13), np.float32)
    for t in range(63):
        s = s + win[:, t]
    mean = s / np.float32(63.0)
    var = np.zeros_like(s)
    for t in range(63):
        d = win[:, t] - mean
        var = var + d * d
    sd = np.sqrt(var / np.float32(63.0))
    nrm = (win - mean[:, None, :]) / (sd[:, None, :] + np.float32(1e-8))
    return device_quantize_frames(nrm)


def device_decisions(n_frames: int, logits: np.ndarray, threshold_pct: float = 80.0, deaf_frames: int = 250,
                     cleared_logit: float | None = None):
    """detect_task's control flow (:171-258) in the frame domain, as a plain loop:
    the window ending at frame e (frames e-62..e) is scored once 64 frames were
    written since the last reset (shared_counter == 64, :38-44,141); a score
    sigmoid(x)*100 >= 80 (:228,245) fires, the task sleeps 5 s (250 frames of 20
    ms, :248) and then clears the buffer (:251-256).  logits[e - 62] is the
    window ending at frame e.  Returns (end_frame, detected) of every scored window.

    cleared_logit (the model's output on the CMVN of an all-zero ring): the
    firmware's extra inference after each sleep.  record_task keeps calling
    xTaskNotifyGive (:141-143) while detect_task sleeps, so when it has cleared
    the ring its ulTaskNotifyTake (:172) returns at once and it scores the
    cleared buffer -- all zeros: the reset and that read happen within the same
    20 ms frame period -- as the window "ending" at the wake frame x + 250.  If
    that fires too, it sleeps and clears again."""
    def fires(x):
        x = np.float32(x)
        pct = np.float32(1.0) / (np.float32(1.0) + np.exp(-x)) * np.float32(100.0)
        return bool(pct >= np.float32(threshold_pct))

    out, reset = [], 0
    e = 62
    while e < n_frames:
        if e - reset < 63:
            e += 1
            continue
        fire = fires(logits[e - 62])
        out.append((e, fire))
        if fire:
            x = e
            while True:
                wake = x + deaf_frames
                reset = wake + 1
                if cleared_logit is None or wake >= n_frames:
                    break
                again = fires(cleared_logit)
                out.append((wake, again))
                if not again:
                    break
                x = wake
            e = reset
            continue
        e += 1
    return out
