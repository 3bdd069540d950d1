"""Streaming wake-word detection.

The audio arrives as a continuous 16 kHz stream; every `hop` samples (480 =
30 ms by default) one more 1 s window is complete and is scored by the fused
HIP path.  The sample ring lives on the device (wk_stream_* in the C ABI,
ring_buffer.c:57-117 overwrite-oldest semantics).  On top, the detector
applies the firmware's decision rule (esp_wake_word_detector.cpp:241-257):
probability >= 0.8 fires, then the detector is deaf for 5 s and restarts from
an empty history (the firmware sleeps 5 s and clears its MFCC ring, so the
next decision sees only audio recorded after that).
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from . import _lib
from ._lib import check, lib

WIN = 16000


@dataclass
class Window:
    end: int          # stream position (samples since start) one past the window's last sample
    logit: float
    prob: float
    detected: bool


class DecisionRule:
    """The firmware's threshold + refractory rule in the sample domain (pure
    host logic, testable without a GPU).  `suppressed_until` is the first
    stream position a new window may START at after a detection."""

    def __init__(self, threshold: float = 0.8, refractory_samples: int = 5 * 16000):
        self.threshold = threshold
        self.refractory = refractory_samples
        self.suppressed_until = 0

    def __call__(self, end: int, logit: float) -> Window:
        prob = 1.0 / (1.0 + math.exp(-logit))
        fire = (end - WIN) >= self.suppressed_until and prob >= self.threshold
        if fire:
            self.suppressed_until = end + self.refractory
        return Window(end, logit, prob, fire)


class StreamingDetector:
    """push(samples) -> list[Window] for the windows the push completed."""

    def __init__(self, model, hop: int = 480, capacity: int = 1 << 16, threshold: float = 0.8,
                 refractory_s: float = 5.0, sample_rate: int = 16000, stream=None):
        import torch
        self._model = model
        self.hop = hop
        self.capacity = capacity
        self.rule = DecisionRule(threshold, int(round(refractory_s * sample_rate)))
        dev = model._h.device
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        self._s = C.c_void_p()
        check(lib().wk_stream_create(model._h.h, hop, capacity, C.c_void_p(st.cuda_stream), C.byref(self._s)),
              "wk_stream_create")
        self._max = (capacity - WIN) // hop + 1
        self._logits = np.zeros(self._max, np.float32)
        self._ends = np.zeros(self._max, np.int64)

    def push(self, samples) -> List[Window]:
        x = np.ascontiguousarray(samples, np.float32).reshape(-1)
        n = C.c_int32(0)
        check(lib().wk_stream_push(self._s, x.ctypes.data_as(C.POINTER(C.c_float)), x.size,
                                   self._logits.ctypes.data_as(C.POINTER(C.c_float)),
                                   self._ends.ctypes.data_as(C.POINTER(C.c_int64)), self._max, C.byref(n)),
              "wk_stream_push")
        return [self.rule(int(self._ends[i]), float(self._logits[i])) for i in range(n.value)]

    def reset(self):
        check(lib().wk_stream_reset(self._s), "wk_stream_reset")
        self.rule.suppressed_until = 0

    def close(self):
        if self._s:
            lib().wk_stream_destroy(self._s)
            self._s = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------------------
# The firmware's detector over an MFCC frame stream (esp_wake_word_detector.cpp)
# ---------------------------------------------------------------------------
FRAME_WIN = 63           # frames per window (MFCC_LEN = 13*63, :3)
N_COEF = 13


def record_front(tdm, device: int = 0, float_out: bool = False):
    """wk_record_front: the firmware record task's sample path
    (esp_wake_word_detector.cpp:102-121) on device.  tdm: int16 48 kHz TDM
    samples of 4 channels, shape (n, 4), (frames, 960, 4) or flat (4n,), n a
    multiple of 3 -> int16 16 kHz samples (n // 3,) on device (and the same
    / 32768 as float32 when float_out)."""
    import torch
    x = tdm
    if isinstance(x, np.ndarray):
        x = torch.from_numpy(np.ascontiguousarray(x))
    if x.dtype != torch.int16:
        raise ValueError(f"TDM samples must be int16, got {x.dtype}")
    x = x.to(f"cuda:{device}").contiguous().reshape(-1)
    if x.numel() % 12:
        raise ValueError("TDM input must hold whole groups of 3 samples x 4 channels")
    n_out = x.numel() // 12
    out = torch.empty((n_out,), dtype=torch.int16, device=x.device)
    f = torch.empty((n_out,), dtype=torch.float32, device=x.device) if float_out else None
    st = torch.cuda.current_stream(x.device)
    check(lib().wk_record_front(C.c_void_p(x.data_ptr()), n_out, C.c_void_p(out.data_ptr()),
                                C.c_void_p(f.data_ptr()) if f is not None else None, C.c_void_p(st.cuda_stream)),
          "wk_record_front")
    return (out, f) if float_out else out


def quantize_frames(mfcc, device: int = 0):
    """wk_quantize_frames: record_task's int8 frame quantisation (:128-131),
    lroundf then saturate -> int8 tensor of mfcc's shape, on device."""
    import torch
    x = torch.as_tensor(mfcc, dtype=torch.float32).to(f"cuda:{device}").contiguous()
    q = torch.empty(x.shape, dtype=torch.int8, device=x.device)
    st = torch.cuda.current_stream(x.device)
    check(lib().wk_quantize_frames(C.c_void_p(x.data_ptr()), x.numel(), C.c_void_p(q.data_ptr()),
                                   C.c_void_p(st.cuda_stream)), "wk_quantize_frames")
    return q


def device_cmvn(frames, device: int = 0):
    """wk_device_cmvn on an MFCC frame stream [n][13] (int8 as the firmware
    stores it, or float MFCC quantised first as record_task :128-131 does):
    returns (int8 [n-62][63][13] -- the firmware's mfcc_cmvn_buffer per window --,
    float [n-62][13][63] -- the same values in wk_cnn's feature layout)."""
    import torch
    x = frames
    if isinstance(x, np.ndarray):
        x = torch.from_numpy(np.ascontiguousarray(x))
    is_i8 = x.dtype == torch.int8
    x = x.to(device=f"cuda:{device}", dtype=torch.int8 if is_i8 else torch.float32).contiguous()
    if x.dim() != 2 or x.shape[1] != N_COEF:
        raise ValueError(f"expected frames (n, 13), got {tuple(x.shape)}")
    nw = max(x.shape[0] - (FRAME_WIN - 1), 0)
    q = torch.empty((nw, FRAME_WIN, N_COEF), dtype=torch.int8, device=x.device)
    f = torch.empty((nw, N_COEF, FRAME_WIN), dtype=torch.float32, device=x.device)
    st = torch.cuda.current_stream(x.device)
    check(lib().wk_device_cmvn(C.c_void_p(x.data_ptr()), _lib.WK_DTYPE_I8 if is_i8 else _lib.WK_DTYPE_F32,
                               x.shape[0], C.c_void_p(q.data_ptr()), C.c_void_p(f.data_ptr()),
                               C.c_void_p(st.cuda_stream)), "wk_device_cmvn")
    return q, f


@dataclass
class FrameWindow:
    end: int          # index (frames since start) of the window's newest frame
    logit: float      # model output (int8 model: raw * 2^-3, as the firmware dequantises it, :226-227)
    pct: float        # sigmoid * 100 (:228)
    detected: bool
    cleared: bool = False   # the post-sleep inference on the just-cleared (all-zero) ring


class FrameDecisionLoop:
    """detect_task's control flow (esp_wake_word_detector.cpp:171-258) in the
    frame domain (host logic, testable without a GPU).  The window ending at
    frame e is scored once 64 frames were written since the last reset
    (shared_counter == 64, :38-44,141 -- the 64th frame overwrites the first, so
    the window is the newest 63); sigmoid*100 >= threshold fires (:245); the
    task then sleeps 5 s = `deaf_frames` frames of 20 ms (:248) and clears the
    ring (:251-256), so the next window needs 64 frames written after that.

    The extra inference after each sleep (cleared_inference=True): record_task
    keeps notifying while detect_task sleeps (:141-143), so right after the
    reset ulTaskNotifyTake (:172) returns at once and the task scores the
    cleared ring -- all zeros, since the reset and that read fall in one 20 ms
    frame period -- as a window at the wake frame (fire frame + deaf_frames).
    `pending` is that frame until it is scored; a firing extra inference sleeps
    and clears again."""

    def __init__(self, threshold_pct: float = 80.0, deaf_frames: int = 250, cleared_inference: bool = True):
        self.threshold = np.float32(threshold_pct)
        self.deaf = deaf_frames
        self.cleared_inference = cleared_inference
        self.reset_at = 0          # first frame written after the last reset
        self.pending: Optional[int] = None

    def scored(self, e: int) -> bool:
        return e - self.reset_at >= FRAME_WIN

    def __call__(self, e: int, logit: float, cleared: bool = False) -> FrameWindow:
        x = np.float32(logit)
        pct = np.float32(1.0) / (np.float32(1.0) + np.exp(-x)) * np.float32(100.0)
        fire = bool(pct >= self.threshold)
        if cleared:
            self.pending = None
        if fire:
            self.reset_at = e + self.deaf + 1
            self.pending = e + self.deaf if self.cleared_inference else None
        return FrameWindow(e, float(x), float(pct), fire, cleared)


class DeviceDetector:
    """The firmware's wake-word loop on an MFCC frame stream, on the GPU:
    push(frames [n][13]) -> the windows it scored.  Each push runs
    wk_device_cmvn over the new windows and the model (normally a
    precision='int8' KWSModel: the device's esp-dl int8 network) in one batch;
    the decision loop then walks them in order.  The MFCC frames themselves come
    from esp-dl's dl::audio::MFCC on the device (a third-party library absent
    here): the caller supplies them, int8 or float."""

    def __init__(self, model, threshold_pct: float = 80.0, refractory_s: float = 5.0, frame_s: float = 0.02,
                 cleared_inference: bool = True):
        self._model = model
        self.loop = FrameDecisionLoop(threshold_pct, int(round(refractory_s / frame_s)), cleared_inference)
        self._tail = None          # the last <= 62 frames of earlier pushes
        self._next = 0             # index of the next frame to arrive
        self._zero_logit = None    # the model on the CMVN of an all-zero ring (computed once)

    def cleared_logit(self) -> float:
        """The model's output on the cleared ring (63 zero frames through the
        device CMVN: all zeros), scored after every sleep."""
        if self._zero_logit is None:
            _, feats = device_cmvn(np.zeros((FRAME_WIN, N_COEF), np.int8), self._model.device)
            self._zero_logit = float(self._model(feats).reshape(-1)[0])
        return self._zero_logit

    def _due(self, before: int, out: List[FrameWindow]) -> None:
        while self.loop.pending is not None and self.loop.pending < before:
            out.append(self.loop(self.loop.pending, self.cleared_logit(), cleared=True))

    def push(self, frames) -> List[FrameWindow]:
        f = np.asarray(frames)
        if f.ndim != 2 or f.shape[1] != N_COEF:
            raise ValueError(f"expected frames (n, 13), got {f.shape}")
        if f.dtype != np.int8:
            f = f.astype(np.float32)
        if self._tail is not None and self._tail.dtype != f.dtype:   # int8 frames as floats quantise to themselves
            f, self._tail = f.astype(np.float32), self._tail.astype(np.float32)
        cat = f if self._tail is None else np.concatenate([self._tail, f])
        first = self._next - (0 if self._tail is None else self._tail.shape[0])   # frame index of cat[0]
        self._next += f.shape[0]
        self._tail = cat[-(FRAME_WIN - 1):].copy()
        out: List[FrameWindow] = []
        ends = np.arange(first + FRAME_WIN - 1, first + cat.shape[0])
        if cat.shape[0] < FRAME_WIN or not any(self.loop.scored(int(e)) for e in ends):
            self._due(self._next, out)   # (reset_at only grows during the walk)
            return out
        _, feats = device_cmvn(cat, self._model.device)
        logits = self._model(feats).reshape(-1).cpu().numpy()
        for e, lg in zip(ends, logits):
            self._due(int(e), out)
            if self.loop.scored(int(e)):
                out.append(self.loop(int(e), float(lg)))
        self._due(self._next, out)
        return out
