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
