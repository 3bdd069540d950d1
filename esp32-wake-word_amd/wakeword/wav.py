"""WAV ingest + waveform augmentation over the native
host loader in libwakeword.so (wk_wav_read / wk_wav_load_batch / wk_augment):
esp_wav.cpp's header walk, torchaudio.load scaling, extract_mfcc.py's
pad_audio and augment_audio_waveform."""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import check, lib


def read_wav(path: str, max_samples: int = 16000) -> Tuple[np.ndarray, Dict[str, int]]:
    """int16 samples (channel 0, at most max_samples -- the reference truncates
    to 16000, esp_wav.cpp:129-133) and the header fields."""
    out = np.zeros(max(max_samples, 1), np.int16)
    info = _lib.WkWavInfo()
    check(lib().wk_wav_read(path.encode(), out.ctypes.data_as(C.c_void_p), max_samples, C.byref(info)), "wk_wav_read")
    meta = {k: getattr(info, k) for k, _ in _lib.WkWavInfo._fields_}
    return out[:info.n_samples].copy(), meta


def load_batch(paths: Sequence[str], pad_to: int = 16000, noise_level: float = 0.005, seed: int = 0,
               out=None) -> Tuple[np.ndarray, List[int]]:
    """(len(paths), pad_to) float32 in [-1, 1): x/32768, trimmed or right-padded
    with N(0, noise_level^2) (pad_audio, extract_mfcc.py:7-23; 0 = zero pad).
    `out` may be a pinned torch tensor or numpy array of that shape."""
    n = len(paths)
    arr = (C.c_char_p * n)(*[p.encode() for p in paths])
    if out is None:
        out = np.zeros((n, pad_to), np.float32)
    ptr = out.data_ptr() if hasattr(out, "data_ptr") else out.ctypes.data
    n_read = np.zeros(max(n, 1), np.int32)
    check(lib().wk_wav_load_batch(arr, n, pad_to, noise_level, seed & 0xFFFFFFFF, C.c_void_p(ptr),
                                  n_read.ctypes.data_as(C.c_void_p)), "wk_wav_load_batch")
    return out, n_read[:n].tolist()


def augment(x: np.ndarray, speed: float = 1.0, volume: float = 1.0, noise_level: float = 0.0, seed: int = 0,
            out_len: int = 16000) -> np.ndarray:
    """augment_audio_waveform (extract_mfcc.py:90-121) for one waveform."""
    x = np.ascontiguousarray(x, np.float32).reshape(-1)
    out = np.zeros(out_len, np.float32)
    check(lib().wk_augment(x.ctypes.data_as(C.c_void_p), x.size, speed, volume, noise_level, seed & 0xFFFFFFFF,
                           out.ctypes.data_as(C.c_void_p), out_len), "wk_augment")
    return out


def augment_variants(x: np.ndarray, noise_level: float = 0.005, seed: int = 0) -> List[np.ndarray]:
    """The reference's five variants: original, speed 0.8 / 1.2 (padded to
    16000), volume 0.7 / 1.3 (clamped)."""
    x = np.asarray(x, np.float32).reshape(-1)
    outs = [x.copy()]
    outs += [augment(x, speed=s, noise_level=noise_level, seed=seed + i, out_len=16000) for i, s in enumerate((0.8, 1.2))]
    outs += [augment(x, volume=v, out_len=x.size) for v in (0.7, 1.3)]
    return outs
