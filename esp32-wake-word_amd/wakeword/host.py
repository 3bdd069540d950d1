"""ctypes binding of libwakeword_host.so (include/wakeword_host.h): the same
wake-word path on the host CPU, for BASELINE config 1 ("single WAV on CPU")
and for callers without a GPU.

This is a separate library the caller asks for -- ``wakeword.host`` /
``python -m wakeword.test --cpu`` -- never a fallback: the GPU package
(``wakeword.lib()``, ``KWSModel``) does not call it, and it does not touch HIP.

    from wakeword import host
    model = host.load_onnx("xiaoa.onnx")          # LightweightKWS on the host
    logits = model.detect(audio)                  # (B, 16000) -> (B,)
    feats = host.mfcc(audio)                      # (B, 13, 63), CMVN'd
    mf = host.extract_mfcc(signal, len(signal))   # mfcc.h on the host, mode A

Reference interfaces: ml_models/src/wakeModel.py:29-34 (forward),
ml_models/src/extract_mfcc.py:137-175 + :47-88 (mode B + CMVN),
main/esp_mfcc/mfcc.c:431-527 (extract_mfcc), :297-427 (single frame).
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from typing import Dict, Optional, Sequence

import numpy as np

from .onnx_reader import read_onnx, xiaoa_state_dict

_PKG = os.path.dirname(os.path.abspath(__file__))
HOST_LIB_PATH = os.environ.get("WAKEWORD_HOST_LIB", os.path.join(_PKG, "libwakeword_host.so"))
STATE_KEYS = ("conv_layers.0.weight", "conv_layers.3.weight", "conv_layers.6.weight", "classifier.0.weight",
              "classifier.2.weight")
WK_NUM_WEIGHTS = 40224

# Every symbol include/wakeword_host.h declares (tests/test_host.py checks the export table).
EXPORTS = ("wkh_create", "wkh_destroy", "wkh_mfcc", "wkh_cnn", "wkh_forward", "wkh_esp_mfcc", "wkh_set_threads",
           "wkh_last_error")
MFCC_H = ("extract_mfcc", "free_mfcc", "analyze_mfcc_range", "flow_extract_mfcc_single_frame")
WAV = ("wk_wav_read", "wk_wav_load_batch", "wk_augment")   # wk_wav.cpp, the same host loader libwakeword.so carries


class HostError(RuntimeError):
    pass


_lock = threading.Lock()
_lib = None
_fp = C.POINTER(C.c_float)


def lib():
    """Load libwakeword_host.so once (RTLD_LOCAL: its mfcc.h symbols never
    shadow libwakeword.so's)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(HOST_LIB_PATH):
                try:   # built on demand (wakeword.build.build() does not fail on it)
                    from .build import build_host
                    build_host()
                except (RuntimeError, OSError) as e:
                    raise HostError(f"{HOST_LIB_PATH} not found and could not be built: {e}") from e
            L = C.CDLL(HOST_LIB_PATH, mode=C.RTLD_LOCAL)
            vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
            L.wkh_create.argtypes = [_fp, C.POINTER(vp)]
            L.wkh_destroy.argtypes = [vp]
            L.wkh_mfcc.argtypes = [_fp, i64, i32, i64, i32, _fp]
            L.wkh_cnn.argtypes = [vp, _fp, i64, _fp]
            L.wkh_forward.argtypes = [vp, _fp, i64, i32, i64, _fp, _fp]
            L.wkh_esp_mfcc.argtypes = [_fp, i64, i32, i64, i32, i32, i32, i32, i32, i32, i32, C.c_float, _fp]
            L.wkh_set_threads.argtypes = [i32]
            L.wkh_set_threads.restype = i32
            L.wkh_last_error.restype = C.c_char_p
            for name in ("wkh_create", "wkh_destroy", "wkh_mfcc", "wkh_cnn", "wkh_forward", "wkh_esp_mfcc"):
                getattr(L, name).restype = i32
            L.extract_mfcc.argtypes = [_fp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
            L.extract_mfcc.restype = _fp
            L.flow_extract_mfcc_single_frame.argtypes = [_fp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
            L.flow_extract_mfcc_single_frame.restype = _fp
            L.free_mfcc.argtypes = [_fp]
            L.analyze_mfcc_range.argtypes = [_fp, C.c_int, C.c_char_p]
            L.wk_wav_load_batch.argtypes = [C.POINTER(C.c_char_p), i32, i32, C.c_float, C.c_uint32, vp, vp]
            L.wk_wav_load_batch.restype = i32
            _lib = L
    return _lib


def check(status: int, what: str) -> None:
    if status != 0:
        raise HostError(f"{what}: status {status} ({lib().wkh_last_error().decode()})")


def set_threads(n: int) -> int:
    """Host threads for batch calls (0 = hardware concurrency); returns the value in effect."""
    return int(lib().wkh_set_threads(int(n)))


def _f32(x, ndim: int) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    if a.ndim == ndim - 1:
        a = a[None]
    if a.ndim != ndim:
        raise ValueError(f"expected {ndim - 1}-d or {ndim}-d input, got shape {a.shape}")
    return a


def load_batch(paths: Sequence[str], pad_to: int = 16000, noise_level: float = 0.005, seed: int = 0):
    """WAV files -> ((len(paths), pad_to) float32, samples read per file): the
    same native loader as wakeword.wav.load_batch (esp_wav.cpp header walk,
    x / 32768, pad_audio with the loader's seeded N(0, noise_level^2) pad)."""
    n = len(paths)
    out = np.zeros((n, pad_to), np.float32)
    if n == 0:
        return out, []
    arr = (C.c_char_p * n)(*[p.encode() for p in paths])
    n_read = np.zeros(n, np.int32)
    check(lib().wk_wav_load_batch(arr, n, pad_to, noise_level, seed & 0xFFFFFFFF, out.ctypes.data_as(C.c_void_p),
                                  n_read.ctypes.data_as(C.c_void_p)), "wk_wav_load_batch")
    return out, n_read.tolist()


def mfcc(wave_batch, cmvn: bool = True) -> np.ndarray:
    """Mode B (torchaudio MFCC + normalize_mfcc('cmvn')): (B, 16000) -> (B, 13, 63)."""
    x = _f32(wave_batch, 2)
    out = np.empty((x.shape[0], 13, 63), np.float32)
    check(lib().wkh_mfcc(x.ctypes.data_as(_fp), x.shape[0], x.shape[1], x.shape[1], int(bool(cmvn)),
                         out.ctypes.data_as(_fp)), "wkh_mfcc")
    return out


def esp_mfcc(signals, sampling_rate: int = 16000, frame_size: int = 320, hop_size: int = 256, n_fft: int = 512,
             n_filters: int = 40, n_mfcc: int = 13, esp_dsp_packing: bool = True,
             pre_emphasis: float = 0.97) -> np.ndarray:
    """Mode A (mfcc.c) at any parameter set: (B, L) -> (B, n_frames, n_mfcc)."""
    x = _f32(signals, 2)
    nf = (x.shape[1] - frame_size) // hop_size + 1 if hop_size >= 1 and x.shape[1] >= frame_size else 0
    out = np.empty((x.shape[0], max(nf, 0), n_mfcc), np.float32)
    check(lib().wkh_esp_mfcc(x.ctypes.data_as(_fp), x.shape[0], x.shape[1], x.shape[1], sampling_rate, frame_size,
                             hop_size, n_fft, n_filters, n_mfcc, int(bool(esp_dsp_packing)), float(pre_emphasis),
                             out.ctypes.data_as(_fp)), "wkh_esp_mfcc")
    return out


def extract_mfcc(signal, signal_len: Optional[int] = None, sampling_rate: int = 16000, frame_size: int = 320,
                 hop_size: int = 256, n_fft: int = 512, n_filters: int = 40, n_mfcc: int = 13):
    """mfcc.h's extract_mfcc on the host (malloc'd block copied out, then
    free_mfcc): (n_frames, n_mfcc) float32, or None where the reference
    returns NULL."""
    x = np.ascontiguousarray(np.asarray(signal, np.float32))
    if x.ndim != 1:
        raise ValueError(f"signal must be 1-D, got shape {x.shape}")
    n = int(x.shape[0] if signal_len is None else signal_len)
    if n > x.shape[0]:   # the C side would read past the array
        raise ValueError(f"signal_len {n} exceeds the signal's {x.shape[0]} samples")
    L = lib()
    p = L.extract_mfcc(x.ctypes.data_as(_fp), n, sampling_rate, frame_size, hop_size, n_fft, n_filters, n_mfcc)
    if not p:
        return None
    nf = (n - frame_size) // hop_size + 1
    out = np.ctypeslib.as_array(p, shape=(nf, n_mfcc)).copy()
    L.free_mfcc(p)
    return out


class HostKWS:
    """LightweightKWS (wakeModel.py:4-34) on the host: forward((B,13,63)) ->
    (B,1), detect(audio (B,16000)) -> (B,) logits, ONNX-style run()."""

    def __init__(self, state_dict: Dict[str, np.ndarray]):
        self._sd = {k: np.asarray(state_dict[k], np.float32) for k in STATE_KEYS}
        blob = np.ascontiguousarray(np.concatenate([self._sd[k].reshape(-1) for k in STATE_KEYS]), np.float32)
        if blob.size != WK_NUM_WEIGHTS:
            raise ValueError(f"weight blob has {blob.size} floats, expected {WK_NUM_WEIGHTS}")
        h = C.c_void_p()
        check(lib().wkh_create(blob.ctypes.data_as(_fp), C.byref(h)), "wkh_create")
        self._h = h

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                lib().wkh_destroy(self._h)
                self._h = None
        except Exception:
            pass

    def state_dict(self) -> Dict[str, np.ndarray]:
        return dict(self._sd)

    def eval(self):
        return self

    def __call__(self, x):
        return self.forward(x)

    def forward(self, x) -> np.ndarray:
        f = _f32(x, 3)
        if f.shape[1:] != (13, 63):
            raise ValueError(f"expected (B, 13, 63) features, got {f.shape}")
        out = np.empty((f.shape[0],), np.float32)
        check(lib().wkh_cnn(self._h, f.ctypes.data_as(_fp), f.shape[0], out.ctypes.data_as(_fp)), "wkh_cnn")
        return out[:, None]

    def run(self, output_names: Optional[Sequence[str]], input_feed: Dict[str, object]):
        """onnxruntime-style: {"input.1": (B,13,63)} -> [(B,1)] (output "22")."""
        return [self.forward(input_feed["input.1"])]

    def detect(self, audio, return_features: bool = False):
        x = _f32(audio, 2)
        logits = np.empty((x.shape[0],), np.float32)
        feats = np.empty((x.shape[0], 13, 63), np.float32) if return_features else None
        check(lib().wkh_forward(self._h, x.ctypes.data_as(_fp), x.shape[0], x.shape[1], x.shape[1],
                                logits.ctypes.data_as(_fp), feats.ctypes.data_as(_fp) if feats is not None else None),
              "wkh_forward")
        return (logits, feats) if return_features else logits

    def probability(self, audio) -> np.ndarray:
        return 1.0 / (1.0 + np.exp(-self.detect(audio).astype(np.float64)))


def load_onnx(path: str) -> HostKWS:
    """xiaoa.onnx -> HostKWS (the ONNX reader of the GPU package; no onnxruntime)."""
    inits, _, _ = read_onnx(path)
    return HostKWS(xiaoa_state_dict(inits))
