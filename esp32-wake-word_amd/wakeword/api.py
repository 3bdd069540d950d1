"""Python host side of the wake-word path -- mirrors the reference's call surface.

Reference surface kept (paths relative to the reference root):
  * ``LightweightKWS(num_classes=1)`` state-dict keys + ``forward(x (B,13,63)) -> (B,1)``
    (ml_models/src/wakeModel.py:4-34)          -> ``KWSModel`` / ``load_onnx``
  * ONNX I/O names ``input.1`` -> ``22`` (ml_models/xiaoa.onnx) -> ``KWSModel.run``
  * ``pad_audio`` / ``normalize_mfcc`` / MFCC front-end (ml_models/src/extract_mfcc.py)
  * sigmoid + threshold of the callers (ml_models/main.py:53,
    esp_wake_word_detector.cpp:227-245)         -> ``probability`` / ``detect``

All compute goes through libwakeword.so (HIP kernels).  Torch is used only as
the device-memory / stream container; numpy inputs are uploaded to device.
"""
from __future__ import annotations

import ctypes as C
import wave
from typing import Dict, Iterable, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import check, lib
from .onnx_reader import read_onnx, xiaoa_state_dict

_MODES = {"torchaudio": _lib.WK_MODE_TORCHAUDIO_CMVN, "torchaudio_cmvn": _lib.WK_MODE_TORCHAUDIO_CMVN,
          "b": _lib.WK_MODE_TORCHAUDIO_CMVN, "esp": _lib.WK_MODE_ESP_MFCC, "esp_mfcc": _lib.WK_MODE_ESP_MFCC,
          "a": _lib.WK_MODE_ESP_MFCC}
_NORM = {"standardization": 0, "minmax": 1, "cmvn": 2}
STATE_KEYS = ("conv_layers.0.weight", "conv_layers.3.weight", "conv_layers.6.weight",
              "classifier.0.weight", "classifier.2.weight")


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise _lib.WakewordError("no HIP device visible: the wake-word path runs on MI355X only")
    return torch


def _stream(torch, device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _as_device(x, dtype, device):
    """numpy / torch (any device) -> contiguous torch tensor of `dtype` on `device`."""
    torch = _torch()
    if isinstance(x, np.ndarray):
        x = torch.from_numpy(np.ascontiguousarray(x))
    x = x.to(device=device, dtype=dtype)
    return x.contiguous()


def pack_weights(sd: Dict[str, np.ndarray]) -> np.ndarray:
    """Concatenate the state dict in the WK_NUM_WEIGHTS order of wakeword.h."""
    blob = np.concatenate([np.ascontiguousarray(sd[k], np.float32).reshape(-1) for k in STATE_KEYS])
    if blob.size != _lib.WK_NUM_WEIGHTS:
        raise ValueError(f"weight blob has {blob.size} floats, expected {_lib.WK_NUM_WEIGHTS}")
    return blob


class _Handle:
    def __init__(self, mode: int, weights: Optional[np.ndarray], device: int, precision: int = 0,
                 esp_dsp_packing: int = 1, cmvn: int = 1):
        L = lib()
        cfg = _lib.WkConfig(mode, precision, esp_dsp_packing, device, cmvn)
        h = C.c_void_p()
        wptr = weights.ctypes.data_as(C.c_void_p) if weights is not None else None
        check(L.wk_create(C.byref(cfg), wptr, C.byref(h)), "wk_create")
        self.h = h
        self.device = device
        self.mode = mode

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().wk_destroy(self.h)
                self.h = None
        except Exception:
            pass


_fe_handles: Dict[tuple, _Handle] = {}


def _frontend_handle(mode: int, device: int, esp_dsp_packing: int, cmvn: int) -> _Handle:
    key = (mode, device, esp_dsp_packing, cmvn)
    if key not in _fe_handles:
        _fe_handles[key] = _Handle(mode, None, device, 0, esp_dsp_packing, cmvn)
    return _fe_handles[key]


def mfcc(wave_batch, mode: str = "torchaudio", cmvn: bool = True, esp_dsp_packing: bool = True, device: int = 0):
    """MFCC front-end on device.

    mode 'torchaudio' (B): (B, 16000) -> (B, 13, 63), CMVN'd when cmvn=True
      (extract_mfcc.py:171-175).
    mode 'esp' (A): (B, L) -> (B, (L-320)//256+1, 13) (mfcc.c:431-527).
    Input float32 (or int16, scaled by 1/32768) numpy or torch; returns a torch
    tensor on cuda:<device>."""
    torch = _torch()
    m = _MODES[mode]
    x = wave_batch
    is_i16 = (isinstance(x, np.ndarray) and x.dtype == np.int16) or (hasattr(x, "dtype") and str(x.dtype) == "torch.int16")
    x = _as_device(x, torch.int16 if is_i16 else torch.float32, f"cuda:{device}")
    if x.dim() == 1:
        x = x.unsqueeze(0)
    B, L = x.shape
    if m == _lib.WK_MODE_TORCHAUDIO_CMVN:
        out = torch.empty((B, 13, 63), dtype=torch.float32, device=x.device)
    else:
        out = torch.empty((B, (L - 320) // 256 + 1, 13), dtype=torch.float32, device=x.device)
    h = _frontend_handle(m, device, int(esp_dsp_packing), int(cmvn))
    check(lib().wk_mfcc(h.h, C.c_void_p(x.data_ptr()), _lib.WK_DTYPE_I16 if is_i16 else _lib.WK_DTYPE_F32, B, L, L,
                        C.c_void_p(out.data_ptr()), _stream(torch, x.device)), "wk_mfcc")
    return out


def normalize_mfcc(m, method: str = "standardization", device: int = 0):
    """normalize_mfcc(mfcc (n_mfcc, T) or (B, n_mfcc, T), method) on device
    (extract_mfcc.py:47-88; unknown methods pass through unchanged)."""
    torch = _torch()
    x = _as_device(m, torch.float32, f"cuda:{device}")
    squeeze = x.dim() == 2
    if squeeze:
        x = x.unsqueeze(0)
    out = torch.empty_like(x)
    code = _NORM.get(method, 3)
    check(lib().wk_normalize(C.c_void_p(x.data_ptr()), C.c_void_p(out.data_ptr()), x.shape[0], x.shape[1],
                             x.shape[2], code, _stream(torch, x.device)), "wk_normalize")
    return out[0] if squeeze else out


def pad_audio(audio, target_length: int = 16000, add_noise_to_pad: bool = True, noise_level: float = 0.005,
              generator=None):
    """extract_mfcc.py:7-23 (host-side data preparation, outside the kernel):
    trim to target_length or right-pad with N(0, noise_level^2) noise / zeros."""
    import torch
    a = torch.as_tensor(audio, dtype=torch.float32)
    if a.dim() == 1:
        a = a.unsqueeze(0)
    n = a.shape[1]
    if n < target_length:
        pad = target_length - n
        if add_noise_to_pad:
            noise = torch.randn(a.shape[0], pad, generator=generator) * noise_level
            a = torch.cat([a, noise], dim=1)
        else:
            a = torch.nn.functional.pad(a, (0, pad))
    elif n > target_length:
        a = a[:, :target_length]
    return a


def load_wav(path: str) -> np.ndarray:
    """16-bit PCM mono WAV -> float32 in [-1, 1) (torchaudio.load scaling)."""
    with wave.open(path) as w:
        if w.getsampwidth() != 2:
            raise ValueError(f"{path}: only 16-bit PCM is supported")
        raw = np.frombuffer(w.readframes(w.getnframes()), "<i2")
        ch = w.getnchannels()
    if ch > 1:
        raw = raw.reshape(-1, ch)[:, 0]
    return raw.astype(np.float32) / 32768.0


class KWSModel:
    """LightweightKWS(num_classes=1) on MI355X (wakeModel.py:4-34)."""

    input_names = ("input.1",)
    output_names = ("22",)

    def __init__(self, state_dict: Dict[str, np.ndarray], device: int = 0, precision: str = "fp32"):
        self._sd = {k: np.ascontiguousarray(state_dict[k], np.float32) for k in STATE_KEYS}
        self.device = device
        self.precision = precision
        self._h = _Handle(_lib.WK_MODE_TORCHAUDIO_CMVN, pack_weights(self._sd), device,
                          {"fp32": _lib.WK_PREC_FP32, "bf16": _lib.WK_PREC_BF16, "int8": _lib.WK_PREC_INT8,
                           "bf16x3": _lib.WK_PREC_BF16X3}[precision])

    # -- nn.Module-like surface ------------------------------------------------
    def state_dict(self) -> Dict[str, np.ndarray]:
        return {k: v.copy() for k, v in self._sd.items()}

    def eval(self):
        return self

    def __call__(self, x):
        return self.forward(x)

    def forward(self, x):
        """x (B, 13, 63) CMVN'd MFCC -> logits (B, 1), torch on cuda."""
        torch = _torch()
        x = _as_device(x, torch.float32, f"cuda:{self.device}")
        if x.dim() != 3 or tuple(x.shape[1:]) != (13, 63):
            raise ValueError(f"expected (B, 13, 63) features, got {tuple(x.shape)}")
        out = torch.empty((x.shape[0],), dtype=torch.float32, device=x.device)
        check(lib().wk_cnn(self._h.h, C.c_void_p(x.data_ptr()), x.shape[0], C.c_void_p(out.data_ptr()),
                           _stream(torch, x.device)), "wk_cnn")
        return out.unsqueeze(1)

    # -- ONNX-runtime-like surface --------------------------------------------
    def run(self, output_names: Optional[Sequence[str]], input_feed: Dict[str, object]):
        x = input_feed[self.input_names[0]]
        y = self.forward(x).cpu().numpy()
        return [y]

    # -- end to end ------------------------------------------------------------
    def detect(self, audio, return_features: bool = False):
        """audio (B, 16000) float32/int16 -> logits (B,) (features too if asked):
        preemphasis -> MFCC -> CMVN -> CNN, all on device."""
        torch = _torch()
        is_i16 = (isinstance(audio, np.ndarray) and audio.dtype == np.int16) or \
            (hasattr(audio, "dtype") and str(audio.dtype) == "torch.int16")
        x = _as_device(audio, torch.int16 if is_i16 else torch.float32, f"cuda:{self.device}")
        if x.dim() == 1:
            x = x.unsqueeze(0)
        B, L = x.shape
        out = torch.empty((B,), dtype=torch.float32, device=x.device)
        feats = torch.empty((B, 13, 63), dtype=torch.float32, device=x.device) if return_features else None
        check(lib().wk_forward(self._h.h, C.c_void_p(x.data_ptr()), _lib.WK_DTYPE_I16 if is_i16 else _lib.WK_DTYPE_F32,
                               B, L, L, C.c_void_p(out.data_ptr()),
                               C.c_void_p(feats.data_ptr()) if feats is not None else None,
                               _stream(torch, x.device)), "wk_forward")
        return (out, feats) if return_features else out

    def probability(self, audio):
        return _torch().sigmoid(self.detect(audio))

    def check_device_errors(self) -> None:
        """Synchronise the device and raise WakewordError if a fused launch on
        this model since the last check reported a role hand-off failure (its
        logits are then invalid; wk_check_device_errors in include/wakeword.h)."""
        flags = C.c_uint32(0)
        check(lib().wk_check_device_errors(self._h.h, C.byref(flags)), "wk_check_device_errors")


def load_onnx(path: str, device: int = 0, precision: str = "fp32") -> KWSModel:
    """Load ``xiaoa.onnx`` (ml_models/xiaoa.onnx) into a device-resident KWSModel."""
    inits, inputs, outputs = read_onnx(path)
    m = KWSModel(xiaoa_state_dict(inits), device=device, precision=precision)
    if inputs:
        m.input_names = tuple(inputs)
    if outputs:
        m.output_names = tuple(outputs)
    return m


def synth_clips(seed: int, first: int, count: int, n: int = 16000, device: int = 0):
    """Device generator of SURVEY 8(d) synthetic clips -> torch (count, n) on cuda."""
    torch = _torch()
    out = torch.empty((count, n), dtype=torch.float32, device=f"cuda:{device}")
    check(lib().wk_synth_clips(seed & 0xFFFFFFFF, first, count, n, C.c_void_p(out.data_ptr()),
                               _stream(torch, out.device)), "wk_synth_clips")
    return out


def extract_mfcc(signal: Iterable[float], signal_len: Optional[int] = None, sampling_rate: int = 16000,
                 frame_size: int = 320, hop_size: int = 256, n_fft: int = 512, n_filters: int = 40,
                 n_mfcc: int = 13) -> Optional[np.ndarray]:
    """The mfcc.h C entry point (through the C ABI): returns (n_frames, n_mfcc) or None."""
    sig = np.ascontiguousarray(signal, np.float32)
    n = int(signal_len if signal_len is not None else sig.size)
    L = lib()
    p = L.extract_mfcc(sig.ctypes.data_as(C.POINTER(C.c_float)), n, sampling_rate, frame_size, hop_size, n_fft,
                       n_filters, n_mfcc)
    if not p:
        return None
    nf = (n - frame_size) // hop_size + 1
    out = np.ctypeslib.as_array(p, shape=(nf * n_mfcc,)).copy().reshape(nf, n_mfcc)
    L.free_mfcc(p)
    return out


class EspMfcc:
    """mfcc.c's mode-A MFCC at any parameter set, batched on the GPU
    (wk_esp_mfcc: tables built once per object with the reference's formulas,
    main/esp_mfcc/mfcc.c:144-234,298-527).  ``m(signals, hop_size)`` maps a
    (B, L) float batch to (B, (L - frame_size) // hop_size + 1, n_mfcc) on
    device; pre_emphasis 0.97 is extract_mfcc's, 0 the single-frame variant's."""

    def __init__(self, sampling_rate: int = 16000, frame_size: int = 320, n_fft: int = 512, n_filters: int = 40,
                 n_mfcc: int = 13, esp_dsp_packing: bool = True, device: int = 0):
        self.frame_size, self.n_mfcc, self.device = frame_size, n_mfcc, device
        self._m = C.c_void_p()
        check(lib().wk_esp_mfcc_create(sampling_rate, frame_size, n_fft, n_filters, n_mfcc, int(esp_dsp_packing),
                                       device, C.byref(self._m)), "wk_esp_mfcc_create")

    def __call__(self, signals, hop_size: int, pre_emphasis: float = 0.97):
        torch = _torch()
        x = _as_device(signals, torch.float32, self.device)
        if x.dim() == 1:
            x = x.unsqueeze(0)
        B, L = x.shape
        nf = (L - self.frame_size) // hop_size + 1 if L >= self.frame_size and hop_size > 0 else 0
        out = torch.empty((B, max(nf, 0), self.n_mfcc), dtype=torch.float32, device=x.device)
        check(lib().wk_esp_mfcc_run(self._m, C.c_void_p(x.data_ptr()), B, L, L, hop_size, pre_emphasis,
                                    C.c_void_p(out.data_ptr()), _stream(torch, self.device)), "wk_esp_mfcc_run")
        return out

    def __del__(self):
        m = getattr(self, "_m", None)
        if m and m.value:
            lib().wk_esp_mfcc_destroy(m)
            self._m = C.c_void_p()


_DEFAULT_MODELS: Dict[tuple, "KWSModel"] = {}


def detect(wave_batch, onnx: Optional[str] = None, device: int = 0, precision: str = "fp32"):
    """(B, 16000) float32/int16 audio -> logits (B,) on device, with a cached
    model per (onnx, device, precision); onnx defaults to $WAKEWORD_ONNX or the
    xiaoa.onnx kept with the test fixtures (wakeword.test.default_onnx)."""
    from .test import default_onnx
    key = (onnx or default_onnx(), device, precision)
    if key not in _DEFAULT_MODELS:
        _DEFAULT_MODELS[key] = load_onnx(key[0], device=device, precision=precision)
    return _DEFAULT_MODELS[key].detect(wave_batch)
