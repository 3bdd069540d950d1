"""ctypes binding of libwakeword.so (the C ABI declared in include/wakeword.h).

The library is the product: every compute entry point below runs a HIP kernel.
There is no CPU fallback -- if the library is missing, ``lib()`` raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("WAKEWORD_LIB", os.path.join(_PKG, "libwakeword.so"))

WK_OK = 0
WK_MODE_TORCHAUDIO_CMVN = 0
WK_MODE_ESP_MFCC = 1
WK_DTYPE_F32 = 0
WK_DTYPE_I16 = 1
WK_DTYPE_I8 = 2
WK_PREC_FP32 = 0
WK_PREC_BF16 = 1
WK_PREC_INT8 = 2
WK_PREC_BF16X3 = 3
WK_NUM_WEIGHTS = 40224

# Every symbol include/wakeword.h declares (checked by tests/test_abi.py).
EXPORTS = ("wk_create", "wk_destroy", "wk_mfcc", "wk_cnn", "wk_forward", "wk_synth_clips", "wk_normalize",
           "wk_status_string", "wk_last_error", "wk_abi_version", "extract_mfcc", "free_mfcc",
           "analyze_mfcc_range", "wk_stream_create", "wk_stream_destroy", "wk_stream_reset", "wk_stream_push",
           "wk_ctc_num_weights", "wk_ctc_create", "wk_ctc_destroy", "wk_ctc_features", "wk_ctc_forward",
           "wk_wav_read", "wk_wav_load_batch", "wk_augment", "flow_extract_mfcc_single_frame", "wk_device_cmvn",
           "wk_check_device_errors", "wk_ctc_frame_argmax", "wk_record_front", "wk_quantize_frames",
           "wk_ctc_profile", "wk_ctc_stage_times", "wk_ctc_transcribe", "wk_esp_mfcc_create", "wk_esp_mfcc_run",
           "wk_esp_mfcc_destroy")


class WkConfig(C.Structure):
    _fields_ = [("mode", C.c_int32), ("precision", C.c_int32), ("esp_dsp_packing", C.c_int32),
                ("device", C.c_int32), ("cmvn", C.c_int32)]


class WkCtcConfig(C.Structure):
    _fields_ = [("vocab", C.c_int32), ("hidden", C.c_int32), ("layers", C.c_int32), ("n_mels", C.c_int32),
                ("device", C.c_int32), ("precision", C.c_int32)]


class WkWavInfo(C.Structure):
    _fields_ = [("sample_rate", C.c_int32), ("channels", C.c_int32), ("bits_per_sample", C.c_int32),
                ("data_samples", C.c_int32), ("n_samples", C.c_int32)]


class WakewordError(RuntimeError):
    pass


_lock = threading.Lock()
_lib = None


def _declare(L):
    vp, i32, i64, u32, fp = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.POINTER(C.c_float)
    L.wk_create.argtypes = [C.POINTER(WkConfig), vp, C.POINTER(vp)]
    L.wk_destroy.argtypes = [vp]
    L.wk_mfcc.argtypes = [vp, vp, i32, i64, i32, i64, vp, vp]
    L.wk_cnn.argtypes = [vp, vp, i64, vp, vp]
    L.wk_forward.argtypes = [vp, vp, i32, i64, i32, i64, vp, vp, vp]
    L.wk_synth_clips.argtypes = [u32, i64, i64, i32, vp, vp]
    L.wk_normalize.argtypes = [vp, vp, i64, i32, i32, i32, vp]
    L.wk_status_string.argtypes = [i32]
    L.wk_status_string.restype = C.c_char_p
    L.wk_last_error.restype = C.c_char_p
    L.wk_abi_version.restype = i32
    L.extract_mfcc.argtypes = [fp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    L.extract_mfcc.restype = fp
    L.free_mfcc.argtypes = [fp]
    L.analyze_mfcc_range.argtypes = [fp, C.c_int, C.c_char_p]
    L.flow_extract_mfcc_single_frame.argtypes = [fp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    L.flow_extract_mfcc_single_frame.restype = fp
    L.wk_stream_create.argtypes = [vp, i32, i32, vp, C.POINTER(vp)]
    L.wk_stream_destroy.argtypes = [vp]
    L.wk_stream_reset.argtypes = [vp]
    L.wk_stream_push.argtypes = [vp, fp, i64, fp, C.POINTER(i64), i32, C.POINTER(i32)]
    L.wk_ctc_num_weights.argtypes = [C.POINTER(WkCtcConfig)]
    L.wk_ctc_num_weights.restype = i64
    L.wk_ctc_create.argtypes = [C.POINTER(WkCtcConfig), vp, C.POINTER(vp)]
    L.wk_ctc_destroy.argtypes = [vp]
    L.wk_ctc_features.argtypes = [vp, vp, i64, i32, i32, i64, vp, vp]
    L.wk_ctc_forward.argtypes = [vp, vp, i64, i32, vp, vp, vp, vp]
    L.wk_ctc_transcribe.argtypes = [vp, vp, i64, i32, i32, i64, vp, vp, vp]
    L.wk_ctc_frame_argmax.argtypes = [vp, i64, i32, vp, vp]
    L.wk_record_front.argtypes = [vp, i64, vp, vp, vp]
    L.wk_quantize_frames.argtypes = [vp, i64, vp, vp]
    L.wk_ctc_profile.argtypes = [vp, i32]
    L.wk_ctc_stage_times.argtypes = [vp, vp, vp]
    L.wk_wav_read.argtypes = [C.c_char_p, vp, i32, C.POINTER(WkWavInfo)]
    L.wk_wav_load_batch.argtypes = [C.POINTER(C.c_char_p), i32, i32, C.c_float, u32, vp, vp]
    L.wk_augment.argtypes = [vp, i32, C.c_float, C.c_float, C.c_float, u32, vp, i32]
    L.wk_device_cmvn.argtypes = [vp, i32, i64, vp, vp, vp]
    L.wk_check_device_errors.argtypes = [vp, C.POINTER(u32)]
    if hasattr(L, "wk_esp_mfcc_create"):   # (absent from pre-round-4 libraries loaded for A/B timing)
        L.wk_esp_mfcc_create.argtypes = [i32, i32, i32, i32, i32, i32, i32, C.POINTER(vp)]
        L.wk_esp_mfcc_run.argtypes = [vp, vp, i64, i32, i64, i32, C.c_float, vp, vp]
        L.wk_esp_mfcc_destroy.argtypes = [vp]
    for name in ("wk_create", "wk_destroy", "wk_mfcc", "wk_cnn", "wk_forward", "wk_synth_clips", "wk_normalize",
                 "wk_stream_create", "wk_stream_destroy", "wk_stream_reset", "wk_stream_push", "wk_ctc_create",
                 "wk_ctc_destroy", "wk_ctc_features", "wk_ctc_forward", "wk_wav_read", "wk_wav_load_batch",
                 "wk_augment", "wk_device_cmvn", "wk_ctc_frame_argmax", "wk_record_front",
                 "wk_quantize_frames", "wk_ctc_profile", "wk_ctc_stage_times", "wk_ctc_transcribe",
                 "wk_esp_mfcc_create", "wk_esp_mfcc_run", "wk_esp_mfcc_destroy"):
        if hasattr(L, name):
            getattr(L, name).restype = i32


def lib():
    """Load libwakeword.so once (after torch, so both share one HIP runtime)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise WakewordError(
                    f"{LIB_PATH} not found: build it with `python -m wakeword.build` (no CPU fallback exists)")
            try:
                import torch  # noqa: F401  (load torch's libamdhip64 first)
            except ImportError:
                pass
            L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
            _declare(L)
            _lib = L
    return _lib


def check(status: int, what: str = "") -> None:
    if status != WK_OK:
        L = lib()
        raise WakewordError(f"{what}: {L.wk_status_string(status).decode()} ({L.wk_last_error().decode()})")
