"""Build / load the C oracle (TEST INFRASTRUCTURE ONLY: tests/, smoke(), bench
cpu_baseline).  gcc -O2 -shared oracle/esp_mfcc_oracle.c -> oracle/_build/."""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "esp_mfcc_oracle.c")
OUT = os.path.join(HERE, "_build", "libesp_mfcc_oracle.so")


def build(force: bool = False) -> str:
    if force or not os.path.exists(OUT) or os.path.getmtime(OUT) < os.path.getmtime(SRC):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        subprocess.check_call(["gcc", "-O2", "-std=gnu99", "-fPIC", "-shared", "-pthread", SRC, "-o", OUT, "-lm"])
    return OUT


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
        fp = C.POINTER(C.c_float)
        _lib.esp_mfcc_oracle.argtypes = [fp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.c_int, fp]
        _lib.esp_mfcc_oracle.restype = C.c_int
        _lib.esp_mfcc_oracle_ex.argtypes = [fp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                            C.c_int, C.c_float, fp]
        _lib.esp_mfcc_oracle_ex.restype = C.c_int
        _lib.esp_mfcc_oracle_fbank.argtypes = [C.c_int, C.c_int, C.c_int, fp]
        _lib.esp_mfcc_oracle_fbank.restype = C.c_int
        _lib.esp_mfcc_oracle_batch.argtypes = [fp, C.c_longlong, C.c_int, C.c_longlong, C.c_int, C.c_int, C.c_int,
                                               C.c_int, C.c_int, C.c_int, C.c_int, C.c_float, C.c_int, fp]
        _lib.esp_mfcc_oracle_batch.restype = C.c_int
    return _lib


def esp_mfcc(x, esp_pack: bool = True, sr: int = 16000, frame: int = 320, hop: int = 256, n_fft: int = 512,
             n_filters: int = 40, n_mfcc: int = 13, pre: float = 0.97) -> np.ndarray:
    """Mode-A MFCC of one signal -> (n_frames, n_mfcc) float32."""
    x = np.ascontiguousarray(x, np.float32)
    nf = (x.shape[0] - frame) // hop + 1
    out = np.zeros((max(nf, 1), n_mfcc), np.float32)
    fp = C.POINTER(C.c_float)
    rc = lib().esp_mfcc_oracle_ex(x.ctypes.data_as(fp), x.shape[0], sr, frame, hop, n_fft, n_filters, n_mfcc,
                                  int(esp_pack), pre, out.ctypes.data_as(fp))
    if rc < 0:
        raise ValueError("esp_mfcc_oracle rejected the arguments")
    return out[:rc]


def esp_mfcc_batch(x, esp_pack: bool = True, n_threads: int = 1, sr: int = 16000, frame: int = 320, hop: int = 256,
                   n_fft: int = 512, n_filters: int = 40, n_mfcc: int = 13, pre: float = 0.97) -> np.ndarray:
    """Mode-A MFCC of (B, L) signals through the FFT path on n_threads host
    threads -> (B, n_frames, n_mfcc) float32 (the timed CPU baseline)."""
    x = np.ascontiguousarray(x, np.float32)
    B, L = x.shape
    nf = (L - frame) // hop + 1
    out = np.zeros((B, nf, n_mfcc), np.float32)
    fp = C.POINTER(C.c_float)
    rc = lib().esp_mfcc_oracle_batch(x.ctypes.data_as(fp), B, L, L, sr, frame, hop, n_fft, n_filters, n_mfcc,
                                     int(esp_pack), pre, n_threads, out.ctypes.data_as(fp))
    if rc < 0:
        raise ValueError("esp_mfcc_oracle_batch rejected the arguments")
    return out


def fbank(sr: int = 16000, n_filters: int = 40, n_fft: int = 512) -> np.ndarray:
    fb = np.zeros((n_filters, n_fft // 2 + 1), np.float32)
    lib().esp_mfcc_oracle_fbank(sr, n_filters, n_fft, fb.ctypes.data_as(C.POINTER(C.c_float)))
    return fb
