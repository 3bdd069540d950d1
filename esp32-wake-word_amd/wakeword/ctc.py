"""GRU-CTC head: the reference's ml_models/ctc.py
inference surface on the HIP path (wk_ctc_* in the C ABI).

    model = wakeword.CTCModel(state_dict_or_flat_weights, vocab=V)
    feats = model.features(audio, n_samples=48000)      # ctc.py:82-107, (B, T, 80)
    tokens, log_probs = model.forward(feats, return_log_probs=True)   # ctc.py:148-152 + 453-471
    tokens = model.transcribe(audio)                     # both
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Union

import numpy as np

from . import _lib
from ._lib import check, lib

MAX_AUDIO_SAMPLES = 8 * 16000   # Config.max_audio_length (ctc.py:29)


class CTCModel:
    def __init__(self, weights: Union[np.ndarray, Dict[str, np.ndarray]], vocab: int, device: int = 0,
                 precision: str = "fp32"):
        if isinstance(weights, dict):
            weights = np.concatenate([np.asarray(v, np.float32).reshape(-1) for v in weights.values()])
        w = np.ascontiguousarray(weights, np.float32)
        L = lib()
        self.cfg = _lib.WkCtcConfig(vocab, 128, 2, 80, device, {"fp32": 0, "fp16": 1}[precision])
        need = L.wk_ctc_num_weights(C.byref(self.cfg))
        if w.size != need:
            raise ValueError(f"expected {need} weights for vocab={vocab}, got {w.size}")
        self.vocab, self.device = vocab, device
        self._h = C.c_void_p()
        check(L.wk_ctc_create(C.byref(self.cfg), w.ctypes.data_as(C.c_void_p), C.byref(self._h)), "wk_ctc_create")

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                lib().wk_ctc_destroy(self._h)
        except Exception:
            pass

    def _stream(self, torch):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def features(self, audio, n_samples: int = MAX_AUDIO_SAMPLES):
        """(B, L) float waveform -> (B, T, 80) on device, T = 1 + n_samples // 160."""
        import torch
        x = torch.as_tensor(audio, dtype=torch.float32).to(f"cuda:{self.device}").contiguous()
        if x.dim() == 1:
            x = x.unsqueeze(0)
        B, L = x.shape
        T = 1 + n_samples // 160
        out = torch.empty((B, T, 80), dtype=torch.float32, device=x.device)
        check(lib().wk_ctc_features(self._h, C.c_void_p(x.data_ptr()), B, L, n_samples, L, C.c_void_p(out.data_ptr()),
                                    self._stream(torch)), "wk_ctc_features")
        return out

    def decode(self, feats, return_log_probs: bool = False):
        """(B, T, 80) -> device tensors, stream-ordered, no host sync: tokens
        (B, T) int32 (row b's first lengths[b] entries are its greedy CTC
        sequence, the rest -1), lengths (B,) int32, and (B, T, V) log-probs
        if asked (else None)."""
        import torch
        f = torch.as_tensor(feats, dtype=torch.float32).to(f"cuda:{self.device}").contiguous()
        B, T, _ = f.shape
        lp = torch.empty((B, T, self.vocab), dtype=torch.float32, device=f.device) if return_log_probs else None
        tok = torch.empty((B, T), dtype=torch.int32, device=f.device)
        ln = torch.empty((B,), dtype=torch.int32, device=f.device)
        check(lib().wk_ctc_forward(self._h, C.c_void_p(f.data_ptr()), B, T,
                                   C.c_void_p(lp.data_ptr()) if lp is not None else None, C.c_void_p(tok.data_ptr()),
                                   C.c_void_p(ln.data_ptr()), self._stream(torch)), "wk_ctc_forward")
        return tok, ln, lp

    def forward(self, feats, return_log_probs: bool = False):
        """(B, T, 80) -> token id lists (greedy CTC, decode_predictions'
        output form), and (B, T, V) log-probs if asked."""
        tok, ln, lp = self.decode(feats, return_log_probs)
        tok, ln = tok.cpu().numpy(), ln.cpu().numpy()
        seqs = [tok[b, :ln[b]].tolist() for b in range(tok.shape[0])]
        return (seqs, lp) if return_log_probs else seqs

    def transcribe(self, audio, n_samples: int = MAX_AUDIO_SAMPLES) -> List[List[int]]:
        return self.forward(self.features(audio, n_samples))
