"""CPU ORACLE for the CTC head -- TEST INFRASTRUCTURE ONLY.

Only tests/ and the CTC benchmark's CPU leg import this module.  It restates
ml_models/ctc.py on torch CPU, fp32:

* X1 ``THCHS30Dataset.extract_features`` (ctc.py:82-107): pad/trim to the
  utterance length (:85-90), torchaudio ``MelSpectrogram(16000, n_fft=400,
  hop_length=160, n_mels=80)`` with torchaudio's defaults (periodic Hann(400),
  center=True / reflect, power 2, HTK mel on [0, 8000], norm None), then
  ln(mel + 1e-8) and ONE global z-score over the whole [80][T] map with the
  unbiased std, skipped when std == 0 (:101-104).  torchaudio is absent from
  this image (a third-party dependency, version unpinned): its MelSpectrogram
  is restated on torch.stft, exactly the op torchaudio calls -> "parity
  unpinned" at the torchaudio boundary, like front-end mode B.
* X2 ``GRU_CTC_Model`` (ctc.py:119-152): built from the same torch.nn modules
  the reference composes (Linear 80->H, LayerNorm(H), ReLU, Dropout [eval:
  identity], GRU(H, H, 2 layers, bidirectional, batch_first), Linear 2H->V,
  log_softmax).  The GRU recurrence is therefore torch's own nn.GRU -- the
  reference's implementation of that step.
* X3 ``decode_predictions`` (ctc.py:453-471): argmax over V, drop blank (0),
  collapse repeats with prev_token updated on every frame.

ctc.py itself cannot be imported (torchaudio, librosa, requests, matplotlib are
absent) and no trained weights exist in the reference (THCHS-30 training needs
the network, ctc.py:180-184), so weights are seeded random initialisations of
the same modules; V is fixed by the caller (the reference builds it from the
corpus at run time, ctc.py:261-278).
"""
from __future__ import annotations

import math
from typing import List

import numpy as np
import torch
import torch.nn as nn

SR, N_FFT, HOP, N_MELS = 16000, 400, 160, 80


def mel_fbanks(n_freqs: int = N_FFT // 2 + 1, n_mels: int = N_MELS) -> torch.Tensor:
    """torchaudio.functional.melscale_fbanks(201, 0, 8000, 80, 16000, None, 'htk'): (201, 80)."""
    all_freqs = torch.linspace(0, SR // 2, n_freqs)
    m_min = 2595.0 * math.log10(1.0 + 0.0 / 700.0)
    m_max = 2595.0 * math.log10(1.0 + (SR / 2) / 700.0)
    m_pts = torch.linspace(m_min, m_max, n_mels + 2)
    f_pts = 700.0 * (10 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return torch.clamp(torch.min(down, up), min=0.0)


def pad_or_trim(x: torch.Tensor, n: int) -> torch.Tensor:
    """ctc.py:85-90 (zero right-pad or truncate to n samples)."""
    if x.shape[-1] > n:
        return x[..., :n]
    return torch.nn.functional.pad(x, (0, n - x.shape[-1]))


@torch.no_grad()
def features(x: torch.Tensor) -> torch.Tensor:
    """(B, L) waveform -> (B, T, 80) z-scored log-mel, T = 1 + L // 160."""
    spec = torch.stft(x, n_fft=N_FFT, hop_length=HOP, win_length=N_FFT, window=torch.hann_window(N_FFT),
                      center=True, pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
    p = spec.abs().pow(2.0)                                  # (B, 201, T)
    mel = torch.matmul(p.transpose(-1, -2), mel_fbanks())    # (B, T, 80)
    mel = torch.log(mel + 1e-8)
    out = []
    for m in mel:                                           # per utterance, as the Dataset does
        if m.std() > 0:
            m = (m - m.mean()) / m.std()
        out.append(m)
    return torch.stack(out)


class GRUCTC(nn.Module):
    """ctc.py:119-152 GRU_CTC_Model, eval mode (Dropout = identity)."""

    def __init__(self, vocab: int, hidden: int = 128, layers: int = 2, n_mels: int = N_MELS):
        super().__init__()
        self.audio_encoder = nn.Sequential(nn.Linear(n_mels, hidden), nn.LayerNorm(hidden), nn.ReLU(), nn.Dropout(0.2))
        self.gru = nn.GRU(input_size=hidden, hidden_size=hidden, num_layers=layers, batch_first=True,
                          dropout=0.2 if layers > 1 else 0.0, bidirectional=True)
        self.output_layer = nn.Linear(2 * hidden, vocab)

    def forward(self, x):
        x = self.audio_encoder(x)
        y, _ = self.gru(x)
        return torch.nn.functional.log_softmax(self.output_layer(y), dim=-1)


def make_model(vocab: int, seed: int = 0, hidden: int = 128, out_scale: float = 4.0) -> GRUCTC:
    """Seeded GRU_CTC_Model (ctc.py:119-146 has no trained weights to load).
    out_scale multiplies the output layer's default nn.Linear init: 4 gives
    the greedy path margins (random init is near-uniform); 1 keeps the init."""
    torch.manual_seed(seed)
    m = GRUCTC(vocab, hidden)
    if out_scale != 1.0:
        with torch.no_grad():
            m.output_layer.weight.mul_(out_scale)
    return m.eval()


def flat_weights(m: GRUCTC) -> np.ndarray:
    """The state dict in its own order, concatenated (the wk_ctc_create blob)."""
    return np.concatenate([v.detach().reshape(-1).numpy().astype(np.float32) for v in m.state_dict().values()])


def greedy_decode(log_probs: torch.Tensor) -> List[List[int]]:
    """ctc.py:453-471 without the idx->char map: token id sequences."""
    _, pred = torch.max(log_probs, dim=2)
    out = []
    for row in pred:
        seq, prev = [], 0
        for tok in row.tolist():
            if tok != 0 and tok != prev:
                seq.append(tok)
            prev = tok
        out.append(seq)
    return out
