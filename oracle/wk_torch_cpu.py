"""CPU baseline: the reference's ml_models CPU path restated on torch (fp32).

TEST / BASELINE INFRASTRUCTURE ONLY (imported by tests/ and bench.py's
cpu_baseline leg, never by the product).

  front-end  ml_models/src/extract_mfcc.py:137-175 -- torchaudio is absent, so
             its MFCC is restated on the ops torchaudio itself uses
             (torch.stft center/reflect with a periodic hamming(320) window,
             HTK mel matmul, log(+1e-6), ortho-DCT matmul), then CMVN :73-80.
  CNN        ml_models/src/wakeModel.py:4-34 (LightweightKWS) written with
             torch.nn.functional ops on the xiaoa.onnx weights.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _fbanks() -> torch.Tensor:
    all_freqs = torch.linspace(0, 8000, 257)
    m_min = 2595.0 * math.log10(1.0)
    m_max = 2595.0 * math.log10(1.0 + 8000.0 / 700.0)
    m_pts = torch.linspace(m_min, m_max, 42)
    f_pts = 700.0 * (10 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return torch.clamp(torch.min(down, up), min=0.0)


def _dct() -> torch.Tensor:
    n = torch.arange(40, dtype=torch.float32)
    k = torch.arange(13, dtype=torch.float32).unsqueeze(1)
    d = torch.cos(math.pi / 40 * (n + 0.5) * k)
    d[0] *= 1.0 / math.sqrt(2.0)
    d *= math.sqrt(2.0 / 40)
    return d.t().contiguous()


class TorchCpuPath:
    def __init__(self, state_dict):
        self.w = {k: torch.as_tensor(v, dtype=torch.float32) for k, v in state_dict.items()}
        self.fb = _fbanks()
        self.dct = _dct()
        self.win = torch.hamming_window(320)

    @torch.no_grad()
    def features(self, x: torch.Tensor) -> torch.Tensor:
        y = x.clone()
        y[..., 1:] -= 0.97 * x[..., :-1]
        spec = torch.stft(y, n_fft=512, hop_length=256, win_length=320, window=self.win, center=True,
                          pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
        p = spec.abs().pow(2.0)
        mel = torch.matmul(p.transpose(-1, -2), self.fb)
        mf = torch.matmul(torch.log(mel + 1e-6), self.dct).transpose(-1, -2)
        mean = mf.mean(dim=-1, keepdim=True)
        std = mf.std(dim=-1, keepdim=True)
        std = torch.where(std == 0, torch.ones_like(std), std)
        return (mf - mean) / (std + 1e-8)

    @torch.no_grad()
    def cnn(self, f: torch.Tensor) -> torch.Tensor:
        h = f
        for k in ("conv_layers.0.weight", "conv_layers.3.weight", "conv_layers.6.weight"):
            h = F.max_pool1d(F.relu(F.conv1d(h, self.w[k], padding=1)), 2)
        g = h.mean(dim=-1)
        g = F.relu(g @ self.w["classifier.0.weight"].t())
        return g @ self.w["classifier.2.weight"].t()

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        return self.cnn(self.features(x))[:, 0]
