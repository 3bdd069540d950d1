"""Generate csrc/wk_tables.h: compile-time constants for the front-end kernels.

Run at development time (python esp32-wake-word_amd/tools/gen_tables.py); the
generated header is committed.  The constants restate, in float32 exactly as
the reference computes them:

* mode B (torchaudio path, ml_models/src/extract_mfcc.py:137-148):
  periodic Hamming(320) (torch.hamming_window), HTK mel filterbank
  (torchaudio.functional.melscale_fbanks, n_freqs 257, 40 mels, norm None),
  DCT-II ortho (torchaudio.functional.create_dct).
* mode A (main/esp_mfcc/mfcc.c): symmetric Hamming alpha=0.53836
  (mfcc.c:118-120), integer-bin triangular filterbank (mfcc.c:144-234),
  DCT-II ortho with scale applied after the sum (mfcc.c:20-64).

The mel stage runs "lane-per-frame" (one lane owns one frame, one wave owns a
contiguous block of filters), so every filterbank weight and every power-bin
offset becomes an immediate in straight-line code: the generator emits one
function per (mode, wave).  Filters are partitioned over the 8 waves of a
workgroup to balance LDS reads + FMAs.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "csrc", "wk_tables.h")
N_WAVES = 8
# Relative mel speed per wave (fused kernel: the front-end waves 0-3 issue
# ahead of 4-7 on each SIMD).
MEL_WAVE_WEIGHTS = [1.0] * N_WAVES
N_MELS = 40
N_MFCC = 13


def f32(x) -> str:
    v = float(np.float32(x))
    if v == 0.0:
        return "0.0f"
    return f"{v!r}f" if "e" in repr(v) or "." in repr(v) else f"{v!r}.0f"


def fb_mode_b() -> np.ndarray:
    """(257, 40) float32, torchaudio.functional.melscale_fbanks(htk) in torch fp32."""
    all_freqs = torch.linspace(0, 8000, 257)
    m_min = 2595.0 * math.log10(1.0 + 0.0 / 700.0)
    m_max = 2595.0 * math.log10(1.0 + 8000.0 / 700.0)
    m_pts = torch.linspace(m_min, m_max, N_MELS + 2)
    f_pts = 700.0 * (10 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return torch.clamp(torch.min(down, up), min=0.0).numpy().astype(np.float32)


def dct_mode_b() -> np.ndarray:
    """(13, 40) float32 = create_dct(13, 40, 'ortho').T in torch fp32."""
    n = torch.arange(float(N_MELS))
    k = torch.arange(float(N_MFCC)).unsqueeze(1)
    dct = torch.cos(math.pi / float(N_MELS) * (n + 0.5) * k)
    dct[0] *= 1.0 / math.sqrt(2.0)
    dct *= math.sqrt(2.0 / float(N_MELS))
    return dct.numpy().astype(np.float32)


def window_mode_b() -> np.ndarray:
    return torch.hamming_window(320).numpy().astype(np.float32)


def window_mode_a() -> np.ndarray:
    i = np.arange(320, dtype=np.float64)
    ang = (2.0 * math.pi * i / 319.0).astype(np.float32)       # double expr -> cosf(float)
    return (np.float32(0.53836) - np.float32(1.0 - 0.53836) * np.cos(ang)).astype(np.float32)


def fb_mode_a() -> np.ndarray:
    """(257, 40) float32, mfcc.c:144-234 with sampling_rate 16000, n_fft 512."""
    def hz_to_mel(f):
        f = np.float32(1.0) if f == 0 else np.float32(f)
        return np.float32(np.float32(1127.0) * np.log1p(np.float32(f / np.float32(700.0))))

    def mel_to_hz(m):
        return np.float32(np.float32(700.0) * (np.power(np.float32(10.0), np.float32(m / np.float32(2595.0))) - np.float32(1.0)))

    n_bins = 257
    low, high = hz_to_mel(0), hz_to_mel(8000)
    mel_pts = [np.float32(low + np.float32(i) * (high - low) / np.float32(N_MELS + 1)) for i in range(N_MELS + 2)]
    hz_pts = [mel_to_hz(m) for m in mel_pts]
    bin_w = np.float32(16000.0 / 512.0)
    bins = [int(math.floor(np.float32(h / bin_w))) for h in hz_pts]
    fb = np.zeros((N_MELS, n_bins), np.float32)
    for i in range(N_MELS):
        l, c, r = bins[i], bins[i + 1], bins[i + 2]
        l, c, r = max(l, 0), max(c, 0), max(r, 0)
        l, c, r = min(l, n_bins - 1), min(c, n_bins - 1), min(r, n_bins - 1)
        if l >= c:
            c = l + 1
        if c >= r:
            r = c + 1
        if r >= n_bins:
            r = n_bins - 1
        for j in range(l, c + 1):
            if 0 <= j < n_bins:
                fb[i, j] = np.float32(j - l) / np.float32(c - l)
        for j in range(c, r + 1):
            if 0 <= j < n_bins:
                fb[i, j] = np.float32(r - j) / np.float32(r - c)
    return fb.T.copy()


def dct_mode_a() -> np.ndarray:
    n = N_MELS
    cos = np.zeros((N_MFCC, n), np.float32)
    for k in range(N_MFCC):
        for i in range(n):
            cos[k, i] = np.cos(np.float32(math.pi * k * (2 * i + 1) / (2.0 * n)))
    return cos


def partition(fb: np.ndarray, n_parts: int, weights=None):
    """Contiguous split of the filters minimising max(cost / weight) over the
    parts, cost = distinct bins + fmas (+ 12 per filter); part p goes to wave p."""
    weights = weights or [1.0] * n_parts
    nz = [np.nonzero(fb[:, m])[0] for m in range(fb.shape[1])]

    def cost(a, b):
        bins = set()
        fm = 0
        for m in range(a, b):
            bins.update(nz[m].tolist())
            fm += len(nz[m])
        return len(bins) + fm + 12 * (b - a)

    M = fb.shape[1]
    INF = 1 << 30
    dp = [[INF] * (M + 1) for _ in range(n_parts + 1)]
    cut = [[0] * (M + 1) for _ in range(n_parts + 1)]
    dp[0][0] = 0
    for p in range(1, n_parts + 1):
        for b in range(1, M + 1):
            for a in range(p - 1, b):
                v = max(dp[p - 1][a], cost(a, b) / weights[p - 1])
                if v < dp[p][b]:
                    dp[p][b], cut[p][b] = v, a
    bounds = []
    b = M
    for p in range(n_parts, 0, -1):
        a = cut[p][b]
        bounds.append((a, b))
        b = a
    return bounds[::-1], dp[n_parts][M]


def emit_mel(fb: np.ndarray, name: str, mode: str, scale: float):
    """One straight-line function per wave: P row -> log-mel row."""
    env = os.environ.get("WK_MEL_WEIGHTS")
    bounds, worst = partition(fb, N_WAVES, [float(v) for v in env.split(",")] if env else MEL_WAVE_WEIGHTS)
    lines = [f"// {name}: filters per wave {bounds}, worst-wave cost {worst:.4g}"]
    for w, (a, b) in enumerate(bounds):
        lines.append(f"__device__ __forceinline__ void {name}_w{w}(const float* __restrict__ p, float* __restrict__ l) {{")
        for m in range(a, b):
            lines.append(f"  float a{m} = 0.0f;")
        bins = sorted(set(int(k) for m in range(a, b) for k in np.nonzero(fb[:, m])[0]))
        for k in bins:
            terms = [(m, fb[k, m]) for m in range(a, b) if fb[k, m] != 0.0]
            lines.append(f"  {{ const float v = p[{k}];" +
                         "".join(f" a{m} = __builtin_fmaf(v, {f32(np.float32(wt) * np.float32(scale))}, a{m});"
                                 for m, wt in terms) + " }")
        for m in range(a, b):
            if mode == "B":
                lines.append(f"  l[{m} * WK_LSTRIDE] = wk::wk_logf(a{m} + 1e-6f);")
            else:
                lines.append(f"  l[{m} * WK_LSTRIDE] = wk::wk_logf(__builtin_fmaxf(a{m}, 1e-12f));")
        lines.append("}")
    lines.append(f"template <int W> __device__ __forceinline__ void {name}_wave(const float* p, float* l);")
    for w in range(N_WAVES):
        lines.append(f"template <> __device__ __forceinline__ void {name}_wave<{w}>(const float* p, float* l) {{ {name}_w{w}(p, l); }}")
    return "\n".join(lines)


def main():
    fbB = fb_mode_b()
    fbA = fb_mode_a()
    dB = dct_mode_b()
    dA = dct_mode_a()
    wB = window_mode_b()
    wA = window_mode_a()
    out = ["// GENERATED by esp32-wake-word_amd/tools/gen_tables.py -- do not edit.",
           "// Constants restated from torchaudio (mode B) and main/esp_mfcc/mfcc.c (mode A).",
           "#pragma once", "", "#ifndef WK_LSTRIDE", "#define WK_LSTRIDE 64  // log-mel image is [mel][frame]", "#endif", ""]
    out.append(f"// nnz(mode B fbank) = {int((fbB != 0).sum())}, nnz(mode A fbank) = {int((fbA != 0).sum())}")
    # The analysis windows in the front-end's lane layout (wk_fe_dev.h fe_rest):
    # element i = sample i of the frame, lane j = (i % 32) // 2, row n1 = i // 32;
    # negated where n1 is odd and j >= 8 (the one-pass transpose's slot order).
    sgn = np.array([-1.0 if ((i % 32) // 2 >= 8 and (i // 32) % 2 == 1) else 1.0 for i in range(320)], np.float32)
    out.append("// analysis windows, signed for the front-end's one-pass FFT transpose (fe_rest)")
    out.append("__constant__ float kWinB[320] = {" + ", ".join(f32(v) for v in wB * sgn) + "};")
    out.append("__constant__ float kWinA[320] = {" + ", ".join(f32(v) for v in wA * sgn) + "};")
    out.append("")
    # Mode B: P holds |U|^2 with U = 2 V  ->  fold the 1/4 into the weights (exact).
    out.append(emit_mel(fbB, "melB", "B", 0.25))
    out.append("")
    # Mode A: P already holds mfcc.c's power (re^2+im^2)/n_fft + 1e-12.
    out.append(emit_mel(fbA, "melA", "A", 1.0))
    out.append("")
    for c in range(N_MFCC):
        body = " ".join(f"s = __builtin_fmaf(l[{m} * WK_LSTRIDE], {f32(dB[c, m])}, s);" for m in range(N_MELS))
        out.append(f"__device__ __forceinline__ float dctB_{c}(const float* __restrict__ l) {{ float s = 0.0f; {body} return s; }}")
    for c in range(N_MFCC):
        scale = math.sqrt(1.0 / N_MELS) if c == 0 else math.sqrt(2.0 / N_MELS)
        body = " ".join(f"s = __builtin_fmaf(l[{m} * WK_LSTRIDE], {f32(dA[c, m])}, s);" for m in range(N_MELS))
        out.append(f"__device__ __forceinline__ float dctA_{c}(const float* __restrict__ l) {{ float s = 0.0f; {body} return {f32(scale)} * s; }}")
    # Mode B DCT as the A operand of a 16x40 fp32 MFMA GEMM (rows 13-15 zero).
    dB16 = np.zeros((16, N_MELS), np.float32)
    dB16[:N_MFCC] = dB
    out.append("__constant__ float kDctB16[16 * 40] = {" + ", ".join(f32(v) for v in dB16.reshape(-1)) + "};")
    out.append("template <bool MODE_B> __device__ __forceinline__ float dct_coef(int c, const float* __restrict__ l) {")
    out.append("  switch (c) {")
    for c in range(N_MFCC):
        out.append(f"    case {c}: return MODE_B ? dctB_{c}(l) : dctA_{c}(l);")
    out.append("    default: return 0.0f;")
    out.append("  }")
    out.append("}")
    out.append("")
    with open(OUT, "w") as fh:
        fh.write("\n".join(out) + "\n")
    np.savez(os.path.join(HERE, "tables_dump.npz"), fbB=fbB, fbA=fbA, dB=dB, dA=dA, wB=wB, wA=wA)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
