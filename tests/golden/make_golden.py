"""Generate the committed golden fixtures under tests/golden/.

Runs ONLY in the build container, where the read-only reference is mounted at
/root/reference.  Nothing here is needed (or possible) on the GPU box: the
outputs are plain data files (npz / json / the reference's own .onnx weights
and a few of its WAVs), committed next to this script.

Sources of truth, in order of strength:
  1. ``ml_models/xiaoa.info`` (esp_ppq export, lines 3153-3224): an int8
     known-answer test for the CNN (input [1,63,13] exp -4 -> output -40
     exp -3) and the int8 weights (round(w_fp32 * 2^-exp)).
  2. The reference's OWN ``LightweightKWS`` (ml_models/src/wakeModel.py:4-34),
     imported here with the xiaoa.onnx weights, for every golden logit.
  3. The front-end (torchaudio, absent) restated twice: numpy float64
     (oracle/wk_oracle.py) and torch.stft float32 (below); they must agree.
     No reference artefact holds torchaudio MFCC values -> front-end parity
     is "unpinned" at that boundary.
"""
from __future__ import annotations

import json
import math
import os
import re
import shutil
import sys
import wave

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "esp32-wake-word_amd"))

from oracle import wk_oracle as O  # noqa: E402
from wakeword.onnx_reader import read_onnx, xiaoa_state_dict  # noqa: E402

WAV_PICK = ["xiaoa_041.wav", "xiaoa_095.wav", "xiaoa_162.wav", "xiaoa_230.wav",
            "xiaoa_419.wav", "xiaoa_550.wav", "xiaoa_734.wav", "xiaoa_995.wav"]


def parse_info(path):
    """Parse esp_ppq's xiaoa.info dump: initializers (int8 + exponent) and the
    test input / output vectors."""
    txt = open(path).read()
    out = {}
    pat = re.compile(r"%(\S+?), shape: \[([0-9, ]*)\], exponents: \[(-?\d+)\].*?value: array\(\[(.*?)\]",
                     re.S)
    for m in pat.finditer(txt):
        name = m.group(1)
        shape = [int(s) for s in m.group(2).split(",") if s.strip()]
        exp = int(m.group(3))
        vals = np.array([int(v) for v in m.group(4).replace("\n", " ").split(",") if v.strip()], np.int64)
        out.setdefault(name, []).append((shape, exp, vals))
    return out


def read_wav(path):
    with wave.open(path) as w:
        assert w.getnchannels() == 1 and w.getsampwidth() == 2 and w.getframerate() == 16000
        return np.frombuffer(w.readframes(w.getnframes()), "<i2").copy()


def torch_mfcc_b(x32: np.ndarray) -> np.ndarray:
    """Independent fp32 restatement of the torchaudio path on torch.stft
    (what torchaudio.transforms.Spectrogram calls internally)."""
    x = torch.from_numpy(np.asarray(x32, np.float32))
    y = x.clone()
    y[..., 1:] -= 0.97 * x[..., :-1]
    spec = torch.stft(y, n_fft=512, hop_length=256, win_length=320, window=torch.hamming_window(320),
                      center=True, pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
    p = spec.abs().pow(2.0)                                    # (..., 257, T)
    all_freqs = torch.linspace(0, 8000, 257)
    m_min = 2595.0 * math.log10(1.0 + 0.0 / 700.0)
    m_max = 2595.0 * math.log10(1.0 + 8000.0 / 700.0)
    m_pts = torch.linspace(m_min, m_max, 42)
    f_pts = 700.0 * (10 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    fb = torch.clamp(torch.min(down, up), min=0.0)
    mel = torch.matmul(p.transpose(-1, -2), fb).transpose(-1, -2)
    mel = torch.log(mel + 1e-6)
    n = torch.arange(40, dtype=torch.float32)
    k = torch.arange(13, dtype=torch.float32).unsqueeze(1)
    dct = torch.cos(math.pi / 40 * (n + 0.5) * k)
    dct[0] *= 1.0 / math.sqrt(2.0)
    dct *= math.sqrt(2.0 / 40)
    mf = torch.matmul(mel.transpose(-1, -2), dct.t()).transpose(-1, -2)
    mean = mf.mean(dim=-1, keepdim=True)
    std = mf.std(dim=-1, keepdim=True)
    std = torch.where(std == 0, torch.ones_like(std), std)
    return ((mf - mean) / (std + 1e-8)).numpy()


def main():
    sys.path.insert(0, os.path.join(REF, "ml_models", "src"))
    import wakeModel  # the reference's own class (wakeModel.py:4-34)

    onnx_path = os.path.join(REF, "ml_models", "xiaoa.onnx")
    shutil.copyfile(onnx_path, os.path.join(HERE, "xiaoa.onnx"))
    inits, ins, outs = read_onnx(onnx_path)
    sd = xiaoa_state_dict(inits)
    ref = wakeModel.LightweightKWS(num_classes=1).eval()
    ref.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})

    def ref_logits(feats):
        with torch.no_grad():
            return ref(torch.from_numpy(np.asarray(feats, np.float32))).numpy()[:, 0]

    # ---- 1. esp_ppq KAT + int8 weights --------------------------------------
    info = parse_info(os.path.join(REF, "ml_models", "xiaoa.info"))
    kat_in_shape, kat_in_exp, kat_in = info["input.1"][-1]
    kat_out_shape, kat_out_exp, kat_out = info["22"][-1]
    kat_in = kat_in[: int(np.prod(kat_in_shape))].reshape(kat_in_shape).astype(np.int8)
    kat_out = kat_out[: int(np.prod(kat_out_shape))].reshape(kat_out_shape).astype(np.int8)
    kat_feats = (kat_in.astype(np.float32) * 2.0 ** kat_in_exp).transpose(0, 2, 1)  # (1,13,63)
    q = {}
    for name in ("conv_layers.0.weight", "conv_layers.3.weight", "conv_layers.6.weight",
                 "onnx::MatMul_23", "onnx::MatMul_24"):
        shape, exp, vals = info[name][0]
        q[name] = (vals[: int(np.prod(shape))].reshape(shape).astype(np.int8), exp)
    np.savez_compressed(
        os.path.join(HERE, "kat.npz"),
        kat_in_int8=kat_in, kat_in_exp=kat_in_exp, kat_out_int8=kat_out, kat_out_exp=kat_out_exp,
        kat_feats=kat_feats, kat_ref_logit=ref_logits(kat_feats),
        **{f"q_{k.replace(':', '_').replace('.', '_')}": v[0] for k, v in q.items()},
        **{f"qexp_{k.replace(':', '_').replace('.', '_')}": v[1] for k, v in q.items()},
    )

    # ---- 2. reference WAVs (a committed subset) ------------------------------
    wav_dir = os.path.join(REF, "audio_data", "flash")
    os.makedirs(os.path.join(HERE, "wav"), exist_ok=True)
    names = sorted(f for f in os.listdir(wav_dir) if f.endswith(".wav"))
    torch.manual_seed(0)
    noise_pads = {}
    for nme in names:
        raw = read_wav(os.path.join(wav_dir, nme))
        n = min(len(raw), 16000)
        noise_pads[nme] = (torch.randn(1, 16000 - n) * 0.005).numpy()[0] if n < 16000 else np.zeros(0, np.float32)
    summary = {"zero_pad_positive": 0, "noise_pad_positive": 0, "n": len(names)}
    rows = {k: [] for k in ("name", "x_noise", "feat_zero", "feat_noise", "feat_zero_torch",
                            "logit_zero", "logit_noise")}
    for nme in names:
        raw = read_wav(os.path.join(wav_dir, nme))
        audio = raw.astype(np.float32) / 32768.0                      # torchaudio.load scaling
        xz = O.pad_audio(audio, 16000, None)
        xn = O.pad_audio(audio, 16000, noise_pads[nme] if len(audio) < 16000 else None)
        fz, fn = O.features_mode_b(xz[None]), O.features_mode_b(xn[None])
        lz, ln_ = ref_logits(fz)[0], ref_logits(fn)[0]
        summary["zero_pad_positive"] += int(lz > 0)
        summary["noise_pad_positive"] += int(ln_ > 0)
        if nme in WAV_PICK:
            shutil.copyfile(os.path.join(wav_dir, nme), os.path.join(HERE, "wav", nme))
            rows["name"].append(nme)
            rows["x_noise"].append(xn)
            rows["feat_zero"].append(fz[0].astype(np.float32))
            rows["feat_noise"].append(fn[0].astype(np.float32))
            rows["feat_zero_torch"].append(torch_mfcc_b(xz[None])[0])
            rows["logit_zero"].append(lz)
            rows["logit_noise"].append(ln_)
    np.savez_compressed(os.path.join(HERE, "wavs.npz"), **{k: np.array(v) for k, v in rows.items()})

    # ---- 3. seeded synthetic clips (config 2 generator) ----------------------
    clips = O.synth_clips(1234, 0, 16)
    feats = O.features_mode_b(clips)
    np.savez_compressed(os.path.join(HERE, "synth.npz"), seed=1234, first=0, count=16,
                        clip_checksum=clips.astype(np.float64).sum(axis=1),
                        feats=feats.astype(np.float32), feats_torch=torch_mfcc_b(clips),
                        logits=ref_logits(feats))

    summary["torch_vs_numpy_feat_maxdiff_wavs"] = float(np.max(np.abs(
        np.array(rows["feat_zero"]) - np.array(rows["feat_zero_torch"]))))
    summary["torch_vs_numpy_feat_maxdiff_synth"] = float(np.max(np.abs(feats - torch_mfcc_b(clips))))
    summary["kat_ref_logit"] = float(ref_logits(kat_feats)[0])
    summary["kat_int8_out_dequant"] = float(kat_out.reshape(-1)[0] * 2.0 ** kat_out_exp)
    with open(os.path.join(HERE, "summary.json"), "w") as fh:
        json.dump(summary, fh, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
