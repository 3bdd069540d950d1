"""Config 1 (BASELINE.json configs[0]): score WAV files end to end.

    python -m wakeword.test file.wav [file2.wav ...] [--onnx xiaoa.onnx]
        [--pad noise|zero] [--seed S] [--threshold 0.5] [--precision fp32|bf16|bf16x3|int8] [--json]
        [--cpu]

The reference's single-file path is WAV -> ``pad_audio`` -> torchaudio MFCC +
CMVN -> ``LightweightKWS`` -> sigmoid > 0.5 (ml_models/src/extract_mfcc.py:7-23,
123-182; ml_models/src/wakeModel.py:29-34; ml_models/main.py:52-53).  Here the
WAV header walk and the pad run on the host (wakeword.wav, the esp_wav.cpp
restatement in libwakeword.so) and everything from pre-emphasis to the logit
runs in the fused HIP kernel on cuda:0.

``--cpu`` runs the same path on the host instead (libwakeword_host.so,
wakeword.host: the C++ host implementation of the WAV loader, mode B and the
CNN, fp32) -- the reference's own config-1 setting, "on CPU, no GPU".  It is
a separate library chosen by this flag, not a fallback: without ``--cpu`` a
missing GPU is an error.

``--pad noise`` (the reference default, add_noise_to_pad=True) draws the pad
from N(0, 0.005^2) with the loader's seeded generator, so a run is
repeatable; ``--pad zero`` pads with zeros.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
from typing import List, Optional, Sequence

import numpy as np

_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEFAULT_ONNX = os.path.join(_REPO, "tests", "golden", "xiaoa.onnx")


def default_onnx() -> str:
    """$WAKEWORD_ONNX, else the xiaoa.onnx kept with the test fixtures."""
    return os.environ.get("WAKEWORD_ONNX", DEFAULT_ONNX)


def prepare(paths: Sequence[str], pad: str = "noise", seed: int = 0, cpu: bool = False) -> np.ndarray:
    """WAV files -> (B, 16000) float32 windows: x/32768, trimmed or right-padded
    as pad_audio does (native loader: wakeword.wav.load_batch, or the host
    library's copy of it with cpu=True)."""
    if cpu:
        from .host import load_batch
    else:
        from .wav import load_batch
    if not paths:
        return np.zeros((0, 16000), np.float32)
    x, _ = load_batch(list(paths), 16000, 0.005 if pad == "noise" else 0.0, seed)
    return x


def score(paths: Sequence[str], onnx: Optional[str] = None, pad: str = "noise", seed: int = 0,
          threshold: float = 0.5, precision: str = "fp32", device: int = 0, cpu: bool = False) -> List[dict]:
    """One result dict per file: logit, probability = sigmoid(logit), decision."""
    x = prepare(paths, pad, seed, cpu)
    if cpu:
        if precision != "fp32":
            raise ValueError("--cpu runs the fp32 path only")
        from . import host
        model = host.load_onnx(onnx or default_onnx())
        logits = model.detect(x) if len(paths) else np.zeros((0,), np.float32)
    else:
        from .api import load_onnx
        model = load_onnx(onnx or default_onnx(), device=device, precision=precision)
        logits = model.detect(x).cpu().numpy() if len(paths) else np.zeros((0,), np.float32)
    out = []
    for p, z in zip(paths, logits):
        prob = 1.0 / (1.0 + math.exp(-float(z)))
        out.append({"file": p, "logit": float(z), "probability": prob, "wake": bool(prob > threshold)})
    return out


def main(argv: Optional[Sequence[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="python -m wakeword.test", description=__doc__.split("\n\n")[0])
    ap.add_argument("wav", nargs="+")
    ap.add_argument("--onnx", default=None, help="xiaoa.onnx (default: $WAKEWORD_ONNX or tests/golden/xiaoa.onnx)")
    ap.add_argument("--pad", choices=("noise", "zero"), default="noise")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--threshold", type=float, default=0.5)
    ap.add_argument("--precision", choices=("fp32", "bf16", "bf16x3", "int8"), default="fp32")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--json", action="store_true", help="one JSON object per file")
    ap.add_argument("--cpu", action="store_true",
                    help="run on the host CPU (libwakeword_host.so) instead of the GPU: config 1's setting")
    a = ap.parse_args(argv)
    res = score(a.wav, a.onnx, a.pad, a.seed, a.threshold, a.precision, a.device, a.cpu)
    for r in res:
        if a.json:
            print(json.dumps(r))
        else:
            print(f"{r['file']}: logit {r['logit']:+.6f}  p {r['probability']:.4f}  "
                  f"{'WAKE' if r['wake'] else '-'}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
