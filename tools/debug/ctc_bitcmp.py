"""Bit-exactness of the CTC head between two library builds (diagnostic):
    WAKEWORD_LIB=<lib A> python tools/debug/ctc_bitcmp.py dump a.npz
    WAKEWORD_LIB=<lib B> python tools/debug/ctc_bitcmp.py dump b.npz
    python tools/debug/ctc_bitcmp.py cmp a.npz b.npz
fp16 and fp32 models (seeded weights, V = 4000): SHA-256 of the log-probs of
256 utterances (in chunks of 64) and the tokens of 4,096 (one-call path)."""
import hashlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]

if sys.argv[1] == "dump":
    import torch
    from wakeword import ctc
    out = {}
    g = torch.Generator(device="cuda:0").manual_seed(5)
    audio = 0.1 * torch.randn((4096, 48000), generator=g, device="cuda:0")
    for prec in ("fp16", "fp32"):
        m = ctc.CTCModel(ctc.random_state_dict(4000, seed=3), 4000, precision=prec)
        h = hashlib.sha256()
        for c in range(0, 256, 64):
            f = m.features(audio[c:c + 64])
            tok, ln, lp = m.decode(f, return_log_probs=True)
            h.update(lp.cpu().numpy().tobytes())
        out[f"lp_sha_{prec}"] = np.frombuffer(h.digest(), np.uint8)
        n = 4096 if prec == "fp16" else 512
        tok, ln = m.decode_audio(audio[:n])
        out[f"tok_{prec}"] = tok.cpu().numpy()
        out[f"len_{prec}"] = ln.cpu().numpy()
    np.savez(sys.argv[2], **out)
else:
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = 0
    for k in a.files:
        d = int((a[k] != b[k]).sum())
        bad += d
        print(f"{k}: {d} differing of {a[k].size}")
    sys.exit(1 if bad else 0)
