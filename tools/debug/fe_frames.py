"""Debug: per-frame error of the raw (no CMVN) mode-B MFCC vs the oracle."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]
from oracle import wk_oracle as O
import wakeword
x = O.synth_clips(1234, 0, 4)
got = wakeword.mfcc(x, cmvn=False).cpu().numpy()
ref = O.mfcc_torchaudio(x)
err = np.abs(got - ref).max(axis=(0, 1))
print("per-frame max err:", np.array2string(err, precision=2, max_line_width=200))
print("worst frames:", np.argsort(-err)[:8])
