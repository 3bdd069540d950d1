"""Diagnostic: constant utterances through the CTC one-call and two-call paths."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "esp32-wake-word_amd"))
import numpy as np, torch
import wakeword
from oracle import wk_ctc_oracle as CO
m = CO.make_model(512, seed=7)
g = wakeword.CTCModel(CO.flat_weights(m), 512, precision="fp16")
n = 8000
B, T = 4, 1 + n // 160
x = np.zeros((B, n), np.float32)
x[0::2] = 0.25
feats = g.features(x, n_samples=n).cpu()
for b in range(B):
    f = feats[b]
    print(b, "min", float(f.min()), "max", float(f.max()), "n_distinct", len(torch.unique(f)), "mean", float(f.mean()))
gf = wakeword.CTCModel(CO.flat_weights(m), 512, precision="fp32")
ff = gf.features(x, n_samples=n).cpu()
for b in range(B):
    f = ff[b]
    print("fp32", b, "min", float(f.min()), "max", float(f.max()), "n_distinct", len(torch.unique(f)))
ref = CO.features(torch.from_numpy(x))
for b in range(B):
    f = ref[b]
    print("oracle", b, "min", float(f.min()), "max", float(f.max()), "n_distinct", len(torch.unique(f)))
tok, ln = g.decode_audio(x, n_samples=n)
one = g.frame_argmax(B, T).cpu()
g.decode(feats.cuda())
two = g.frame_argmax(B, T).cpu()
print("one", one[:, :6].tolist())
print("two", two[:, :6].tolist())
# the un-normalised features fed to decode
raw = feats.clone()
