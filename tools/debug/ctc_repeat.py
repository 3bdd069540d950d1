"""Bit-repeatability of the CTC head at the bench size (diagnostic): the same
batch through features + decode several times; tokens, lengths and log-probs
must be identical run to run."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]
import torch  # noqa: E402
import wakeword  # noqa: E402
from oracle import wk_ctc_oracle as CO  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp16"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
V = 4000
n = 48000
g = wakeword.CTCModel(CO.flat_weights(CO.make_model(V, seed=0)), V, precision=prec)
audio = wakeword.synth_clips(1234, 0, B, n)
ref = None
for r in range(4):
    f = g.features(audio, n_samples=n)
    out = g.decode(f, return_log_probs=True)
    torch.cuda.synchronize()
    flat = [t.clone() for t in out if t is not None]
    if ref is None:
        ref = flat
        print("shapes", [tuple(t.shape) for t in flat if hasattr(t, "shape")])
        continue
    same = [bool(torch.equal(a, b)) for a, b in zip(ref, flat)]
    print(f"rep {r}: identical {same}")
