"""Bit-exactness of a library variant against another (diagnostic):
    WAKEWORD_LIB=<lib A> python tools/debug/bitcmp.py dump a.npz
    WAKEWORD_LIB=<lib B> python tools/debug/bitcmp.py dump b.npz
    python tools/debug/bitcmp.py cmp a.npz b.npz
Dumps logits and features of 8,192 synthetic clips (fp32, bf16, bf16x3) and of
the mode-A / mode-B front-ends, and counts differing values."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]

if sys.argv[1] == "dump":
    import torch
    import wakeword
    x = wakeword.synth_clips(77, 0, 8192)
    out = {}
    for prec in ("fp32", "bf16", "bf16x3"):
        m = wakeword.load_onnx(os.path.join(REPO, "tests", "golden", "xiaoa.onnx"), precision=prec)
        lg, ft = m.detect(x, return_features=True)
        out[f"logits_{prec}"] = lg.cpu().numpy()
        out[f"feats_{prec}"] = ft.cpu().numpy()
    out["mfcc_b"] = wakeword.mfcc(x[:1024], mode="torchaudio").cpu().numpy()
    out["mfcc_a"] = wakeword.mfcc(x[:1024], mode="esp").cpu().numpy()
    torch.cuda.synchronize()
    np.savez(sys.argv[2], **out)
else:
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = 0
    for k in a.files:
        n = int((a[k].view(np.uint32) != b[k].view(np.uint32)).sum())
        bad += n
        print(f"{k}: {n} differing of {a[k].size}")
    sys.exit(1 if bad else 0)
