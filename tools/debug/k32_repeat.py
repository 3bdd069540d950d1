"""Repeatability probe of the fused kernel at full size (the
K = 32 question): N launches of the same 65,536 clips through the library
$WAKEWORD_LIB points at; prints, per repeat, how many logits differ from the
first launch.  Diagnostic tool (tools/debug), not a test.

    WAKEWORD_LIB=variants/var_k32/libwakeword.so python tools/debug/k32_repeat.py bf16 6
"""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(R, "esp32-wake-word_amd"))

import torch  # noqa: E402
import wakeword  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 6
feats = len(sys.argv) > 3 and sys.argv[3] == "feats"   # also write the CMVN'd features (the round-3 probe's setting)
m = wakeword.load_onnx(os.path.join(R, "tests", "golden", "xiaoa.onnx"), precision=prec)
x = wakeword.synth_clips(777, 0, 65536, device=0)
def run():
    if feats:
        lg, f = m.detect(x, return_features=True)
        return lg.reshape(-1).clone(), f.clone()
    return m.detect(x).reshape(-1).clone(), None


ref, fref = run()
counts, fcounts = [], []
for _ in range(n):
    got, f = run()
    counts.append(int((got != ref).sum()))
    if feats:
        fcounts.append(int((f != fref).reshape(f.shape[0], -1).any(dim=1).sum()))
torch.cuda.synchronize()
m.check_device_errors()
tag = os.environ.get("WAKEWORD_LIB", "prod")
print(f"{tag} {prec}{' +feats' if feats else ''}: clips whose logit differs from launch 0, per repeat: {counts}"
      + (f"; clips whose features differ: {fcounts}" if feats else ""), flush=True)
np.save(os.path.join(R, "gpurun_out", f"k32_{prec}_{os.path.basename(os.path.dirname(tag)) or 'prod'}.npy"),
        ref.cpu().numpy())
