"""Run-to-run and precision-to-precision logit differences at full batch
(diagnostic): which clips differ, and where they sit (clip % grid, clip // grid)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]
import torch  # noqa: E402
import wakeword  # noqa: E402

onnx = os.path.join(REPO, "tests", "golden", "xiaoa.onnx")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
x = wakeword.synth_clips(1234, 0, B)
G = torch.cuda.get_device_properties(0).multi_processor_count
precs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["fp32", "bf16", "bf16x3"]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
for prec in precs:
    m = wakeword.load_onnx(onnx, precision=prec)
    ref = m.detect(x).reshape(-1).cpu().numpy()
    for r in range(reps):
        got = m.detect(x).reshape(-1).cpu().numpy()
        d = np.abs(got - ref)
        bad = np.nonzero(d != 0)[0]
        print(f"{prec} rep {r}: {bad.size} clips differ from rep 0, max {d.max():.3g}", flush=True)
        for i in bad[:6]:
            print(f"   clip {i}: cu-slot {i % G} iter {i // G}  {ref[i]:.5f} {got[i]:.5f}")
