"""Per-phase cycle breakdown of the fused kernel (diagnostic library built by
tools/debug/build_diag.sh; run with WAKEWORD_LIB pointing at it)."""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]
import torch  # noqa: E402
import wakeword  # noqa: E402
from wakeword import _lib  # noqa: E402

L = _lib.lib()
L.wk_debug_stamps.argtypes = [C.c_void_p, C.c_int]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
model = wakeword.load_onnx(os.path.join(REPO, "tests", "golden", "xiaoa.onnx"), precision=prec)
x = wakeword.synth_clips(1234, 0, B)
model.detect(x)
torch.cuda.synchronize()
buf = np.zeros((16, 16), np.uint64)
L.wk_debug_stamps(buf.ctypes.data, 1)
reps = 3
for _ in range(reps):
    model.detect(x)
torch.cuda.synchronize()
L.wk_debug_stamps(buf.ctypes.data, 1)
grid = min(B, 256)
clips_per_wg = B / grid
# stamp ids: wk_fused.hip fe_role (0, 1, 7-10) and wk_fe_dev.h fe_rest (2-6); cnn_role 0-8
fe = ["stage0", "pf_issue", "dft1", "tw+trW", "trR", "dft2", "split", "sync_P", "mel", "p_wait", "L_free", "vm_wait"]
cnn = ["dct+waitL", "conv1", "sync1", "conv2", "sync2", "conv3", "sync3", "fc1+sync", "fc2"]
print(f"cycles per clip per wave (B={B}, grid={grid}, reps={reps}, precision={prec})")
for w in range(8):
    row = buf[w, :12].astype(np.float64) / (grid * reps * clips_per_wg)
    print(f"FE  w{w}: " + " ".join(f"{n}={v:5.0f}" for n, v in zip(fe, row)) + f"  total={row.sum():6.0f}")
for w in range(8):
    row = buf[8 + w, :9].astype(np.float64) / (grid * reps * clips_per_wg)
    print(f"CNN w{w}: " + "  ".join(f"{n}={v:6.0f}" for n, v in zip(cnn, row)) + f"  total={row.sum():7.0f}")
