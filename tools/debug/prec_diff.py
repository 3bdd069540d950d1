"""Compare a precision mode against the fp32 path clip by clip at full size
and report which clips exceed a tolerance, with their workgroup slot, per-WG
iteration and CNN-batch position (diagnostic)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]
import torch  # noqa: E402
import wakeword  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16x3"
tol = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-3
B = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
onnx = os.path.join(REPO, "tests", "golden", "xiaoa.onnx")
m = wakeword.load_onnx(onnx, precision=prec)
m32 = wakeword.load_onnx(onnx)
x = wakeword.synth_clips(1234, 0, B)
G = torch.cuda.get_device_properties(0).multi_processor_count
b = m32.detect(x).reshape(-1)
a = m.detect(x).reshape(-1)
a2 = m.detect(x).reshape(-1)
import ctypes as C
from wakeword import _lib
fl = C.c_uint32(0)
st = _lib.lib().wk_check_device_errors(m._h.h, C.byref(fl))
print(f"device error check: status {st} flags {fl.value}")
print(f"{prec}: repeat identical: {bool((a == a2).all())}; max |d| vs fp32 {(a - b).abs().max().item():.3g}")
bad = ((a - b).abs() > tol).nonzero().flatten().tolist()
print(f"{len(bad)} clips over {tol}")
from collections import Counter
print("iter", Counter(i // G for i in bad).most_common(10))
print("batch clip", Counter((i // G) % 4 for i in bad).most_common(4))
print("slot", Counter(i % G for i in bad).most_common(10))
for i in bad[:12]:
    print(f"  clip {i}: slot {i % G} iter {i // G} batch {(i // G) // 4} pos {(i // G) % 4}: {b[i].item():.5f} -> {a[i].item():.5f}")
