"""For clips whose features differ from the clean fp32 run, test whether the
corrupted features equal another clip's clean features (diagnostic)."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]
import torch  # noqa: E402
import wakeword  # noqa: E402
from wakeword import _lib  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
B = 65536
onnx = os.path.join(REPO, "tests", "golden", "xiaoa.onnx")
x = wakeword.synth_clips(1234, 0, B)
L = _lib.lib()
st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
G = torch.cuda.get_device_properties(0).multi_processor_count


def run(m):
    lg = torch.empty(B, device="cuda")
    ft = torch.empty((B, 13, 63), device="cuda")
    _lib.check(L.wk_forward(m._h.h, C.c_void_p(x.data_ptr()), 0, B, 16000, 16000, C.c_void_p(lg.data_ptr()),
                            C.c_void_p(ft.data_ptr()), st), "fwd")
    torch.cuda.synchronize()
    return lg, ft


_, f0 = run(wakeword.load_onnx(onnx))
_, f1 = run(wakeword.load_onnx(onnx, precision=prec))
bad = (f1 != f0).reshape(B, -1).any(1).nonzero().flatten().tolist()
print(f"{len(bad)} clips with different features")
flat0 = f0.reshape(B, -1)
for i in bad[:10]:
    d = (flat0 - f1[i].reshape(1, -1)).abs().max(1).values
    j = int(d.argmin())
    print(f"clip {i} (slot {i % G} iter {i // G}): closest clean clip {j} (slot {j % G} iter {j // G}) "
          f"max|d| {d[j].item():.3g}; own {d[i].item():.3g}")
    # per-frame: which frames differ
    fr = (f1[i] != f0[i]).any(0).nonzero().flatten().tolist()
    print(f"   frames differing: {len(fr)}: {fr[:10]}")
