"""Repeat one full-size fused launch with the feature output enabled and report
which clips' features / logits change between repeats (diagnostic)."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]
import torch  # noqa: E402
import wakeword  # noqa: E402
from wakeword import _lib  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16x3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
B = 65536
m = wakeword.load_onnx(os.path.join(REPO, "tests", "golden", "xiaoa.onnx"), precision=prec)
x = wakeword.synth_clips(1234, 0, B)
L = _lib.lib()
st = C.c_void_p(torch.cuda.current_stream().cuda_stream)


def run():
    lg = torch.empty(B, device="cuda")
    ft = torch.empty((B, 13, 63), device="cuda")
    _lib.check(L.wk_forward(m._h.h, C.c_void_p(x.data_ptr()), 0, B, 16000, 16000, C.c_void_p(lg.data_ptr()),
                            C.c_void_p(ft.data_ptr()), st), "fwd")
    torch.cuda.synchronize()
    return lg, ft


lg0, ft0 = run()
G = torch.cuda.get_device_properties(0).multi_processor_count
for r in range(reps):
    lg, ft = run()
    dl = (lg != lg0).nonzero().flatten().tolist()
    df = (ft != ft0).reshape(B, -1).any(1).nonzero().flatten().tolist()
    print(f"rep {r}: logits differ at {dl[:8]}, features differ at {df[:8]}", flush=True)
    for i in df[:4]:
        d = (ft[i] != ft0[i])
        rows = d.any(1).nonzero().flatten().tolist()
        cols = d.any(0).nonzero().flatten().tolist()
        print(f"   clip {i}: slot {i % G} iter {i // G} (batch clip {(i // G) % 4}) logit {lg0[i].item():.5f} -> "
              f"{lg[i].item():.5f}; coefficients {rows}, frames {cols[:20]}{'...' if len(cols) > 20 else ''}, "
              f"max |d| {(ft[i] - ft0[i]).abs().max().item():.3g}")
