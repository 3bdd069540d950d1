"""Time the standalone front-end kernel (wk_mfcc, mode B + CMVN; 8-wave
workgroups, 2 per CU) on the bench workload, for comparison with the fused
kernel's front-end role alone (WAKEWORD_FUSED_EXP=1)."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]
import torch  # noqa: E402
import wakeword  # noqa: E402
from wakeword import _lib  # noqa: E402
from wakeword.api import _frontend_handle  # noqa: E402

B = 65536
x = wakeword.synth_clips(1234, 0, B)
out = torch.empty((B, 13, 63), device="cuda")
h = _frontend_handle(_lib.WK_MODE_TORCHAUDIO_CMVN, 0, 1, 1)
L = _lib.lib()
st = torch.cuda.current_stream()
sp = C.c_void_p(st.cuda_stream)


def run():
    _lib.check(L.wk_mfcc(h.h, C.c_void_p(x.data_ptr()), 0, B, 16000, 16000, C.c_void_p(out.data_ptr()), sp), "mfcc")


for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
n = 10
e0.record(st)
for _ in range(n):
    run()
e1.record(st)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / n
print(f"standalone front-end: {ms:.4f} ms per {B} clips = {B / ms / 1e3:.2f} M clips/s")
