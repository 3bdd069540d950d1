"""Where does a streaming push's latency go?  (diagnostic)
kernel: fused kernel duration for one window (HIP events); launch+sync: one
wk_forward on a resident window + stream sync, wall; push: wk_stream_push wall
(C call only) and StreamingDetector.push wall (Python)."""
import ctypes as C
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import wakeword  # noqa: E402
from wakeword import _lib  # noqa: E402

m = wakeword.load_onnx(os.path.join(REPO, "tests", "golden", "xiaoa.onnx"))
L = _lib.lib()
x = wakeword.synth_clips(1, 0, 4)
lg = torch.empty(4, device="cuda")
st = torch.cuda.current_stream()
sp = C.c_void_p(st.cuda_stream)


def fwd(b=1):
    L.wk_forward(m._h.h, C.c_void_p(x.data_ptr()), 0, b, 16000, 16000, C.c_void_p(lg.data_ptr()), None, sp)


for b in (1, 2, 4):
    ts = []
    for i in range(200):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fwd(b)
        e1.record(st)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    print(f"kernel (events) batch {b}: p50 {np.percentile(ts[20:], 50):.1f} us")
ts = []
for i in range(300):
    t0 = time.perf_counter()
    fwd()
    st.synchronize()
    ts.append((time.perf_counter() - t0) * 1e6)
print(f"wk_forward + sync wall: p50 {np.percentile(ts[20:], 50):.1f} us")
ts = []
for i in range(300):
    t0 = time.perf_counter()
    fwd()
    while not st.query():
        pass
    ts.append((time.perf_counter() - t0) * 1e6)
print(f"wk_forward + spin on hipStreamQuery wall: p50 {np.percentile(ts[20:], 50):.1f} us")
for name, wait in (("sync", st.synchronize), ("spin", lambda: [None for _ in iter(st.query, True)])):
    ts = []
    for i in range(300):
        t0 = time.perf_counter()
        lg.zero_()
        wait()
        ts.append((time.perf_counter() - t0) * 1e6)
    print(f"trivial kernel (fill) + {name} wall: p50 {np.percentile(ts[20:], 50):.1f} us")
det = wakeword.StreamingDetector(m, hop=480)
audio = wakeword.synth_clips(1234, 0, 20).reshape(-1).cpu().numpy()
det.push(audio[:16000])
ts, tc = [], []
buf = np.zeros(64, np.float32)
ends = np.zeros(64, np.int64)
n = C.c_int32(0)
for p in range(16000, audio.size, 480):
    chunk = np.ascontiguousarray(audio[p:p + 480])
    t0 = time.perf_counter()
    L.wk_stream_push(det._s, chunk.ctypes.data_as(C.POINTER(C.c_float)), chunk.size,
                     buf.ctypes.data_as(C.POINTER(C.c_float)), ends.ctypes.data_as(C.POINTER(C.c_int64)), 64,
                     C.byref(n))
    tc.append((time.perf_counter() - t0) * 1e6)
print(f"wk_stream_push (C call) wall: p50 {np.percentile(tc[20:], 50):.1f} us")
for p in range(0, audio.size, 480):
    t0 = time.perf_counter()
    det.push(audio[p:p + 480])
    ts.append((time.perf_counter() - t0) * 1e6)
print(f"StreamingDetector.push wall: p50 {np.percentile(ts[40:], 50):.1f} us")
