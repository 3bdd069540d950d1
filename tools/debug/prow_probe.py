"""Power-row snapshots of the fused kernel (the K = 32
question), from a library built with -DWK_DIAG_PROW (tools/debug/build_variant.sh
<name> -DWK_DIAG_PROW [-DWK_MFMA_K32 -DWK_ALLOW_K32_DIAG]).  Diagnostic tool,
not a test.

For each of `n` full-size launches (65,536 clips, precision bf16 by default)
the kernel records, for the first P = 32 clips of every workgroup (clip
b + 256 i of workgroup b, i < P; -DWK_PROW_CLIPS), A = the power
bins each front-end lane wrote (read back right after its round), B = the
rows just before the mel, C = the rows after the mel.  Printed:
  * within each launch, the (clip, frame) rows where A != B or B != C: the
    LDS changed between the front-end's write and the mel's read;
  * across launches, the rows where A differs from launch 0's A: the
    front-end computed different power values from the same audio.
"""
import ctypes as C
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(R, "esp32-wake-word_amd"))

import torch  # noqa: E402
import wakeword  # noqa: E402
from wakeword import _lib  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
L = _lib.lib()
L.wk_debug_prow_buffer.argtypes = [C.c_void_p]
L.wk_debug_lmel_buffer.argtypes = [C.c_void_p]
L.wk_debug_epi_bad.argtypes = [C.c_void_p, C.c_int]
m = wakeword.load_onnx(os.path.join(R, "tests", "golden", "xiaoa.onnx"), precision=prec)
x = wakeword.synth_clips(777, 0, 65536, device=0)
grid = 256   # (the fused launch's grid on a 256-CU MI355X: min(batch, n_cu))
P = int(os.environ.get("WK_PROW_CLIPS", "32"))
buf = torch.full((3, grid * P, 64, 257), float("nan"), dtype=torch.float32, device="cuda:0")
# slot s = b * P + i  <->  global clip b + grid * i
slot_clip = np.array([(s_ // P) + grid * (s_ % P) for s_ in range(grid * P)])
lbuf = torch.full((2, grid * P, 40, 64), float("nan"), dtype=torch.float32, device="cuda:0")
assert L.wk_debug_prow_buffer(C.c_void_p(buf.data_ptr())) == 0
assert L.wk_debug_lmel_buffer(C.c_void_p(lbuf.data_ptr())) == 0
bad = C.c_uint(0)
L.wk_debug_epi_bad(C.byref(bad), 1)
snaps, lsnaps, logits = [], [], []
for _ in range(n):
    buf.fill_(float("nan"))
    lbuf.fill_(float("nan"))
    lg, _f = m.detect(x, return_features=True)
    torch.cuda.synchronize()
    snaps.append(buf[:, :, :63].cpu().numpy().copy())
    lsnaps.append(lbuf[:, :, :, :63].cpu().numpy().copy())
    logits.append(lg.reshape(-1).cpu().numpy().copy())
L.wk_debug_prow_buffer(None)
L.wk_debug_lmel_buffer(None)
L.wk_debug_epi_bad(C.byref(bad), 1)
print(f"epilogue bounds check over {n} launches: {'an epilogue store left its image' if bad.value else 'every store inside its image'}")
m.check_device_errors()
tag = os.path.basename(os.path.dirname(os.environ.get("WAKEWORD_LIB", "prod")))
for r, s in enumerate(snaps):
    a, b, c = s
    ab = ~((a == b) | (np.isnan(a) & np.isnan(b)))
    bc = ~((b == c) | (np.isnan(b) & np.isnan(c)))
    rows_ab = int(ab.any(axis=2).sum())
    rows_bc = int(bc.any(axis=2).sum())
    da = ~((a == snaps[0][0]) | (np.isnan(a) & np.isnan(snaps[0][0])))
    rows_a0 = int(da.any(axis=2).sum())
    clips_lg = int((logits[r] != logits[0]).sum())
    msg = (f"{tag} {prec} launch {r}: rows with A!=B {rows_ab}, B!=C {rows_bc}; rows whose A differs from launch 0 "
           f"{rows_a0} (of {a.shape[0] * a.shape[1]}); clips whose logit differs from launch 0 {clips_lg} (of 65536)")
    diff_clips = logits[r] != logits[0]
    mon = diff_clips[slot_clip]                     # monitored slots whose logit differs
    a_rows = da.any(axis=2).any(axis=1)             # slots whose power rows (A) differ from launch 0
    msg += (f"; monitored clips {len(slot_clip)}, of them logit differs {int(mon.sum())}, "
            f"power rows (A) differ {int(a_rows.sum())}, both {int((mon & a_rows).sum())}")
    d, e = lsnaps[r]
    de = ~((d == e) | (np.isnan(d) & np.isnan(e)))
    dl = ~((d == lsnaps[0][0]) | (np.isnan(d) & np.isnan(lsnaps[0][0])))
    msg += (f"; log-mel images: D!=E (hand-off) {int(de.any(axis=(1, 2)).sum())} of {d.shape[0]}, "
            f"D differs from launch 0 {int(dl.any(axis=(1, 2)).sum())} (of them logit differs "
            f"{int((dl.any(axis=(1, 2)) & mon).sum())})")
    print(msg, flush=True)
    if rows_ab:
        cl, fr = np.nonzero(ab.any(axis=2))
        print("   A!=B at (clip slot, frame):", list(zip(cl[:8].tolist(), fr[:8].tolist())),
              "bins:", np.nonzero(ab[cl[0], fr[0]])[0][:16].tolist())
    if rows_a0:
        cl, fr = np.nonzero(da.any(axis=2))
        bins = np.nonzero(da[cl[0], fr[0]])[0]
        print("   A differs at (clip slot, frame):", list(zip(cl[:8].tolist(), fr[:8].tolist())), "bins:", bins[:16].tolist(),
              "frames hist:", np.bincount(fr, minlength=63).tolist())
