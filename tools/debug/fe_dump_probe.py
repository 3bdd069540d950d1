"""Front-end register dumps of the fused kernel (the K = 32
question), from a library built with -DWK_DIAG -DWK_DIAG_PROW
-DWK_PROW_CLIPS=4 -DWK_DIAG_FEDUMP [-DWK_DIAG_K32_SPIN=0|1 -DWK_ALLOW_K32_DIAG]
and run with WAKEWORD_FUSED_EXP=1 (front-end role alone, the CNN waves
replaced by the bare MFMA stream).  Diagnostic tool, not a test.

For `n` full-size launches the kernel stores, for the first P clips of every
workgroup, each front-end lane's 16 complex registers at four points of
fe_rest (k = 0 stage-0 output, 1 after the first DFT16, 2 after the LDS
transpose, 3 after the second DFT16).  Printed per launch and point: how many
(clip, frame) blocks differ from launch 0, and for the first point where they
do, the lanes (0-15 of the frame's group) and registers that differ.
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
P = int(os.environ.get("WK_PROW_CLIPS", "4"))
L = _lib.lib()
L.wk_debug_fe_buffer.argtypes = [C.c_void_p]
m = wakeword.load_onnx(os.path.join(R, "tests", "golden", "xiaoa.onnx"), precision=prec)
x = wakeword.synth_clips(777, 0, 65536, device=0)
grid = 256
buf = torch.full((grid * P, 64, 4, 16, 32), float("nan"), dtype=torch.float32, device="cuda:0")
assert L.wk_debug_fe_buffer(C.c_void_p(buf.data_ptr())) == 0
snaps = []
for _ in range(n):
    buf.fill_(float("nan"))
    m.detect(x)
    torch.cuda.synchronize()
    snaps.append(buf[:, :63].cpu().numpy().copy())
L.wk_debug_fe_buffer(None)
m.check_device_errors()
tag = os.path.basename(os.path.dirname(os.environ.get("WAKEWORD_LIB", "prod")))
ref = snaps[0]
for r in range(1, n):
    s = snaps[r]
    diff = ~((s == ref) | (np.isnan(s) & np.isnan(ref)))       # [clip, frame, k, lane, 32]
    per_k = [int(diff[:, :, k].any(axis=(2, 3)).sum()) for k in range(4)]
    print(f"{tag} launch {r}: (clip, frame) blocks differing from launch 0 at points 0-3: {per_k} "
          f"(of {s.shape[0] * s.shape[1]})", flush=True)
    for k in range(4):
        blk = diff[:, :, k].any(axis=(2, 3))
        if not blk.any():
            continue
        fr = np.nonzero(blk)[1]
        lanes = diff[:, :, k].any(axis=(0, 1, 3))
        regs = diff[:, :, k].any(axis=(0, 1, 2))
        first_k_only = blk & ~(diff[:, :, k - 1].any(axis=(2, 3)) if k else np.zeros_like(blk))
        print(f"   point {k}: frames {np.bincount(fr, minlength=63)[44:].tolist()} (from 44), "
              f"lanes {np.nonzero(lanes)[0].tolist()}, floats {np.nonzero(regs)[0].tolist()}, "
              f"new at this point {int(first_k_only.sum())}", flush=True)
        if k == int(np.argmax([v > 0 for v in per_k])):
            c, f = np.argwhere(first_k_only)[0] if first_k_only.any() else np.argwhere(blk)[0]
            d = diff[c, f, k]
            print(f"   first block (clip slot {c}, frame {f}): lanes {np.nonzero(d.any(1))[0].tolist()}, "
                  f"floats {np.nonzero(d.any(0))[0].tolist()}; values now/launch 0 (lane, float): "
                  + ", ".join(f"({l},{q}) {s[c, f, k, l, q]:.6g}/{ref[c, f, k, l, q]:.6g}"
                              for l, q in np.argwhere(d)[:6]), flush=True)
