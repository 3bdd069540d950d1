"""K=32 bf16 MFMA corruption probe.  Repeats one full-size
fused launch with the feature output on and, on a -DWK_DEBUG_LOGMEL library,
the log-mel image of every clip as the front-end left it (fe) and as the DCT
read it (cnn).  For every clip whose features change between repeats it
reports whether the log-mel the DCT read changed (buffer overwritten before
or during the DCT's read) or not (the DCT / its MFMAs computed differently
from the same input), and whether the front-end's own copy changed.

    WAKEWORD_LIB=<variant .so> python tools/debug/k32_probe.py [bf16|bf16x3] [reps]
"""
import ctypes as C
import os
import sys
from collections import Counter

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]
import torch  # noqa: E402
import wakeword  # noqa: E402
from wakeword import _lib  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
B = 65536
m = wakeword.load_onnx(os.path.join(REPO, "tests", "golden", "xiaoa.onnx"), precision=prec)
x = wakeword.synth_clips(1234, 0, B)
L = _lib.lib()
dbg = hasattr(L, "wk_debug_logmel_set")
st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
G = torch.cuda.get_device_properties(0).multi_processor_count
print(f"precision {prec}, {reps} repeats, debug log-mel copies: {dbg}, lib {_lib.LIB_PATH}", flush=True)


def run():
    lg = torch.empty(B, device="cuda")
    ft = torch.empty((B, 13, 63), device="cuda")
    fe = cn = None
    if dbg:
        fe = torch.full((B, 40, 64), float("nan"), device="cuda")
        cn = torch.full((B, 40, 64), float("nan"), device="cuda")
        assert L.wk_debug_logmel_set(C.c_void_p(fe.data_ptr()), C.c_void_p(cn.data_ptr())) == 0
    _lib.check(L.wk_forward(m._h.h, C.c_void_p(x.data_ptr()), 0, B, 16000, 16000, C.c_void_p(lg.data_ptr()),
                            C.c_void_p(ft.data_ptr()), st), "fwd")
    torch.cuda.synchronize()
    return lg, ft, fe, cn


def rows_differ(a, b):
    a, b = a[..., :63], b[..., :63]
    return ((a != b) & ~(torch.isnan(a) & torch.isnan(b))).reshape(a.shape[0], -1).any(1)


lg0, ft0, fe0, cn0 = run()
tot = Counter()
for r in range(reps):
    lg, ft, fe, cn = run()
    bad = (ft != ft0).reshape(B, -1).any(1)
    idx = bad.nonzero().flatten().tolist()
    line = f"rep {r}: {len(idx)} clips with changed features, {int((lg != lg0).sum())} changed logits"
    if dbg:
        have = ~torch.isnan(fe[:, 0, 0])
        cn_chg = rows_differ(cn, cn0)
        fe_chg = rows_differ(fe, fe0) & have
        self_mis = rows_differ(cn, fe) & have
        line += (f"; cnn-copy changed in {int(cn_chg.sum())}, fe-copy changed in {int(fe_chg.sum())}, "
                 f"cnn != fe (same run) in {int(self_mis.sum())}")
        for i in idx:
            key = ("cnn-in changed" if bool(cn_chg[i]) else "cnn-in same") + "/" + \
                  ("fe changed" if bool(fe_chg[i]) else ("fe same" if bool(have[i]) else "fe n/a"))
            tot[key] += 1
    print(line, flush=True)
    for i in idx[:3]:
        d = ft[i] != ft0[i]
        msg = (f"   clip {i}: slot {i % G} iter {i // G} (batch clip {(i // G) % 4}) coef {d.any(1).nonzero().flatten().tolist()} "
               f"frames {d.any(0).nonzero().flatten().tolist()[:12]} max|d| {(ft[i] - ft0[i]).abs().max().item():.3g}")
        if dbg:
            dc = (cn[i, :, :63] != cn0[i, :, :63])
            msg += (f"; cnn-in differs at mel {dc.any(1).nonzero().flatten().tolist()[:8]} "
                    f"frames {dc.any(0).nonzero().flatten().tolist()[:12]}")
        print(msg, flush=True)
print("classification of changed clips:", dict(tot))
if hasattr(L, "wk_debug_epi_get"):
    bad = (C.c_uint32 * 8)()
    assert L.wk_debug_epi_get(bad, 0) == 0
    print("epilogue stores out of bounds:", bad[0], "first (kind, lane, co0, clip, t0/r, idx, lim):", list(bad)[1:])
m.check_device_errors()
