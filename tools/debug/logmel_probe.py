"""Where does a clip's log-mel go wrong?  Needs a -DWK_DEBUG_LOGMEL library
(WAKEWORD_LIB): the fused kernel copies each clip's log-mel image as the
front-end left it (after all 8 front-end waves finished its mel) and as the
DCT read it.  Compares both with a clean run (fp32 convolutions)."""
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
G = torch.cuda.get_device_properties(0).multi_processor_count


def run(m):
    fe = torch.full((B, 40, 64), float("nan"), device="cuda")
    cn = torch.full((B, 40, 64), float("nan"), device="cuda")
    assert L.wk_debug_logmel_set(C.c_void_p(fe.data_ptr()), C.c_void_p(cn.data_ptr())) == 0
    lg = m.detect(x)
    torch.cuda.synchronize()
    return lg, fe, cn


l0, fe0, cn0 = run(wakeword.load_onnx(onnx))
l1, fe1, cn1 = run(wakeword.load_onnx(onnx, precision=prec))
ok = ~torch.isnan(fe0[:, 0, 0])
print("fe copies present:", int(ok.sum()), "of", B)
sel = lambda t: t[..., :63]   # column 63 is the padding frame
d_fe = (sel(fe1) != sel(fe0)).reshape(B, -1).any(1) & ok
d_cn = (sel(cn1) != sel(cn0)).reshape(B, -1).any(1)
print(f"clean run: fe vs cnn copies differ in {int(((sel(fe0) != sel(cn0)).reshape(B, -1).any(1) & ok).sum())} clips")
print(f"{prec} run: fe vs cnn copies differ in {int(((sel(fe1) != sel(cn1)).reshape(B, -1).any(1) & ok).sum())} clips")
print(f"{prec} vs clean: fe copy differs in {int(d_fe.sum())} clips, cnn copy in {int(d_cn.sum())} clips")
bad = d_cn.nonzero().flatten().tolist()
for i in bad[:6]:
    dd = (sel(cn1[i]) != sel(cn0[i]))
    rows = dd.any(1).nonzero().flatten().tolist()
    cols = dd.any(0).nonzero().flatten().tolist()
    print(f" clip {i} (slot {i % G} iter {i // G} pos {(i // G) % 4}): mel rows {rows}, frames {cols[:16]}..., "
          f"fe-copy differs: {bool(d_fe[i])}, max|d| {(sel(cn1[i]) - sel(cn0[i])).abs().max().item():.3g}")

from collections import Counter
fr, rw, nfr = Counter(), Counter(), Counter()
for i in bad:
    dd = (sel(cn1[i]) != sel(cn0[i]))
    cols = dd.any(0).nonzero().flatten().tolist()
    nfr[len(cols)] += 1
    for c in cols:
        fr[c] += 1
    for r in dd.any(1).nonzero().flatten().tolist():
        rw[r] += 1
print("frames per bad clip:", sorted(nfr.items()))
print("frame histogram:", sorted(fr.items()))
print("mel-row histogram:", sorted(rw.items()))
