"""Health of the fused kernel's role hand-off protocol and the handle's shared
state:
- every bounded spin that times out raises a flag in the handle's host-visible
  error word; wk_check_device_errors reports it (clean runs must read 0);
- the INT8 / unfused path's per-handle feature workspace is ordered across
  streams, so one handle used from two streams gives the single-stream logits."""
import ctypes as C
import os

import numpy as np
import pytest

from oracle import wk_oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("precision", ["fp32", "bf16", "bf16x3"])
def test_error_word_clean_at_scale(gpu, golden_dir, precision):
    import wakeword
    from wakeword import _lib
    m = wakeword.load_onnx(os.path.join(golden_dir, "xiaoa.onnx"), precision=precision)
    x = wakeword.synth_clips(99, 0, 65536, device=0)
    for _ in range(3):
        m.detect(x)
    feats = wakeword.mfcc(x[:8192])
    for _ in range(3):
        m(feats)                # wk_cnn: the same CNN role, two per workgroup, reports to the same word
    flags = C.c_uint32(123)
    assert _lib.lib().wk_check_device_errors(m._h.h, C.byref(flags)) == 0
    assert flags.value == 0
    m.check_device_errors()   # the Python surface raises on a nonzero word


def test_check_device_errors_rejects_null_handle(gpu):
    from wakeword import _lib
    assert _lib.lib().wk_check_device_errors(None, None) == 1


def test_int8_workspace_ordered_across_streams(gpu, golden_dir):
    """Two streams, one INT8 handle, no caller-side sync between them: each
    call's features go through the handle's workspace, which the library
    orders with an event.  Results equal the one-stream results."""
    import torch
    import wakeword
    m = wakeword.load_onnx(os.path.join(golden_dir, "xiaoa.onnx"), precision="int8")
    xa = torch.from_numpy(O.synth_clips(5, 0, 20000, 16000)).cuda()
    xb = torch.from_numpy(O.synth_clips(6, 0, 20000, 16000)).cuda()
    ref_a = m.detect(xa).clone()
    ref_b = m.detect(xb).clone()
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for _ in range(3):
        with torch.cuda.stream(s1):
            a = m.detect(xa)
        with torch.cuda.stream(s2):
            b = m.detect(xb)
        outs.append((a, b))
    torch.cuda.synchronize()
    for a, b in outs:
        assert torch.equal(a, ref_a) and torch.equal(b, ref_b)
