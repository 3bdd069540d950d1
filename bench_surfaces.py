"""Throughput of the drop-in call surfaces besides the fused hot path (not the
driver's bench.py line): the front-end alone (wk_mfcc, both definitions) and the
CNN alone on given features (wk_cnn = LightweightKWS.forward / ONNX run).
Inputs resident in HBM, B clips per launch, HIP-event timing on the launch
stream.  Prints one JSON line."""
import argparse
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    import torch
    import wakeword
    from wakeword import _lib
    L = _lib.lib()
    B = args.batch
    st = torch.cuda.current_stream()
    sp = C.c_void_p(st.cuda_stream)
    x = wakeword.synth_clips(1234, 0, B)
    feats = torch.empty((B, 13, 63), device="cuda")
    logits = torch.empty(B, device="cuda")

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(args.steps):
            fn()
        e1.record(st)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / args.steps
        return {"ms": round(ms, 4), "windows_per_s": round(B / (ms * 1e-3), 1)}

    out = {"metric": "call-surface throughput (windows/s, 1 MI355X)", "batch": B}
    hb = wakeword.api._frontend_handle(_lib.WK_MODE_TORCHAUDIO_CMVN, 0, 1, 1)
    out["wk_mfcc_mode_b_cmvn"] = timed(lambda: _lib.check(L.wk_mfcc(
        hb.h, C.c_void_p(x.data_ptr()), 0, B, 16000, 16000, C.c_void_p(feats.data_ptr()), sp), "wk_mfcc"))
    featsA = torch.empty((B, 62, 13), device="cuda")
    ha = wakeword.api._frontend_handle(_lib.WK_MODE_ESP_MFCC, 0, 1, 0)
    out["wk_mfcc_mode_a"] = timed(lambda: _lib.check(L.wk_mfcc(
        ha.h, C.c_void_p(x.data_ptr()), 0, B, 16000, 16000, C.c_void_p(featsA.data_ptr()), sp), "wk_mfcc"))
    for prec in ("fp32", "int8"):
        m = wakeword.load_onnx(os.path.join(REPO, "tests", "golden", "xiaoa.onnx"), precision=prec)
        out[f"wk_cnn_{prec}"] = timed(lambda: _lib.check(L.wk_cnn(
            m._h.h, C.c_void_p(feats.data_ptr()), B, C.c_void_p(logits.data_ptr()), sp), "wk_cnn"))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
