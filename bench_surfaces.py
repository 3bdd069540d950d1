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
    ap.add_argument("--cpu-clips", type=int, default=4096,
                    help="clips in the mode-A CPU baseline sample (0: skip)")
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
    if args.cpu_clips > 0:
        # the mode-A front-end (mfcc.c) on the host, single-threaded
        # and on the host's cores, beside wk_mfcc mode A: the C restatement
        # (oracle/esp_mfcc_oracle.c, float radix-2 FFT path) on the same clips
        import time
        from oracle import build_oracle as EO
        xs = x[:args.cpu_clips].cpu().numpy()
        cores = min(16, len(os.sched_getaffinity(0)))
        res = {}
        for nt, n in ((1, max(1, args.cpu_clips // 8)), (cores, args.cpu_clips)):
            EO.esp_mfcc_batch(xs[:min(n, 64)], n_threads=nt)
            t0 = time.perf_counter()
            EO.esp_mfcc_batch(xs[:n], n_threads=nt)
            res[f"threads_{nt}"] = round(n / (time.perf_counter() - t0), 1)
        gpu = out["wk_mfcc_mode_a"]["windows_per_s"]
        out["cpu_baseline_mode_a"] = {
            "value": res[f"threads_{cores}"], "unit": "windows/s", "cores": cores, "kind": "port",
            "single_thread": res["threads_1"], "gpu_over_cpu": round(gpu / res[f"threads_{cores}"], 1),
            "sample": f"{args.cpu_clips} clips ({max(1, args.cpu_clips // 8)} single-threaded) of the device "
                      "generator, mfcc.c restated in C with a float radix-2 FFT (oracle/esp_mfcc_oracle.c, "
                      "esp_mfcc_oracle_batch), gcc -O2, pthreads"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
