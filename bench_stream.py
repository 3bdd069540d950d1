"""Streaming benchmark, SURVEY 8(d) config 3 (not the driver's bench.py line).

One continuous 16 kHz stream (default 60 s, the device generator's clips laid
end to end), 1 s windows every 30 ms (hop 480):
  * latency: the stream is pushed hop by hop through wk_stream_push (host
    samples -> device ring -> fused kernel on the newest window -> logit on the
    host); per-push wall time = window available on host -> logit on host.
    p50 / p90 / p99 reported.
  * throughput: the whole backlog as one strided launch over the resident
    stream (clip_stride = hop, overlapping windows), windows/s.
Prints one JSON line."""
import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]


def run_stream(seconds=60, hop=480, backlog_seconds=3600, device=0, model=None):
    """Config 3: push latency (p50/p90/p99) and backlog throughput; returns the line's dict."""
    import numpy as np
    import torch
    import wakeword
    from wakeword import _lib

    if model is None:
        model = wakeword.load_onnx(os.path.join(REPO, "tests", "golden", "xiaoa.onnx"), device=device)
    audio = wakeword.synth_clips(1234, 0, seconds, device=device).reshape(-1).cpu().numpy()
    det = wakeword.StreamingDetector(model, hop=hop)
    lat = []
    for p in range(0, audio.size, hop):
        t0 = time.perf_counter()
        out = det.push(audio[p:p + hop])
        if out:
            lat.append(time.perf_counter() - t0)
    det.close()
    lat = np.asarray(lat[10:]) * 1e3   # drop warm-up pushes

    # throughput: a long resident stream scored as one backlog of overlapping windows
    dev = wakeword.synth_clips(1234, 0, backlog_seconds, device=device).reshape(-1)
    n = (dev.numel() - 16000) // hop + 1
    logits = torch.empty(n, dtype=torch.float32, device=dev.device)
    st = torch.cuda.current_stream(dev.device)

    def run():
        _lib.check(_lib.lib().wk_forward(model._h.h, C.c_void_p(dev.data_ptr()), _lib.WK_DTYPE_F32, n, 16000,
                                         hop, C.c_void_p(logits.data_ptr()), None,
                                         C.c_void_p(st.cuda_stream)), "wk_forward")
    run()
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    thr = n * reps / (time.perf_counter() - t0)
    return {
        "metric": "streaming 1 s windows @ 30 ms hop (config 3)",
        "p50_latency_ms": round(float(np.percentile(lat, 50)), 4),
        "p90_latency_ms": round(float(np.percentile(lat, 90)), 4),
        "p99_latency_ms": round(float(np.percentile(lat, 99)), 4),
        "latency_windows": int(lat.size),
        "throughput_windows_per_s": round(thr, 1),
        "throughput_stream_seconds": backlog_seconds,
        "realtime_factor": round(thr * hop / 16000.0, 1),
        "hop": hop, "dtype": "f32", "data": "synthetic stream (device generator clips end to end)",
        "n_gpus": 1}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=int, default=60)
    ap.add_argument("--hop", type=int, default=480)
    ap.add_argument("--backlog-seconds", type=int, default=3600, help="stream length for the throughput leg")
    args = ap.parse_args()
    print(json.dumps(run_stream(args.seconds, args.hop, args.backlog_seconds)))


if __name__ == "__main__":
    main()
