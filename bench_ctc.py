"""CTC-head benchmark, SURVEY 8(d) config 5 (not the driver's bench.py line).

B utterances of 3 s (48,000 samples, T = 301 frames at hop 160), synthetic
(device generator), seeded GRU_CTC_Model weights (the reference ships none),
fixed V.  One step = log-mel front-end + encoder + 2-layer BiGRU + output
layer + argmax + greedy decode, inputs resident in HBM and the token
sequences left there (CTCModel.decode; forward() adds the host list form).  Prints
one JSON line with utterances/s, the per-stage split, and the torch-CPU
oracle timed on a bounded sample of the same workload."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--vocab", type=int, default=4000)
    ap.add_argument("--seconds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-utts", type=int, default=8)
    ap.add_argument("--precision", default="fp16", choices=["fp32", "fp16"],
                    help="GEMM operand precision (config 5 names fp16; fp32 is the parity mode)")
    args = ap.parse_args()
    import torch
    import wakeword
    from oracle import wk_ctc_oracle as CO

    n = args.seconds * 16000
    m = CO.make_model(args.vocab, seed=0)
    g = wakeword.CTCModel(CO.flat_weights(m), args.vocab, precision=args.precision)
    audio = wakeword.synth_clips(1234, 0, args.batch, n)
    for _ in range(args.warmup):
        g.transcribe(audio, n_samples=n)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    t_fe = t_all = 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ev[0].record()
        f = g.features(audio, n_samples=n)
        ev[1].record()
        g.decode(f)   # tokens + lengths stay in HBM (the host list form is forward())
        ev[2].record()
        torch.cuda.synchronize()
        t_fe += ev[0].elapsed_time(ev[1])
        t_all += ev[0].elapsed_time(ev[2])
    el = time.perf_counter() - t0
    value = args.batch * args.steps / el

    # CPU baseline: the torch-CPU oracle on a bounded sample
    x = torch.from_numpy(audio[:args.cpu_utts].cpu().numpy())
    with torch.no_grad():
        CO.greedy_decode(m(CO.features(x[:1])))
        c0 = time.perf_counter()
        CO.greedy_decode(m(CO.features(x)))
        cpu = args.cpu_utts / (time.perf_counter() - c0)
    print(json.dumps({
        "metric": "CTC utterances/s (3 s @16 kHz, log-mel 80 -> BiGRU x2 H128 -> greedy CTC), config 5",
        "value": round(value, 1), "unit": "utterances/s", "audio_seconds_per_s": round(value * args.seconds, 1),
        "batch": args.batch, "vocab": args.vocab, "T": 1 + n // 160, "steps": args.steps,
        "ms_per_step": round(el / args.steps * 1e3, 3), "frontend_ms": round(t_fe / args.steps, 3),
        "model_ms": round((t_all - t_fe) / args.steps, 3),
        "dtype": "f32" if args.precision == "fp32" else "f16 GEMM operands / f32 accumulate + recurrence",
        "data": "synthetic (device generator), seeded weights",
        "cpu_baseline": {"value": round(cpu, 2), "unit": "utterances/s", "cores": torch.get_num_threads(),
                         "kind": "port", "sample": f"{args.cpu_utts} utterances, torch-CPU oracle (oracle/wk_ctc_oracle.py)"},
    }))


if __name__ == "__main__":
    main()
