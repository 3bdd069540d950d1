"""CTC-head benchmark, SURVEY 8(d) config 5 (not the driver's bench.py line).

B utterances of 3 s (48,000 samples, T = 301 frames at hop 160), synthetic
(device generator), seeded GRU_CTC_Model weights (the reference ships none),
fixed V.  One step = log-mel front-end + encoder + 2-layer BiGRU + output
layer + argmax + greedy decode, inputs resident in HBM and the token
sequences left there: one wk_ctc_transcribe call (CTCModel.decode_audio; in
fp16 mode the z-score is folded into the encoder), or with --separate the
reference's two steps, wk_ctc_features then wk_ctc_forward.

Prints one JSON line: utterances/s over the timed steps, and per stage (HIP
events on the launch stream, wk_ctc_profile) the mean duration with its
algorithmic bytes or flops against the MI355X roofline that bounds it, the
PMC-measured HBM traffic (profiles/ctc_hbm_traffic.json) and which stages are
library code; `roofline` is the dominant stage's.  The torch-CPU oracle is
timed on a bounded sample of the same workload as the reported CPU baseline.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]

PEAK_HBM_GBS = 8000.0
PEAK_F16_TFLOPS = 2500.0      # MI355X dense fp16 MFMA
PEAK_F32_TFLOPS = 157.3
STAGES = ["logmel", "zscore", "encoder", "proj0", "gru0", "proj1", "gru1", "output", "decode"]
H, MELS = 128, 80


def stage_work(B, T, V, n_samples, f16, zfold=False):
    """(algorithmic HBM bytes, algorithmic flop) per launch of each stage (the
    compulsory reads and writes of its inputs and outputs; weights, read once
    through L2, are counted once)."""
    rows = B * T
    a = 2 if f16 else 4                       # activation bytes after the encoder
    gi = 2 if f16 else 4
    out = {
        "logmel": (B * n_samples * 4 + rows * MELS * 4, rows * 4600 + rows * MELS * 2 * 6),
        # (zfold: only the per-utterance statistics from the log-mel passes' partials)
        "zscore": ((rows + 5) // 6 * 16 + B * 8, B * 4 * ((T + 5) // 6 + 1)) if zfold else (2 * rows * MELS * 4, rows * MELS * 5),
        "encoder": (rows * MELS * 4 + rows * H * a + (H * MELS) * 4, rows * H * MELS * 2),
        "proj0": (rows * H * a + rows * 6 * H * gi + 6 * H * H * a, rows * 6 * H * H * 2),
        "gru0": (rows * 6 * H * gi + rows * 2 * H * a, rows * 2 * 3 * H * H * 2),
        "proj1": (rows * 2 * H * a + rows * 6 * H * gi + 6 * H * 2 * H * a, rows * 6 * H * 2 * H * 2),
        "gru1": (rows * 6 * H * gi + rows * 2 * H * a, rows * 2 * 3 * H * H * 2),
        "output": (rows * 2 * H * a + V * 2 * H * a + rows * 4, rows * V * 2 * H * 2),
        "decode": (2 * rows * 4 + B * 4, 0),
    }
    return out


def bound_of(stage, f16, fused=False):
    # the fused recurrence does the projection's MFMA work too: priced on the matrix cores
    return "mfma" if stage == "output" or (fused and stage in ("gru0", "gru1")) else "hbm"


def load_traffic(tag):
    p = os.path.join(REPO, "profiles", "ctc_hbm_traffic.json")
    try:
        with open(p) as fh:
            d = json.load(fh)
        return d.get(tag, {}), d.get("source")
    except (OSError, ValueError):
        return {}, None


def run_ctc(batch=4096, vocab=4000, seconds=3, steps=5, warmup=1, precision="fp16", separate=False, device=0,
            keep=None):
    """Config 5 on the HIP path: the timed steps, then the per-stage profile.
    Returns the JSON line's dict (no CPU baseline).  Weights are seeded
    random GRU_CTC_Model weights (wakeword.ctc.random_state_dict: the
    reference ships none).  keep: optional dict that receives the model and
    the audio (the CPU-baseline leg reuses them)."""
    import torch
    import wakeword
    from wakeword import _lib
    from wakeword.ctc import random_state_dict

    f16 = precision == "fp16"
    n = seconds * 16000
    T = 1 + n // 160
    B, V = batch, vocab
    sd = random_state_dict(V, seed=0)
    g = wakeword.CTCModel(sd, V, device=device, precision=precision)
    audio = wakeword.synth_clips(1234, 0, B, n, device=device)
    if keep is not None:
        keep.update(state_dict=sd, audio=audio)
    if separate:
        def step():
            tok, ln, _ = g.decode(g.features(audio, n_samples=n))
            return tok, ln
    else:
        def step():
            return g.decode_audio(audio, n_samples=n)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()

    # timed region: the whole step, host clock, no per-stage events
    t0 = time.perf_counter()
    for _ in range(steps):
        tok, ln = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    value = B * steps / el
    assert int(ln.min()) >= 0 and int(ln.max()) <= T

    # per-stage durations: the same steps again with HIP events around each stage
    L = _lib.lib()
    _lib.check(L.wk_ctc_profile(g._h, 1), "wk_ctc_profile")
    for _ in range(steps):
        step()
    ms = (C.c_double * len(STAGES))()
    cnt = (C.c_int64 * len(STAGES))()
    _lib.check(L.wk_ctc_stage_times(g._h, ms, cnt), "wk_ctc_stage_times")
    _lib.check(L.wk_ctc_profile(g._h, 0), "wk_ctc_profile")
    zfold = f16 and not separate and T >= 6
    work = stage_work(B, T, V, n, f16, zfold)
    fused = f16 and cnt[STAGES.index("proj0")] == 0
    if fused:
        # projection fused into the recurrence: the layer reads its input rows
        # instead of the gate inputs and does the projection's flops too.  Each
        # direction's recurrence reads every input row once, at opposite ends
        # of the sequence (step t forward, step T-1-t backward), so the
        # compulsory reads are 2 x the input: the two reads of a row lie ~|2t-T|
        # steps (4.2 MB of layer-1 input per step) apart, beyond L2 and, but for
        # the middle rows, the Infinity Cache.  Reading the input once needs the
        # unfused projection, whose [rows][768] gate tensor (3 x the input's
        # bytes at layer 1, 6 x at layer 0) is written and read back.
        rows = B * T
        for l, din in ((0, H), (1, 2 * H)):
            by_g, fl_g = work[f"gru{l}"]
            by_p, fl_p = work[f"proj{l}"]
            work[f"gru{l}"] = (2 * rows * din * 2 + rows * 2 * H * 2 + 6 * H * din * 2, fl_g + fl_p)
    traffic, traffic_src = load_traffic(precision)
    kernels = {}
    for i, s in enumerate(STAGES):
        if cnt[i] == 0:
            continue
        avg = ms[i] / cnt[i]
        by, fl = work[s]
        bound = bound_of(s, f16, fused)
        if bound == "mfma":
            ach, peak, unit = fl / (avg * 1e-3) / 1e12, PEAK_F16_TFLOPS if f16 else PEAK_F32_TFLOPS, "TFLOP/s"
        else:
            ach, peak, unit = by / (avg * 1e-3) / 1e9, PEAK_HBM_GBS, "GB/s"
        kernels[s] = {"ms": round(avg, 4), "bound": bound, "achieved": round(ach, 1), "peak": peak, "unit": unit,
                      "frac": round(ach / peak, 4), "algorithmic_bytes": by, "algorithmic_flop": fl,
                      "traffic": traffic.get(s)}
    dom = max(kernels, key=lambda k: kernels[k]["ms"])
    d = kernels[dom]
    line = {
        "metric": "CTC utterances/s (3 s @16 kHz, log-mel 80 -> BiGRU x2 H128 -> greedy CTC), config 5",
        "value": round(value, 1), "unit": "utterances/s", "higher_is_better": True,
        "audio_seconds_per_s": round(value * seconds, 1), "n_gpus": 1,
        "steps": steps, "warmup": warmup, "ms_per_step": round(el / steps * 1e3, 3),
        "dtype": "f32" if not f16 else "f16 GEMM/MFMA operands, f32 accumulate, f32 gate math and front-end",
        "data": "synthetic (device generator), seeded GRU_CTC_Model weights (the reference ships none)",
        "config": {"workload": "config5: CTC head, 3 s utterances", "batch": B, "vocab": V, "T": T,
                   "precision": precision,
                   "call": "wk_ctc_features + wk_ctc_forward" if separate else "wk_ctc_transcribe"
                   + (" (z-score folded into the encoder)" if zfold else "")},
        "roofline": {"kernel": dom, "bound": d["bound"], "achieved": d["achieved"], "peak": d["peak"],
                     "unit": d["unit"], "frac": d["frac"], "traffic": d["traffic"]},
        "kernels": kernels,
        "stage_sum_ms": round(sum(k["ms"] for k in kernels.values()), 4),
    }
    if traffic_src:
        line["traffic_source"] = traffic_src
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--vocab", type=int, default=4000)
    ap.add_argument("--seconds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-utts", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--precision", default="fp16", choices=["fp32", "fp16"],
                    help="GEMM operand precision (config 5 names fp16; fp32 is the parity mode)")
    ap.add_argument("--separate", action="store_true",
                    help="time wk_ctc_features + wk_ctc_forward instead of the one-call wk_ctc_transcribe")
    args = ap.parse_args()
    keep = {}
    line = run_ctc(args.batch, args.vocab, args.seconds, args.steps, args.warmup, args.precision, args.separate,
                   keep=keep)
    if not args.no_cpu_baseline:
        import torch
        from oracle import wk_ctc_oracle as CO
        m = CO.make_model(args.vocab, seed=0)   # the same seeded weights (wakeword.ctc.random_state_dict)
        x = torch.from_numpy(keep["audio"][:args.cpu_utts].cpu().numpy())
        with torch.no_grad():
            CO.greedy_decode(m(CO.features(x[:2])))
            c0 = time.perf_counter()
            CO.greedy_decode(m(CO.features(x)))
            cpu = args.cpu_utts / (time.perf_counter() - c0)
        line["cpu_baseline"] = {"value": round(cpu, 2), "unit": "utterances/s", "cores": torch.get_num_threads(),
                                "host_cpus": len(os.sched_getaffinity(0)), "kind": "port",
                                "sample": f"{args.cpu_utts} utterances of {args.seconds} s in one batch, torch-CPU "
                                          f"oracle (oracle/wk_ctc_oracle.py: torch.stft log-mel, nn.GRU, "
                                          f"V={args.vocab})"}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
