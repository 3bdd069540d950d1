"""Every BASELINE.json config at its stated size, through the C ABI, against the
oracle.

  config 1  single WAV CLI               tests/test_gpu_parity.py::test_cli_config1_golden_wavs
  config 2  B = 65,536 fused fp32        tests/test_gpu_parity.py::test_full_size_batch_sample_parity
  config 3  30 s stream, hop 480          test_config3_stream_30s_hop480 (below)
  config 4  131,072 clips per rank, bf16  test_config4_bf16_rank_shard (below)
  config 5  CTC B = 4096, T = 301, V = 4000, fp16   test_config5_ctc_full_batch (below)

Sampled oracle parity at full size (a spread of windows / utterances through
the CPU oracle), plus size-independent properties over the whole batch
(finite outputs, decision agreement with the fp32 path, streaming == batch bit
for bit, argmax-only tokens == log-prob-path tokens).  Tolerances are the
ones stated in the per-path tests: fp32 logits 1e-3, bf16 0.05, CTC fp16
log-probs 0.05 with identical argmax on frames whose oracle top-2 margin
exceeds 0.2.
"""
import os

import numpy as np
import pytest

from oracle import wk_oracle as O

pytestmark = pytest.mark.gpu

LOGIT_ATOL = 1e-3
BF16_LOGIT_ATOL = 0.05
CTC16_LOGP_ATOL = 0.05
CTC16_MARGIN = 0.2
WIN = 16000


# ---------------------------------------------------------------- config 3
def test_config3_stream_30s_hop480(gpu, golden_dir, xiaoa_sd):
    """A continuous 30 s stream pushed 30 ms at a time (the hop), as a
    device feeding the ring: every window is scored exactly once, in order,
    bit-identical to the batch path over the same samples, and a spread of
    windows matches the oracle."""
    import ctypes as C
    import torch
    import wakeword
    from wakeword import _lib
    hop, seconds = 480, 30
    audio = O.synth_clips(2024, 0, seconds).reshape(-1)           # 480,000 samples
    n_win = (audio.size - WIN) // hop + 1
    assert n_win == 967
    model = wakeword.load_onnx(os.path.join(golden_dir, "xiaoa.onnx"))
    d = torch.from_numpy(audio).cuda()
    ref = torch.empty(n_win, dtype=torch.float32, device="cuda")
    _lib.check(_lib.lib().wk_forward(model._h.h, C.c_void_p(d.data_ptr()), _lib.WK_DTYPE_F32, n_win, WIN, hop,
                                     C.c_void_p(ref.data_ptr()), None,
                                     C.c_void_p(torch.cuda.current_stream().cuda_stream)), "wk_forward")
    ref = ref.cpu().numpy()
    det = wakeword.StreamingDetector(model, hop=hop, capacity=1 << 15)
    ends, logits = [], []
    for p in range(0, audio.size, hop):
        for w in det.push(audio[p:p + hop]):
            ends.append(w.end)
            logits.append(w.logit)
    det.close()
    assert ends == [WIN + k * hop for k in range(n_win)]
    np.testing.assert_array_equal(np.asarray(logits, np.float32), ref)
    idx = np.linspace(0, n_win - 1, 8).astype(int)
    clips = np.stack([audio[k * hop:k * hop + WIN] for k in idx]).astype(np.float64)
    want = O.detect_mode_b(clips, xiaoa_sd)
    assert np.abs(ref[idx] - want).max() < LOGIT_ATOL
    model.check_device_errors()


# ---------------------------------------------------------------- config 4
def test_config4_bf16_rank_shard(gpu, golden_dir, xiaoa_sd):
    """Config 4 at its per-rank size: 131,072 clips of rank 3's shard of the
    1,048,576-clip job (global clip indices from weak_shard, so the device
    generator gives the clips an 8-rank run scores there), bf16
    convolutions.  All logits finite; a spread sample within 0.05 of the
    oracle; every clip within 0.05 of the fp32 path with the same decision
    wherever the fp32 logit is not within 0.05 of the threshold."""
    import torch
    import wakeword
    from wakeword.shard import weak_shard
    per_rank, rank = 131072, 3
    first, count = weak_shard(per_rank, rank)
    assert (first, count) == (rank * per_rank, per_rank)
    x = wakeword.synth_clips(1234, first, count, device=0)
    m16 = wakeword.load_onnx(os.path.join(golden_dir, "xiaoa.onnx"), precision="bf16")
    m32 = wakeword.load_onnx(os.path.join(golden_dir, "xiaoa.onnx"))
    a = m16.detect(x).reshape(-1)
    b = m32.detect(x).reshape(-1)
    m16.check_device_errors()
    m32.check_device_errors()
    assert bool(torch.isfinite(a).all()) and bool(torch.isfinite(b).all())
    d = (a - b).abs()
    assert d.max().item() <= BF16_LOGIT_ATOL, d.max().item()
    confident = b.abs() > BF16_LOGIT_ATOL
    assert bool(((a > 0) == (b > 0))[confident].all())
    idx = np.linspace(0, count - 1, 16).astype(int)
    xs = O.synth_clips(1234, first, 1, 16000)
    assert np.abs(x[0].cpu().numpy() - xs[0]).max() < 1e-5   # device generator keyed on the global index
    clips = x[torch.from_numpy(idx).cuda()].cpu().numpy().astype(np.float64)
    ref = O.detect_mode_b(clips, xiaoa_sd)
    a_np = a.cpu().numpy()
    assert np.abs(a_np[idx] - ref).max() <= BF16_LOGIT_ATOL
    assert np.abs(b.cpu().numpy()[idx] - ref).max() <= LOGIT_ATOL


# ---------------------------------------------------------------- config 5
def test_config5_ctc_full_batch():
    """Config 5 at its bench size: B = 4096 utterances of 3 s (T = 301),
    V = 4000, fp16.  The timed path (features -> decode, argmax-only output
    kernel) and the log-prob path give identical tokens and lengths for all
    4096 utterances; all lengths are in range and all log-probs finite; 16
    utterances spread over the batch match the torch-CPU oracle (log-probs
    within 0.05, argmax identical on frames whose oracle top-2 margin exceeds
    0.2, and the greedy tokens equal to decode_predictions of the oracle for
    every utterance whose frames are all that confident)."""
    import torch
    import wakeword
    from oracle import wk_ctc_oracle as CO
    B, V, n = 4096, 4000, 48000
    T = 1 + n // 160
    m = CO.make_model(V, seed=0)
    g = wakeword.CTCModel(m.state_dict(), V, precision="fp16")
    audio = wakeword.synth_clips(1234, 0, B, n)
    feats = g.features(audio, n_samples=n)
    assert feats.shape == (B, T, 80)
    tok, ln, _ = g.decode(feats)
    tok, ln = tok.clone(), ln.clone()
    tok2, ln2, lp = g.decode(feats, return_log_probs=True)
    assert torch.equal(ln, ln2) and torch.equal(tok, tok2)
    assert int(ln.min()) >= 0 and int(ln.max()) <= T
    assert bool(torch.isfinite(lp).all())
    idx = torch.linspace(0, B - 1, 16).long()
    x_s = torch.from_numpy(audio[idx.cuda()].cpu().numpy())
    f_ref = CO.features(x_s)
    np.testing.assert_allclose(feats[idx.cuda()].cpu().numpy(), f_ref.numpy(), atol=2e-3)
    with torch.no_grad():
        ref_lp = m(f_ref)
    lp_s = lp[idx.cuda()].cpu()
    del lp
    assert np.abs((lp_s - ref_lp).numpy()).max() <= CTC16_LOGP_ATOL
    top2 = torch.topk(ref_lp, 2, dim=-1).values
    ok = (top2[..., 0] - top2[..., 1]) > CTC16_MARGIN
    assert (lp_s.argmax(-1) == ref_lp.argmax(-1))[ok].all()
    # per-frame argmax of the timed path (decode_predictions' `predictions`):
    # the oracle's argmax on every confident frame, and the device tokens are
    # exactly its blank-drop / repeat-collapse for all 4096 utterances
    tok, ln, _ = g.decode(feats)
    pred = g.frame_argmax(B, T)
    pred_s = pred[idx.cuda()].cpu()
    assert (pred_s == ref_lp.argmax(-1))[ok].all()
    assert float(ok.float().mean()) > 0.1      # the sample has confident frames to check
    p = pred.cpu().numpy()
    keep = (p != 0) & (p != np.concatenate([np.zeros((B, 1), p.dtype), p[:, :-1]], axis=1))
    tok_np, ln_np = tok.cpu().numpy(), ln.cpu().numpy()
    np.testing.assert_array_equal(ln_np, keep.sum(1))
    assert np.array_equal(tok_np[np.arange(T)[None, :] < ln_np[:, None]], p[keep])
    assert (tok_np[np.arange(T)[None, :] >= ln_np[:, None]] == -1).all()
    # and where the oracle's whole utterance is confident, the tokens are its greedy decode
    ref_seqs = CO.greedy_decode(ref_lp)
    for j in range(len(idx)):
        if bool(ok[j].all()):
            b = int(idx[j])
            assert tok_np[b, :ln_np[b]].tolist() == ref_seqs[j]
    # the one-call path bench_ctc.py times (wk_ctc_transcribe: z-score folded
    # into the encoder): the oracle's argmax on every confident frame, and the
    # two-call path's frame decisions except at float-rounding near-ties
    tok3, ln3 = g.decode_audio(audio, n_samples=n)
    pred3 = g.frame_argmax(B, T).cpu()
    assert (pred3[idx] == ref_lp.argmax(-1))[ok].all()
    agree = float((pred3.numpy() == p).mean())
    assert agree > 0.999, agree
    assert int(ln3.min()) >= 0 and int(ln3.max()) <= T


def test_config5_repeatable_at_scale():
    """Config 5's timed path, bit for bit run to run at its bench size
    (B = 4096, T = 301, V = 4000, fp16): four one-call transcriptions
    (log-mel, encoder, fused GRU layers, decode-only output kernel, near-tie
    re-scoring) give identical tokens, lengths and per-frame argmax, and so do
    three two-call decodes of one feature tensor.  The CTC kernels run the
    K = 32 f16 MFMA beside VALU work on the same SIMDs, the combination that
    changes the fused kernel's front-end values (DESIGN 5.1, K = 32): this is
    the at-scale check that it does not touch them."""
    import torch
    import wakeword
    from oracle import wk_ctc_oracle as CO
    B, V, n = 4096, 4000, 48000
    T = 1 + n // 160
    g = wakeword.CTCModel(CO.make_model(V, seed=2).state_dict(), V, precision="fp16")
    audio = wakeword.synth_clips(4321, 0, B, n)
    ref = None
    for _ in range(4):
        tok, ln = g.decode_audio(audio, n_samples=n)
        got = (tok.clone(), ln.clone(), g.frame_argmax(B, T))
        if ref is None:
            ref = got
        else:
            diff = [int((a != b).sum()) for a, b in zip(ref, got)]
            assert diff == [0, 0, 0], diff
    feats = g.features(audio, n_samples=n)
    ref = None
    for _ in range(3):
        tok, ln, _ = g.decode(feats)
        got = (tok.clone(), ln.clone(), g.frame_argmax(B, T))
        if ref is None:
            ref = got
        else:
            diff = [int((a != b).sum()) for a, b in zip(ref, got)]
            assert diff == [0, 0, 0], diff
    torch.cuda.synchronize()


def _edit_distance(a, b):
    """Levenshtein distance between two token sequences."""
    prev = list(range(len(b) + 1))
    for i, x in enumerate(a, 1):
        cur = [i] + [0] * len(b)
        for j, y in enumerate(b, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (x != y))
        prev = cur
    return prev[-1]


# ((precision, out_scale, mix), bounds): the oracle model's output layer at 4x
# its default init (the margins the other config-5 tests rely on) and at the
# default nn.Linear init (near-uniform logits over V = 4000: near-ties
# everywhere).  Bounds: minimum exact-sequence match rate, maximum mean edit
# distance per utterance (tokens), minimum frame-argmax agreement, over 64
# utterances of ~120 oracle tokens x 301 frames.  Round 4's fp16 path flipped
# about one frame decision in 800 at near-ties (0.750 / 0.33 / 0.99875 at x4);
# round 5 re-scores the output layer's near-ties in fp32.
# mix: "out32" = the fp16 path with an fp32 output layer, "out16" = the fp32
# path with the fp16 output kernel (WAKEWORD_CTC_MIX), "norescore" = the
# re-scoring off (WAKEWORD_CTC_RESCORE=0): the attribution table of DESIGN 5.3.
#
# The counts are chaotic at the level of a few sequences: every flip is a
# near-tie, so a perturbation far below the fp16 noise moves them.  Round 5
# measured them under two summation orders of the z-score statistics (per-pass
# partials, profiles/r05c_ctc_decisions.txt; per-wave running sums,
# profiles/r05g_ctc_decisions.txt), both exact to ~1e-7 relative: fp16 x4 went
# 56 -> 52 exact sequences while its re-scoring-off variant went 48 -> 50.  The
# sequence bounds are the lower of the two minus one or two sequences; the
# hard parity assertion is on the margins: a decision may differ from the
# oracle's only where the oracle's own top-2 log-prob margin is below
# CTC_FLIP_MARGIN (fp16: measured at most 8.0e-4; fp32: 9.5e-7, an fp32
# rounding-level tie decided by summation order).
CTC_DECISION_BOUNDS = {
    # product paths
    ("fp16", 4.0, ""): (0.78, 0.32, 0.9988),           # measured 56 / 52 of 64, 0.141 / 0.250, 0.99922 / 0.99907
    ("fp16", 1.0, ""): (0.66, 0.52, 0.9982),           # measured 49 / 44, 0.375 / 0.438, 0.99886 / 0.99849
    ("fp32", 4.0, ""): (0.96, 0.05, 0.9999),           # measured 63 / 63, 0.016, 0.99995
    # attribution: re-scoring off, one stage's precision swapped
    ("fp16", 4.0, "norescore"): (0.70, 0.40, 0.9985),  # measured 48 / 50, 0.328 / 0.328, 0.99875 / 0.99881
    ("fp16", 1.0, "norescore"): (0.66, 0.52, 0.9982),  # measured 49 / 45, 0.406 / 0.438, 0.99881 / 0.99855
    ("fp16", 4.0, "out32"): (0.78, 0.32, 0.9988),      # measured 56 / 52, 0.141 / 0.250, 0.99922 / 0.99907
    ("fp32", 4.0, "out16+norescore"): (0.75, 0.35, 0.9985),   # measured 51 / 51, 0.297, 0.99891
}
CTC_FLIP_MARGIN = {"fp16": 2e-3, "fp32": 1e-5}


@pytest.mark.parametrize("precision,out_scale,mix", list(CTC_DECISION_BOUNDS))
def test_config5_decision_parity(precision, out_scale, mix, monkeypatch):
    """Config 5's product output is the token sequence (decode_predictions,
    ctc.py:453-471).  For 64 utterances spread over the B = 4096 batch, the
    one-call path bench_ctc.py times (wk_ctc_transcribe; fp16 is the bench's
    precision) against greedy_decode of the torch-CPU oracle: the
    exact-sequence match rate, the mean token edit distance per utterance and
    the frame-argmax agreement are printed and held to CTC_DECISION_BOUNDS."""
    import torch
    import wakeword
    from oracle import wk_ctc_oracle as CO
    for part in mix.split("+") if mix else []:
        if part == "norescore":
            monkeypatch.setenv("WAKEWORD_CTC_RESCORE", "0")
        else:
            monkeypatch.setenv("WAKEWORD_CTC_MIX", part)
    B, V, n = 4096, 4000, 48000
    T = 1 + n // 160
    m = CO.make_model(V, seed=0, out_scale=out_scale)
    g = wakeword.CTCModel(m.state_dict(), V, precision=precision)
    audio = wakeword.synth_clips(1234, 0, B, n)
    tok, ln = g.decode_audio(audio, n_samples=n)
    pred = g.frame_argmax(B, T).cpu()
    tok, ln = tok.cpu().numpy(), ln.cpu().numpy()
    idx = torch.linspace(0, B - 1, 64).long()
    x_s = torch.from_numpy(audio[idx.cuda()].cpu().numpy())
    with torch.no_grad():
        ref_lp = m(CO.features(x_s))
    ref_seqs = CO.greedy_decode(ref_lp)
    exact, dist, ntok = 0, 0, 0
    for j, b in enumerate(idx.tolist()):
        got = tok[b, :ln[b]].tolist()
        exact += got == ref_seqs[j]
        dist += _edit_distance(got, ref_seqs[j])
        ntok += len(ref_seqs[j])
    frame_agree = float((pred[idx] == ref_lp.argmax(-1)).float().mean())
    match, mean_dist = exact / len(idx), dist / len(idx)
    # the oracle's top-2 log-prob margin at every frame whose decision differs (a near-tie or not)
    flip = (pred[idx] != ref_lp.argmax(-1))
    top2 = ref_lp.topk(2, dim=-1).values
    margins = (top2[..., 0] - top2[..., 1])[flip]
    print(f"\nconfig5 flipped frames: {int(flip.sum())}, oracle top-2 margins at them: max "
          f"{float(margins.max()) if margins.numel() else 0.0:.2e}, median "
          f"{float(margins.median()) if margins.numel() else 0.0:.2e}")
    print(f"\nconfig5 decisions ({precision}{'+' + mix if mix else ''}, out_scale {out_scale}): exact-sequence match "
          f"{match:.4f} ({exact}/{len(idx)}), mean edit distance {mean_dist:.3f} tokens per utterance "
          f"(oracle mean length {ntok / len(idx):.1f}), frame-argmax agreement {frame_agree:.5f}")
    lo_match, hi_dist, lo_frame = CTC_DECISION_BOUNDS[(precision, out_scale, mix)]
    assert match >= lo_match and mean_dist <= hi_dist and frame_agree >= lo_frame, (match, mean_dist, frame_agree)
    # confident frames decide exactly as the oracle does (the fp16 margin wherever an fp16 stage is in the path)
    bound = CTC_FLIP_MARGIN["fp16" if precision == "fp16" or "out16" in mix else "fp32"]
    assert margins.numel() == 0 or float(margins.max()) <= bound, float(margins.max())


@pytest.mark.gpu
def test_bench_line_carries_every_config(gpu):
    """The driver's bench line (bench.py, N = 1) holds the headline and the
    config 4 / 5 / 3 keys, each measured (no error entry)."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["value"] > 0 and line["roofline"]["frac"] > 0
    for key in ("config4", "config5", "config3"):
        assert key in line and "error" not in line[key], (key, line.get(key))
    assert line["config4"]["batch_per_gpu"] == 131_072 and line["config4"]["value"] > 0
    assert line["config5"]["value"] > 0 and line["config5"]["output_kernel"]["frac"] > 0
    assert line["config3"]["p50_latency_ms"] > 0
