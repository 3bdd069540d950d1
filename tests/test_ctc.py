"""CTC head (ml_models/ctc.py) through the C ABI against the
torch-CPU oracle (oracle/wk_ctc_oracle.py: torch.stft restatement of
torchaudio's MelSpectrogram -- parity unpinned at that boundary -- and the
torch.nn modules GRU_CTC_Model is built from, with seeded weights; the
reference ships no trained CTC weights)."""
import numpy as np
import pytest
import torch

from oracle import wk_ctc_oracle as CO
from oracle import wk_oracle as O

FEAT_ATOL = 2e-3      # z-scored log-mel (unit scale)
LOGP_ATOL = 2e-3      # log_softmax outputs, fp32 end to end
V = 512


def test_greedy_decode_semantics():
    lp = torch.full((1, 9, 6), -10.0)
    for t, k in enumerate([0, 3, 3, 0, 3, 5, 5, 1, 1]):
        lp[0, t, k] = 0.0
    assert CO.greedy_decode(lp) == [[3, 3, 5, 1]]    # blank separates repeats; prev updated on blanks


def test_oracle_feature_shapes_and_zscore():
    x = torch.from_numpy(O.synth_clips(3, 0, 2, 48000))
    f = CO.features(x)
    assert f.shape == (2, 301, 80)
    assert abs(float(f[0].mean())) < 1e-4 and abs(float(f[0].std()) - 1.0) < 1e-4


@pytest.fixture(scope="module")
def ctc():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    import wakeword
    m = CO.make_model(V, seed=7)
    return m, wakeword.CTCModel(CO.flat_weights(m), V)


@pytest.mark.gpu
@pytest.mark.parametrize("n_valid,n_samples", [(48000, 48000), (30000, 48000), (48000, 128000), (60000, 48000), (400, 480)])
def test_ctc_features_match_oracle(ctc, n_valid, n_samples):
    _, g = ctc
    x = O.synth_clips(11, 0, 5, n_valid)
    got = g.features(x, n_samples=n_samples).cpu().numpy()
    ref = CO.features(CO.pad_or_trim(torch.from_numpy(x), n_samples)).numpy()
    assert got.shape == ref.shape == (5, 1 + n_samples // 160, 80)
    assert np.abs(got - ref).max() <= FEAT_ATOL


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 5, 17, 40])
def test_ctc_forward_matches_oracle(ctc, B):
    m, g = ctc
    x = torch.from_numpy(O.synth_clips(5, 0, B, 48000))
    feats = CO.features(x)
    with torch.no_grad():
        ref_lp = m(feats)
    seqs, lp = g.forward(feats, return_log_probs=True)
    lp = lp.cpu()
    assert np.abs((lp - ref_lp).numpy()).max() <= LOGP_ATOL
    # greedy tokens: identical wherever the oracle's top-2 margin is not a near-tie
    top2 = torch.topk(ref_lp, 2, dim=-1).values
    margin = (top2[..., 0] - top2[..., 1]).min().item()
    if margin > 10 * LOGP_ATOL:
        assert seqs == CO.greedy_decode(ref_lp)
    else:
        ok = (top2[..., 0] - top2[..., 1]) > 10 * LOGP_ATOL
        assert (lp.argmax(-1) == ref_lp.argmax(-1))[ok].all()


@pytest.mark.gpu
def test_ctc_end_to_end_and_bad_args(ctc):
    import wakeword
    m, g = ctc
    x = O.synth_clips(21, 0, 3, 48000)
    seqs = g.transcribe(x, n_samples=48000)
    with torch.no_grad():
        ref = CO.greedy_decode(m(CO.features(torch.from_numpy(x))))
    assert len(seqs) == 3 and all(isinstance(s, list) for s in seqs)
    agree = sum(a == b for a, b in zip(seqs, ref))
    assert agree >= 2       # near-tie frames may flip one token; see test_ctc_forward_matches_oracle
    with pytest.raises(ValueError):
        wakeword.CTCModel(np.zeros(10, np.float32), V)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "fp16"])
def test_ctc_argmax_only_path_matches_log_prob_path(ctc, precision):
    """Without log-probs the output layer takes the argmax-only kernel (no
    log-sum-exp): its tokens must equal the log_softmax path's exactly (both
    take the first maximum of logit + bias)."""
    import wakeword
    m, _ = ctc
    g = wakeword.CTCModel(CO.flat_weights(m), V, precision=precision)
    feats = CO.features(torch.from_numpy(O.synth_clips(7, 0, 33, 48000)))
    seqs_lp, _ = g.forward(feats, return_log_probs=True)
    seqs = g.forward(feats)
    assert seqs == seqs_lp


@pytest.mark.gpu
def test_ctc_fp16_gemm_mode(ctc):
    """precision='fp16' (config 5): GEMM operands in fp16, fp32 accumulation and
    recurrence -- looser log-prob bound, same decisions on confident frames."""
    import wakeword
    m, _ = ctc
    g16 = wakeword.CTCModel(CO.flat_weights(m), V, precision="fp16")
    feats = CO.features(torch.from_numpy(O.synth_clips(5, 0, 9, 48000)))
    with torch.no_grad():
        ref_lp = m(feats)
    _, lp = g16.forward(feats, return_log_probs=True)
    lp = lp.cpu()
    assert np.abs((lp - ref_lp).numpy()).max() <= 0.05
    top2 = torch.topk(ref_lp, 2, dim=-1).values
    ok = (top2[..., 0] - top2[..., 1]) > 0.2
    assert (lp.argmax(-1) == ref_lp.argmax(-1))[ok].all()


@pytest.mark.gpu
@pytest.mark.parametrize("vocab", [37, 100, 4000, 4100])
def test_ctc_fp16_ragged_vocab(vocab):
    """The fused fp16 output layer + argmax walks V in 64-column tiles: a
    vocabulary that is not a multiple of 64 (and a large one) must give the
    oracle's decisions on confident frames, with and without log-probs.
    (V > 4096 takes the untagged compare-and-select epilogue.)"""
    import wakeword
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    m = CO.make_model(vocab, seed=11)
    g16 = wakeword.CTCModel(CO.flat_weights(m), vocab, precision="fp16")
    feats = CO.features(torch.from_numpy(O.synth_clips(13, 0, 3, 48000)))
    with torch.no_grad():
        ref_lp = m(feats)
    seqs_lp, lp = g16.forward(feats, return_log_probs=True)
    seqs = g16.forward(feats)
    assert seqs == seqs_lp
    lp = lp.cpu()
    assert lp.shape[-1] == vocab and np.abs((lp - ref_lp).numpy()).max() <= 0.05
    top2 = torch.topk(ref_lp, 2, dim=-1).values
    ok = (top2[..., 0] - top2[..., 1]) > 0.2
    assert (lp.argmax(-1) == ref_lp.argmax(-1))[ok].all()


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "fp16"])
def test_ctc_bit_repeatable_at_scale(precision):
    """Several hundred utterances through features + BiGRU + output layer,
    three times: tokens, lengths and log-probs bit-identical run to run (the
    persistent recurrence and the fused output kernel carry no timing
    dependence)."""
    import wakeword
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    m = CO.make_model(V, seed=3)
    g = wakeword.CTCModel(CO.flat_weights(m), V, precision=precision)
    audio = wakeword.synth_clips(77, 0, 384, 48000)
    ref = None
    for _ in range(3):
        out = [t.clone() for t in g.decode(g.features(audio, n_samples=48000), return_log_probs=True)]
        if ref is None:
            ref = out
        else:
            assert all(torch.equal(a, b) for a, b in zip(ref, out))


@pytest.mark.gpu
def test_ctc_fp16_batch_split_invariant():
    """fp16 argmax-only decode of 400 utterances (120,400 time-major rows, more
    output-layer blocks than CUs) gives the same tokens and lengths as four
    100-utterance batches: a row's result does not depend on the batch it
    came in (row order, block boundaries, GRU batch tiles)."""
    import wakeword
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    m = CO.make_model(V, seed=5)
    g = wakeword.CTCModel(CO.flat_weights(m), V, precision="fp16")
    audio = wakeword.synth_clips(91, 0, 400, 48000)
    feats = g.features(audio, n_samples=48000)
    tok, ln, _ = g.decode(feats)
    tok, ln = tok.clone(), ln.clone()
    for i in range(4):
        t4, l4, _ = g.decode(feats[100 * i:100 * (i + 1)].contiguous())
        assert torch.equal(l4, ln[100 * i:100 * (i + 1)])
        assert torch.equal(t4, tok[100 * i:100 * (i + 1)])


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "fp16"])
def test_ctc_long_utterance_and_device_decode(ctc, precision):
    """8 s utterances (T = 801, Config.max_audio_length): the z-score's
    streaming path (more values than its register cache holds) and the
    wave-per-utterance greedy decode across 13 64-frame chunks.  The device
    tokens must equal decode_predictions applied to the device's own
    log-probs, and the log-probs must track the oracle."""
    import wakeword
    m, _ = ctc
    g = wakeword.CTCModel(CO.flat_weights(m), V, precision=precision)
    x = O.synth_clips(17, 0, 3, 128000)
    feats = g.features(x, n_samples=128000)
    ref_f = CO.features(torch.from_numpy(x))
    assert feats.shape == ref_f.shape == (3, 801, 80)
    assert np.abs(feats.cpu().numpy() - ref_f.numpy()).max() <= FEAT_ATOL
    seqs, lp = g.forward(feats, return_log_probs=True)
    lp = lp.cpu()
    if precision == "fp32":
        # one kernel computes both the argmax and the log-probs; in fp16 mode the
        # log-probs come from fp16-rounded logits, so their own argmax can break
        # near-ties differently from the fp32 accumulators the tokens use
        assert seqs == CO.greedy_decode(lp)
    with torch.no_grad():
        ref_lp = m(ref_f)
    assert np.abs((lp - ref_lp).numpy()).max() <= (LOGP_ATOL if precision == "fp32" else 0.05)
    assert seqs == g.forward(feats)   # the argmax-only kernel agrees with the log-prob path


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "fp16"])
def test_ctc_transcribe_one_call(ctc, precision):
    """wk_ctc_transcribe (audio -> tokens in one call) against the two calls
    it stands for.  fp32, and fp16 with T < 6: the same kernels, identical
    tokens.  fp16 with T >= 6 folds the z-score into the encoder (statistics
    from the log-mel passes): the oracle's argmax on every confident frame,
    for a batch whose log-mel passes straddle utterances (T = 301 = 1 mod 6)
    and which holds a silent utterance (std 0: left un-normalised)."""
    import wakeword
    m, _ = ctc
    g = wakeword.CTCModel(CO.flat_weights(m), V, precision=precision)
    x = O.synth_clips(23, 0, 7, 48000)
    x[3] = 0.0
    tok, ln = g.decode_audio(x, n_samples=48000)
    pred = g.frame_argmax(7, 301).cpu()
    assert int(ln.min()) >= 0 and int(ln.max()) <= 301
    t2, l2, _ = g.decode(g.features(x, n_samples=48000))
    pred2 = g.frame_argmax(7, 301).cpu()
    if precision == "fp32":
        assert torch.equal(tok, t2) and torch.equal(ln, l2)
    else:
        feats = CO.features(torch.from_numpy(np.delete(x, 3, axis=0)))
        with torch.no_grad():
            ref_lp = m(feats)
        top2 = torch.topk(ref_lp, 2, dim=-1).values
        ok = (top2[..., 0] - top2[..., 1]) > 0.2
        live = [0, 1, 2, 4, 5, 6]
        assert (pred[live] == ref_lp.argmax(-1))[ok].all()
        assert (pred[live] == pred2[live])[ok].all()
    # T = 4 (< 6): the unfused sequence in both modes
    xs = O.synth_clips(29, 0, 9, 480)
    tok, ln = g.decode_audio(xs, n_samples=480)
    t2, l2, _ = g.decode(g.features(xs, n_samples=480))
    assert torch.equal(tok, t2) and torch.equal(ln, l2)


@pytest.mark.gpu
@pytest.mark.parametrize("n_samples", [800, 960, 1920, 8000])
def test_ctc_transcribe_short_utterances(ctc, n_samples):
    """The folded z-score at small T (6, 7, 13, 51 frames): log-mel passes of
    6 rows start mid-utterance and straddle two utterances in every pattern;
    the fp16 one-call path must give the oracle's argmax on confident frames
    for all 11 utterances."""
    import wakeword
    m, _ = ctc
    g = wakeword.CTCModel(CO.flat_weights(m), V, precision="fp16")
    B, T = 11, 1 + n_samples // 160
    x = O.synth_clips(31, 0, B, n_samples)
    tok, ln = g.decode_audio(x, n_samples=n_samples)
    pred = g.frame_argmax(B, T).cpu()
    with torch.no_grad():
        ref_lp = m(CO.features(torch.from_numpy(x)))
    top2 = torch.topk(ref_lp, 2, dim=-1).values
    ok = (top2[..., 0] - top2[..., 1]) > 0.2
    assert (pred == ref_lp.argmax(-1))[ok].all()
    assert int(ln.min()) >= 0 and int(ln.max()) <= T


def test_ctc_state_dict_bound_by_name():
    """CTCModel binds a GRU_CTC_Model state dict by key (ctc.py:119-146), in any
    order; missing, unexpected or mis-shaped keys are rejected (host-only)."""
    import random
    from wakeword.ctc import ctc_state_dict_spec, pack_state_dict
    m = CO.make_model(37, seed=2)
    sd = m.state_dict()
    assert [k for k, _ in ctc_state_dict_spec(37)] == list(sd.keys())
    assert [s for _, s in ctc_state_dict_spec(37)] == [tuple(v.shape) for v in sd.values()]
    keys = list(sd.keys())
    random.Random(0).shuffle(keys)
    shuffled = {k: sd[k] for k in keys}
    assert np.array_equal(pack_state_dict(shuffled, 37), CO.flat_weights(m))
    with pytest.raises(ValueError, match="missing"):
        pack_state_dict({k: v for k, v in sd.items() if k != "gru.bias_hh_l1"}, 37)
    with pytest.raises(ValueError, match="unexpected"):
        pack_state_dict({**sd, "gru.weight_ih_l2": sd["gru.weight_ih_l1"]}, 37)
    bad = dict(sd)
    bad["gru.weight_hh_l0"], bad["gru.weight_ih_l0"] = sd["gru.weight_ih_l0"].T, sd["gru.weight_hh_l0"]
    assert bad["gru.weight_hh_l0"].shape == (128, 384)
    with pytest.raises(ValueError, match="shape"):
        pack_state_dict(bad, 37)
    with pytest.raises(ValueError, match="shape"):
        pack_state_dict(sd, 40)         # vocab disagrees with output_layer


def test_random_state_dict_equals_oracle_seeded_model():
    """wakeword.ctc.random_state_dict (the bench's config-5 weights, no oracle
    import on the product side) draws the same values as the oracle's seeded
    GRU_CTC_Model, in its state-dict order, and leaves torch's global RNG as
    it found it (host-only)."""
    from wakeword.ctc import ctc_state_dict_spec, random_state_dict
    before = torch.random.get_rng_state()
    sd = random_state_dict(53, seed=3)
    assert torch.equal(before, torch.random.get_rng_state())
    ref = CO.make_model(53, seed=3).state_dict()
    assert list(sd) == list(ref) == [k for k, _ in ctc_state_dict_spec(53)]
    for k in sd:
        np.testing.assert_array_equal(sd[k], ref[k].numpy())


def test_ctc_decode_predictions_text_round_trip():
    """decode_predictions (ctc.py:453-471): argmax, blank drop, repeat collapse,
    idx_to_char with "<unk>" for unmapped ids -- text equals the oracle's token
    ids mapped through the same vocabulary."""
    from wakeword.ctc import decode_predictions, greedy_tokens, tokens_to_text
    vocab = {"<blank>": 0, "<unk>": 1}
    for ch in "你好小爱同学abc":
        vocab[ch] = len(vocab)
    idx_to_char = {i: c for c, i in vocab.items()}
    text = "小爱同学你好"
    ids = [vocab[c] for c in text]
    frames = []
    for i in ids:                               # each char for 2 frames, blank between
        frames += [i, i, 0]
    lp = torch.full((1, len(frames), len(vocab) + 3), -9.0)
    for t, k in enumerate(frames):
        lp[0, t, k] = 0.0
    assert decode_predictions(lp, idx_to_char) == [text]
    assert greedy_tokens(lp) == CO.greedy_decode(lp)
    lp2 = torch.randn(4, 50, len(vocab) + 3, generator=torch.Generator().manual_seed(3))
    seqs = CO.greedy_decode(lp2)
    assert decode_predictions(lp2, idx_to_char) == tokens_to_text(seqs, idx_to_char)
    assert any("<unk>" in s for s in decode_predictions(lp2, idx_to_char))   # ids past the map


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 33, 200])
def test_ctc_fp16_fused_projection_matches_gemm_path(B, monkeypatch):
    """fp16 mode computes the GRU input projections inside the recurrence (no
    projection GEMM, fp32 gate pre-activations); WAKEWORD_CTC_GEMM=1 keeps the
    separate GEMM (fp16 gate pre-activations).  Both track the oracle within
    the fp16 bound and agree with each other on confident frames; ragged B
    (workgroups own 32 utterances) included."""
    import wakeword
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    m = CO.make_model(V, seed=13)
    g_fused = wakeword.CTCModel(m.state_dict(), V, precision="fp16")
    monkeypatch.setenv("WAKEWORD_CTC_GEMM", "1")
    g_gemm = wakeword.CTCModel(m.state_dict(), V, precision="fp16")
    monkeypatch.delenv("WAKEWORD_CTC_GEMM")
    feats = CO.features(torch.from_numpy(O.synth_clips(19, 0, B, 48000)))
    with torch.no_grad():
        ref_lp = m(feats)
    _, lp_f = g_fused.forward(feats, return_log_probs=True)
    _, lp_g = g_gemm.forward(feats, return_log_probs=True)
    lp_f, lp_g = lp_f.cpu(), lp_g.cpu()
    assert np.abs((lp_f - ref_lp).numpy()).max() <= 0.05
    assert np.abs((lp_g - ref_lp).numpy()).max() <= 0.05
    top2 = torch.topk(ref_lp, 2, dim=-1).values
    ok = (top2[..., 0] - top2[..., 1]) > 0.2
    assert (lp_f.argmax(-1) == ref_lp.argmax(-1))[ok].all()
    # fp32 gate pre-activations: the fused path is at least as close to the oracle
    assert np.abs((lp_f - ref_lp).numpy()).mean() <= np.abs((lp_g - ref_lp).numpy()).mean() * 1.05


@pytest.mark.gpu
@pytest.mark.parametrize("precision,rows", [("fp32", "zero"), ("fp16", "zero"), ("fp16", "equal")])
@pytest.mark.parametrize("level", [-1.0, 1.0])
def test_ctc_argmax_ties_keep_first_index(precision, rows, level):
    """torch.argmax (ctc.py:454) keeps the FIRST of equal maxima.  Output rows
    40 and 300 get the same bias, on top at a negative (level -1) or positive
    (+1) level, and either zero weights (every logit is then its bias exactly,
    whatever the GEMM's order: both paths) or identical weight rows (the fp16
    output kernel computes both columns with the same instruction sequence, so
    their logits are bit-identical).  Every frame's argmax must be 40: the
    fp16 path's column-tagged epilogue as the fp32 path's compare-and-select
    (advisor finding, round 3: negative ties went to the later column)."""
    import wakeword
    m = CO.make_model(V, seed=3)
    with torch.no_grad():
        w, b = m.output_layer.weight, m.output_layer.bias
        if rows == "zero":
            w.zero_()
        else:
            w.mul_(0.01)
            w[300] = w[40]
        b.fill_(level - 4.0)
        b[40] = level
        b[300] = level
    g = wakeword.CTCModel(CO.flat_weights(m), V, precision=precision)
    x = torch.from_numpy(O.synth_clips(8, 0, 6, 48000))
    feats = CO.features(x)
    with torch.no_grad():
        ref = m(feats)
    # the oracle: rows 40 and 300 on top and equal (up to the CPU GEMM's own order)
    assert (ref.topk(2, -1).indices.sort(-1).values == torch.tensor([40, 300])).all()
    assert float((ref[..., 40] - ref[..., 300]).abs().max()) < 1e-5
    if rows == "zero":
        assert (ref.argmax(-1) == 40).all()
    seqs = g.forward(feats)
    fa = g.frame_argmax(6, feats.shape[1]).cpu()
    assert (fa == 40).all(), torch.unique(fa)
    assert seqs == [[40]] * 6


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n", [("silent", 8000), ("dc", 8000), ("dc_and_silent", 7840)])
def test_ctc_transcribe_constant_inputs(ctc, kind, n):
    """Constant audio through the one-call path (the z-score folded into the
    encoder, statistics from the log-mel partials, with the exact two-pass
    fallback for a variance within the partials' rounding) against the
    two-call path (features() z-scored by its own double-precision kernel,
    ctc.py:101-104): digital silence (std 0: left un-normalised by both), a DC
    offset (non-silent, the log-mel far from constant) and a batch alternating
    the two.  The mixed batch uses T = 50: the log-mel kernel transforms two
    consecutive frames per complex FFT, and with an odd T the last frame of
    one utterance shares its FFT with the first of the next, which puts
    ~eps^2 of the DC frame's power (above the 1e-8 floor) into the silent
    frame -- a constant utterance is then only constant to rounding, and its
    z-score (noise / noise, as torch's own for silence) is ill-conditioned."""
    import wakeword
    m, _ = ctc
    g = wakeword.CTCModel(CO.flat_weights(m), V, precision="fp16")
    B, T = 4, 1 + n // 160
    x = np.zeros((B, n), np.float32)
    if kind == "dc":
        x[:] = 0.25
    elif kind == "dc_and_silent":
        x[0::2] = 0.25
    tok, ln = g.decode_audio(x, n_samples=n)
    one = g.frame_argmax(B, T).cpu()
    feats = g.features(x, n_samples=n)
    if kind != "dc":
        silent = feats[1::2] if kind == "dc_and_silent" else feats
        assert float((silent - float(np.log(1e-8))).abs().max()) < 1e-5   # the un-normalised floor ln(1e-8)
    g.decode(feats)
    two = g.frame_argmax(B, T).cpu()
    assert torch.equal(one, two)
    assert int(ln.min()) >= 0 and int(ln.max()) <= T
