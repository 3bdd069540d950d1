"""GRU-CTC head: the reference's ml_models/ctc.py
inference surface on the HIP path (wk_ctc_* in the C ABI).

    model = wakeword.CTCModel(state_dict_or_flat_weights, vocab=V, idx_to_char=None)
    feats = model.features(audio, n_samples=48000)      # ctc.py:82-107, (B, T, 80)
    tokens, log_probs = model.forward(feats, return_log_probs=True)   # ctc.py:148-152 + 453-471
    tokens = model.transcribe(audio)                     # both
    texts = model.decode_predictions(log_probs)          # ctc.py:453-471 (idx_to_char map)
    texts = model.transcribe_text(audio)                 # device decode, then the map

A state dict is bound BY NAME: its keys must be exactly GRU_CTC_Model's
(ctc_state_dict_spec(), ctc.py:119-146: audio_encoder.{0,1}, gru.*_l{k}[_reverse],
output_layer) with the module's shapes; any order is accepted, missing, extra
or mis-shaped entries raise ValueError.  A flat blob must already be in that
order (wk_ctc_create's layout, include/wakeword.h).
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Mapping, Optional, Sequence, Tuple, Union

import numpy as np

from . import _lib
from ._lib import check, lib

MAX_AUDIO_SAMPLES = 8 * 16000   # Config.max_audio_length (ctc.py:29)
BLANK = 0                       # ctc.py:458 (prev_token = 0 = blank_idx)


def ctc_state_dict_spec(vocab: int, hidden: int = 128, layers: int = 2, n_mels: int = 80) -> List[Tuple[str, tuple]]:
    """(key, shape) of GRU_CTC_Model's state dict in registration order
    (ctc.py:119-146: audio_encoder = Sequential(Linear, LayerNorm, ReLU,
    Dropout), nn.GRU(bidirectional, num_layers=layers), output_layer) -- the
    order wk_ctc_create's flat blob concatenates."""
    spec = [("audio_encoder.0.weight", (hidden, n_mels)), ("audio_encoder.0.bias", (hidden,)),
            ("audio_encoder.1.weight", (hidden,)), ("audio_encoder.1.bias", (hidden,))]
    for k in range(layers):
        d_in = hidden if k == 0 else 2 * hidden
        for sfx in ("", "_reverse"):
            spec += [(f"gru.weight_ih_l{k}{sfx}", (3 * hidden, d_in)), (f"gru.weight_hh_l{k}{sfx}", (3 * hidden, hidden)),
                     (f"gru.bias_ih_l{k}{sfx}", (3 * hidden,)), (f"gru.bias_hh_l{k}{sfx}", (3 * hidden,))]
    spec += [("output_layer.weight", (vocab, 2 * hidden)), ("output_layer.bias", (vocab,))]
    return spec


def random_state_dict(vocab: int, seed: int = 0, hidden: int = 128, layers: int = 2, n_mels: int = 80,
                      out_scale: float = 4.0) -> Dict[str, np.ndarray]:
    """Seeded random GRU_CTC_Model weights (the reference ships no trained CTC
    weights; ctc.py:119-146).  torch's default initialisers, drawn in the
    module's registration order after torch.manual_seed(seed) -- nn.Linear,
    nn.LayerNorm, nn.GRU(bidirectional), nn.Linear -- so a torch model built
    the same way holds the same values.  out_scale multiplies the output
    layer's weight: 4 gives the greedy path decision margins (a default init is
    near-uniform over V)."""
    import torch
    from torch import nn
    gen_state = torch.random.get_rng_state()
    try:
        torch.manual_seed(seed)
        enc = nn.Linear(n_mels, hidden)
        ln = nn.LayerNorm(hidden)
        gru = nn.GRU(input_size=hidden, hidden_size=hidden, num_layers=layers, batch_first=True,
                     dropout=0.2 if layers > 1 else 0.0, bidirectional=True)
        out = nn.Linear(2 * hidden, vocab)
    finally:
        torch.random.set_rng_state(gen_state)
    sd = {"audio_encoder.0.weight": enc.weight, "audio_encoder.0.bias": enc.bias,
          "audio_encoder.1.weight": ln.weight, "audio_encoder.1.bias": ln.bias}
    sd.update({f"gru.{k}": v for k, v in gru.state_dict().items()})
    sd["output_layer.weight"] = out.weight * out_scale
    sd["output_layer.bias"] = out.bias
    return {k: v.detach().numpy().astype(np.float32) for k, v in sd.items()}


def _as_f32(v) -> np.ndarray:
    if hasattr(v, "detach"):          # torch tensor (any device)
        v = v.detach().cpu().numpy()
    return np.asarray(v, np.float32)


def pack_state_dict(sd: Mapping[str, object], vocab: int, hidden: int = 128, layers: int = 2,
                    n_mels: int = 80) -> np.ndarray:
    """Bind a GRU_CTC_Model state dict by name into wk_ctc_create's blob.
    Raises ValueError naming every missing, unexpected or mis-shaped key."""
    spec = ctc_state_dict_spec(vocab, hidden, layers, n_mels)
    want = dict(spec)
    missing = [k for k, _ in spec if k not in sd]
    extra = [k for k in sd if k not in want]
    if missing or extra:
        raise ValueError(f"GRU_CTC_Model state dict mismatch: missing {missing}, unexpected {extra}")
    parts = []
    for k, shape in spec:
        a = _as_f32(sd[k])
        if tuple(a.shape) != shape:
            raise ValueError(f"{k}: expected shape {shape}, got {tuple(a.shape)}")
        parts.append(a.reshape(-1))
    return np.concatenate(parts)


def tokens_to_text(seqs: Sequence[Sequence[int]], idx_to_char: Mapping[int, str]) -> List[str]:
    """decode_predictions' last step (ctc.py:468): ids -> characters, unknown
    ids as "<unk>", joined."""
    return ["".join(idx_to_char.get(int(i), "<unk>") for i in seq) for seq in seqs]


def greedy_tokens(log_probs) -> List[List[int]]:
    """ctc.py:454-466: first argmax per frame, blank (0) dropped, repeats
    collapsed with prev_token updated on every frame (blanks included)."""
    import torch
    pred = torch.as_tensor(log_probs).argmax(dim=-1).cpu().numpy()
    if pred.ndim == 1:
        pred = pred[None]
    seqs = []
    for row in pred:
        keep = (row != BLANK) & (row != np.concatenate([[BLANK], row[:-1]]))
        seqs.append(row[keep].tolist())
    return seqs


def decode_predictions(log_probs, idx_to_char: Mapping[int, str]) -> List[str]:
    """THCHS30Trainer.decode_predictions (ctc.py:453-471) on (B, T, V)
    log-probs (host-side; the batched device decode is CTCModel.decode)."""
    return tokens_to_text(greedy_tokens(log_probs), idx_to_char)


class CTCModel:
    def __init__(self, weights: Union[np.ndarray, Mapping[str, np.ndarray]], vocab: int, device: int = 0,
                 precision: str = "fp32", idx_to_char: Optional[Mapping[int, str]] = None):
        if hasattr(weights, "state_dict") and callable(weights.state_dict):   # an nn.Module (GRU_CTC_Model)
            weights = weights.state_dict()
        if isinstance(weights, Mapping):
            weights = pack_state_dict(weights, vocab)
        if precision not in ("fp32", "fp16"):
            raise ValueError(f"precision must be 'fp32' or 'fp16', got {precision!r}")
        self.idx_to_char = dict(idx_to_char) if idx_to_char is not None else None
        w = np.ascontiguousarray(_as_f32(weights).reshape(-1))
        L = lib()
        self.cfg = _lib.WkCtcConfig(vocab, 128, 2, 80, device, {"fp32": 0, "fp16": 1}[precision])
        need = L.wk_ctc_num_weights(C.byref(self.cfg))
        if w.size != need:
            raise ValueError(f"expected {need} weights for vocab={vocab}, got {w.size}")
        self.vocab, self.device = vocab, device
        self._h = C.c_void_p()
        check(L.wk_ctc_create(C.byref(self.cfg), w.ctypes.data_as(C.c_void_p), C.byref(self._h)), "wk_ctc_create")

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                lib().wk_ctc_destroy(self._h)
        except Exception:
            pass

    def _stream(self, torch):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def features(self, audio, n_samples: int = MAX_AUDIO_SAMPLES):
        """(B, L) float waveform -> (B, T, 80) on device, T = 1 + n_samples // 160."""
        import torch
        x = torch.as_tensor(audio, dtype=torch.float32).to(f"cuda:{self.device}").contiguous()
        if x.dim() == 1:
            x = x.unsqueeze(0)
        B, L = x.shape
        T = 1 + n_samples // 160
        out = torch.empty((B, T, 80), dtype=torch.float32, device=x.device)
        check(lib().wk_ctc_features(self._h, C.c_void_p(x.data_ptr()), B, L, n_samples, L, C.c_void_p(out.data_ptr()),
                                    self._stream(torch)), "wk_ctc_features")
        return out

    def decode(self, feats, return_log_probs: bool = False):
        """(B, T, 80) -> device tensors, stream-ordered, no host sync: tokens
        (B, T) int32 (row b's first lengths[b] entries are its greedy CTC
        sequence, the rest -1), lengths (B,) int32, and (B, T, V) log-probs
        if asked (else None)."""
        import torch
        f = torch.as_tensor(feats, dtype=torch.float32).to(f"cuda:{self.device}").contiguous()
        B, T, _ = f.shape
        lp = torch.empty((B, T, self.vocab), dtype=torch.float32, device=f.device) if return_log_probs else None
        tok = torch.empty((B, T), dtype=torch.int32, device=f.device)
        ln = torch.empty((B,), dtype=torch.int32, device=f.device)
        check(lib().wk_ctc_forward(self._h, C.c_void_p(f.data_ptr()), B, T,
                                   C.c_void_p(lp.data_ptr()) if lp is not None else None, C.c_void_p(tok.data_ptr()),
                                   C.c_void_p(ln.data_ptr()), self._stream(torch)), "wk_ctc_forward")
        return tok, ln, lp

    def decode_audio(self, audio, n_samples: int = MAX_AUDIO_SAMPLES):
        """(B, L) float waveform -> (tokens (B, T) int32, lengths (B,) int32) on
        device, stream-ordered: wk_ctc_transcribe, i.e. features() then
        decode() in one call (fp16 mode: the z-score folded into the encoder)."""
        import torch
        x = torch.as_tensor(audio, dtype=torch.float32).to(f"cuda:{self.device}").contiguous()
        if x.dim() == 1:
            x = x.unsqueeze(0)
        B, L = x.shape
        T = 1 + n_samples // 160
        tok = torch.empty((B, T), dtype=torch.int32, device=x.device)
        ln = torch.empty((B,), dtype=torch.int32, device=x.device)
        check(lib().wk_ctc_transcribe(self._h, C.c_void_p(x.data_ptr()), B, L, n_samples, L, C.c_void_p(tok.data_ptr()),
                                      C.c_void_p(ln.data_ptr()), self._stream(torch)), "wk_ctc_transcribe")
        return tok, ln

    def frame_argmax(self, batch: int, T: int):
        """decode_predictions' per-frame `predictions` (ctc.py:454) of the last
        decode/forward on this model: (batch, T) int32 on device."""
        import torch
        out = torch.empty((batch, T), dtype=torch.int32, device=f"cuda:{self.device}")
        check(lib().wk_ctc_frame_argmax(self._h, batch, T, C.c_void_p(out.data_ptr()), self._stream(torch)),
              "wk_ctc_frame_argmax")
        return out

    def forward(self, feats, return_log_probs: bool = False):
        """(B, T, 80) -> token id lists (greedy CTC, decode_predictions'
        output form), and (B, T, V) log-probs if asked."""
        tok, ln, lp = self.decode(feats, return_log_probs)
        tok, ln = tok.cpu().numpy(), ln.cpu().numpy()
        seqs = [tok[b, :ln[b]].tolist() for b in range(tok.shape[0])]
        return (seqs, lp) if return_log_probs else seqs

    def transcribe(self, audio, n_samples: int = MAX_AUDIO_SAMPLES) -> List[List[int]]:
        """audio -> token id lists (extract_features + model + decode_predictions)."""
        tok, ln = self.decode_audio(audio, n_samples)
        tok, ln = tok.cpu().numpy(), ln.cpu().numpy()
        return [tok[b, :ln[b]].tolist() for b in range(tok.shape[0])]

    def _char_map(self, idx_to_char):
        m = idx_to_char if idx_to_char is not None else self.idx_to_char
        if m is None:
            raise ValueError("no idx_to_char map: pass one here or to CTCModel(...)")
        return m

    def decode_predictions(self, log_probs, idx_to_char: Optional[Mapping[int, str]] = None) -> List[str]:
        """THCHS30Trainer.decode_predictions (ctc.py:453-471) with this model's map."""
        return decode_predictions(log_probs, self._char_map(idx_to_char))

    def transcribe_text(self, audio, n_samples: int = MAX_AUDIO_SAMPLES,
                        idx_to_char: Optional[Mapping[int, str]] = None) -> List[str]:
        """audio -> text: the device greedy decode, then the idx_to_char map."""
        return tokens_to_text(self.transcribe(audio, n_samples), self._char_map(idx_to_char))
