"""CPU tests of libwakeword_host.so (include/wakeword_host.h), the host-CPU
path of BASELINE config 1 and of the mfcc.h drop-in for callers without a GPU.

The library is product code (csrc/wk_host.cpp + csrc/wk_wav.cpp): it never
links or loads anything under oracle/, which here is only the checker.
Parity:
  * mode B + CNN against the golden vectors of the reference's own
    LightweightKWS (tests/golden: synth clips, eight reference WAVs zero- and
    noise-padded, the xiaoa.info KAT features) -- the CNN half is pinned, the
    torchaudio front-end is "parity unpinned" (torchaudio absent; restated);
  * mode A against the C restatement oracle/esp_mfcc_oracle.c at the
    reference configuration and seven general parameter sets, packing on and
    off, the single-frame variant and the NULL paths -- "parity unpinned" at
    the esp-dsp boundary, as for the GPU mode-A tests.
Tolerances (written here): features 5e-4, logits 1e-3, mode A 2e-5 max|x| + 2e-4.
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from oracle import build_oracle as B
from oracle import wk_oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "wakeword_host.h")
FEAT_ATOL, LOGIT_ATOL = 5e-4, 1e-3


def _tol(ref):
    return 2e-5 * np.abs(ref).max() + 2e-4


@pytest.fixture(scope="module")
def host():
    from wakeword import build
    build.build_host()
    from wakeword import host as H
    return H


@pytest.fixture(scope="module")
def model(host, golden_dir):
    return host.load_onnx(os.path.join(golden_dir, "xiaoa.onnx"))


def test_exports_and_no_gpu_or_oracle_dependency(host):
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    declared = set(re.findall(r"\b([A-Za-z_]\w*)\s*\([^;{]*\)\s*;", txt))
    assert declared == set(host.EXPORTS)
    out = subprocess.run(["nm", "-D", "--defined-only", host.HOST_LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (\w+)", out))
    for name in (*host.EXPORTS, *host.MFCC_H, *host.WAV):
        assert name in exported, name
    assert not any("oracle" in s for s in exported)
    deps = subprocess.run(["ldd", host.HOST_LIB_PATH], capture_output=True, text=True).stdout
    assert "amdhip" not in deps and "rocblas" not in deps and "oracle" not in deps, deps


def test_mode_b_features_match_golden(host, golden_dir):
    s = np.load(os.path.join(golden_dir, "synth.npz"))
    x = O.synth_clips(int(s["seed"]), int(s["first"]), int(s["count"]))
    assert np.abs(host.mfcc(x) - s["feats"]).max() < FEAT_ATOL
    raw = host.mfcc(x, cmvn=False)
    assert np.abs(raw - O.mfcc_torchaudio(x)).max() < 1e-3


def test_cnn_matches_reference_module_and_kat(model, golden_dir):
    s = np.load(os.path.join(golden_dir, "synth.npz"))
    assert np.abs(model(s["feats"])[:, 0] - s["logits"]).max() < 1e-4
    k = np.load(os.path.join(golden_dir, "kat.npz"))
    got = float(model(k["kat_feats"])[0, 0])
    assert abs(got - float(k["kat_ref_logit"][0])) < 1e-4
    assert abs(got - float(k["kat_out_int8"].reshape(-1)[0]) * 2.0 ** int(k["kat_out_exp"])) < 0.25
    assert np.array_equal(model.run(None, {"input.1": s["feats"]})[0], model(s["feats"]))


def test_end_to_end_golden_wavs(model, golden_dir):
    g = np.load(os.path.join(golden_dir, "wavs.npz"))
    logits, feats = model.detect(g["x_noise"], return_features=True)
    assert np.abs(feats - g["feat_noise"]).max() < FEAT_ATOL
    assert np.abs(logits - g["logit_noise"]).max() < LOGIT_ATOL


def test_cli_cpu_config1(host, golden_dir, capsys):
    """python -m wakeword.test --cpu: WAV -> zero pad -> logit on the host,
    against the reference LightweightKWS logits of the zero-padded WAVs."""
    import json
    from wakeword import test as cli
    g = np.load(os.path.join(golden_dir, "wavs.npz"))
    paths = [os.path.join(golden_dir, "wav", str(n)) for n in g["name"]]
    assert cli.main([*paths, "--pad", "zero", "--json", "--cpu"]) == 0
    rows = [json.loads(r) for r in capsys.readouterr().out.strip().splitlines()]
    got = np.array([r["logit"] for r in rows])
    assert np.abs(got - g["logit_zero"]).max() < LOGIT_ATOL
    x = cli.prepare(paths, "zero", cpu=True)
    assert np.abs(host.mfcc(x) - g["feat_zero"]).max() < FEAT_ATOL


def test_thread_count_invariance(host, model):
    x = O.synth_clips(7, 0, 37)
    old = host.set_threads(1)
    try:
        a = model.detect(x)
        host.set_threads(5)
        b = model.detect(x)
    finally:
        host.set_threads(old)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("pack", [True, False])
def test_mode_a_reference_config(host, pack):
    x = O.synth_clips(77, 0, 6, 16000)
    got = host.esp_mfcc(x, esp_dsp_packing=pack)
    assert got.shape == (6, 62, 13)
    for i in range(6):
        ref = B.esp_mfcc(x[i], pack)
        assert np.abs(got[i] - ref).max() <= _tol(ref)


GENERAL = [(8000, 200, 80, 256, 26, 12), (16000, 400, 160, 512, 40, 13), (22050, 1024, 512, 1024, 64, 20),
           (16000, 512, 128, 256, 30, 13), (16000, 320, 256, 512, 40, 45), (44100, 2048, 441, 4096, 128, 40),
           (4000, 100, 50, 128, 64, 13)]


@pytest.mark.parametrize("cfg", GENERAL)
def test_extract_mfcc_general_parameters(host, cfg):
    sr, frame, hop, n_fft, nfil, nmfcc = cfg
    L = sr + 777
    x = O.synth_clips(13, 0, 1, L)[0]
    got = host.extract_mfcc(x, L, sr, frame, hop, n_fft, nfil, nmfcc)
    ref = B.esp_mfcc(x, True, sr, frame, hop, n_fft, nfil, nmfcc)
    assert got is not None and got.shape == ref.shape
    assert np.isfinite(got).all()
    assert np.abs(got - ref).max() <= _tol(ref)
    if nmfcc > nfil:
        assert not got[:, nfil:].any()


@pytest.mark.parametrize("L", [320, 575, 16192, 48123])
def test_extract_mfcc_lengths(host, L):
    x = O.synth_clips(5, 0, 1, L)[0]
    got = host.extract_mfcc(x, L)
    ref = B.esp_mfcc(x)
    assert got.shape == ((L - 320) // 256 + 1, 13)
    assert np.abs(got - ref).max() <= _tol(ref)


def test_extract_mfcc_refusals(host):
    """NULL where mfcc.c returns NULL (:434-437) and outside its FFT's domain."""
    x = O.synth_clips(14, 0, 1, 16000)[0]
    assert host.extract_mfcc(x[:100], 100) is None
    assert host.extract_mfcc(x, 16000, 16000, 400, 160, 500, 40, 13) is None
    assert host.extract_mfcc(x, 16000, 16000, 400, 160, 8192, 40, 13) is None
    assert host.extract_mfcc(x, 16000, 16000, 400, 0, 512, 40, 13) is None
    assert host.extract_mfcc(x, 16000, 16000, 400, 160, 512, 0, 13) is None
    assert host.extract_mfcc(x, 16000, 16000, 400, 160, 512, 40, 0) is None
    assert host.extract_mfcc(x, 16000, 16000, 0, 160, 512, 40, 13) is None
    L = host.lib()
    assert not L.extract_mfcc(None, 16000, 16000, 320, 256, 512, 40, 13)
    # the Python wrapper refuses a signal_len past the array (the C side would over-read) and non-1-D input
    with pytest.raises(ValueError):
        host.extract_mfcc(x[:1000], 16000)
    with pytest.raises(ValueError):
        host.extract_mfcc(x.reshape(2, -1))


@pytest.mark.parametrize("cfg", [(16000, 320, 512, 40, 13), (8000, 200, 256, 26, 12), (16000, 512, 512, 64, 13)])
def test_single_frame(host, cfg):
    sr, frame_size, n_fft, nfil, nmfcc = cfg
    L = host.lib()
    fp = C.POINTER(C.c_float)
    frame = O.synth_clips(15, 0, 1, frame_size)[0]
    p = L.flow_extract_mfcc_single_frame(frame.ctypes.data_as(fp), frame_size, sr, n_fft, nfil, nmfcc)
    assert p
    got = np.ctypeslib.as_array(p, shape=(nmfcc,)).copy()
    L.free_mfcc(p)
    ref = B.esp_mfcc(frame, True, sr, frame_size, frame_size, n_fft, nfil, nmfcc, pre=0.0)[0]
    assert np.abs(got - ref).max() <= _tol(ref)
    assert not L.flow_extract_mfcc_single_frame(frame.ctypes.data_as(fp), n_fft + 1, sr, n_fft, nfil, nmfcc)


def test_analyze_mfcc_range(host, capfd):
    L = host.lib()
    v = np.array([1.0, -2.0, np.nan, 4.0], np.float32)
    L.analyze_mfcc_range(v.ctypes.data_as(C.POINTER(C.c_float)), 4, b"t")
    out = capfd.readouterr().out
    assert "min=-2.000000, max=4.000000, avg=1.000000, valid=3/4" in out


def test_bad_arguments(host):
    L = host.lib()
    fp = C.POINTER(C.c_float)
    h = C.c_void_p()
    assert L.wkh_create(None, C.byref(h)) == 1
    assert L.wkh_mfcc(None, 1, 16000, 16000, 1, None) == 1
    x = np.zeros((2, 15000), np.float32)
    out = np.zeros((2, 13, 63), np.float32)
    assert L.wkh_mfcc(x.ctypes.data_as(fp), 2, 15000, 15000, 1, out.ctypes.data_as(fp)) == 1   # mode B: 16000 only
    assert L.wkh_cnn(None, None, 1, None) == 1
    assert b"16000" in L.wkh_last_error() or L.wkh_last_error()
