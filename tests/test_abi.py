"""CPU tests of the C-ABI library: it loads, exports every symbol the header
declares, and rejects bad arguments before touching the GPU."""
import ctypes as C
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "wakeword.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b([A-Za-z_]\w*)\s*\([^;{]*\)\s*;", txt)))


@pytest.fixture(scope="module")
def L():
    from wakeword import _lib
    return _lib.lib()


def test_header_declares_expected_surface():
    fns = declared_functions()
    for name in ("wk_create", "wk_destroy", "wk_mfcc", "wk_cnn", "wk_forward", "extract_mfcc", "free_mfcc",
                 "analyze_mfcc_range"):
        assert name in fns
    # mfcc.h:7-8,13 declare flow_extract_mfcc / test_mfcc but never define them:
    # the replacement must not export phantom symbols.
    assert "flow_extract_mfcc" not in fns and "test_mfcc" not in fns


def test_library_exports_every_declared_symbol(L):
    from wakeword import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (\w+)", out))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    assert set(_lib.EXPORTS) == set(declared_functions())


def test_abi_version_and_strings(L):
    assert L.wk_abi_version() == 1
    assert L.wk_status_string(0) == b"WK_OK"
    assert L.wk_status_string(1) == b"WK_ERR_INVALID_ARG"


def test_bad_arguments_rejected_without_gpu(L):
    from wakeword import _lib
    h = C.c_void_p()
    assert L.wk_create(None, None, C.byref(h)) == 1
    assert L.wk_mfcc(None, None, 0, 1, 16000, 16000, None, None) == 1
    assert L.wk_cnn(None, None, 1, None, None) == 1
    assert L.wk_forward(None, None, 0, 1, 16000, 16000, None, None, None) == 1
    assert L.wk_synth_clips(0, 0, -1, 16000, None, None) == 1
    assert L.wk_normalize(None, None, 1, 13, 63, 9, None) == 1
    # mfcc.c:434-437: NULL signal / too short -> NULL
    assert not L.extract_mfcc(None, 16000, 16000, 320, 256, 512, 40, 13)
    buf = (C.c_float * 100)()
    assert not L.extract_mfcc(buf, 100, 16000, 320, 256, 512, 40, 13)
    cfg = _lib.WkConfig(7, 0, 0, 0, 1)   # bad mode
    assert L.wk_create(C.byref(cfg), None, C.byref(h)) == 1
    # CTC entry points: a NULL handle is rejected before any device work
    assert L.wk_ctc_features(None, None, 1, 48000, 48000, 48000, None, None) == 1
    assert L.wk_ctc_forward(None, None, 1, 301, None, None, None, None) == 1
    assert L.wk_ctc_transcribe(None, None, 1, 48000, 48000, 48000, None, None, None) == 1


def test_analyze_mfcc_range_output(L, capfd):
    import numpy as np
    x = np.array([1.0, -2.0, np.nan, 3.0, np.inf], np.float32)
    L.analyze_mfcc_range(x.ctypes.data_as(C.POINTER(C.c_float)), 5, b"probe")
    out = capfd.readouterr().out
    assert "probe MFCC Range: min=-2.000000, max=3.000000, avg=0.666667, valid=3/5" in out


def test_pack_weights_layout(xiaoa_sd):
    from wakeword.api import pack_weights
    blob = pack_weights(xiaoa_sd)
    assert blob.size == 40224 and blob.dtype.name == "float32"
    assert blob[0] == xiaoa_sd["conv_layers.0.weight"].reshape(-1)[0]
    assert blob[-1] == xiaoa_sd["classifier.2.weight"].reshape(-1)[-1]


def test_every_export_has_a_ctypes_prototype(L):
    """The Python binding declares argument types for every C entry point (an
    undeclared prototype silently truncates int64 / float arguments)."""
    from wakeword import _lib
    no_args = {"wk_last_error", "wk_abi_version"}
    for name in _lib.EXPORTS:
        if name not in no_args:
            assert getattr(L, name).argtypes is not None, name


def test_product_links_only_the_hip_runtime():
    """Every kernel is hand-written: the library needs the HIP runtime and the
    C/C++ runtime, no vendor math library (rocBLAS, hipBLAS(Lt), MIOpen, ...)."""
    from wakeword import _lib
    out = subprocess.run(["readelf", "-d", _lib.LIB_PATH], capture_output=True, text=True).stdout
    needed = re.findall(r"\(NEEDED\)\s+Shared library: \[([^\]]+)\]", out)
    assert any(n.startswith("libamdhip64") for n in needed), needed
    banned = ("rocblas", "hipblas", "miopen", "rocfft", "hipfft", "rccl", "rocsparse", "torch")
    assert not [n for n in needed if any(b in n.lower() for b in banned)], needed
