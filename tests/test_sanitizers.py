"""ASan + UBSan over the host C/C++ that reads untrusted input or is the
checker ("race detection / sanitizers"): the WAV ingest
(csrc/wk_wav.cpp, replacing esp_wav.cpp:8-139) under truncated, corrupted,
odd-chunk and mis-declared files, and the C oracle (oracle/esp_mfcc_oracle.c)
over its edge parameter sets.  Host-only builds with clang (-fsanitize=
address,undefined, -fno-sanitize-recover=all: any report fails the run);
no GPU code is instrumented and nothing here runs on the GPU box."""
import glob
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/llvm/bin/clang++"
CLANGC = "/opt/rocm/llvm/bin/clang"
SAN = ["-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=66",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=67")

pytestmark = pytest.mark.skipif(not os.path.exists(CLANG), reason="ROCm clang not found")


def _run(cmd, sanitized_run=False):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=ENV if sanitized_run else None)
    assert r.returncode == 0, (cmd[0], r.stdout[-3000:], r.stderr[-3000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    return r


def test_wav_ingest_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "wav_harness")
    _run([CLANG, "-std=c++17", *SAN, "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I", os.path.join(REPO, "include"),
          "-I", os.path.join(REPO, "esp32-wake-word_amd", "csrc"), "-x", "c++",
          os.path.join(REPO, "esp32-wake-word_amd", "csrc", "wk_wav.cpp"), "-x", "none",
          os.path.join(REPO, "tests", "sanitize", "wav_harness.cpp"), "-o", exe, "-lpthread"])
    wavs = sorted(glob.glob(os.path.join(REPO, "tests", "golden", "wav", "*.wav")))[:3]
    assert wavs
    r = _run([exe, str(tmp_path), *wavs], sanitized_run=True)
    assert "accepted" in r.stdout


def test_c_oracle_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "oracle_harness")
    _run([CLANGC, *SAN, os.path.join(REPO, "oracle", "esp_mfcc_oracle.c"),
          os.path.join(REPO, "tests", "sanitize", "oracle_harness.c"), "-o", exe, "-lm", "-lpthread"])
    r = _run([exe], sanitized_run=True)
    assert "runs" in r.stdout
