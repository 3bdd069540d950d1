"""CPU test: the K = 32 rule holds in the shipped library's gfx950 ISA.

A kernel that issues a K-doubled MFMA (v_mfma_f32_16x16x32_bf16/f16,
v_mfma_i32_16x16x64_i8, ...) must issue no packed-fp32 VALU op (v_pk_*_f32):
DESIGN.md 5.1 records packed-fp32 results corrupted in lanes 48-63 beside
such an MFMA on the same SIMD.  The check disassembles every kernel of
libwakeword.so (tools/isa_rules.py), so a source or compiler change that
brings the combination back fails here, before any GPU run.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

import isa_rules  # noqa: E402

if not os.path.exists(os.path.join(isa_rules.LLVM_BIN, "llvm-objdump")):
    pytest.skip("llvm-objdump not found", allow_module_level=True)


@pytest.fixture(scope="module")
def stats():
    from wakeword import _lib
    assert os.path.exists(_lib.LIB_PATH), "build libwakeword.so first (python -m wakeword.build)"
    return isa_rules.kernel_stats(_lib.LIB_PATH)


def _find(stats, *parts):
    return [k for k in stats if all(p in k for p in parts)]


def test_every_kernel_obeys_the_k32_rule(stats):
    bad = isa_rules.k32_violations(stats)
    detail = {k: stats[k]["pk_lines"][:4] for k in bad}
    assert not bad, detail


def test_rule_is_not_vacuous(stats):
    # The product's K = 32 users are present and counted: the bf16 / split-bf16
    # fused kernels, the standalone bf16 CNN, the int8 network, the CTC kernels.
    for parts in (("wk_fused_kernel<float, 1",), ("wk_fused_kernel<float, 2",), ("wk_cnn_fused_kernel<1>",),
                  ("wk_cnn_fused_kernel<2>",), ("wk_int8_mfma_kernel",), ("ctc_out_decode16_kernel",)):
        ks = _find(stats, *parts)
        assert ks, parts
        assert all(stats[k]["k32"] > 0 for k in ks), parts
    # ... and the packed-fp32 users are seen too (the fp32 fused kernel's
    # front-end beside its K = 4 fp32 MFMAs, which the rule allows).
    ks = _find(stats, "wk_fused_kernel<float, 0")
    assert ks and all(stats[k]["pk_f32"] > 100 and stats[k]["k32"] == 0 for k in ks)


def test_bf16_family_has_no_packed_fp32(stats):
    for parts in (("wk_fused_kernel<", ", 1, "), ("wk_fused_kernel<", ", 2, "), ("wk_cnn_fused_kernel<1>",),
                  ("wk_cnn_fused_kernel<2>",)):
        for k in _find(stats, *parts):
            assert stats[k]["pk_f32"] == 0, (k, stats[k]["pk_lines"][:4])
