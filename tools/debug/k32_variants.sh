#!/bin/bash
# Diagnostic library variants of the K=32 bf16 MFMA investigation (DESIGN.md 5.1,
# round 3); probes: tools/debug/k32_probe.py via k32_probe_run*.sh.
set -e
B="bash $(dirname "$0")/build_variant.sh"
K="-DWK_MFMA_K32 -DWK_ALLOW_K32_DIAG"
$B k32dbg   $K -DWK_DEBUG_LOGMEL &                      # log-mel copies (front-end / DCT input)
$B k32pad   $K -DWK_K32_PAD &                           # >= 8 wait states after every K=32 MFMA
$B k32noepi $K -DWK_DEBUG_LOGMEL -DWK_ABL_NOEPI &       # no CNN epilogue LDS stores
$B k32gap   $K -DWK_DEBUG_LOGMEL -DWK_ABL_NOGAPST &     # no GAP stores
$B k32pool  $K -DWK_DEBUG_LOGMEL -DWK_ABL_NOPOOLST &    # no pool stores
$B k32chk   $K -DWK_DEBUG_LOGMEL -DWK_EPI_CHECK &       # bounds check of every epilogue store
$B k16dbg   -DWK_DEBUG_LOGMEL &                         # control: the product's K=16 pair
wait
