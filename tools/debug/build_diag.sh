#!/bin/bash
# Diagnostic library with in-kernel s_memtime phase stamps (never the product).
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
cd "$R/esp32-wake-word_amd"
HIPCC=/opt/rocm/bin/hipcc
FL="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -fno-signed-zeros -ffp-contract=fast -fno-slp-vectorize -I $R/include -I csrc -DWK_DIAG"
mkdir -p build/diag
for f in wk_frontend wk_fused wk_fused_xdl wk_misc wk_api wk_ctc wk_int8 wk_esp_mfcc; do $HIPCC $FL -c csrc/$f.hip -o build/diag/$f.o & done; wait
$HIPCC $FL -c csrc/wk_wav.cpp -o build/diag/wk_wav.o || { echo "compile of wk_wav failed"; exit 1; }
$HIPCC --offload-arch=gfx950 -shared -fPIC build/diag/*.o -Wl,-rpath,/opt/rocm/lib -o build/diag/libwakeword_diag.so
echo "$R/esp32-wake-word_amd/build/diag/libwakeword_diag.so"
