#!/bin/bash
# Build a variant of the library with extra compile flags (experiments only):
#   bash tools/debug/build_variant.sh <name> [-DFOO=1 ...]  -> build/var_<name>/libwakeword.so
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
NAME=$1; shift
cd "$R/esp32-wake-word_amd"
HIPCC=/opt/rocm/bin/hipcc
FL="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -fno-signed-zeros -ffp-contract=fast -fno-slp-vectorize -I $R/include -I csrc $*"
D=$R/variants/var_$NAME
mkdir -p $D
rm -f $D/*.o
for f in wk_frontend wk_fused wk_fused_xdl wk_misc wk_api wk_ctc wk_int8 wk_esp_mfcc; do $HIPCC $FL -c csrc/$f.hip -o $D/$f.o & done; wait
$HIPCC $FL -c csrc/wk_wav.cpp -o $D/wk_wav.o || { echo "compile of wk_wav failed"; exit 1; }
for f in wk_frontend wk_fused wk_fused_xdl wk_misc wk_api wk_ctc wk_int8 wk_esp_mfcc; do [ -f $D/$f.o ] || { echo "compile of $f failed"; exit 1; }; done
$HIPCC --offload-arch=gfx950 -shared -fPIC $D/*.o -Wl,-rpath,/opt/rocm/lib -o $D/libwakeword.so
echo "$D/libwakeword.so"
