#!/bin/bash
# Device ISA of every product translation unit with the product flags (for
# "the product ISA did not change" checks):  bash tools/isa_snapshot.sh <dir>
# then  diff -r <dir1> <dir2>  (comments and blank lines stripped).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
D=${1:?outdir}
mkdir -p "$D"
FL="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -fno-signed-zeros -ffp-contract=fast -fno-slp-vectorize -I $R/include -I $R/esp32-wake-word_amd/csrc"
for f in wk_frontend wk_fused wk_fused_xdl wk_misc wk_api wk_ctc wk_int8 wk_esp_mfcc; do
  /opt/rocm/bin/hipcc $FL --cuda-device-only -S "$R/esp32-wake-word_amd/csrc/$f.hip" -o "$D/$f.raw.s" 2>/dev/null &
done
wait
for f in "$D"/*.raw.s; do
  grep -v '^\s*;' "$f" | grep -v '^\s*$' | grep -v '\.file\|\.ident\|amdhsa.version\|\.loc\b\|__hip_cuid' > "${f%.raw.s}.s"
  rm "$f"
done
