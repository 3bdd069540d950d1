#!/bin/bash
# Build libwakeword.so of a git revision (A/B base for a change in the working
# tree):  bash tools/debug/build_rev.sh <rev> <name> [-DFLAG ...]
#   -> variants/var_<name>/libwakeword.so   (time it with ab.sh prod <name>)
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
REV=$1; NAME=$2; shift 2
WT=/tmp/wk_rev_$NAME
rm -rf "$WT"; git -C "$R" worktree prune
git -C "$R" worktree add --detach "$WT" "$REV" > /dev/null
cd "$WT/esp32-wake-word_amd"
HIPCC=/opt/rocm/bin/hipcc
FL="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -fno-signed-zeros -ffp-contract=fast -fno-slp-vectorize -I $WT/include -I csrc $*"
D=$R/variants/var_$NAME
mkdir -p "$D"; rm -f "$D"/*.o
SRCS=$(ls csrc/*.hip csrc/wk_wav.cpp 2>/dev/null)
for f in $SRCS; do $HIPCC $FL -c $f -o "$D/$(basename ${f%.*}).o" & done; wait
for f in $SRCS; do [ -f "$D/$(basename ${f%.*}).o" ] || { echo "compile of $f failed"; exit 1; }; done
LIBS="-Wl,-rpath,/opt/rocm/lib"
grep -q rocblas csrc/wk_ctc.hip && LIBS="-L/opt/rocm/lib -lrocblas $LIBS"   # (revisions before the hand-written CTC GEMM)
$HIPCC --offload-arch=gfx950 -shared -fPIC "$D"/*.o $LIBS -o "$D/libwakeword.so"
rm -f "$D"/*.o
git -C "$R" worktree remove --force "$WT"
echo "$D/libwakeword.so"
