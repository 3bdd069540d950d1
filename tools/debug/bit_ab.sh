#!/bin/bash
# Bit compare of variants against the first one (bitcmp.py: logits and
# features of every precision, both MFCC modes), then ab4.sh's timing.
#   bash tools/debug/bit_ab.sh base name2 ...   ("prod" = the in-tree library)
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
cd "$R"
O=gpurun_out/bit_ab; mkdir -p $O
lib() { if [ "$1" = prod ]; then echo $R/esp32-wake-word_amd/wakeword/libwakeword.so; else echo $R/variants/var_$1/libwakeword.so; fi; }
for v in "$@"; do
  WAKEWORD_LIB=$(lib $v) timeout -k 10 200 python tools/debug/bitcmp.py dump $O/$v.npz > $O/dump_$v.log 2>&1 || { tail -5 $O/dump_$v.log; rm -f $O/*.npz; exit 1; }
done
rc=0
for v in "${@:2}"; do echo "$v vs $1:"; python tools/debug/bitcmp.py cmp $O/$1.npz $O/$v.npz || rc=1; done
rm -f $O/*.npz   # the dumps would exceed gpurun's copy-back limit
[ $rc = 0 ] && bash tools/debug/ab4.sh "$@"
