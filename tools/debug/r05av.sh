# round 5: the product with the bf16-family fused kernel in its own unit
# (scalar-fp32 front-end): GPU suite, then A/B against the all-packed build
# (-DWK_FE_PACKED_ALL) in bf16, bf16x3 and fp32
set -o pipefail
O=$PWD/gpurun_out/r05av
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1 || { tail -20 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
for p in bf16 bf16x3 fp32; do
  echo "== $p" >> $O/ab.txt
  AB_ARGS="--precision $p" timeout -k 10 400 bash tools/debug/ab.sh prod pk >> $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
done
cat $O/ab.txt
