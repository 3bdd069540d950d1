# round 5 final bundle, part 1: GPU suite, then the headline (fp32) and config-4 (bf16) profile bundles
set -o pipefail
O=$PWD/gpurun_out/r05k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -20 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
bash tools/profile_round.sh r05 || exit $?
bash tools/profile_round.sh r05_bf16 --precision bf16 || exit $?
