set -o pipefail
O=$PWD/gpurun_out/r04s
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/gputest.log 2>&1; rc=$?; tail -2 $O/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
bash tools/profile_round.sh r04s || exit $?
bash tools/pmc_census.sh $O/census > $O/census.log 2>&1 || exit $?
python tools/pmc_census.py $O/census --json $O/census.json > $O/census.txt 2>&1
bash tools/debug/ab.sh prod sleep1 sleep4 prod sleep1 sleep4 2>&1 | tee $O/ab.txt
