set -o pipefail
O=$PWD/gpurun_out/r04q
mkdir -p $O
bash tools/round_bundle.sh r04q || exit $?
bash tools/pmc_census.sh $O/census > $O/census.log 2>&1 || exit $?
python tools/pmc_census.py $O/census --json $O/census.json > $O/census.txt 2>&1
