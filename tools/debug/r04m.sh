set -o pipefail
O=$PWD/gpurun_out/r04m
mkdir -p $O
bash tools/debug/ctc_ab.sh encg4 encu2 encg4u2 2>&1 | tee $O/ctc_ab.txt
