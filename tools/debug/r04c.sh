set -o pipefail
bash tools/debug/ab.sh base prod 2>&1 | tee gpurun_out/r04b/ab_fp32.txt
AB_ARGS="--precision bf16" bash tools/debug/ab.sh base prod 2>&1 | tee gpurun_out/r04b/ab_bf16.txt
