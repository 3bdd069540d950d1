# round 5: CTC PMC bundle on the decode-only output kernel
set -o pipefail
timeout -k 10 900 bash tools/ctc_pmc.sh r05q > gpurun_out/ctcpmc_r05q.log 2>&1 || { tail -5 gpurun_out/ctcpmc_r05q.log; exit 1; }
tail -14 gpurun_out/ctcpmc_r05q.log
