set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_ctc.py -m gpu -x -q -k "transcribe" --timeout 120 --timeout-method thread > gpurun_out/tshort.log 2>&1; rc=$?; tail -15 gpurun_out/tshort.log; exit $rc
