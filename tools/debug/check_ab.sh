#!/bin/bash
# GPU round trip for a kernel change: the -m gpu suite on the in-tree library,
# then an A/B bench of the in-tree library against build/var_<name> variants.
#   bash tools/debug/check_ab.sh <variant...>      (AB_ARGS passes bench flags)
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?; tail -3 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
bash tools/debug/ab.sh prod "$@"
