#!/bin/bash
# Front-end occupancy experiment: the standalone front-end kernel at 1 and 2
# workgroups per CU (2 / 4 front-end waves per SIMD, same code), the fused kernel's front-end
# role alone, and issue PMC for both occupancies.  Needs the WK_DIAG library in variants/var_diag.
set -o pipefail
R=/root/repo; O=$R/gpurun_out/r06d; mkdir -p $O; cd $R
export WAKEWORD_LIB=$R/variants/var_diag/libwakeword.so   # (bash tools/debug/build_diag.sh, copied there: build/ does not travel)
for pass in 1 2; do for w in 1 2; do
  WAKEWORD_FE_WG_PER_CU=$w timeout -k 10 120 python tools/debug/fe_rate.py > $O/fe_wg${w}_p$pass.txt 2>&1 || exit $?
  echo "wg/cu=$w pass $pass: $(tail -1 $O/fe_wg${w}_p$pass.txt)"
done; done
EXPS=1 PRECS=fp32 bash tools/debug/roles.sh || exit $?
cd /tmp && export TMPDIR=/tmp
for w in 1 2; do
  WAKEWORD_FE_WG_PER_CU=$w timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d $O/pmc_wg$w -o run --output-format csv -- python3 $R/tools/debug/fe_rate.py > $O/pmc_wg$w.log 2>&1 || exit $?
done
echo done
