# round 5, K = 32 question: does the K = 32 MFMA's register placement matter?
# (probe modes 4-6: A/B, everything, or the accumulator in AGPRs), on the
# reproducing VALU loop (variant 1312: DFT16 twiddles + row pass) and the full DFT16
set -o pipefail
O=$PWD/gpurun_out/r05aq
mkdir -p $O
for v in 1312 32; do
  XDL_PROBE_MODES=0123456 timeout -k 10 120 ./tools/debug/xdl_probe 2 20000 $v >> $O/probe13.txt 2>&1 || { cat $O/probe13.txt; exit 1; }
done
grep -v "^workgroup" $O/probe13.txt | sed 's/by lane:.*by output float/by output float/' | cut -c1-200
