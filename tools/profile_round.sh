#!/bin/bash
# Round-end measurement bundle (run on the GPU box through gpurun):
#   bash tools/profile_round.sh <tag> [bench args...]   (e.g. --precision bf16)
# writes into gpurun_out/prof_<tag>/ (gpurun merges only gpurun_out/ back); then,
# in the build container, `bash tools/profile_round.sh <tag> --collect` copies
# the summaries into profiles/:
#   <tag>_bench.json          bench.py line (default config, with cpu_baseline)
#   <tag>_kernel_stats.csv    rocprofv3 --kernel-trace --stats of the same bench command
#   <tag>_bench_profiled.json the bench line printed under rocprofv3
#   <tag>_pmc.json            per-kernel PMC means (tools/pmc_summary.py)
#   hbm_traffic.json          HBM bytes per window of the fused kernel (read by bench.py)
set -e -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:?tag}
OUT=$R/gpurun_out/prof_$TAG
if [ "$2" = "--collect" ]; then
  mkdir -p "$R/profiles"
  grep "^{\"metric\"" "$OUT/bench.log" | tail -1 > "$R/profiles/${TAG}_bench.json"
  grep "^{\"metric\"" "$OUT/prof.log" | tail -1 > "$R/profiles/${TAG}_bench_profiled.json"
  cp "$OUT/trace/run_kernel_stats.csv" "$R/profiles/${TAG}_kernel_stats.csv"
  cp "$OUT/pmc_summary.txt" "$R/profiles/${TAG}_pmc_summary.txt"
  cp "$OUT/${TAG}_pmc.json" "$R/profiles/${TAG}_pmc.json"
  cp "$OUT"/hbm_traffic*.json "$R/profiles/"
  exit 0
fi
shift
BARGS="$*"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 bench.py $BARGS > "$OUT/bench.log" 2> "$OUT/bench.err"
echo "bench: $(tail -1 $OUT/bench.log | cut -c1-200)"
cd /tmp && export TMPDIR=/tmp
# 40 timed steps so the 2 warm-up launches weigh little in the kernel's mean; the
# profiled bench line (prof.log) carries the same command's own HIP-event launch time
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-extras --steps 40 --warmup 2 $BARGS > "$OUT/prof.log" 2>&1
cd "$R"
timeout -k 10 900 bash tools/profile_pmc.sh "$OUT/pmc" --steps 2 --warmup 1 --no-cpu-baseline --no-extras $BARGS > "$OUT/pmc.log" 2>&1
python3 tools/pmc_summary.py "$OUT/pmc" --json "$OUT/${TAG}_pmc.json" > "$OUT/pmc_summary.txt"
case "$BARGS" in *bf16x3*) BF=2; TF=hbm_traffic_bf16x3.json ;; *bf16*) BF=1; TF=hbm_traffic_bf16.json ;; *) BF=0; TF=hbm_traffic.json ;; esac
python3 - "$OUT/${TAG}_pmc.json" "$OUT/$TF" "$TAG" "$BF" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
kname = f"wk_fused_kernel<float, {sys.argv[4]}, false>"
k = next(v for n, v in d.items() if n.startswith(kname))
B = 65536   # bench default batch (tools/profile_pmc.sh runs the default bench)
rd, wr = k["hbm_read_bytes_corrected"], k.get("hbm_write_bytes", 0.0)
json.dump({"bytes_per_window": (rd + wr) / B, "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
           "batch": B, "source": f"profiles/{sys.argv[3]}_pmc.json (rocprofv3 --pmc FETCH_SIZE x2 gfx950 "
           f"correction + WRITE_SIZE, {kname})"}, open(sys.argv[2], "w"), indent=1)
print("hbm bytes/window", (rd + wr) / B)
PY
