"""Map the per-kernel PMC means of a bench_ctc.py run (tools/pmc_summary.py
--json) to bench_ctc's stages: HBM bytes per launch = corrected FETCH_SIZE
(x2 on gfx950) + WRITE_SIZE.  Kernels launched once per layer (the GRU
recurrence, the projection GEMM) give both layers' stages their mean.

    python tools/ctc_traffic.py pmc.json <source-name> > profiles/ctc_hbm_traffic.json
"""
import json
import sys

MAP = [("ctc_logmel_fft", ["logmel"]), ("ctc_zscore_kernel", ["zscore"]), ("ctc_zstats_kernel", ["zscore"]),
       ("ctc_encoder16_kernel", ["encoder"]), ("ctc_encoder_kernel", ["encoder"]),
       ("ctc_proj16_kernel", ["proj0", "proj1"]), ("Cijk", ["proj0", "proj1"]),
       ("ctc_gru16x_kernelILi128", ["gru0"]), ("ctc_gru16x_kernelILi256", ["gru1"]),
       ("ctc_gru16_kernel", ["gru0", "gru1"]), ("ctc_gru_kernel", ["gru0", "gru1"]),
       ("ctc_out_argmax16_kernel", ["output"]), ("ctc_out_decode16_kernel", ["output"]),
       ("ctc_greedy_kernel", ["decode"])]


def main():
    pmc = json.load(open(sys.argv[1]))
    per = {}
    for name, rec in pmc.items():
        if "hbm_read_bytes_corrected" not in rec or "hbm_write_bytes" not in rec:
            continue
        for key, stages in MAP:
            if key in name:
                for s in stages:   # several kernel names on one stage (e.g. rocBLAS per K): their mean
                    per.setdefault(s, []).append(rec["hbm_read_bytes_corrected"] + rec["hbm_write_bytes"])
                break
    out = {s: sum(v) / len(v) for s, v in per.items()}
    print(json.dumps({"fp16": {k: round(v) for k, v in out.items()},
                      "source": sys.argv[2] if len(sys.argv) > 2 else sys.argv[1],
                      "note": "HBM bytes per launch: 2 x FETCH_SIZE + WRITE_SIZE (rocprofv3 --pmc, separate passes)"},
                     indent=1))


if __name__ == "__main__":
    main()
