"""Per-kernel register / spill / LDS table of one translation unit (dev tool).

    python tools/res_usage.py wk_fused.hip [extra hipcc flags...]
"""
import os
import re
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-fno-signed-zeros",
       "-ffp-contract=fast", "-fno-slp-vectorize", "-I", f"{R}/include", "-I", f"{R}/esp32-wake-word_amd/csrc",
       *sys.argv[2:], "-c", f"{R}/esp32-wake-word_amd/csrc/{src}", "-o", "/tmp/res_usage.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    if "error" in line and "remark" not in line:
        print(line)
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt"], input=v, capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    else:
        cur[k] = v
for r in rows:
    print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('VGPRs Spill', '?'):>3} vspill {r.get('SGPRs Spill', '?'):>3} sspill "
          f"{r.get('LDS Size [bytes/block]', '?'):>6} lds  {r['name'][:120]}")
