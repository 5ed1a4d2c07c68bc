"""Per-kernel VGPR / AGPR / SGPR / spill / LDS table of one translation unit, from hipcc's
kernel-resource-usage remarks (gfx950):  python tools/res_table.py FILE.hip [REGEX]"""
import os
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else "."
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC",
       "-I" + os.path.join(root, "include"), "-Rpass-analysis=kernel-resource-usage",
       "-c", src, "-o", "/tmp/res_table.o"] + sys.argv[3:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for ln in out.splitlines():
    m = re.search(r"Function Name: (\S+)", ln)
    if m:
        cur = {"fn": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark: +(VGPRs|AGPRs|SGPRs|VGPRs Spill|SGPRs Spill|LDS Size \[bytes/block\]): (\d+)", ln)
    if m and cur is not None:
        cur[m.group(1)] = m.group(2)
for r in rows:
    if re.search(flt, r["fn"]):
        g = lambda k: r.get(k, "?")
        print(f"{g('VGPRs'):>4}v {g('AGPRs'):>3}a {g('SGPRs'):>3}s spill v{g('VGPRs Spill')}/s{g('SGPRs Spill')} "
              f"lds {g('LDS Size [bytes/block]'):>6}  {r['fn'][:120]}")
