"""Per-kernel VGPRs / spills / occupancy of a .hip file for gfx950 (hipcc resource-usage remarks).

    python scripts/kres.py clustermachinelearningforhospitalnetworks_apache_spark_amd/_native/csrc/glm.hip [filter]
"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
inc = src.rsplit("/", 1)[0]
r = subprocess.run(["hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-I", inc, "-c", src,
                    "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
cur = {}
rows = []
for line in r.stderr.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (.*?) \[", line)
    if not m:
        if "error" in line:
            print(line)
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    else:
        cur[k] = v
for c in rows:
    name = re.sub(r"\(anonymous namespace\)::", "", c["name"])
    name = re.sub(r"^void ", "", name)
    name = name.split("(")[0]
    if flt in name:
        print(f"{name:70s} vgpr={c.get('VGPRs')} spill={c.get('VGPRs Spill')} occ={c.get('Occupancy [waves/SIMD]')}")
