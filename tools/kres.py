"""Per-kernel VGPR / scratch / occupancy / LDS of one HIP source (hipcc -Rpass-analysis=kernel-resource-usage).
    python tools/kres.py torch-optical-flow_amd/csrc/conv_s32.hip [regex] [-D...]"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("-D") else ".")
defs = [a for a in sys.argv[2:] if a.startswith("-D")]
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Iinclude", "-I../../include",
                      "-fno-slp-vectorize", "-fno-vectorize", *defs, "-c", src, "-o", "/dev/null",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = {}
for line in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        if cur and pat.search(cur["name"]):
            print(f"{cur['name'][:80]:80s} vgpr {cur.get('VGPRs')} agpr {cur.get('AGPRs')} scratch {cur.get('ScratchSize [bytes/lane]')} occ {cur.get('Occupancy [waves/SIMD]')} lds {cur.get('LDS Size [bytes/block]')}")
        cur = {"name": re.sub(r"_ZN5oflow12_GLOBAL__N_1\d+", "", v)}
    else:
        cur[k] = v
if cur and pat.search(cur["name"]):
    print(f"{cur['name'][:80]:80s} vgpr {cur.get('VGPRs')} agpr {cur.get('AGPRs')} scratch {cur.get('ScratchSize [bytes/lane]')} occ {cur.get('Occupancy [waves/SIMD]')} lds {cur.get('LDS Size [bytes/block]')}")
