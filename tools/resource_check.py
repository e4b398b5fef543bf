"""Compile one HIP translation unit with -Rpass-analysis=kernel-resource-usage and list kernels whose
name matches a pattern: VGPRs, AGPRs, scratch (spills), occupancy.
  python tools/resource_check.py whisper_context_biasing_amd/csrc/k_gemm_bf16.hip gemm_dec [--all]"""
import re
import subprocess
import sys

src, pat = sys.argv[1], sys.argv[2]
show_all = "--all" in sys.argv
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                    "-c", src, "-o", "/tmp/_rc.o", "-Rpass-analysis=kernel-resource-usage"],
                   capture_output=True, text=True)
cur, rows = None, []
for line in r.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split()[0]] = int(m.group(2))
for c in rows:
    if pat in c["name"] and (show_all or c.get("ScratchSize", 0) > 0 or c.get("VGPRs", 0) + c.get("AGPRs", 0) > 256):
        print(f"{c['name'][:90]:90s} VGPR {c.get('VGPRs')} AGPR {c.get('AGPRs')} scratch {c.get('ScratchSize')} occ {c.get('Occupancy')}")
print(f"{sum(pat in c['name'] for c in rows)} kernels matched; rc {r.returncode}")
