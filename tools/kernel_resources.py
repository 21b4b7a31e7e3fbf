"""VGPRs / scratch / occupancy of every trace_kernel instantiation, from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (a build of csrc/trace_kernel.hip for
gfx950 with the Makefile's flags). Usage: python tools/kernel_resources.py [filter]"""
import re
import subprocess
import sys

PKG = __file__.rsplit("/tools/", 1)[0] + "/gpu-ray-tracing_amd"
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-fgpu-flush-denormals-to-zero",
       "-ffp-contract=off", "-fno-slp-vectorize", "-I../include", "-c", "csrc/trace_kernel.hip", "-o", "/tmp/_tk.o",
       "--offload-device-only", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
txt = subprocess.run(cmd, cwd=PKG, capture_output=True, text=True).stderr
flt = sys.argv[1] if len(sys.argv) > 1 else ""
name = None
rows = {}
for line in txt.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = m.group(1)
        rows[name] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\S+) \[", line)
    if m and name:
        rows[name][m.group(1).strip()] = m.group(2)
for n, r in rows.items():
    if "trace_kernel" in n and flt in n:
        print(f"{n[:70]:70s} VGPR {r.get('VGPRs')} scratch {r.get('ScratchSize')} occ {r.get('Occupancy')} "
              f"spill {r.get('VGPRs Spill')}")
