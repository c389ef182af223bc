#!/usr/bin/env python
"""Print per-kernel VGPR / SGPR / occupancy / LDS from hipcc -Rpass-analysis=kernel-resource-usage."""
import re, subprocess, sys
src = sys.argv[1] if len(sys.argv) > 1 else "non-iid-topology-simulator_amd/csrc/niidmix.hip"
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17",
                      "--cuda-device-only", "-c", "-o", "/dev/null", src,
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark:\s+([^:]+):\s*(.*?)\s*\[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    n = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    n = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "")).replace("void ", "")
    if flt in n:
        print(f"{n:48s} VGPR {r.get('VGPRs','?'):>4} AGPR {r.get('AGPRs','?'):>3} SGPR {r.get('TotalSGPRs','?'):>4} "
              f"occ {r.get('Occupancy [waves/SIMD]','?')} LDS {r.get('LDS Size [bytes/block]','?')} "
              f"spill {r.get('VGPRs Spill','?')}/{r.get('SGPRs Spill','?')}")
