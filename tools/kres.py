"""Per-kernel resource table of one HIP source (VGPRs, AGPRs, scratch, occupancy, LDS) from the
compiler's kernel-resource-usage remarks.  usage: python tools/kres.py csrc/remap.hip [name-filter]"""
import os
import re
import subprocess
import sys

src = os.path.abspath(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "--offload-arch=gfx950", "-x", "hip",
       "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True, cwd=os.path.dirname(src)).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?)(?: \[-Rpass)", line)
    if not m:
        continue
    body = m.group(1).strip()
    if body.startswith("Function Name:"):
        name = body.split(":", 1)[1].strip()
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        cur = {"name": dem.replace("gtfv3::(anonymous namespace)::", "")}
        rows.append(cur)
    elif cur is not None and ":" in body:
        k, v = body.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if flt and flt not in r["name"]:
        continue
    print(f"{r.get('VGPRs', '?'):>4} v {r.get('AGPRs', '?'):>3} a {r.get('ScratchSize [bytes/lane]', '?'):>4} scr "
          f"{r.get('Occupancy [waves/SIMD]', '?'):>2} occ {r.get('LDS Size [bytes/block]', '?'):>6} lds  {r['name'][:110]}")
