"""Per-kernel VGPR/AGPR/LDS/occupancy/spill report for a .hip file (hipcc remarks)."""
import re, subprocess, sys
src = sys.argv[1]; extra = sys.argv[2:]
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o",
                    "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage", *extra], capture_output=True, text=True)
cur = None; info = {}
for line in r.stderr.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m: continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip(); info[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1); info[cur][k.strip()] = v.strip()
for f, d in info.items():
    name = subprocess.run(["c++filt", f], capture_output=True, text=True).stdout.strip()
    name = name.replace("(anonymous namespace)::", "")
    print(f"{d.get('VGPRs','?'):>4} v {d.get('AGPRs','?'):>3} a  occ {d.get('Occupancy [waves/SIMD]','?'):>2}  "
          f"lds {d.get('LDS Size [bytes/block]','?'):>6}  spill {d.get('VGPRs Spill','?')}/{d.get('ScratchSize [bytes/lane]','?')}  {name[:90]}")
if r.returncode: print(r.stderr[-2000:])
