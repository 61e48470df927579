"""Per-kernel resource usage (VGPR/SGPR/spill/LDS) from a hipcc -S device assembly file."""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
meta = s[s.index("amdhsa.kernels:"):]
for m in re.finditer(r"\.name:\s+(\S+)\n(.*?)(?=\n  - |\n\.end_amdgpu_metadata)", meta, re.S):
    name, body = m.group(1), m.group(2)
    if pat and not re.search(pat, name):
        continue
    f = dict(re.findall(r"\.(vgpr_count|sgpr_count|vgpr_spill_count|group_segment_fixed_size|agpr_count):\s+(\d+)", body))
    print(f"{name[:90]:90s} vgpr={f.get('vgpr_count')} agpr={f.get('agpr_count')} sgpr={f.get('sgpr_count')} spill={f.get('vgpr_spill_count')}")
