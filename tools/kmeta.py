"""Register counts and spills per kernel from a gfx950 assembly file's metadata
(developer tool): python tools/kmeta.py file.s [name-substring]"""
import re
import sys

txt = open(sys.argv[1]).read()
meta = txt[txt.find("amdhsa.kernels:"):]
for rec in re.split(r"\n  - ", meta)[1:]:
    f = dict(re.findall(r"\.(\w+):\s+(\S+)", rec))
    name = f.get("name", "?")
    if len(sys.argv) > 2 and sys.argv[2] not in name:
        continue
    print(f"{name[:90]:90s} vgpr {f.get('vgpr_count')} agpr {f.get('agpr_count')} "
          f"spill {f.get('vgpr_spill_count')} sgpr {f.get('sgpr_count')} lds {f.get('group_segment_fixed_size')}")
