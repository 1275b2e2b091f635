"""Dev tool: per-kernel VGPR / AGPR / spill / LDS counts from the AMDGPU metadata of a hipcc -S listing.

usage: python tools/kmeta.py listing.s [kernel-substring ...]"""
import re
import sys

txt = open(sys.argv[1]).read()
pats = sys.argv[2:]
for blk in re.split(r"\n\s+- \.agpr_count:", txt)[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if pats and not any(p in name for p in pats):
        continue
    g = lambda k: (re.search(r"\.%s:\s+(\d+)" % k, blk) or [None, "?"])[1]
    agpr = blk.split("\n", 1)[0].strip()
    print(f"{name[:90]:90s} vgpr={g('vgpr_count')} agpr={agpr} vspill={g('vgpr_spill_count')} "
          f"sspill={g('sgpr_spill_count')} lds={g('group_segment_fixed_size')}")
