"""Per-kernel register / LDS / scratch metadata from a `hipcc --cuda-device-only -S` listing."""
import re, sys
txt = open(sys.argv[1]).read()
meta = txt[txt.find('amdhsa.kernels:'):]
for blk in re.split(r'\n  - ', meta)[1:]:
    name = re.search(r'\.name:\s+(\S+)', blk)
    if not name or not any(p in name.group(1) for p in sys.argv[2:] or ['']):
        continue
    g = lambda k: (re.search(r'\.' + k + r':\s+(\d+)', blk) or [None, '?'])[1]
    print(f"{name.group(1)[:60]:60s} vgpr {g('vgpr_count'):>4} sgpr {g('sgpr_count'):>4} lds {g('group_segment_fixed_size'):>6} "
          f"scratch {g('private_segment_fixed_size'):>4} spill {g('vgpr_spill_count')}")
