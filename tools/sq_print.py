"""Print the SQ instruction/occupancy mix per kernel from a tools/summarize_pmc.py summary:
    python tools/sq_print.py <summary.json> [name-filter,...]
(quad-cycle counters, guides/MI355X_MICROARCH.md: cyc/wave is in units of 4 cycles)."""
import json
import sys

d = json.load(open(sys.argv[1]))
flt = sys.argv[2].split(",") if len(sys.argv) > 2 else []
for k, r in d.items():
    if flt and not any(f in k for f in flt):
        continue
    wc, w = r.get("SQ_WAVE_CYCLES", 0), r.get("SQ_WAVES", 0)
    if not wc or not w:
        continue
    print(k[:44], "waves", int(w), "cyc/wave", int(wc / w),
          "active %.2f parked %.2f stalled %.2f valu-active %.2f" % (
              r["SQ_ACTIVE_INST_ANY"] / wc, r["SQ_WAIT_ANY"] / wc, r["SQ_WAIT_INST_ANY"] / wc,
              r["SQ_ACTIVE_INST_VALU"] / wc),
          "valu/wave", int(r["SQ_INSTS_VALU"] / w), "salu/wave", int(r["SQ_INSTS_SALU"] / w))
