#!/usr/bin/env python3
"""Refresh pmc/*.json (the PMC traffic bench.py reports as `roofline.traffic` and the step's
bytes per particle-step) from one round's committed profile summaries.

    python tools/refresh_pmc.py <tag>      # reads profiles/<tag>_pmc_summary.json, _pmc_step_bytes.json

bench.py reads pmc/ because profiles/ is not read at run time; the copies name their source
so the line's `traffic` is traceable to the round that measured it."""
import json
import pathlib
import sys

REPO = pathlib.Path(__file__).resolve().parents[1]
tag = sys.argv[1]
summ = REPO / "profiles" / f"{tag}_pmc_summary.json"
step = REPO / "profiles" / f"{tag}_pmc_step_bytes.json"
d = json.loads(summ.read_text())
props = [(k, r) for k, r in d.items() if "k_ssm2d_prop" in k]
assert props, f"no k_ssm2d_prop in {summ}"
k, r = max(props, key=lambda kr: kr[1]["dispatches"])
out = {"kernel": k,
       "bytes_per_launch": r.get("hbm_read_bytes_corrected", 0.0) + r.get("hbm_write_bytes", 0.0),
       "read_bytes_corrected": r.get("hbm_read_bytes_corrected", 0.0),
       "write_bytes": r.get("hbm_write_bytes", 0.0),
       "dispatches": r["dispatches"],
       "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of "
                 "`bench.py --steps 2 --warmup 1 --no-cpu-baseline`; FETCH_SIZE x 2 (gfx950 wide-read "
                 "correction, MI355X_MICROARCH.md HBM section), KB -> bytes; mean per dispatch "
                 "(tools/gpu.sh prof_passes)",
       "source": str(summ.relative_to(REPO)), "n_particles": 1000000, "T": 100}
(REPO / "pmc" / "pmc_propagate_bytes.json").write_text(json.dumps(out, indent=1) + "\n")
s = json.loads(step.read_text())
s["source"] = str(step.relative_to(REPO))
(REPO / "pmc" / "pmc_step_bytes.json").write_text(json.dumps(s, indent=1) + "\n")
print(f"pmc/ refreshed from {tag}: propagate {out['bytes_per_launch'] / 1e6:.1f} MB a launch, "
      f"{s['bytes_per_particle_step']:.1f} B a particle-step")
