#!/usr/bin/env python3
"""HBM bytes per particle-step of the whole fused C2 run from a PMC summary.

    python tools/pmc_step_bytes.py PMC_SUMMARY.json N T OUT.json

For every kernel of the run: mean corrected bytes per dispatch (tools/summarize_pmc.py:
FETCH_SIZE x 2 on gfx950 + WRITE_SIZE) x its dispatches per run (dispatches / the number of
trace-back dispatches, one per run), summed and divided by N x T. The CDF work and the
trace-back are included: this is the `traffic` beside SURVEY.md §8(d)'s 104 algorithmic
bytes per particle-step."""
import json
import sys

d = json.load(open(sys.argv[1]))
N, T = int(sys.argv[2]), int(sys.argv[3])
runs = sum(r["dispatches"] for k, r in d.items() if "k_ssm2d_final" in k)
assert runs > 0, "no trace-back dispatches in the summary"
per_kernel = {}
for k, r in d.items():
    if not any(x in k for x in ("k_ssm2d_prop", "k_rs_sums_t", "k_rs_fill_fused", "k_ssm2d_final")):
        continue
    b = r.get("hbm_read_bytes_corrected", 0.0) + r.get("hbm_write_bytes", 0.0)
    per_kernel[k.split("(")[0]] = b * r["dispatches"] / runs / (N * T)
out = {"n_particles": N, "T": T, "bytes_per_particle_step": sum(per_kernel.values()),
       "per_kernel": per_kernel, "source": sys.argv[1],
       "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes (tools/gpu.sh round); "
                 "FETCH_SIZE x 2 (gfx950 wide-read correction), per dispatch x dispatches per run / (N T)"}
json.dump(out, open(sys.argv[4], "w"), indent=1)
print(json.dumps(out))
