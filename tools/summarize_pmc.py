#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs into per-kernel averages (per dispatch).

    python tools/summarize_pmc.py OUT.json DIR [DIR ...]

FETCH_SIZE / WRITE_SIZE are reported in KB by rocprofv3. On gfx950 FETCH_SIZE counts
exactly half of the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md §HBM),
so `hbm_read_bytes_corrected` = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16-B/lane
streaming stores. Both are per dispatch.
"""
import collections
import csv
import json
import pathlib
import sys


def main():
    out = pathlib.Path(sys.argv[1])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[2:]:
        for f in pathlib.Path(d).rglob("*counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, cs in agg.items():
        if "rocclr" in k or "k_delay" in k:
            continue
        row = {c: sum(v) / len(v) for c, v in cs.items()}
        row["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in row:
            row["hbm_read_bytes_corrected"] = 2.0 * row["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in row:
            row["hbm_write_bytes"] = row["WRITE_SIZE"] * 1024
        res[k] = row
    out.write_text(json.dumps(res, indent=1, sort_keys=True))
    for k, r in res.items():
        print(k[:50], {c: round(v, 1) for c, v in r.items() if c in ("hbm_read_bytes_corrected", "hbm_write_bytes", "SQ_INSTS_VALU", "SQ_WAVES")})


if __name__ == "__main__":
    main()
