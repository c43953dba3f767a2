#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes into per-launch HBM bytes (profiles/<round>/pmc_step.json).
gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reads 1/2 of the bytes of a
wide (16 B/lane) coalesced stream -> x2; WRITE_SIZE is exact for 16-B stores.  Units: KB."""
import csv
import glob
import json
import statistics
import sys
from collections import defaultdict


def load(pattern, counter):
    out = defaultdict(list)
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"]
            key = ("k_step" if "k_step" in name else "k_rollout" if "k_rollout" in name else None)
            if key is None:
                continue
            out[(key, int(r["Grid_Size"]) if "Grid_Size" in r else int(r.get("Grid_Size_X", 0)))].append(
                float(r["Counter_Value"]))
    return out


def main(fetch_glob, write_glob, out_path):
    fe, wr = load(fetch_glob, "FETCH_SIZE"), load(write_glob, "WRITE_SIZE")
    res = {}
    for key in sorted(set(fe) | set(wr)):
        kern, grid = key
        f = statistics.median(fe.get(key, [0.0]))
        w = statistics.median(wr.get(key, [0.0]))
        res[f"{kern}@{grid}"] = {"kernel": kern, "boards": grid, "dispatches": len(fe.get(key, [])),
                                 "fetch_kb_raw": f, "write_kb": w,
                                 "hbm_bytes_per_launch": (2 * f + w) * 1024}
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
