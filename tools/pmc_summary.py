#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/gpu_pmc.sh) into profiles/<round>/pmc.json.

HBM bytes per launch (MI355X_MICROARCH.md, HBM section, gfx950): FETCH_SIZE reads 1/2 of the
bytes of a wide (16 B/lane) coalesced read stream -> x2; WRITE_SIZE is exact for 16-B stores.
Units: KB.  Infinity-Cache hits are counted, so at 64k boards (the working set fits in the
256 MiB cache) the numbers are memory-side traffic, not HBM-only; the 4M-board rows are past it.
Issue counters (one SQ pass): per wave and env step, VALU / SALU instructions and the wave's
cycles (quad-cycles, as SQ reports them); issue_util = (VALU + SALU active) / wave cycles.
Usage: pmc_summary.py <out.json> <pass-dir>[:suffix] [...]  (a suffix is appended to the keys of
that pass, e.g. k_rollout@65536x64 + "r8" for the ring of 8 launches' rows)."""
import csv
import glob
import json
import os
import re
import statistics
import sys
from collections import defaultdict

SHAPES = {65536: 64, 1 << 22: 16}  # tools/pmc_step.py: boards -> rollout K


def kernel_key(name: str, grid: int):
    if "k_rollout_ws" in name:  # 512-thread workgroups of 256 boards: two work-items per board
        return f"k_rollout_ws@{grid // 2}x{SHAPES.get(grid // 2, 0)}"
    if "k_rollout" in name:
        return f"k_rollout@{grid}x{SHAPES.get(grid, 0)}"
    if "k_step" in name:
        return f"k_step@{grid}"
    return None


def steps_of(key: str) -> int:
    """Env steps per work-item in one launch of `key`: K of a rollout key "k_rollout@<N>x<K>"
    (optionally suffixed "r<launches>", e.g. "k_rollout@65536x64r8" -> 64), 1 for k_step.  (Round
    4 stripped every digit here and always returned 1, so its issue block was per launch.)"""
    m = re.fullmatch(r"k_rollout(?:_ws)?@\d+x(\d+)(?:r\d+)?", key)
    return int(m.group(1)) if m and int(m.group(1)) > 0 else 1


def load(dirs):
    vals = defaultdict(lambda: defaultdict(list))  # key -> counter -> [per dispatch]
    for spec in dirs:
        d, _, suffix = spec.partition(":")
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(float)  # (dispatch, counter) -> summed over dimensions
            meta = {}
            for r in csv.DictReader(open(f)):
                grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
                key = kernel_key(r["Kernel_Name"], grid)
                if key is None:
                    continue
                key += suffix
                did = r.get("Dispatch_Id") or r.get("Correlation_Id")
                per[(did, r["Counter_Name"])] += float(r["Counter_Value"])
                meta[did] = key
            for (did, cn), v in per.items():
                vals[meta[did]][cn].append(v)
    return vals


def provenance() -> str:
    import socket
    import subprocess
    import time
    gpu = ""
    try:
        out = subprocess.run(["rocm-smi", "--showproductname"], capture_output=True, text=True,
                             timeout=30).stdout
        gpu = next((l.split(":")[-1].strip() for l in out.splitlines() if "Card Series" in l), "")
    except Exception:
        pass
    return (f"rocprofv3 --pmc passes (tools/gpu_pmc.sh) on {socket.gethostname()} {gpu}, "
            f"{time.strftime('%Y-%m-%d %H:%M UTC', time.gmtime())}")


def main(out_path, *dirs):
    vals = load(dirs)
    res = {"_provenance": provenance()}
    for key in sorted(vals):
        c = {cn: statistics.median(v) for cn, v in vals[key].items()}
        rec = {"dispatches": max(len(v) for v in vals[key].values())}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            rec.update(fetch_kb_raw=c["FETCH_SIZE"], write_kb=c["WRITE_SIZE"],
                       hbm_bytes_per_launch=(2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
        if "SQ_WAVES" in c and c["SQ_WAVES"] > 0:
            steps = steps_of(key)
            # (k_rollout_ws: SQ_WAVES counts the compute and the store waves)
            per = lambda n: c.get(n, 0.0) / c["SQ_WAVES"] / steps  # noqa: E731
            rec["issue"] = {
                "valu_insts_per_wave_step": per("SQ_INSTS_VALU"),
                "salu_insts_per_wave_step": per("SQ_INSTS_SALU"),
                "valu_active_quads_per_wave_step": per("SQ_ACTIVE_INST_VALU"),
                "salu_active_quads_per_wave_step": per("SQ_ACTIVE_INST_SCA"),
                "wave_quads_per_wave_step": per("SQ_WAVE_CYCLES"),
                "issue_util": (c.get("SQ_ACTIVE_INST_VALU", 0) + c.get("SQ_ACTIVE_INST_SCA", 0))
                / max(c.get("SQ_WAVE_CYCLES", 1), 1),
            }
        res[key] = rec
    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], *sys.argv[2:])
