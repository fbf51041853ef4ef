#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into profiles/pmc_summary.json.

usage: pmc_summary.py OUT.json DIR [DIR ...]
Each DIR is one `rocprofv3 --pmc ... --output-format csv` pass (counters in
*_counter_collection.csv).  Per kernel instance (named like bench.py's labels:
rowgemm_128x128, wgrad_64x64, ...) it reports the per-dispatch average of every counter and

  hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024

following MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB and on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced stream, so it is doubled.
Clock estimate: GRBM_GUI_ACTIVE / 8 XCDs / kernel duration.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    """rocprofv3 kernel name -> bench.py label (rowgemm_BMxBNxBK / wgrad_BMxBNxBKP)."""
    m = re.search(r"rowgemm_x3_row3_kernel<\d+, (\d+)[,>]", name)
    if m:  # tap-row halo x3 GEMM (tiles 4 / 5)
        return f"x3r3_256x{m.group(1)}"
    m = re.search(r"wgrad_x3_row3_kernel<(\d+), (\d+)", name)
    if m:  # split-bf16 f32 GEMMs (kernels_gemm_x3.hip)
        return f"wx3r3_{m.group(1)}x{m.group(2)}"
    m = re.search(r"WTileX3<(\d+), (\d+),", name)
    if m:
        return f"wx3_{m.group(1)}x{m.group(2)}"
    m = re.search(r"TileX3<(\d+), (\d+),", name)
    if m:
        return f"x3_{m.group(1)}x{m.group(2)}"
    m = re.search(r"Wr3PipeTile<(\d+), (\d+), \d+, \d+, (\d+)", name)
    if m:
        return f"wgrad3p_{m.group(1)}x{m.group(2)}x{m.group(3)}"
    m = re.search(r"PipeTile<(\d+), (\d+), \d+, \d+, \d+", name)
    if m:
        return f"rowgemm_{m.group(1)}x{m.group(2)}x32p"
    m = re.search(r"row3_kernel.*?(?:Row|Wg)Tile<(\d+), (\d+), \d+, \d+, (\d+)", name)
    if m:
        fam = "wgrad3" if "wgrad_row3" in name else "rowgemm3"
        return f"{fam}_{m.group(1)}x{m.group(2)}x{m.group(3)}"
    m = re.search(r"RowTile<(\d+), (\d+), \d+, \d+, (\d+), (true|false)", name)
    if m:
        return f"rowgemm_{m.group(1)}x{m.group(2)}x{m.group(3)}{'d' if m.group(4) == 'true' else ''}"
    m = re.search(r"WgTile<(\d+), (\d+), \d+, \d+, (\d+)", name)
    if m:
        return f"wgrad_{m.group(1)}x{m.group(2)}x{m.group(3)}"
    if "rowgemm16_row3_kernel" in name:  # tap-row halo bf16 GEMM (tile 19)
        return "rg16r3_256x256s2"
    if "rowgemm16_pp_kernel" in name:    # ping-pong bf16 GEMM (tile 18)
        return "rg16pp_256x256s2"
    m = re.search(r"(?<!W)Tile16<(\d+), (\d+), \d+, \d+, (\d+), \d+[,>]", name)
    if m:
        return f"rg16_{m.group(1)}x{m.group(2)}s{m.group(3)}"
    m = re.search(r"WTile16<(\d+), (\d+), \d+, \d+, \d+, (\d+), \d+>", name)
    if m:
        return f"wg16_{m.group(1)}x{m.group(2)}s{m.group(3)}"
    m = re.search(r"::(\w+?)_kernel", name)
    return m.group(1) if m else name[:60]


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                k = short(row.get("Kernel_Name", ""))
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                if row.get("Start_Timestamp") and row.get("End_Timestamp"):
                    dur[k].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    res = {}
    for k, cs in acc.items():
        e = {c: sum(v) / len(v) for c, v in cs.items()}
        e["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["hbm_bytes_per_launch"] = (2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
        if dur[k]:
            e["avg_duration_ns_profiled"] = sum(dur[k]) / len(dur[k])
            if "GRBM_GUI_ACTIVE" in e:
                e["clock_ghz_est"] = e["GRBM_GUI_ACTIVE"] / 8 / e["avg_duration_ns_profiled"]
        res[k] = e
    json.dump({"source": dirs, "kernels": res}, open(out, "w"), indent=1, sort_keys=True)
    for k, e in sorted(res.items(), key=lambda kv: -kv[1].get("avg_duration_ns_profiled", 0))[:12]:
        print(k, {c: round(v, 3) if isinstance(v, float) else v for c, v in e.items()})


if __name__ == "__main__":
    main()
