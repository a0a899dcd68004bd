#!/usr/bin/env python
"""HBM traffic per launch of one kernel from rocprofv3 --pmc pass directories (FETCH_SIZE pass and
WRITE_SIZE pass run separately, MI355X_MICROARCH.md "HBM"): bytes = 2 * FETCH_SIZE * 1024 (gfx950
tallies 128-B requests at 64 B) + WRITE_SIZE * 1024, averaged over the kernel's dispatches.
    python tools/pmc_traffic.py <pass_dir> <kernel-substring> <out.json> [note]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_dispatch(d, kname, counter):
    vals = defaultdict(float)
    for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            if kname in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals[(f, row["Dispatch_Id"])] += float(row["Counter_Value"])
    return list(vals.values())


def main(d, kname, out, note=""):
    fetch = per_dispatch(d, kname, "FETCH_SIZE")
    write = per_dispatch(d, kname, "WRITE_SIZE")
    hit = per_dispatch(d, kname, "TCC_HIT_sum")
    miss = per_dispatch(d, kname, "TCC_MISS_sum")
    mean = lambda v: sum(v) / len(v) if v else None  # noqa: E731
    res = {"kernel": kname, "dispatches": len(fetch),
           "fetch_bytes_per_launch": 2.0 * 1024.0 * mean(fetch),
           "write_bytes_per_launch": 1024.0 * mean(write),
           "l2_hit_rate": (sum(hit) / (sum(hit) + sum(miss))) if hit and miss else None,
           "correction": "FETCH_SIZE x2 (gfx950: 128-B requests counted as 64 B), KB -> B",
           "note": note}
    res["traffic_bytes_per_launch"] = res["fetch_bytes_per_launch"] + res["write_bytes_per_launch"]
    # per dispatch (capture order within each pass), for launches of different sizes
    res["per_dispatch_fetch_bytes"] = [round(2.0 * 1024.0 * v) for v in fetch]
    res["per_dispatch_write_bytes"] = [round(1024.0 * v) for v in write]
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:])
