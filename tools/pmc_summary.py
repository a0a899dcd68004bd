#!/usr/bin/env python
"""Average PMC counters per dispatch of a kernel across tools/pmc_passes.sh pass directories.
    python tools/pmc_summary.py gpurun_out/pmc_dir <kernel-substring>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, kname):
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
        per = defaultdict(float)   # (dispatch, counter) -> summed value
        for row in csv.DictReader(open(f)):
            if kname not in row["Kernel_Name"]:
                continue
            per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
        for (disp, cn), v in per.items():
            vals[cn].append(v)
    for cn, v in sorted(vals.items()):
        print(f"{cn:28s} dispatches {len(v):4d}  mean {sum(v) / len(v):16.1f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
