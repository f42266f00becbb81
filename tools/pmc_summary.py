#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc csv passes (tools/gpu/pmc_conv.sh) per kernel: mean counter value per
dispatch of the named kernel substring.  usage: pmc_summary.py KERNEL_SUBSTR dir1 [dir2 ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def collect(kern, dirs):
    vals = defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for row in csv.DictReader(open(f)):
                if kern in row["Kernel_Name"]:
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


if __name__ == "__main__":
    kern, dirs = sys.argv[1], sys.argv[2:]
    for k, v in sorted(collect(kern, dirs).items()):
        print(f"{k:28s} {v:16.1f}")
