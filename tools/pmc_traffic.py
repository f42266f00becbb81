#!/usr/bin/env python3
"""Per-kernel HBM traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE csv passes
(tools/gpu/pmc_bench_traffic.sh).  FETCH_SIZE x 2: on gfx950 it reports half the bytes of wide
(16 B/lane) coalesced reads (MI355X_MICROARCH.md, HBM); WRITE_SIZE as reported (exact for 16-B
stores; the conv epilogue's 4-B stores are not calibrated).  Both in KB per dispatch.
usage: pmc_traffic.py FETCH_DIR WRITE_DIR [kernel-substring ...]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def load(d, counter):
    per = defaultdict(list)
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == counter:
                name = re.sub(r"\(.*", "", row["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", ""))
                per[name].append(float(row["Counter_Value"]) * 1024.0)
    return per


def main():
    fd, wd = sys.argv[1], sys.argv[2]
    fetch, write = load(fd, "FETCH_SIZE"), load(wd, "WRITE_SIZE")
    print(f"{'kernel':60s} {'calls':>6s} {'read MB/launch (x2)':>20s} {'write MB/launch':>16s}")
    tot = {}
    for k in sorted(set(fetch) | set(write), key=lambda k: -sum(fetch.get(k, [0])) - sum(write.get(k, [0]))):
        f, w = fetch.get(k, []), write.get(k, [])
        n = max(len(f), len(w))
        rf = 2.0 * sum(f) / max(1, len(f)) / 1e6
        rw = sum(w) / max(1, len(w)) / 1e6
        tot[k] = (n, rf, rw)
        print(f"{k[:60]:60s} {n:6d} {rf:20.2f} {rw:16.2f}")
    # the launches bench.py's roofline times: the implicit-GEMM convs (k_conv<...>, k_conv3g<...>, ...)
    conv = [v for k, v in tot.items() if re.match(r"tcx::(k_conv(3g|3p|3l|3lg|3lb|3m|3mb|4s2h|4s2g)?|k_lin1x1)<", k)]
    n = sum(v[0] for v in conv)
    if n:
        avg = sum(v[0] * (v[1] + v[2]) for v in conv) / n
        print(f"\nconv launches (k_conv<>, k_conv3g<>, k_conv3l<>, k_conv3lg<>, k_conv3lb<>, k_conv3m<>, k_conv3mb<>, k_conv3p<>, k_conv4s2h<>, k_conv4s2g<>, k_lin1x1<>): {n}, average HBM bytes per launch (read x2 + write) = "
              f"{avg:.1f} MB")


if __name__ == "__main__":
    main()
