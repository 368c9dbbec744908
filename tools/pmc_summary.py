#!/usr/bin/env python3
"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes (separate runs) into per-kernel
HBM traffic per launch, with the gfx950 correction of MI355X_MICROARCH.md (HBM
section): FETCH_SIZE reports half the bytes of coalesced streaming reads -> x2 (calibrated on
gfx950 for 4-, 8- and 16-B-per-lane loads by tools/pmc_calib.hip, profiles/r02_pmc_calibration.json);
WRITE_SIZE taken as is; both counters are in KiB.

    tools/pmc_summary.py FETCH_DIR WRITE_DIR OUT_JSON
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def load(d, counter):
    out = defaultdict(list)
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            m = re.search(r"::(\w+(?:<[^>]*>)?)\(", r["Kernel_Name"])
            out[m.group(1) if m else r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return out


def main():
    fd, wd, out = sys.argv[1:4]
    fetch, write = load(fd, "FETCH_SIZE"), load(wd, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) & set(write)):
        f = sum(fetch[k]) / len(fetch[k])
        w = sum(write[k]) / len(write[k])
        res[k] = dict(fetch_kib=f, write_kib=w, launches=len(fetch[k]),
                      traffic_bytes=(2.0 * f + w) * 1024.0,
                      note="FETCH_SIZE x2 + WRITE_SIZE (factors calibrated for 4-, 8- and 16-B/lane loads and 8-B/lane stores: profiles/r02_pmc_calibration.json)")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
