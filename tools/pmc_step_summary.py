#!/usr/bin/env python3
"""Reduce tools/pmc_step.sh output: per kernel family the mean duration, VGPR / LDS, waves per
SIMD the registers allow, issue-state shares (SQ_* over SQ_WAVE_CYCLES), L2 hit rate and HBM
traffic (FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md HBM section).

    tools/pmc_step_summary.py gpurun_out/TAG > profiles/TAG_pmc_step.json
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict


def kname(s):
    m = re.search(r"::(\w+(?:<[^>]*>)?)\(", s)
    return m.group(1) if m else s.split("(")[0]


def counters(d):
    out = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            out[kname(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def trace(d):
    out = defaultdict(lambda: dict(ns=[], vgpr=0, agpr=0, lds=0, sgpr=0))
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = out[kname(r["Kernel_Name"])]
            k["ns"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
            k["vgpr"] = int(r.get("Arch_VGPR_Count", r.get("VGPR_Count", 0)) or 0)
            k["agpr"] = int(r.get("Accum_VGPR_Count", 0) or 0)
            k["lds"] = int(r.get("LDS_Block_Size", r.get("Lds_Size", 0)) or 0)
            k["sgpr"] = int(r.get("SGPR_Count", 0) or 0)
    return out


def waves(v):
    for lim, w in ((64, 8), (72, 7), (80, 6), (96, 5), (128, 4), (168, 3), (256, 2)):
        if v <= lim:
            return w
    return 1


def main():
    base = sys.argv[1]
    tr = trace(base + "_kt")
    c = {}
    for p in ("sqa", "sqb", "tcc", "fetch", "write"):
        for k, v in counters(base + "_" + p).items():
            c.setdefault(k, {}).update({n: sum(x) / len(x) for n, x in v.items()})
    res = {}
    for k, t in sorted(tr.items(), key=lambda kv: -sum(kv[1]["ns"])):
        x = c.get(k, {})
        wc = x.get("SQ_WAVE_CYCLES", 0) or 1
        r = dict(launches=len(t["ns"]), mean_us=sum(t["ns"]) / len(t["ns"]) / 1e3, total_ms=sum(t["ns"]) / 1e6,
                 vgpr=t["vgpr"], agpr=t["agpr"], lds=t["lds"], waves_per_simd=waves(t["vgpr"] + t["agpr"]))
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM",
                  "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            if n in x:
                r[n.lower() + "_frac"] = x[n] / wc
        if "SQ_BUSY_CYCLES" in x and "SQ_WAVE_CYCLES" in x:
            r["avg_waves_in_flight"] = x["SQ_WAVE_CYCLES"] / max(x["SQ_BUSY_CYCLES"], 1)
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_WAVES"):
            if n in x:
                r[n.lower()] = x[n]
        if "TCC_HIT_sum" in x:
            r["l2_hit"] = x["TCC_HIT_sum"] / max(x["TCC_HIT_sum"] + x["TCC_MISS_sum"], 1)
        if "FETCH_SIZE" in x and "WRITE_SIZE" in x:
            r["hbm_bytes"] = (2.0 * x["FETCH_SIZE"] + x["WRITE_SIZE"]) * 1024.0
            r["hbm_tbs"] = r["hbm_bytes"] / (r["mean_us"] * 1e-6) / 1e12
        res[k] = r
    json.dump(res, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
