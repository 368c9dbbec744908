#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 PMC counters from rocpd SQLite outputs.

    tools/pmc_db.py DB [DB ...]   -> table: kernel, launches, mean duration, counters
"""
import re
import sqlite3
import sys
from collections import defaultdict


def load(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
    rows = c.execute("select * from counters_collection").fetchall()
    out = defaultdict(lambda: defaultdict(list))
    for r in rows:
        d = dict(zip(cols, r))
        name = d.get("kernel_name") or d.get("name")
        m = re.search(r"::(\w+)\(", name or "")
        k = m.group(1) if m else name
        out[k][d["counter_name"]].append(float(d["value"]))
    durs = defaultdict(list)
    kcols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    for r in c.execute("select * from kernels").fetchall():
        d = dict(zip(kcols, r))
        m = re.search(r"::(\w+)\(", d.get("name") or "")
        durs[m.group(1) if m else d.get("name")].append((d["end"] - d["start"]) * 1e-3)
    return out, durs


def main():
    allc = defaultdict(dict)
    alld = {}
    for db in sys.argv[1:]:
        out, durs = load(db)
        for k, cs in out.items():
            for cn, vals in cs.items():
                allc[k][cn] = sum(vals) / len(vals)
        for k, v in durs.items():
            alld.setdefault(k, v)
    order = sorted(allc, key=lambda k: -sum(alld.get(k, [0])))
    for k in order[:25]:
        d = alld.get(k, [0])
        print(f"{k:24s} n={len(d):4d} us={sum(d)/max(len(d),1):8.1f} " +
              " ".join(f"{cn}={v:.4g}" for cn, v in sorted(allc[k].items())))


if __name__ == "__main__":
    main()
