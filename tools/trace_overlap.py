"""Concurrency of a multi-stream step from a rocprofv3 --kernel-trace CSV: per step, the time
with no kernel running (gaps), with one, and with two or more, and the largest gaps with the
kernels on either side.  usage: python tools/trace_overlap.py run_kernel_trace.csv [first_kernel]"""
import csv
import re
import sys

from trace_stats import short


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    first = sys.argv[2] if len(sys.argv) > 2 else "prep_k"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == first]
    rows = rows[idx[1]:idx[-1]]  # whole steps after the first
    nstep = len(idx) - 2
    ev = []
    for r in rows:
        ev.append((int(r["Start_Timestamp"]), 1, r))
        ev.append((int(r["End_Timestamp"]), -1, r))
    ev.sort(key=lambda e: (e[0], e[1]))
    t0, act, acc = ev[0][0], 0, {0: 0, 1: 0, 2: 0}
    last_end, gaps = None, []
    prev = ev[0][0]
    for t, d, r in ev:
        acc[min(act, 2)] += t - prev
        if act == 0 and last_end is not None and d == 1:
            gaps.append((t - last_end[0], short(last_end[1]["Kernel_Name"]), short(r["Kernel_Name"])))
        act += d
        if act == 0:
            last_end = (t, r)
        prev = t
    span = (ev[-1][0] - t0) / 1e6 / nstep
    print(f"steps {nstep} span/step {span:.2f} ms: idle {acc[0] / 1e6 / nstep:.2f}  one kernel {acc[1] / 1e6 / nstep:.2f}"
          f"  two+ {acc[2] / 1e6 / nstep:.2f} ms")
    agg = {}
    for g, a, b in gaps:
        k = (a, b)
        agg[k] = (agg.get(k, (0, 0))[0] + g, agg.get(k, (0, 0))[1] + 1)
    print("largest idle transitions (total us per step, count per step):")
    for (a, b), (g, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:25]:
        print(f"  {g / 1e3 / nstep:8.1f} us {n / nstep:5.1f}x  {a} -> {b}")


if __name__ == "__main__":
    main()
