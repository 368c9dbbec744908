"""Per-kernel device time per step from a rocprofv3 --kernel-trace CSV.
usage: python tools/trace_stats.py run_kernel_trace.csv [first_step_kernel]
Steps are delimited by the step's first kernel (prep_k); the first step is skipped."""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    m = re.search(r'gtfv3::(?:\(anonymous namespace\)::)?([A-Za-z0-9_]+)(<[^(]*>)?', n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:40]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    first = sys.argv[2] if len(sys.argv) > 2 else "prep_k"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == first]
    rows = rows[idx[1]:]  # drop the first (cold) step
    nstep = len(idx) - 1
    tot, cnt = defaultdict(float), defaultdict(int)
    for r in rows:
        k = short(r["Kernel_Name"])
        tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        cnt[k] += 1
    span = (max(int(r["End_Timestamp"]) for r in rows) - int(rows[0]["Start_Timestamp"])) / 1e6
    busy = sum(tot.values())
    print(f"steps {nstep}  span/step {span / nstep:.2f} ms  busy/step {busy / nstep:.2f} ms")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"{k:40s} {v / nstep:7.3f} ms/step  {cnt[k] // nstep:4d} launches  {v / cnt[k] * 1e3:8.1f} us/launch")


if __name__ == "__main__":
    main()
