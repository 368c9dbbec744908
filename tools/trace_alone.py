"""Which kernels run alone in a multi-stream step: from a rocprofv3 --kernel-trace CSV, per
kernel, the time per step during which it was the only kernel on the device (the step's serial
part: shortening these shortens the step) and the time it shared the device.
usage: python tools/trace_alone.py run_kernel_trace.csv [first_kernel]"""
import csv
import sys

from trace_stats import short


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    first = sys.argv[2] if len(sys.argv) > 2 else "prep_k"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == first]
    rows = rows[idx[1]:idx[-1]]
    nstep = len(idx) - 2
    ev = []
    for n, r in enumerate(rows):
        ev.append((int(r["Start_Timestamp"]), 1, n))
        ev.append((int(r["End_Timestamp"]), -1, n))
    ev.sort(key=lambda e: (e[0], e[1]))
    active, prev = set(), ev[0][0]
    alone, shared, idle = {}, {}, 0
    for t, dlt, n in ev:
        dt = t - prev
        if len(active) == 1:
            k = short(rows[next(iter(active))]["Kernel_Name"])
            alone[k] = alone.get(k, 0) + dt
        elif len(active) > 1:
            for m in active:
                k = short(rows[m]["Kernel_Name"])
                shared[k] = shared.get(k, 0) + dt / len(active)
        else:
            idle += dt
        if dlt > 0:
            active.add(n)
        else:
            active.discard(n)
        prev = t
    span = (ev[-1][0] - ev[0][0]) / 1e6 / nstep
    tot_alone = sum(alone.values()) / 1e6 / nstep
    print(f"steps {nstep}: span {span:.2f} ms/step, one kernel alone {tot_alone:.2f}, idle {idle / 1e6 / nstep:.2f}")
    print(f"{'kernel':44s} {'alone ms/step':>14s} {'shared share':>13s}")
    for k in sorted(alone, key=lambda k: -alone[k])[:30]:
        print(f"{k[:44]:44s} {alone[k] / 1e6 / nstep:14.3f} {shared.get(k, 0) / 1e6 / nstep:13.3f}")


if __name__ == "__main__":
    main()
