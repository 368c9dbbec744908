"""Timeline of the last geos_gtfv3 run call in a rocprofv3 trace of tools/bridge_bench.py
(--kernel-trace --memory-copy-trace [--hip-trace], csv): when the uploads before the step, the
step's kernels, the uploads beside it and the copies back ran, and how much of the copy-back
traffic overlapped the step.

    python tools/bridge_timeline.py <dir>/<prefix>   (reads <prefix>_kernel_trace.csv, ...)
"""
import csv
import re
import sys


def load(prefix):
    ev = []
    for r in csv.DictReader(open(prefix + "_kernel_trace.csv")):
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace("gtfv3::", "")
        n = re.sub(r"\(.*", "", n)
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", n, r["Stream_Id"]))
    for r in csv.DictReader(open(prefix + "_memory_copy_trace.csv")):
        d = "H2D" if r["Direction"].endswith("HOST_TO_DEVICE") else "D2H"
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "M", d, r["Stream_Id"]))
    api = []
    try:
        for r in csv.DictReader(open(prefix + "_hip_api_trace.csv")):
            api.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]))
    except FileNotFoundError:
        pass
    ev.sort()
    return ev, api


def main():
    ev, api = load(sys.argv[1])
    # the last call: from the last run of upload kernels before the last prep_k (the step's first)
    p = max(i for i, e in enumerate(ev) if e[3].startswith("prep_k"))
    i = p - 1
    while i > 0 and ev[i][3].startswith("fort_move<") and ", true>" in ev[i][3]:
        i -= 1
    t0 = ev[i + 1][0]
    step0 = ev[p][0]
    step_k = [e for e in ev[p:] if e[2] == "K" and not e[3].startswith("fort_move")]
    step1 = max(e[1] for e in step_k if e[3].startswith(("c2l_k",)))
    call = [e for e in ev if e[0] >= t0]
    end = max(e[1] for e in call)
    ms = lambda t: (t - t0) / 1e6  # noqa: E731
    up_crit = [e for e in call if e[0] < step0 and e[3].startswith("fort_move") and ", true>" in e[3]]
    side_up = [e for e in call if e[0] >= step0 and ((e[2] == "M" and e[3] == "H2D")
                                                      or (e[3].startswith("fort_move") and ", true>" in e[3]))]
    down = [e for e in call if (e[2] == "M" and e[3] == "D2H") or (e[3].startswith("fort_move") and ", false>" in e[3])]
    acoustic_end = max(e[1] for e in step_k if e[3].startswith("nhpgrad"))
    print(f"call: {ms(end):.2f} ms from the first upload kernel to the last copy back")
    print(f"uploads before the step (zero-copy kernels): {ms(up_crit[0][0]):.2f} - {ms(up_crit[-1][1]):.2f} ms, "
          f"{len(up_crit)} launches")
    print(f"step kernels: {ms(step0):.2f} - {ms(step1):.2f} ms ({(step1 - step0) / 1e6:.2f} ms; acoustic sub-steps "
          f"end at {ms(acoustic_end):.2f})")
    if side_up:
        print(f"uploads beside the step: {ms(side_up[0][0]):.2f} - {ms(max(e[1] for e in side_up)):.2f} ms, "
              f"{sum(1 for e in side_up if e[2] == 'M')} DMAs")
    d2h = [e for e in down if e[2] == "M"]
    busy_in = sum(min(e[1], step1) - e[0] for e in d2h if e[0] < step1) / 1e6
    busy = sum(e[1] - e[0] for e in d2h) / 1e6
    print(f"copies back: first at {ms(down[0][0]):.2f} ms, last ends {ms(max(e[1] for e in down)):.2f} ms; "
          f"DMA busy {busy:.2f} ms, {busy_in:.2f} ms of it before the step's last kernel")
    # per-millisecond activity around the step's end
    if api:
        long_calls = [(a, b, f) for a, b, f in api if a >= t0 and b - a > 200000]
        for a, b, f in long_calls:
            print(f"host call > 0.2 ms: {f} at {ms(a):.2f} for {(b - a) / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
