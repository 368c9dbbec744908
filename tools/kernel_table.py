"""Markdown per-kernel table for DESIGN §4 from one round's profiles:
   profiles/<R>_bench_kernel_events.json (bench.py --kernel-report), <R>_rocprof_kernel_stats.csv
   (rocprofv3 --kernel-trace --stats) and <R>_pmc_traffic.json (tools/pmc_summary.py).
   usage: tools/kernel_table.py R [N_ROWS]"""
import csv
import json
import re
import sys

R = sys.argv[1]
n_rows = int(sys.argv[2]) if len(sys.argv) > 2 else 22
ev = json.load(open(f"profiles/{R}_bench_kernel_events.json"))
pmc = json.load(open(f"profiles/{R}_pmc_traffic.json"))
rp = {}
for r in csv.DictReader(open(f"profiles/{R}_rocprof_kernel_stats.csv")):
    rp[r["Name"]] = r
# launch name -> device kernel (template arguments as rocprof / PMC print them)
DEV = {
    "tp_march_thermo<6, in>": "tp_march<6, false, true, 3, 1, 2, 2>",
    "tp_march_thermo<6, ex>": "tp_march<6, false, true, 3, 1, 2, 1>",
    "tp_march_uv<6>": "tp_march<6, true, false, 1, 3, 0, 0>",
    "tp_march_zh<6>": "tp_march<6, true, false, 1, 4, 0, 0>",
    "tp_march_tracer<6, 2>": "tp_march<6, true, true, 2, 2, 0, 0>",
    "ds_ke": "ds_ke_ld<6, true>",
    "cs_transport_ke": "cs_transport_ke_ld",
    "cs_update": "cs_update_ld",
    "cs_tmp": "cs_tmp_ld",
    "cs_cgrid": "cs_cgrid_kl",
    "a2b_edge_k": "a2b_edge2_k",
    "halo_local_kernel": "halo_local_kernel<",
}


def dev_name(launch):
    name = launch.strip("()")
    if name in DEV:
        return DEV[name]
    return re.sub(r"<M, NB, PART, (\w+)>", "<", name)


def find(table, dn):
    for k in table:
        base = re.sub(r"^void ", "", k)
        base = re.sub(r"^gtfv3::\(anonymous namespace\)::|^gtfv3::", "", base)
        if base.startswith(dn) and (dn.endswith("<") or base[len(dn):len(dn) + 1] in ("(", "")):
            yield k


rows = sorted(ev.items(), key=lambda kv: -kv[1]["ms_per_step"])
total = sum(v["ms_per_step"] for v in ev.values())
print("| Kernel | Launches/step | ms/step | µs/launch (rocprof) | alg. GB/launch | alg. TB/s | frac | PMC GB/launch |")
print("|---|---|---|---|---|---|---|---|")
shown = 0.0
for name, v in rows[:n_rows]:
    dn = dev_name(name)
    lps = v["launches"] / 3.0 if "launches" in v else 0
    rk = list(find(rp, dn))
    us = sum(float(rp[k]["TotalDurationNs"]) for k in rk) / max(1, sum(int(rp[k]["Calls"]) for k in rk)) / 1e3 if rk else None
    pk = list(find(pmc, dn))
    pg = (sum(pmc[k]["traffic_bytes"] * pmc[k]["launches"] for k in pk) / sum(pmc[k]["launches"] for k in pk) / 1e9
          if pk else None)
    bpl = v.get("bytes_per_launch") or 0.0
    tbs = (v.get("gbs") or 0.0) / 1e3
    print(f"| `{name.strip('()')}` | {lps:.0f} | {v['ms_per_step']:.2f} | {us:.0f} | {bpl / 1e9:.2f} | {tbs:.2f} | "
          f"{tbs / 8.0:.2f} | {'–' if pg is None else f'{pg:.2f}'} |" if us is not None else
          f"| `{name.strip('()')}` | {lps:.0f} | {v['ms_per_step']:.2f} | – | {bpl / 1e9:.2f} | {tbs:.2f} | {tbs / 8.0:.2f} | "
          f"{'–' if pg is None else f'{pg:.2f}'} |")
    shown += v["ms_per_step"]
print(f"| other ({len(rows) - n_rows} kernels) | | {total - shown:.2f} | | | | | |")
