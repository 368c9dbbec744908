#!/usr/bin/env python3
"""The CPU baseline at the headline configuration: one
oracle fv_dynamics step (oracle/fv_dynamics.py, numpy fp64, single-threaded) of Held-Suarez
C180 L72, nq = 4, 6 tiles in one process, with the host's CPU count and the process's
affinity recorded.  Too long for bench.py's default run (minutes of one core), so it is run
once per round and its JSON line committed under profiles/.

    OMP_NUM_THREADS=1 OPENBLAS_NUM_THREADS=1 python tools/cpu_baseline_c180.py > profiles/rNN_cpu_c180.json
"""
import json
import os
import platform
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import gtfv3_pkg  # noqa: E402


def main():
    npx = int(sys.argv[1]) if len(sys.argv) > 1 else 181
    pkg = gtfv3_pkg.load()
    dt = 450.0 * 180.0 / (npx - 1)
    r = bench.cpu_baseline(pkg, npx, 72, 4, dt, procs=1)  # one replica: one host core
    r["host"] = platform.processor() or platform.machine()
    r["threads_env"] = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS")}
    print(json.dumps(r))


if __name__ == "__main__":
    main()
