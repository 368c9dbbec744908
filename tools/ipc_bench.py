"""Several ranks per GPU over the IPC transport (csrc/ipc.cpp): N rank processes share the one
GPU, each stepping its sub-domains of C180 L72; prints each rank's median step time (ms) and
the job's (max over ranks).  usage: python tools/ipc_bench.py NRANKS LX LY [STEPS]"""
import importlib
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rank_main(rank, nranks, key, lx, ly, steps):
    sys.path.insert(0, ROOT)
    pkg = importlib.import_module("geosongpu-ci_amd")
    state = importlib.import_module(pkg.__name__ + ".state")
    d = pkg.Domain(rank, nranks, bytes.fromhex(key), npx=181, npz=72, nq=4, layout_x=lx, layout_y=ly, dt=450.0,
                   ipc=1)
    ak, bk, ks = state.hybrid_levels(72)
    st = state.jablonowski_williamson(d, ak, bk)
    d.set_vertical(ak, bk, ks)
    for k, v in st.items():
        d.upload(k, v)
    d.step(1)
    d.sync()
    times = []
    for _ in range(steps):
        t0 = time.perf_counter()
        d.step(1)
        d.sync()
        times.append(1e3 * (time.perf_counter() - t0))
    print(f"RANK {rank} {statistics.median(times):.2f}", flush=True)
    d.close()


if __name__ == "__main__":
    if sys.argv[1] == "--rank":
        rank_main(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], int(sys.argv[5]), int(sys.argv[6]), int(sys.argv[7]))
        sys.exit(0)
    n, lx, ly = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    key = os.urandom(128).hex()
    ps = [subprocess.Popen([sys.executable, __file__, "--rank", str(r), str(n), key, str(lx), str(ly), str(steps)],
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(n)]
    res = []
    for p in ps:
        o, _ = p.communicate(timeout=600)
        if p.returncode != 0:
            print(o[-2000:])
            sys.exit(p.returncode)
        res += [float(line.split()[2]) for line in o.splitlines() if line.startswith("RANK")]
        for line in o.splitlines():
            if line.startswith("ipc rank"):
                print(line)
    print(f"{n} ranks on one GPU (layout {lx}x{ly}, C180 L72, wall time per step incl. host waits): "
          f"median over ranks {statistics.median(res):.2f} ms, max {max(res):.2f} ms")
