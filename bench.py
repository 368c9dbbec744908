#!/usr/bin/env python3
"""Benchmark: grid-cell-updates/sec per dycore step, Held-Suarez C180 L72 (BASELINE.json).

One "step" is one fv_dynamics call (= one geos_gtfv3 run: n_split=6 acoustic
sub-steps, tracer_2d_1l, vertical remap) on device-resident fp64 state.  At N=1
the whole C180 L72 cubed sphere (6 tiles) lives on one MI355X; for N>1 one
process per GPU (torch.distributed / RCCL over xGMI), the 6*layout^2 sub-domains
split evenly across ranks, halos exchanged with RCCL send/recv (strong scaling:
the global grid is fixed).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (the driver's N>1 launch)

Prints ONE JSON line on rank 0 (contract in DESIGN.md §Measurement):
  value            whole-job cells*levels advanced per second (max-over-ranks time)
  roofline         dominant kernel: algorithmic bytes per launch / its mean HIP-event
                   duration over the timed steps, against 8 TB/s HBM; and the whole step:
                   step_bytes (every kernel's algorithmic bytes, bytes_manifest.yaml, as
                   registered by the launchers on the probe step) / ms_per_step -> step_frac
  cpu_baseline     the numpy oracle (oracle/fv_dynamics.py) timed for one step on a
                   bounded sample (C48 L72, 6 tiles, ~20 s per core) on the host, rank 0
                   only, as --cpu-procs concurrent single-threaded replicas (one per core);
                   the host's CPU count and this process's affinity are recorded
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md

# Algorithmic HBM bytes come from the library: each launcher registers its
# kernel's bytes per launch (distinct fields read + written once over the compute
# domain; formulas in DESIGN.md §4) with the event timer.


def family(kernel):
    """kernel family: the launch name without template arguments ("(tp_march<6, true,
    false>)" -> "tp_march"); the roofline reports the family with the most device time"""
    return kernel.strip("()").split("<")[0]


def families(kstats):
    """{family: (total_ms, launches, algorithmic_bytes)} summed over instantiations"""
    out = {}
    for k, (ms, n, b) in kstats.items():
        t = out.get(family(k), (0.0, 0, 0.0))
        out[family(k)] = (t[0] + ms, t[1] + n, t[2] + b)
    return out


def march_ex_fraction(nx, subs, mout=58):
    """share of the column marches' outputs (columns 0 .. nx of every sub-domain) in tile-edge
    spans (tp.hip plan_spans: [0, 2] at a west tile edge, [nx-3, nx] at an east one, all of a
    sub-domain too narrow for both), the tile-edge kernel's part of the thermo march"""
    nex = 0
    for s in subs:
        we, ee = s["ioff"] == 0, s["ioff"] + nx == s["N"]
        lo, hi = (3 if we else 0), (nx - 4 if ee else nx)
        nex += nx + 1 if hi < lo else (3 if we else 0) + (4 if ee else 0)
    return nex / (len(subs) * (nx + 1))


def manifest_step_bytes(nx, ny, nsub, npz, nq, n_split, pitch, nj, fex=0.5, alternatives=False):
    """Algorithmic bytes of one step from bytes_manifest.yaml (evaluated independently of
    the launchers' registration; tests/test_bytes_manifest.py compares the two).  Families
    marked `alternative_to` (a fused form the benchmark step does not run by default) are
    left out of the step unless `alternatives`."""
    import yaml
    with open(os.path.join(ROOT, "bytes_manifest.yaml")) as f:
        man = yaml.safe_load(f)["families"]
    env = dict(C=nsub * nx * ny, X=nsub * (nx + 1) * ny, Y=nsub * nx * (ny + 1), K=nsub * (nx + 1) * (ny + 1),
               L=npz, L1=npz + 1, nq=nq, ns=n_split, nsub=nsub, nx=nx, ny=ny, pitch=pitch, nj=nj, fex=fex)
    out = {}
    for fam, spec in man.items():
        if "same_as" in spec:  # an alternative form of another family (counted once, there)
            continue
        if "alternative_to" in spec and not alternatives:
            continue
        kinds = spec.get("launches") or ([spec] if "doubles" in spec else [])
        out[fam] = sum(8.0 * eval(k["n"], {}, env) * eval(k["doubles"], {}, env) for k in kinds)
    return out


def manifest_family(fam):
    """the manifest family whose bytes a kernel family registers (level-loop and other
    alternative forms name the one-level form they replace with `same_as`)"""
    import yaml
    with open(os.path.join(ROOT, "bytes_manifest.yaml")) as f:
        man = yaml.safe_load(f)["families"]
    spec = man.get(fam)
    return spec["same_as"] if isinstance(spec, dict) and "same_as" in spec else fam


# launch names (GT_LAUNCH_N) whose kernel symbol, as rocprof records it, differs
LAUNCH_SYMBOL = {
    "tp_march_thermo<6, ex>": "tp_march<6, false, true, 3, 1, 2, 1>",
    "tp_march_thermo<6, in>": "tp_march<6, false, true, 3, 1, 2, 2>",
    "tp_march_thermo<5, ex>": "tp_march<5, false, true, 3, 1, 2, 1>",
    "tp_march_thermo<5, in>": "tp_march<5, false, true, 3, 1, 2, 2>",
    "tp_march_uv<6>": "tp_march<6, true, false, 1, 3, 0, 0>",
    "tp_march_zh<6>": "tp_march<6, true, false, 1, 4, 0, 0>",
    "tp_march_tracer<6, 2>": "tp_march<6, true, true, 2, 2, 0, 0>",
    "ds_ke": "ds_ke_ld<6, true>",
    "cs_transport_ke": "cs_transport_ke_ld",
    "cs_update": "cs_update_ld",
    "cs_tmp": "cs_tmp_ld",
}


def pmc_traffic(fam, launches):
    """HBM bytes per launch of kernel family `fam` (launch-weighted over the instantiations
    timed, `launches` = {launch name: count}) from the newest committed PMC summary
    (profiles/rNN_pmc_traffic.json, made by tools/pmc_summary.py from separate
    FETCH_SIZE / WRITE_SIZE rocprofv3 passes of this same command); None if absent."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    for f in reversed(files):
        with open(f) as fh:
            t = json.load(fh)
        keys = {k: LAUNCH_SYMBOL.get(k.strip("()"), k.strip("()")).replace(" ", "") for k in launches}
        tk = {k.replace(" ", ""): v for k, v in t.items()}
        for k, v in keys.items():  # rocprof spells out defaulted template arguments
            if v not in tk and v.endswith(">"):
                ext = [x for x in tk if x.startswith(v[:-1] + ",")]
                if len(ext) == 1:
                    keys[k] = ext[0]
        if keys and all(v in tk for v in keys.values()):
            tot = sum(tk[keys[k]]["traffic_bytes"] * n for k, n in launches.items())
            return tot / sum(launches.values()), os.path.basename(f)
    return None, None


def state_check(d, ptop, names=("ps", "pt", "delp", "u", "w")):
    """After the timed steps: the state must be finite and physically bounded, else the run
    has diverged and its throughput means nothing (raises).  Returns the bounds and a
    checksum (fp64 sums of the compute-domain fields) for the JSON line."""
    NG = 3
    n_x, n_y = d.nx, d.ny
    out = {}
    for k in names:
        a = d.download(k)[..., NG:NG + n_y, NG:NG + n_x]
        if not np.all(np.isfinite(a)):
            raise SystemExit(f"bench: state field {k} is not finite after the timed steps")
        out[k] = a
    pt, dp, ps = out["pt"], out["delp"], out["ps"]
    ok = (150.0 < pt.min() and pt.max() < 400.0 and dp.min() > 0.0 and 3.0e4 < ps.min() and ps.max() < 1.2e5
          and np.abs(out["u"]).max() < 200.0)
    res = dict(finite=True, bounded=bool(ok), pt_min=float(pt.min()), pt_max=float(pt.max()),
               ps_min=float(ps.min()), ps_max=float(ps.max()), max_abs_u=float(np.abs(out["u"]).max()),
               max_abs_w=float(np.abs(out["w"]).max()),
               checksum={k: float(v.sum(dtype=np.float64)) for k, v in out.items()})
    if not ok:
        raise SystemExit(f"bench: state out of physical bounds after the timed steps: {res}")
    return res


def layout_for(n):
    """(layout_x, layout_y) for n ranks: 6*lx*ly sub-domains divisible by n"""
    # bands of full tile width (1 x ly): the x-marching kernels keep C180's strip
    # efficiency; with all 24 sub-domains on one GPU 1x4 ran 52.4 ms/step, 2x2 54.7
    return {1: (1, 1), 2: (1, 1), 3: (1, 1), 6: (1, 1), 4: (1, 2), 8: (1, 4), 12: (1, 2), 24: (1, 4)}.get(n, (2, 2))


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--npx", type=int, default=181)
    p.add_argument("--npz", type=int, default=72)
    p.add_argument("--nq", type=int, default=4)
    p.add_argument("--layout", default="", help="sub-domain layout per tile, e.g. 2x2 (default: by rank count)")
    p.add_argument("--dt", type=float, default=0.0, help="dt_atmos (default 450 s x 180 / N: C180 450 s)")
    p.add_argument("--cpu-npx", type=int, default=0,
                   help="cpu_baseline sample grid npx (default 49: C48 L72, 6 tiles, ~20 s of one host core; "
                        "13 with --moist, ~40 s)")
    p.add_argument("--cpu-procs", type=int, default=16,
                   help="cpu_baseline: concurrent single-threaded oracle replicas (= host cores used)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-kernel-timing", action="store_true")
    p.add_argument("--kernel-report", default="", help="write per-kernel stats JSON here")
    p.add_argument("--streams", type=int, default=3, choices=(1, 3),
                   help="streams of the timed steps (3: wind stages, update_dz_d and the tracer "
                        "transport beside the main chain; 1: everything on one stream)")
    p.add_argument("--rank-proxy", type=int, default=0,
                   help="measurement aid, one GPU: run rank 0 of an N-rank layout alone with the null "
                        "transport (each cross-rank receive answered by the rank's own send, as device copies) -- "
                        "the per-GPU compute time of an N-GPU run without the xGMI transfers; not a "
                        "numerical result")
    p.add_argument("--roofline-steps", type=int, default=3,
                   help="steps of the single-stream roofline pass after the timed region")
    p.add_argument("--moist", action="store_true",
                   help="Aquaplanet configuration: nq=6 moist tracers and the moist physics (aer_activation, "
                        "evap_subl_pdf, GFDL microphysics, radcouple) after every fv_dynamics call, inside the "
                        "timed region")
    p.add_argument("--geos-log", default="", help="also write a GEOS-style log (geoslog.py) of K individually "
                   "synchronised steps run after the timed region, for tcn.benchmark's parse_geos_log")
    return p.parse_args()


def _cpu_replica(args):
    """one oracle step in a child process (numpy only: the child never loads the HIP library)"""
    st, ak, bk, grid, nl, moist, cd_info, barrier = args
    from oracle import fv_dynamics as fvd
    g = fvd.Grid(*grid)
    barrier.wait()
    t0 = time.perf_counter()
    out = fvd.fv_dynamics(st, ak, bk, g, nl)
    if moist:
        from oracle import NG
        from oracle import geos_moist as gm
        nsub, ny, nx, npz, dt = cd_info
        cd = (Ellipsis, slice(NG, NG + ny), slice(NG, NG + nx))  # the compute domain (the padded
        for s in range(nsub):                                    # plane's outer cells are not state)
            q = out["q"][s]
            sp = [q[n * npz:(n + 1) * npz][cd] for n in range(6)]
            gm.aquaplanet_physics(dt, out["pt"][s][cd], *sp, out["delp"][s][cd], out["delz"][s][cd],
                                  out["pe"][s][cd], out["w"][s][cd])
    return time.perf_counter() - t0


def cpu_baseline(pkg, npx, npz, nq, dt, moist=False, procs=8):
    """The oracle fv_dynamics step (+ the oracle moist column step with --moist) of a bounded
    sample, timed on the host: `procs` single-threaded processes each run the same step at
    once (the oracle's tiles exchange halos every acoustic sub-step inside one process, so
    a step does not split over processes; concurrent replicas measure what `procs` host
    cores sustain).  value = sum over replicas of cells / own step time."""
    import importlib
    import multiprocessing as mp

    state = importlib.import_module(pkg.__name__ + ".state")
    d = pkg.Domain(npx=npx, npz=npz, nq=nq, host_only=1, dt=dt)
    ak, bk, ks = state.hybrid_levels(npz)
    st = state.jablonowski_williamson(d, ak, bk)
    if moist:
        state.aquaplanet_tracers(d, st, ak, bk)
    from oracle import grid as og  # the oracle's own grid (tests/test_oracle_grid.py pins grid.cpp to it)
    ms, sc = og.domain_metrics(d.subs, d.nx, d.ny, d.N, d.pitch, d.nj)
    grid = (d.N, 1, 1, ms, sc["corner_w"], sc["da_min_c"], d.nj, d.pitch)
    nl = dict(n_split=6, dt_atmos=dt, hord_mt=6, hord_vt=6, hord_tm=6, hord_dp=6, hord_tr=6, dddmp=0.2, d2_bg=0.0,
              p_fac=0.05, dz_min=2.0, fill=1, nq=nq)
    cd_info = (d.nsub, d.ny, d.nx, npz, dt)
    cells = 6 * d.N * d.N * npz
    N = d.N
    d.close()
    env = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")}
    for k in env:
        os.environ[k] = "1"  # one core per replica; the spawned children inherit this
    try:
        ctx = mp.get_context("spawn")  # fresh interpreters: nothing of this process's GPU state
        with ctx.Manager() as man:
            bar = man.Barrier(procs)
            # close + join, not the context manager: Pool.__exit__ calls terminate(), which
            # SIGTERMs the replicas, and under rocprofv3 each then logs an abort trace
            pool = ctx.Pool(procs)
            try:
                els = pool.map(_cpu_replica, [(st, ak, bk, grid, nl, moist, cd_info, bar)] * procs)
                pool.close()
            except BaseException:
                pool.terminate()
                raise
            finally:
                pool.join()
    finally:
        for k, v in env.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        aff = sorted(os.sched_getaffinity(0))
    except AttributeError:
        aff = []
    return dict(value=sum(cells / e for e in els), unit="grid-cell-updates/s", cores=procs, kind="port",
                host_cpus=os.cpu_count(), affinity=f"{len(aff)} cpus ({aff[0]}-{aff[-1]})" if aff else None,
                per_core=cells / float(np.median(els)),
                sample=f"one fv_dynamics step{' + moist physics' if moist else ''}, C{N} L{npz} nq={nq}, "
                       f"6 tiles, numpy fp64 oracle (oracle/fv_dynamics.py), {procs} concurrent single-threaded "
                       f"replicas (one per core), step times {min(els):.1f}-{max(els):.1f} s")


def main():
    a = parse()
    if a.dt <= 0.0:
        a.dt = 450.0 * 180.0 / (a.npx - 1)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import torch
    import torch.distributed as dist

    import gtfv3_pkg
    pkg = gtfv3_pkg.load()
    import importlib
    state = importlib.import_module(pkg.__name__ + ".state")

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs an MI355X (no GPU visible)")
    torch.cuda.set_device(local)
    nccl_id = None
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        obj = [pkg.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        nccl_id = obj[0]
    proxy = a.rank_proxy if world == 1 and a.rank_proxy > 1 else 0
    lx, ly = (tuple(int(v) for v in a.layout.split("x")) if a.layout else layout_for(proxy or world))
    t_init = time.perf_counter()
    nq = max(a.nq, 6) if a.moist else a.nq
    if proxy:
        d = pkg.Domain(0, proxy, None, npx=a.npx, npz=a.npz, nq=nq, layout_x=lx, layout_y=ly, dt=a.dt, loopback=-1)
    else:
        d = pkg.Domain(rank, world, nccl_id, npx=a.npx, npz=a.npz, nq=nq, layout_x=lx, layout_y=ly, dt=a.dt)
    ak, bk, ks = state.hybrid_levels(a.npz)
    # large tracer sets (the C720 L137 x 54 configuration's per-GPU share) go up one tracer
    # at a time, so the host never holds all of them
    big_q = nq > 8 and not a.moist
    st = state.jablonowski_williamson(d, ak, bk, tracers=1 if big_q else None)
    if a.moist:
        state.aquaplanet_tracers(d, st, ak, bk)
    d.set_vertical(ak, bk, ks)
    for k, v in st.items():
        if k == "q" and big_q:
            d.create("q", nq * a.npz)
            d.upload_levels("q", 0, v)
            for iq in range(1, nq):
                d.upload_levels("q", iq * a.npz, state.tracer_planes(d, iq))
        else:
            d.upload(k, v)
    del st
    torch.cuda.synchronize()
    t_init = time.perf_counter() - t_init

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    def one_step():
        d.step(1)
        if a.moist:
            d.stencil("aquaplanet_physics", [], [a.dt])

    # Timed region: the steps alone (no events).  The roofline comes from a separate pass
    # afterwards on ONE stream: with the step's side streams two kernels share the chip and
    # each one's event span stretches, so per-kernel durations are only meaningful unoverlapped.
    d.set_streams(a.streams)
    for i in range(a.warmup):
        one_step()
    barrier()
    d.step_times(reset=True)  # the warm-up steps' device times are dropped
    t0 = time.perf_counter()
    for _ in range(a.steps):
        one_step()
    d.sync()
    barrier()
    el = time.perf_counter() - t0
    # per-step device times of the same K steps (HIP events on the library stream around each
    # fv_dynamics call, read after the timed region): the metric's median (report.py:152-153)
    per_step = d.step_times(reset=True)

    # Roofline pass (single stream): one step with every kernel bracketed by HIP events on
    # the library stream (the dominant family by device time, and every launcher's registered
    # algorithmic bytes = step_bytes), then --roofline-steps steps bracketing only that family
    # (so its events do not perturb its neighbours); --kernel-report: every kernel, all steps.
    kstats, dominant, step_bytes = {}, None, None
    if not a.no_kernel_timing:
        d.set_streams(1)
        d.kernel_timing_filter(None)
        d.kernel_timing(True)
        one_step()
        ks = d.kernel_stats()
        d.kernel_timing(False)
        step_bytes = sum(v[2] for v in ks.values())
        fam = families(ks)
        dominant = max(fam.items(), key=lambda kv: kv[1][0])[0] if fam else None
        d.kernel_timing_filter(None if a.kernel_report else dominant)
        d.kernel_timing(True)
        for _ in range(a.roofline_steps):
            one_step()
        kstats = d.kernel_stats()
        d.kernel_timing(False)
        d.kernel_timing_filter(None)
        d.set_streams(a.streams)
        barrier()
    med = float(np.median(per_step)) if len(per_step) == a.steps else None
    if world > 1:
        t = torch.tensor([el, med if med is not None else -1.0], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t[0].item())
        med = float(t[1].item()) if float(t[1].item()) > 0 else None

    N, npz = d.N, d.npz
    cells = 6 * N * N * npz
    value = cells * a.steps / el
    ms_step = 1000.0 * el / a.steps  # wall mean of the K timed steps (value's time base)
    step_stats = None
    if per_step and med is not None:
        step_stats = dict(median_ms=med, min_ms=float(np.min(per_step)), max_ms=float(np.max(per_step)),
                          mean_ms=float(np.mean(per_step)), wall_mean_ms=ms_step, n=len(per_step),
                          source="HIP events on the library stream around each fv_dynamics call of the "
                                 "timed steps (rank max of the median)" +
                                 ("; excludes the moist physics stencil" if a.moist else ""))

    roof = None
    if kstats:
        fam = families(kstats)
        name, (tot, n, byt) = max(fam.items(), key=lambda kv: kv[1][0])
        rsteps = a.roofline_steps
        avg_ms = tot / n
        traffic, src = pmc_traffic(name, {k: v[1] for k, v in kstats.items() if family(k) == name})
        ach = byt / (tot * 1e-3) / 1e9 if byt > 0 else None
        roof = dict(bound="hbm", kernel=name, achieved=ach, peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=ach / HBM_PEAK_GBS if ach else None, traffic=traffic, traffic_source=src,
                    bytes_per_launch=byt / n if byt > 0 else None, avg_ms=avg_ms,
                    launches_per_step=n / rsteps, share_of_step=tot / rsteps / ms_step,
                    measured=f"HIP events on the library stream around each launch, {rsteps} steps of a "
                             f"single-stream pass after the timed region")
        # the dominant single kernel (one instantiation, by launch name) of the all-kernel pass,
        # beside the dominant family above (the C and D grid Riemann solvers are one family;
        # the marches' template forms are separate families)
        kname, (kms, kn, kb) = max(ks.items(), key=lambda kv: kv[1][0])
        kach = kb / (kms * 1e-3) / 1e9 if kb > 0 else None
        roof["dominant_kernel"] = dict(kernel=kname.strip("()"), family=family(kname), ms_per_step=kms,
                                       launches_per_step=kn, achieved=kach,
                                       frac=kach / HBM_PEAK_GBS if kach else None,
                                       measured="HIP events, one single-stream step with every kernel timed")
        if step_bytes:
            man = manifest_step_bytes(d.nx, d.ny, d.nsub, npz, nq, 6, d.pitch, d.nj,
                                      march_ex_fraction(d.nx, d.subs))
            roof.update(step_bytes=step_bytes, step_bytes_manifest=sum(man.values()),
                        step_achieved=step_bytes / (ms_step * 1e-3) / 1e9,
                        step_frac=step_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS)
        if a.kernel_report and rank == 0:
            with open(a.kernel_report, "w") as f:
                json.dump({k: dict(ms_total=v[0], launches=v[1], ms_per_step=v[0] / rsteps,
                                   bytes_per_step=v[2] / rsteps, bytes_per_launch=v[2] / v[1],
                                   gbs=(v[2] / (v[0] * 1e-3) / 1e9) if v[2] > 0 else None)
                           for k, v in sorted(kstats.items(), key=lambda kv: -kv[1][0])}, f, indent=1)

    if a.geos_log:
        d.kernel_timing(False)
        per_step = []
        for _ in range(a.steps):
            barrier()
            t1 = time.perf_counter()
            one_step()
            d.sync()
            barrier()
            per_step.append(time.perf_counter() - t1)
        if rank == 0:
            geoslog = importlib.import_module(pkg.__name__ + ".geoslog")
            t_fin = time.perf_counter()
            geoslog.write_geos_log(a.geos_log, npx=d.N + 1, npz=d.npz, layout_x=lx, layout_y=ly,
                                   backend="hip-gfx950-f64", step_seconds=per_step, init_s=t_init,
                                   run_s=sum(per_step), finalize_s=time.perf_counter() - t_fin)

    if proxy:
        try:
            check = state_check(d, ak[0])
        except SystemExit as e:  # remote halos never refreshed: the state is not meaningful
            check = dict(not_checked=str(e)[:80])
    else:
        check = state_check(d, ak[0])  # every rank checks its own sub-domains

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        # the moist oracle's column loops are ~40x slower per cell than its dycore: C12 with --moist
        cpu_npx = a.cpu_npx if a.cpu_npx > 0 else (13 if a.moist else 49)
        cpu = cpu_baseline(pkg, cpu_npx, a.npz, nq, a.dt, a.moist, max(1, a.cpu_procs))

    if rank == 0:
        out = {
            "metric": "grid-cell-updates/sec per dycore step, " +
                      (f"Aquaplanet C{N} L{npz} + moist physics" if a.moist else f"Held-Suarez C{N} L{npz}") +
                      (f" with {nq} tracers" if nq != 4 and not a.moist else ""),
            "value": value,
            "unit": "grid-cell-updates/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            # the metric's step time is the median of per-step times (report.py:152-153); with
            # --moist the physics is outside those events, so the wall mean stands in
            "ms_per_step": step_stats["median_ms"] if step_stats and not a.moist else ms_step,
            "step_times": step_stats,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (Jablonowski-Williamson baroclinic state on an analytic hybrid L%d grid)" % npz,
            "config": {"workload": (f"Aquaplanet C{N} L{npz} dycore step + moist physics (aer_activation, "
                                    f"evap_subl_pdf, GFDL microphysics, radcouple)"
                                    if a.moist else f"Held-Suarez C{N} L{npz} dycore step (fv_dynamics)") +
                                   f", 6 tiles on {world} MI355X", "npx": N + 1, "npz": npz, "nq": nq,
                       "layout": f"{lx}x{ly}",
                       "dt_atmos": a.dt, "n_split": 6, "k_split": 1, "cells_per_step": cells,
                       "tracer_cell_updates_per_step": cells * nq},
            "roofline": roof,
            "cpu_baseline": cpu,
            "state_check": check,
        }
        if proxy:
            out["metric"] += f" (rank proxy: one rank of {proxy}, no xGMI transfer; not a measured N-GPU run)"
            out["rank_proxy"] = proxy
        print(json.dumps(out))
    d.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
