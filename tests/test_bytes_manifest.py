"""bytes_manifest.yaml (the committed field set of every kernel family) is
complete and agrees with the algorithmic bytes the launchers register with the event timer,
as recorded in the newest committed per-kernel report (profiles/rNN_bench_kernel_events.json
of `bench.py --kernel-report` at C180 L72, nq = 4, one GPU)."""
import glob
import json
import os

import yaml

from conftest import ROOT

import bench


def _newest_report():
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_bench_kernel_events.json")), reverse=True):
        rep = json.load(open(f))
        if all("bytes_per_step" in v for v in rep.values()):
            return f, rep
    return None, None


def test_manifest_covers_every_kernel_of_the_step():
    man = yaml.safe_load(open(os.path.join(ROOT, "bytes_manifest.yaml")))["families"]
    f, rep = _newest_report()
    assert rep, "no per-kernel report with registered bytes under profiles/"
    missing = [k.strip("()") for k in rep if k.strip("()") not in man and not k.startswith("__amd")]
    assert not missing, f"kernel families without a manifest entry: {missing}"


def test_manifest_matches_registered_bytes():
    f, rep = _newest_report()
    # the thermo march's tile-edge / interior kernels split the bytes by their output columns
    fex = bench.march_ex_fraction(180, [dict(ioff=0, N=180)] * 6)
    man = bench.manifest_step_bytes(180, 180, 6, 72, 4, 6, 192, 187, fex, alternatives=True)
    for k, v in rep.items():
        fam = k.strip("()")
        if fam.startswith("__amd") or fam == "halo_local_kernel":
            continue
        want = man[bench.manifest_family(fam)]
        got = v["bytes_per_step"]
        assert abs(got - want) <= 1e-9 * max(want, 1.0), f"{fam}: manifest {want:.6e} B/step, registered {got:.6e}"


def test_manifest_step_total_c180():
    man = bench.manifest_step_bytes(180, 180, 6, 72, 4, 6, 192, 187)
    total = sum(man.values())
    # the whole-step figure the bench divides by its step time (order 1e11 B at C180 L72)
    assert 5e10 < total < 5e11
