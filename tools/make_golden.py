#!/usr/bin/env python3
"""Capture golden vectors from the reference's own Python.

Runs ONLY in the build container, where the read-only reference checkout sits at
/root/reference; the GPU box never runs this.  It imports the reference modules
that import cleanly here (tcn.benchmark.*, tcn.py_ftn_interface.argument), feeds
them inputs, and commits their OUTPUTS as small JSON / text fixtures under
tests/golden/ (no reference source is copied):

  geos_log_sample.log / geos_log_parsed.json  G2: parse_geos_log (geos_log_parser.py:7-71)
        of a log written by geosongpu-ci_amd/geoslog.py, plus report.py's
        "Dycore (median)" (np.median of the per-step timings, report.py:152-153)
  extract_numerics.json   G4: string_trf.extract_numerics / grep on GEOS profiler lines
  bridge_abi.json         G1+G3: the geos_gtfv3 init/run/finalize argument lists of
        example_def_dycore.yaml:1-71 mapped through Argument.c_type /
        f90_type_definition (argument.py:54-86)

    python tools/make_golden.py
"""
import json
import os
import sys
import tempfile

import numpy as np
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
OUT = os.path.join(ROOT, "tests", "golden")

sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(REF, "src"))


def log_inputs():
    # fixed, representative inputs: C180 L72, 2x2 layout, 8 steps with a slow first one
    return dict(npx=181, npz=72, layout_x=2, layout_y=2, backend="hip-gfx950-f64",
                step_seconds=[0.412345, 0.0751, 0.0749, 0.07502, 0.0748, 0.0753, 0.07499, 0.0750],
                init_s=3.25, run_s=1.0302, finalize_s=0.0125)


def main():
    import gtfv3_pkg
    from tcn.benchmark.geos_log_parser import parse_geos_log
    from tcn.benchmark.string_trf import extract_numerics, grep
    from tcn.py_ftn_interface.argument import Argument

    geoslog = __import__(gtfv3_pkg.load().__name__ + ".geoslog", fromlist=["x"])
    os.makedirs(OUT, exist_ok=True)

    # ---- G2: parse_geos_log on our emitted log
    inp = log_inputs()
    text = geoslog.format_geos_log(**inp)
    with open(os.path.join(OUT, "geos_log_sample.log"), "w") as f:
        f.write(text)
    b = parse_geos_log(os.path.join(OUT, "geos_log_sample.log"))
    parsed = dict(backend=b.backend, grid_resolution=list(b.grid_resolution), node_setup=list(b.node_setup),
                  fv_dyncore_timings=list(b.fv_dyncore_timings), global_init_time=b.global_init_time,
                  global_run_time=b.global_run_time, global_finalize_time=b.global_finalize_time,
                  dycore_median=float(np.median(b.fv_dyncore_timings)))
    with open(os.path.join(OUT, "geos_log_parsed.json"), "w") as f:
        json.dump(dict(inputs=inp, parsed=parsed), f, indent=1)

    # ---- G4: extract_numerics / grep on representative GEOS lines
    samples = [" 0 , geos_gtfv3 0.075123", " Resolution of dynamics restart = 180 1080 72",
               " --Run  97.12  1234.5", "----------FV_DYNAMICS   1.0e+01  -3.5E-2  .25  7.",
               "GOCART2G  12.5 3", "  backend : dace:gpu"]
    en = {s: extract_numerics([s]) for s in samples}
    with tempfile.NamedTemporaryFile("w", suffix=".log", delete=False) as f:
        f.write("\n".join(["head --Run 1 2", "Model Throughput", "x --Run 3 4", "y --Run 5 6", "END", "z --Run 7"])
                + "\n")
        tmp = f.name
    gr = dict(plain=grep(tmp, "--Run"), excluded=grep(tmp, "--Run", exclude_pattern=True),
              started=grep(tmp, "--Run", start_patterns=["Model Throughput"]),
              ended=grep(tmp, "--Run", start_patterns=["Model Throughput"], end_pattern="END"))
    os.unlink(tmp)
    with open(os.path.join(OUT, "extract_numerics.json"), "w") as f:
        json.dump(dict(extract_numerics=en, grep_lines=["head --Run 1 2", "Model Throughput", "x --Run 3 4",
                                                        "y --Run 5 6", "END", "z --Run 7"], grep=gr), f, indent=1)

    # ---- G1 + G3: bridge argument lists through the reference type map
    spec = yaml.safe_load(open(os.path.join(REF, "src/tcn/py_ftn_interface/example_def_dycore.yaml")))
    funcs = {}
    for fname, fdef in spec["functions"].items():
        args = []
        for group in ("inputs", "inouts", "outputs"):
            fd = fdef if isinstance(fdef, dict) else {}  # "finalize: None"
            for name, typ in (fd.get(group) or {}).items():
                a = Argument(name, typ)
                args.append(dict(name=name, group=group, yaml_type=typ, c_type=a.c_type,
                                 f90=a.f90_type_definition))
        funcs[f"{spec['name']}_{fname}_c"] = args
    tmap = {t: dict(c_type=Argument("x", t).c_type, f90=Argument("x", t).f90_type_definition)
            for t in ("int", "float", "double", "array_int", "array_float", "array_double", "MPI")}
    with open(os.path.join(OUT, "bridge_abi.json"), "w") as f:
        json.dump(dict(functions=funcs, type_map=tmap), f, indent=1)
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
