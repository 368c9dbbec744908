"""GEOS-log-compatible benchmark output.

The reference measures the dycore by scanning GEOS stdout logs
(src/tcn/benchmark/geos_log_parser.py:7-71) and reports the median of the
per-step `geos_gtfv3` timings (report.py:152-158).  `write_geos_log` emits the
lines that parser reads, so a run of this build drops into the existing
benchmark workflow unchanged:

  Resource Parameter: NX: <nx>               geos_log_parser.py:48-52
  Resource Parameter: NY: <6*ny>             geos_log_parser.py:53-58 (NY/6 = layout_y)
   RUN_GTFV3:1                               geos_log_parser.py:11
   backend : <name>                          geos_log_parser.py:15-21
   Resolution of dynamics restart = N 6N L   geos_log_parser.py:40-47 (exactly 3 numerics)
   0 , geos_gtfv3 <seconds>                  geos_log_parser.py:24-26 (one line per step)
  Model Throughput / --Initialize / --Run / --Finalize   geos_log_parser.py:60-71 (2nd numeric)

`parse_dycore_log` restates the part of parse_geos_log that reads those lines
(same grep/extract_numerics semantics, string_trf.py:10-49) and
`report_dycore` is the reference's pairwise "Dycore (median)" comparison without
the FV GridComp term that divides by zero in report.py:134-150.
tests/test_golden.py checks both against the reference parser's own output,
captured by tools/make_golden.py into tests/golden/.
"""
import itertools
import re
from typing import Dict, List, Optional, Sequence

# string_trf.py:5-8 (the same verbose pattern)
_NUMERIC = re.compile(r"[-+]? (?: (?: \d* \. \d+ ) | (?: \d+ \.? ) )(?: [Ee] [+-]? \d+ ) ?", re.VERBOSE)


def extract_numerics(strings: Sequence[str]) -> List[float]:
    """All numeric literals of the strings, in order (string_trf.py:10-17)."""
    return [float(r) for s in strings for r in _NUMERIC.findall(s)]


def _grep(lines, pattern, exclude_pattern=False, start_patterns=None, end_pattern=None, expected=True):
    """string_trf.py:20-49 (without the starts_with variant the dycore lines never need)."""
    out = []
    sp = list(start_patterns) if start_patterns else None
    start = sp.pop(0) if sp else None
    for line in lines:
        if start and start in line:
            start = sp.pop(0) if sp else None
        if end_pattern and end_pattern in line:
            break
        if not start and pattern in line:
            if exclude_pattern:
                line = "".join(line.split(pattern)[1:])
            if line != "":
                out.append(line)
    if expected and not out:
        raise RuntimeError(f"Expecting {pattern} to be found")
    return out


def format_geos_log(npx: int, npz: int, layout_x: int, layout_y: int, backend: str,
                    step_seconds: Sequence[float], init_s: float, run_s: float, finalize_s: float) -> str:
    """Text of a GEOS-style stdout log for one dycore benchmark run."""
    n = npx - 1
    ln = [
        f" Resource Parameter: NX: {layout_x}",
        f" Resource Parameter: NY: {6 * layout_y}",
        " RUN_GTFV3:1",
        f" backend : {backend}",
        f" Resolution of dynamics restart = {n} {6 * n} {npz}",
    ]
    ln += [f" 0 , geos_gtfv3 {t:.6f}" for t in step_seconds]
    tot = init_s + run_s + finalize_s
    pct = (lambda x: 100.0 * x / tot) if tot > 0 else (lambda x: 0.0)
    ln += [
        " Model Throughput",
        f" --Initialize  {pct(init_s):.2f}  {init_s:.6f}",
        f" --Run  {pct(run_s):.2f}  {run_s:.6f}",
        f" --Finalize  {pct(finalize_s):.2f}  {finalize_s:.6f}",
        " GEOSgcm Run Status: 0",
    ]
    return "\n".join(ln) + "\n"


def grep_text(text: str, pattern: str, **kw) -> List[str]:
    """string_trf.grep over an in-memory log."""
    return _grep(text.splitlines(keepends=True), pattern, **kw)


def write_geos_log(path: str, **kw) -> None:
    with open(path, "w") as f:
        f.write(format_geos_log(**kw))


def parse_dycore_log(text: str) -> Dict:
    """backend, grid_resolution, node_setup, fv_dyncore_timings and the global
    init/run/finalize times, as parse_geos_log (geos_log_parser.py:7-71) fills them."""
    lines = text.splitlines(keepends=True)
    b: Dict = {}
    gt = _grep(lines, "RUN_GTFV3:1", exclude_pattern=True, expected=False) != []
    if not gt:
        b["backend"] = "fortran"
        b["fv_dyncore_timings"] = extract_numerics(_grep(lines, " 0: fv_dynamics", True, expected=False))
    else:
        g = _grep(lines, "backend : ", exclude_pattern=True, expected=False)
        b["backend"] = ("gtfv3_" + g[0].strip().replace("\n", "").replace(":", "")) if g else \
            "gtfv3 (details failed to parse)"
        b["fv_dyncore_timings"] = extract_numerics(_grep(lines, " 0 , geos_gtfv3", True))
    gs = extract_numerics(_grep(lines, "Resolution of dynamics restart"))
    assert len(gs) == 3
    b["grid_resolution"] = [int(x) for x in gs]
    nx = extract_numerics(_grep(lines, "Resource Parameter: NX:", True))
    ny = extract_numerics(_grep(lines, "Resource Parameter: NY:", True))
    assert len(nx) == 1 and len(ny) == 1
    NX, NY = int(nx[0]), int(ny[0])
    b["node_setup"] = [NX, int(NY / 6), int(NX * (NY / 6) * 6)]
    for key, pat in (("global_init_time", "--Initialize"), ("global_run_time", "--Run"),
                     ("global_finalize_time", "--Finalize")):
        b[key] = extract_numerics(_grep(lines, pat, start_patterns=["Model Throughput"]))[1]
    return b


def dycore_median(b: Dict) -> float:
    """report.py:152-153: np.median of the per-step dycore timings."""
    t = sorted(b["fv_dyncore_timings"])
    n = len(t)
    return t[n // 2] if n % 2 else 0.5 * (t[n // 2 - 1] + t[n // 2])


def report_dycore(benches: Sequence[Dict], names: Optional[Sequence[str]] = None) -> str:
    """Pairwise speed-up lines ("Global RUN", "Dycore (median)") in the spirit of
    report.py:95-204, minus the FV GridComp comparison that crashes there."""
    def cmp(a, b, label):
        if a <= 0 or b <= 0:
            return f"  {label}: n/a\n"
        return f"  {label}: {a:.4f}s vs {b:.4f}s -> x{a / b:.2f}\n"

    out = ""
    names = names or [b["backend"] for b in benches]
    for (na, a), (nb, b) in itertools.combinations(list(zip(names, benches)), 2):
        out += f"{na} vs {nb}\n\n"
        out += cmp(a["global_run_time"], b["global_run_time"], "Global RUN")
        out += cmp(dycore_median(a), dycore_median(b), "Dycore (median)")
        out += "\n"
    return out
