"""Golden vectors captured from the reference's own Python by tools/make_golden.py
(SURVEY.md §8c G1-G4): the benchmark-log contract (parse_geos_log,
geos_log_parser.py:7-71; report.py:152-153), the string helpers it is built on
(string_trf.py:10-49), and the bridge argument lists through the reference type
map (example_def_dycore.yaml:1-71, argument.py:54-86).  CPU only."""
import json
import os
import re

import pytest

from conftest import ROOT

GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def geoslog(pkg):
    import importlib
    return importlib.import_module(pkg.__name__ + ".geoslog")


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_log_writer_reproduces_golden_text(geoslog):
    g = _load("geos_log_parsed.json")
    with open(os.path.join(GOLD, "geos_log_sample.log")) as f:
        assert geoslog.format_geos_log(**g["inputs"]) == f.read()


def test_log_parse_matches_reference_parser(geoslog):
    g = _load("geos_log_parsed.json")
    ref = g["parsed"]
    got = geoslog.parse_dycore_log(geoslog.format_geos_log(**g["inputs"]))
    for k in ("backend", "grid_resolution", "node_setup", "fv_dyncore_timings", "global_init_time",
              "global_run_time", "global_finalize_time"):
        assert got[k] == ref[k], k
    assert geoslog.dycore_median(got) == ref["dycore_median"]
    # the rounded per-step seconds the log carries are the parsed timings
    assert ref["fv_dyncore_timings"] == [round(t, 6) for t in g["inputs"]["step_seconds"]]


def test_report_has_no_zero_division(geoslog):
    g = _load("geos_log_parsed.json")
    b = geoslog.parse_dycore_log(geoslog.format_geos_log(**g["inputs"]))
    txt = geoslog.report_dycore([b, b], names=["A", "B"])
    assert "Dycore (median)" in txt and "x1.00" in txt


def test_extract_numerics_and_grep(geoslog):
    g = _load("extract_numerics.json")
    for s, want in g["extract_numerics"].items():
        assert geoslog.extract_numerics([s]) == want, s
    text = "\n".join(g["grep_lines"]) + "\n"
    assert geoslog.grep_text(text, "--Run") == g["grep"]["plain"]
    assert geoslog.grep_text(text, "--Run", exclude_pattern=True) == g["grep"]["excluded"]
    assert geoslog.grep_text(text, "--Run", start_patterns=["Model Throughput"]) == g["grep"]["started"]
    assert geoslog.grep_text(text, "--Run", start_patterns=["Model Throughput"], end_pattern="END") == \
        g["grep"]["ended"]


def _prototype(txt, name):
    m = re.search(r"void " + name + r"\((.*?)\);", txt, flags=re.S)
    body = m.group(1).strip()
    if body == "void":
        return []
    out = []
    for a in body.split(","):
        a = a.strip()
        typ, nm = a.rsplit(" ", 1)
        if nm.startswith("*"):
            typ, nm = typ + "*", nm[1:]
        out.append((nm, typ.replace(" ", "")))
    return out


def test_bridge_header_matches_reference_type_map():
    g = _load("bridge_abi.json")
    txt = open(os.path.join(ROOT, "include", "geos_gtfv3_interface.h")).read()
    for fn, args in g["functions"].items():
        got = _prototype(txt, fn)
        assert [n for n, _ in got] == [a["name"] for a in args], fn
        assert [t for _, t in got] == [a["c_type"] for a in args], fn
    # fp64 twin: same names, array_float -> array_double through the same map
    want = [(a["name"], g["type_map"]["array_double"]["c_type"] if a["yaml_type"] == "array_float" else a["c_type"])
            for a in g["functions"]["geos_gtfv3_run_c"]]
    assert _prototype(txt, "geos_gtfv3_run_f64_c") == want
