"""Serialbox savepoint ingestion (geosongpu-ci_amd/serialbox.py) on CPU:
archive round trips through the restated binary format, the reference converter's
transformations (serialbox_dat_to_netcdf.py:47-52 fill value, :131-152 tracer halo strip,
:101-104 rank count from the namelist layout) and the FVDynamics-In -> dycore-state mapping.
No GEOS dump exists here: parity against real archives is unpinned."""
import importlib
import os

import numpy as np
import pytest


@pytest.fixture(scope="module")
def sb(pkg):
    return importlib.import_module(pkg.__name__ + ".serialbox")


def test_archive_round_trip(sb, tmp_path):
    r = np.random.default_rng(3)
    w = sb.SerialboxWriter(str(tmp_path), "Generator_rank0", {"nx": 12})
    a0, a1 = r.standard_normal((7, 6, 3)), r.standard_normal((7, 6, 3))
    w.write("u", "FVDynamics-In", a0, {"i_call": 0})
    w.write("u", "FVDynamics-In", a1, {"i_call": 1})
    w.write("ks", "FVDynamics-In", np.array([5], dtype=np.int32), {"i_call": 0})
    w.write("u", "FVDynamics-Out", a0 * 2, {"i_call": 0})
    w.close()
    rd = sb.SerialboxReader(str(tmp_path), "Generator_rank0")
    sps = rd.get_savepoint("FVDynamics-In")
    assert [s.meta_info["i_call"] for s in sps] == [0, 1]
    assert sorted(rd.fields_at_savepoint(sps[0])) == ["ks", "u"]
    assert np.array_equal(rd.read("u", sps[0]), a0) and np.array_equal(rd.read("u", sps[1]), a1)
    assert rd.read("ks", sps[0]).dtype == np.int32
    assert np.array_equal(rd.read("u", rd.get_savepoint("FVDynamics-Out")[0]), a0 * 2)
    assert rd.global_meta_info["nx"] == 12
    # column-major records (the Fortran frontend's order)
    raw = np.fromfile(os.path.join(tmp_path, "Generator_rank0_u.dat"), dtype="<f8", count=a0.size)
    assert np.array_equal(raw, a0.ravel(order="F"))
    # corrupted record -> checksum error
    with open(os.path.join(tmp_path, "Generator_rank0_u.dat"), "r+b") as f:
        f.write(b"\\0" * 8)
    with pytest.raises(ValueError, match="checksum"):
        rd.read("u", sps[0])


def test_reads_hand_written_upstream_layout(sb, tmp_path):
    """A MetaData / ArchiveMetaData pair written by hand in Serialbox 2.6's own layout
    (SavepointVector::toJSON, FieldMap::toJSON, BinaryArchive::updateMetaData: records are
    [offset, checksum], MD5 when the library was built without OpenSSL), not by this
    module's writer."""
    import hashlib
    import json
    r = np.random.default_rng(11)
    delp = r.standard_normal((5, 4, 2))
    ks = np.array([7], dtype=np.int32)
    b_delp = np.asfortranarray(delp).tobytes(order="F")
    # two records of delp; the second one is the one the savepoint points at
    with open(tmp_path / "Generator_rank0_delp.dat", "wb") as f:
        f.write(b"\x00" * len(b_delp) + b_delp)
    with open(tmp_path / "Generator_rank0_ks.dat", "wb") as f:
        f.write(ks.tobytes())
    meta = {
        "serialbox_version": 20600, "prefix": "Generator_rank0",
        "global_meta_info": {"layout": {"type_id": 2, "value": 1}},
        "savepoint_vector": {
            "savepoints": [{"name": "FVDynamics-In", "meta_info": {"i_call": {"type_id": 2, "value": 0}}},
                           {"name": "Driver-In", "meta_info": {}}],
            "fields_per_savepoint": [{"delp": 1, "ks": 0}, None]},
        "field_map": {"delp": {"type_id": 5, "dims": [5, 4, 2], "meta_info": {}},
                      "ks": {"type_id": 2, "dims": [1], "meta_info": {}}},
    }
    arch = {"serialbox_version": 20600, "archive_name": "Binary", "archive_version": 0, "hash_algorithm": "MD5",
            "fields_table": {"delp": [[0, hashlib.md5(b"\x00" * len(b_delp)).hexdigest()],
                                      [len(b_delp), hashlib.md5(b_delp).hexdigest().upper()]],
                             "ks": [[0, hashlib.md5(ks.tobytes()).hexdigest()]]}}
    (tmp_path / "MetaData-Generator_rank0.json").write_text(json.dumps(meta))
    (tmp_path / "ArchiveMetaData-Generator_rank0.json").write_text(json.dumps(arch))
    rd = sb.SerialboxReader(str(tmp_path), "Generator_rank0")
    sp = rd.get_savepoint("FVDynamics-In")[0]
    assert sp.meta_info == {"i_call": 0}
    assert np.array_equal(rd.read("delp", sp), delp)
    assert int(rd.read("ks", sp)[0]) == 7
    assert rd.fields_at_savepoint(rd.get_savepoint("Driver-In")[0]) == []
    # this module's writer emits the same record order
    w = sb.SerialboxWriter(str(tmp_path / "w"), "p")
    w.write("delp", "s", delp)
    w.close()
    rec = json.loads((tmp_path / "w" / "ArchiveMetaData-p.json").read_text())["fields_table"]["delp"][0]
    assert isinstance(rec[0], int) and isinstance(rec[1], str)


def test_namelist_reader(sb, tmp_path):
    p = tmp_path / "input.nml"
    p.write_text("&fv_core_nml\n  layout = 2, 3  ! comment\n  npx = 49, hydrostatic = .false.\n"
                 "  dddmp = 0.2d0\n  grid_file = 'x.nc'\n/\n&other\n a=1\n/\n")
    nml = sb.read_namelist(str(p))
    assert nml["fv_core_nml"]["layout"] == [2, 3]
    assert nml["fv_core_nml"]["npx"] == 49 and nml["fv_core_nml"]["hydrostatic"] is False
    assert nml["fv_core_nml"]["dddmp"] == 0.2 and nml["fv_core_nml"]["grid_file"] == "x.nc"
    assert nml["other"]["a"] == 1


def test_dat_to_netcdf_matches_reference_converter(sb, tmp_path):
    from scipy.io import netcdf_file
    src, dst = tmp_path / "in", tmp_path / "out"
    src.mkdir()
    (src / "input.nml").write_text("&fv_core_nml\n layout = 1, 1\n/\n")
    r = np.random.default_rng(9)
    want = {}
    for rank in range(6):
        w = sb.SerialboxWriter(str(src), f"Generator_rank{rank}")
        for call in range(2):
            qv = r.standard_normal((18, 18, 4))
            qv[0, 0, 0] = 1e40  # the fill value the converter zeroes
            delp = r.standard_normal((18, 18, 4))
            w.write("qvapor", "FVDynamics-In", qv, {"i_call": call})
            w.write("delp", "FVDynamics-In", delp, {"i_call": call})
            w.write("bdt", "FVDynamics-In", np.array([900.0]), {"i_call": call})
            want[(rank, call)] = (qv, delp)
        w.close()
    files = sb.dat_to_netcdf(str(src), str(dst))
    assert [os.path.basename(f) for f in files] == ["FVDynamics-In.nc"]
    with netcdf_file(files[0], "r", mmap=False) as nc:
        q = nc.variables["qvapor"][:].copy()
        dp = nc.variables["delp"][:].copy()
        bdt = nc.variables["bdt"][:].copy()
    assert q.shape == (2, 6, 12, 12, 4) and dp.shape == (2, 6, 18, 18, 4) and bdt.shape == (2, 6)
    for (rank, call), (qv, delp) in want.items():
        ref = qv.copy()
        ref[ref == 1e40] = 0.0
        assert np.array_equal(q[call, rank], ref[3:-3, 3:-3])
        assert np.array_equal(dp[call, rank], delp)
    assert np.all(bdt == 900.0)


def test_fv_dynamics_in_to_state(pkg, sb, tmp_path):
    d = pkg.Domain(npx=13, npz=3, nq=6, host_only=1)
    N, ng = 12, 3
    r = np.random.default_rng(1)
    w = sb.SerialboxWriter(str(tmp_path), "Generator_rank0")
    delp = r.standard_normal((N + 2 * ng, N + 2 * ng, 3))
    u = r.standard_normal((N + 2 * ng, N + 2 * ng + 1, 3))
    pe = r.standard_normal((N + 2, 4, N + 2))  # (is-1:ie+1, npz+1, js-1:je+1)
    w.write("delp", "FVDynamics-In", delp)
    w.write("u", "FVDynamics-In", u)
    w.write("pe", "FVDynamics-In", pe)
    for t in sb.FV_DYNAMICS_TRACERS:
        w.write(t, "FVDynamics-In", np.full((N + 2 * ng, N + 2 * ng, 3), float(len(t))))
    w.close()
    rd = sb.SerialboxReader(str(tmp_path), "Generator_rank0")
    st = sb.fv_dynamics_state(rd, rd.get_savepoint("FVDynamics-In")[0], d)
    # Fortran (isd:ied, jsd:jed, k) -> [k, j + NG, i + NG] from the data-domain corner
    assert np.array_equal(st["delp"][:, :N + 2 * ng, :N + 2 * ng], np.transpose(delp, (2, 1, 0)))
    assert np.array_equal(st["u"][:, :N + 2 * ng + 1, :N + 2 * ng], np.transpose(u, (2, 1, 0)))
    # pe is (i, k, j) in the dump, its section starts one point outside the compute domain
    assert np.array_equal(st["pe"][:, ng - 1:ng + N + 1, ng - 1:ng + N + 1], np.transpose(pe, (1, 2, 0)))
    assert st["q"].shape[0] == 6 * 3 and st["q"][3, ng, ng] == len("qliquid")


def _write_archive(pkg, sb, path, nq=6):
    """FVDynamics-In from the synthetic JW state (six tiles, one prefix each) and
    FVDynamics-Out from one oracle step of it, as a GEOS serialization run would write."""
    import importlib as il
    import sys
    from conftest import metrics_of, oracle_scalars
    from oracle import fv_dynamics as fvd
    state = il.import_module(pkg.__name__ + ".state")
    npz, npx = 10, 13
    d = pkg.Domain(npx=npx, npz=npz, nq=nq, host_only=1)
    ak, bk, ks = state.hybrid_levels(npz)
    st = state.jablonowski_williamson(d, ak, bk)
    ms = metrics_of(d)
    sc = oracle_scalars(d)
    g = fvd.Grid(d.N, 1, 1, ms, sc["corner_w"], sc["da_min_c"], d.nj, d.pitch)
    nl = dict(n_split=6, dt_atmos=900.0, hord_mt=6, hord_vt=6, hord_tm=6, hord_dp=6, hord_tr=6, dddmp=0.2,
              d2_bg=0.0, p_fac=0.05, dz_min=2.0, fill=1, nq=nq)
    out = fvd.fv_dynamics({k: v.copy() for k, v in st.items()}, ak, bk, g, nl)
    (path / "input.nml").write_text("&fv_core_nml\n layout = 1, 1\n n_split = 6\n hord_mt = 6, hord_vt = 6\n"
                                    " hord_tm = 6, hord_dp = 6, hord_tr = 6\n dddmp = 0.2\n p_fac = 0.05\n/\n")
    for r in range(6):
        w = sb.SerialboxWriter(str(path), f"Generator_rank{r}")
        for name, a in sb.state_to_savepoint(st, r, d.N).items():
            w.write(name, "FVDynamics-In", a)
        for name, v in (("ak", ak), ("bk", bk)):
            w.write(name, "FVDynamics-In", np.asarray(v))
        w.write("ks", "FVDynamics-In", np.array([ks], dtype=np.int32))
        w.write("bdt", "FVDynamics-In", np.array([900.0]))
        w.write("nq", "FVDynamics-In", np.array([nq], dtype=np.int32))
        for name, a in sb.state_to_savepoint(out, r, d.N).items():
            w.write(name, "FVDynamics-Out", a)
        w.close()


def test_parity_runner_round_trip_oracle(pkg, sb, tmp_path, capsys):
    """tools/serialbox_parity.py with the oracle engine reproduces an oracle-written
    FVDynamics-Out exactly (the savepoint <-> state mappings are inverse to each other)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import serialbox_parity
    _write_archive(pkg, sb, tmp_path)
    assert serialbox_parity.main([str(tmp_path), "--engine", "oracle", "--rtol", "0"]) == 0
    lines = [ln for ln in capsys.readouterr().out.splitlines() if "max |diff|" in ln]
    assert len(lines) >= 20 and all("FAIL" not in ln for ln in lines)


@pytest.mark.gpu
def test_parity_runner_hip_against_oracle_dump(pkg, require_gpu, sb, tmp_path):
    """The HIP step on a serialized FVDynamics-In matches the dump's FVDynamics-Out within
    1e-9 (here the dump is the oracle's; with a GEOS dump the CI bar is 1e-4)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import serialbox_parity
    _write_archive(pkg, sb, tmp_path)
    assert serialbox_parity.main([str(tmp_path), "--engine", "hip", "--rtol", "1e-9"]) == 0
