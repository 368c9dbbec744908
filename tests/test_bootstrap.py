"""The bridge's ncclUniqueId bootstrap (csrc/bridge.hip share_unique_id), on CPU with two
processes: over the caller's Fortran MPI communicator (the reference's C shim takes the
handle by value and calls MPI_Comm_f2c, base.py:89-96; argument.py:57-58,83-84) with an
MPICH-ABI test double of MPI, and without MPI through a job-stamped id file that a stale
file from another job cannot satisfy (bridge.hip:161)."""
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT

CHILD = r"""
import ctypes, os, sys
if os.environ.get("FAKE_MPI_SO"):
    ctypes.CDLL(os.environ["FAKE_MPI_SO"], mode=ctypes.RTLD_GLOBAL)
sys.path.insert(0, os.environ["GT_ROOT"])
import gtfv3_pkg
import importlib
M = importlib.import_module(gtfv3_pkg.load().__name__ + "._lib")
L = M.lib()
rank = ctypes.c_int(-1); size = ctypes.c_int(-1)
buf = ctypes.create_string_buffer(bytes(range(7, 7 + 128)) if os.environ["ROLE"] == "0" else b"\0" * 128, 128)
rc = L.gtfv3_bootstrap_id(ctypes.c_void_p(int(os.environ["COMM"])), buf, ctypes.byref(rank), ctypes.byref(size))
if rc != 0:
    print("ERR", M.last_error()); sys.exit(3)
print("OK", rank.value, size.value, buf.raw.hex(), flush=True)
if os.environ.get("DONE_AFTER"):  # the real bridge removes its id file once the comm exists
    import time
    while not os.path.exists(os.environ["DONE_AFTER"]):
        time.sleep(0.01)
    L.gtfv3_bootstrap_done()
"""


def _spawn(env_extra):
    env = dict(os.environ, GT_ROOT=ROOT, **env_extra)
    return subprocess.Popen([sys.executable, "-c", CHILD], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                            text=True)


def _finish(p):
    out, err = p.communicate(timeout=120)
    assert p.returncode == 0, out + err
    tag, rank, size, hx = out.strip().splitlines()[-1].split()
    return int(rank), int(size), bytes.fromhex(hx)


WANT = bytes(range(7, 7 + 128))


def test_bootstrap_over_fortran_mpi_comm(pkg, tmp_path):
    so = tmp_path / "libfakempi.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-O1", "-o", str(so), os.path.join(ROOT, "tests", "native",
                                                                                "fake_mpi.c")], check=True)
    handle = 0x44000000  # MPICH's Fortran MPI_COMM_WORLD
    base = dict(FAKE_MPI_SO=str(so), FAKE_MPI_DIR=str(tmp_path), FAKE_MPI_SIZE="2", COMM=str(handle))
    # no env rank variables and no id file: the rank must come from the communicator
    for v in ("RANK", "WORLD_SIZE", "GTFV3_RANK", "GTFV3_WORLD_SIZE", "GTFV3_NCCL_ID_FILE"):
        base[v] = ""
    p1 = _spawn(dict(base, FAKE_MPI_RANK="1", ROLE="1"))
    p0 = _spawn(dict(base, FAKE_MPI_RANK="0", ROLE="0"))
    r0, r1 = _finish(p0), _finish(p1)
    assert r0 == (0, 2, WANT) and r1 == (1, 2, WANT)
    log = (tmp_path / "log.1").read_text().split("\n")
    assert f"f2c {handle} 0" in log
    assert f"bcast {handle} {0x4c00010d * 1000 + 128}" in log


def test_bootstrap_id_file_ignores_stale_job(pkg, tmp_path):
    idf = tmp_path / "nccl.id"
    # a complete id record of an earlier job is already there
    stale = b"GTFV3ID1" + (len(b"GTFV3_JOB_TOKEN=old")).to_bytes(4, "little") + b"GTFV3_JOB_TOKEN=old" + b"\xee" * 128
    idf.write_bytes(stale)
    base = dict(GTFV3_NCCL_ID_FILE=str(idf), GTFV3_JOB_TOKEN="new", GTFV3_WORLD_SIZE="2", COMM="0")
    p1 = _spawn(dict(base, GTFV3_RANK="1", ROLE="1"))
    time.sleep(1.0)  # rank 1 polls the stale file first
    assert p1.poll() is None, "rank 1 must not accept the stale job's id"
    go = tmp_path / "go"
    p0 = _spawn(dict(base, GTFV3_RANK="0", ROLE="0", DONE_AFTER=str(go)))
    r1 = _finish(p1)
    go.write_text("1")
    r0 = _finish(p0)
    assert r0 == (0, 2, WANT) and r1 == (1, 2, WANT)
    assert not idf.exists(), "rank 0 removes its id file at finalize"


def test_bootstrap_id_file_needs_token(pkg, tmp_path):
    env = dict(GTFV3_NCCL_ID_FILE=str(tmp_path / "x.id"), GTFV3_WORLD_SIZE="2", GTFV3_RANK="1", COMM="0", ROLE="1")
    for v in ("GTFV3_JOB_TOKEN", "SLURM_JOB_ID", "PBS_JOBID", "TORCHELASTIC_RUN_ID", "MASTER_PORT"):
        env[v] = ""
    p = _spawn(env)
    out, err = p.communicate(timeout=120)
    assert p.returncode == 3 and "job token" in out
