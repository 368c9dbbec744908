"""Serialbox savepoint ingestion: read the GEOS/FV3 serialized savepoints
(`geos_build/serialize`, e.g. the C24 experiment of `xp_C24_make.sh:9-26`) without the
serialbox library, convert them to NetCDF the way the reference's converter does
(src/tcn/validation/serialbox/serialbox_dat_to_netcdf.py:69-176), and map an
`FVDynamics-In` savepoint onto this package's dycore state so that a dump of the real model
can be stepped on the GPU and compared with its `FVDynamics-Out`.

Serialbox 2 binary archive, restated (Serialbox 2.6, BinaryArchive + MetaDataSerializer):
  MetaData-<prefix>.json         savepoints (name + meta-info), the fields stored at each
                                 savepoint (field -> id in that field's archive table), and
                                 the field map (type id, dims, meta-info)
  ArchiveMetaData-<prefix>.json  per field the table of stored records [byte offset, checksum]
                                 (BinaryArchive::updateMetaData writes FileOffsetType{offset,
                                 checksum} in that order; a [checksum, offset] record, as an
                                 early writer of this module emitted, is recognised by type)
  <prefix>_<field>.dat           the records, raw little-endian values, column-major
                                 (the Fortran frontend's order, first dimension fastest)
with one prefix per rank, "Generator_rank<r>" (serialbox_dat_to_netcdf.py:61-64).
Type ids: 1 bool, 2 int32, 3 int64, 4 float32, 5 float64.

The serialbox library, xarray, netCDF4 and f90nml are not installable here: the
reader/writer below restates the format, NetCDF output is NetCDF-3 through scipy.io, and the
namelist reader handles the `&fv_core_nml layout = a, b` entries the converter uses.  No
GEOS dump exists in this container, so the format is exercised by round trips through the
writer (tests/test_serialbox.py): "parity unpinned" against real archives.
"""
import hashlib
import json
import os
import re

import numpy as np

TYPE_DTYPE = {1: np.dtype("bool"), 2: np.dtype("<i4"), 3: np.dtype("<i8"), 4: np.dtype("<f4"), 5: np.dtype("<f8")}
DTYPE_TYPE = {np.dtype(v).str: k for k, v in TYPE_DTYPE.items()}
# the converter's savepoints whose tracer fields carry a 3-point halo it strips
# (serialbox_dat_to_netcdf.py:131-152)
HALO_SAVEPOINTS = ("FVDynamics-In", "FVDynamics-Out", "Driver-In", "Driver-Out")
HALO_TRACERS = ("qvapor", "qliquid", "qice", "qrain", "qsnow", "qgraupel", "qo3mr", "qsgs_tke")


def _meta_value(v):
    if isinstance(v, dict) and "value" in v:
        return v["value"]
    return v


def _record(r):
    """(byte offset, checksum) of one fields_table record: Serialbox's order is [offset,
    checksum]; a [checksum, offset] pair is told apart by the element types"""
    a, b = r
    if isinstance(a, str) and not isinstance(b, str):
        a, b = b, a
    return int(a), (b or "")


class Savepoint:
    def __init__(self, name, meta):
        self.name = name
        self.meta_info = {k: _meta_value(v) for k, v in (meta or {}).items()}

    def __repr__(self):
        return f"Savepoint({self.name}, {self.meta_info})"


class SerialboxReader:
    """Serializer(OpenModeKind.Read, path, prefix) restated: savepoint_list, get_savepoint,
    fields_at_savepoint, read."""

    def __init__(self, path, prefix):
        self.path, self.prefix = path, prefix
        with open(os.path.join(path, f"MetaData-{prefix}.json")) as f:
            self.meta = json.load(f)
        with open(os.path.join(path, f"ArchiveMetaData-{prefix}.json")) as f:
            self.archive = json.load(f)
        spv = self.meta["savepoint_vector"]
        self._sps = [Savepoint(s["name"], s.get("meta_info")) for s in spv["savepoints"]]
        self._fields = [f or {} for f in spv["fields_per_savepoint"]]
        self.field_map = self.meta["field_map"]
        self.global_meta_info = {k: _meta_value(v) for k, v in self.meta.get("global_meta_info", {}).items()}

    def savepoint_list(self):
        return list(self._sps)

    def get_savepoint(self, name):
        return [s for s in self._sps if s.name == name]

    def fields_at_savepoint(self, sp):
        return list(self._fields[self._index(sp)].keys())

    def _index(self, sp):
        for n, s in enumerate(self._sps):
            if s is sp or (s.name == sp.name and s.meta_info == sp.meta_info):
                return n
        raise KeyError(f"no savepoint {sp}")

    def read(self, field, sp, verify=True):
        rec = self._fields[self._index(sp)][field]
        info = self.field_map[field]
        dt = TYPE_DTYPE[int(info["type_id"])]
        dims = [int(x) for x in info["dims"]]
        n = int(np.prod(dims)) if dims else 1
        offset, checksum = _record(self.archive["fields_table"][field][rec])
        with open(os.path.join(self.path, f"{self.prefix}_{field}.dat"), "rb") as f:
            f.seek(int(offset))
            raw = f.read(n * dt.itemsize)
        algo = str(self.archive.get("hash_algorithm", "SHA256")).lower().replace("-", "")
        if verify and checksum and algo in ("sha256", "md5") and \
                hashlib.new(algo, raw).hexdigest().lower() != checksum.lower():
            raise ValueError(f"{field} at {sp}: checksum mismatch")
        return np.frombuffer(raw, dtype=dt).reshape(dims, order="F").copy()


class SerialboxWriter:
    """Writes the same archive layout (savepoints in call order, records appended)."""

    def __init__(self, path, prefix, global_meta_info=None):
        os.makedirs(path, exist_ok=True)
        self.path, self.prefix = path, prefix
        self.sps, self.fields, self.field_map, self.table = [], [], {}, {}
        self.gmi = dict(global_meta_info or {})

    def write(self, field, sp_name, data, sp_meta=None):
        a = np.asarray(data)
        if a.dtype == np.float64 or a.dtype == np.float32 or a.dtype == np.int32 or a.dtype == np.int64 or \
                a.dtype == np.bool_:
            pass
        else:
            a = a.astype(np.float64)
        key = (sp_name, json.dumps(sp_meta or {}, sort_keys=True))
        idx = next((n for n, s in enumerate(self.sps) if (s[0], s[2]) == key), None)
        if idx is None:
            self.sps.append((sp_name, dict(sp_meta or {}), key[1]))
            self.fields.append({})
            idx = len(self.sps) - 1
        tid = DTYPE_TYPE[a.dtype.newbyteorder("<").str if a.dtype.byteorder not in "<|" else a.dtype.str]
        dims = list(a.shape)
        prev = self.field_map.get(field)
        if prev and (prev["dims"] != dims or prev["type_id"] != tid):
            raise ValueError(f"{field}: dims / type differ from earlier records")
        self.field_map[field] = {"type_id": tid, "dims": dims, "meta_info": {}}
        raw = np.asfortranarray(a).astype(TYPE_DTYPE[tid]).tobytes(order="F")
        fn = os.path.join(self.path, f"{self.prefix}_{field}.dat")
        offset = os.path.getsize(fn) if os.path.exists(fn) else 0
        with open(fn, "ab") as f:
            f.write(raw)
        self.table.setdefault(field, []).append([offset, hashlib.sha256(raw).hexdigest()])
        self.fields[idx][field] = len(self.table[field]) - 1

    def close(self):
        meta = {
            "serialbox_version": 20602,
            "prefix": self.prefix,
            "global_meta_info": {k: {"type_id": 5 if isinstance(v, float) else 2, "value": v}
                                 for k, v in self.gmi.items()},
            "savepoint_vector": {
                "savepoints": [{"name": n, "meta_info": {k: {"type_id": 2, "value": v} for k, v in m.items()}}
                               for n, m, _ in self.sps],
                "fields_per_savepoint": self.fields,
            },
            "field_map": self.field_map,
        }
        arch = {"serialbox_version": 20602, "archive_name": "Binary", "archive_version": 0,
                "hash_algorithm": "SHA256", "fields_table": self.table}
        with open(os.path.join(self.path, f"MetaData-{self.prefix}.json"), "w") as f:
            json.dump(meta, f)
        with open(os.path.join(self.path, f"ArchiveMetaData-{self.prefix}.json"), "w") as f:
            json.dump(arch, f)


def _nml_value(x):
    xl = x.strip().lower()
    if xl in (".true.", "t", ".t.", "true"):
        return True
    if xl in (".false.", "f", ".f.", "false"):
        return False
    if re.fullmatch(r"[-+]?\d+", xl):
        return int(xl)
    try:
        return float(xl.replace("d", "e"))
    except ValueError:
        return x.strip().strip("'\"")


def read_namelist(path):
    """{group: {key: value}} of a Fortran namelist (the `&fv_core_nml ... /` groups the
    converter reads with f90nml): integers, reals (1.0d0 too), logicals, strings, lists."""
    txt = re.sub(r"!.*", "", open(path).read())
    out = {}
    for g, body in re.findall(r"&(\w+)(.*?)(?:^\s*/|/\s*$)", txt, flags=re.S | re.M):
        grp = out.setdefault(g.lower(), {})
        keys = list(re.finditer(r"(\w+(?:\(\d+(?::\d+)?\))?)\s*=", body))
        for n, m in enumerate(keys):
            end = keys[n + 1].start() if n + 1 < len(keys) else len(body)
            vals = [v for v in (t.strip() for t in body[m.end():end].replace("\n", ",").split(",")) if v]
            conv = [_nml_value(v) for v in vals]
            grp[m.group(1).lower()] = conv[0] if len(conv) == 1 else conv
    return out


def read_serialized_data(reader, sp, name):
    """serialbox_dat_to_netcdf.py:47-52: scalars unwrapped, the 1e40 fill value -> 0"""
    data = reader.read(name, sp)
    if data.size == 1:
        return data.reshape(-1)[0]
    data = data.astype(np.float64) if data.dtype.kind == "f" else data
    if data.dtype.kind == "f":
        data[data == 1e40] = 0.0
    return data


def dat_to_netcdf(data_path, output_path, do_only_rank=-1, do_only_savepoint=-1):
    """The reference converter (serialbox_dat_to_netcdf.py:69-176) without serialbox /
    xarray: one NetCDF-3 file per savepoint name, each variable (savepoint, rank, dims...),
    tracer halos stripped on the FVDynamics / Driver savepoints.  Returns the file paths."""
    from scipy.io import netcdf_file
    import shutil
    os.makedirs(output_path, exist_ok=True)
    nml_in = os.path.join(data_path, "input.nml")
    nml_out = os.path.join(output_path, "input.nml")
    if os.path.abspath(nml_in) != os.path.abspath(nml_out):
        shutil.copyfile(nml_in, nml_out)
    layout = read_namelist(nml_out)["fv_core_nml"]["layout"]
    total_ranks = 6 * layout[0] * layout[1]
    r0 = SerialboxReader(data_path, "Generator_rank0")
    names = sorted({sp.name for sp in r0.savepoint_list()})
    written = []
    for spn in names:
        fields = list(r0.fields_at_savepoint(r0.get_savepoint(spn)[0]))
        ranks = [do_only_rank] if do_only_rank >= 0 else list(range(total_ranks))
        per_rank = []
        for rk in ranks:
            rd = SerialboxReader(data_path, f"Generator_rank{rk}")
            sps = rd.get_savepoint(spn)
            sel = sps if do_only_savepoint < 0 else [sps[do_only_savepoint]]
            per_rank.append({f: [read_serialized_data(rd, sp, f) for sp in sel] for f in set(fields)})
        nsp = len(per_rank[0][fields[0]]) if fields else 0
        if nsp == 0:
            continue
        path = os.path.join(output_path, f"{spn}.nc")
        with netcdf_file(path, "w") as nc:
            nc.createDimension("savepoint", nsp)
            nc.createDimension("rank", len(ranks))
            for var in sorted(set(fields) - {"rank"}):
                first = np.asarray(per_rank[0][var][0])
                data = np.full([nsp, len(ranks)] + list(first.shape), np.nan)
                for r, rdat in enumerate(per_rank):
                    for s in range(nsp):
                        data[s, r] = rdat[var][s]
                if spn in HALO_SAVEPOINTS and var in HALO_TRACERS:
                    data = data[:, :, 3:-3, 3:-3, ...]
                dims = ["savepoint", "rank"]
                for i, n in enumerate(data.shape[2:]):
                    dn = f"dim_{var}_{i}"
                    nc.createDimension(dn, n)
                    dims.append(dn)
                v = nc.createVariable(var, "d", tuple(dims))
                v[...] = data
        written.append(path)
    return written


# pyFV3's FVDynamics savepoint names -> this package's state fields (D-grid winds, T, delp,
# the six GFDL tracers in the order qv ql qr qi qs qg, the accumulated fluxes)
FV_DYNAMICS_FIELDS = {
    "u": "u", "v": "v", "w": "w", "delz": "delz", "pt": "pt", "delp": "delp", "ps": "ps", "pe": "pe",
    "pk": "pk", "peln": "peln", "pkz": "pkz", "phis": "phis", "q_con": "q_con", "omga": "omga", "ua": "ua",
    "va": "va", "uc": "uc", "vc": "vc", "mfxd": "mfx", "mfyd": "mfy", "cxd": "cx", "cyd": "cy",
    "diss_estd": "diss_est",
}
FV_DYNAMICS_TRACERS = ("qvapor", "qliquid", "qrain", "qice", "qsnow", "qgraupel")


def fv_dynamics_state(reader, sp, dom, tile_of_rank=0):
    """Host arrays (nsub=1 slice of the Domain layout) of one rank's FVDynamics-In savepoint:
    Fortran (isd:ied, jsd:jed[, k]) fields go to [k, j + NG, i + NG] of the padded plane;
    pe / peln keep FV3's (i, k, j) order in the dump and are permuted like the bridge does."""
    from .domain import NG
    out = {}
    for sname, name in FV_DYNAMICS_FIELDS.items():
        if sname not in reader.fields_at_savepoint(sp):
            continue
        a = np.asarray(read_serialized_data(reader, sp, sname), dtype=np.float64)
        if a.ndim == 2:
            a = a[:, :, None]
        if name in ("pe", "peln"):
            a = np.transpose(a, (0, 2, 1))
        ni, nj, nk = a.shape
        plane = np.zeros((nk, dom.nj, dom.pitch))
        i0 = NG - (ni - dom.nx) // 2
        j0 = NG - (nj - dom.ny) // 2
        plane[:, j0:j0 + nj, i0:i0 + ni] = np.transpose(a, (2, 1, 0))
        out[name] = plane
    tr = [t for t in FV_DYNAMICS_TRACERS if t in reader.fields_at_savepoint(sp)]
    if tr:
        qs = []
        for t in tr:
            a = np.asarray(read_serialized_data(reader, sp, t), dtype=np.float64)
            ni, nj, nk = a.shape
            plane = np.zeros((nk, dom.nj, dom.pitch))
            i0, j0 = NG - (ni - dom.nx) // 2, NG - (nj - dom.ny) // 2
            plane[:, j0:j0 + nj, i0:i0 + ni] = np.transpose(a, (2, 1, 0))
            qs.append(plane)
        out["q"] = np.concatenate(qs, axis=0)
    return out


# Fortran sections of the FVDynamics savepoint fields (FV3 declarations):
# (i0, i1, j0, j1) relative to the compute domain 0..n-1, kind "c"/"x"/"y"/"e"(pe-like) and
# level count key
def _sections(n):
    d, e = -3, n - 1 + 3
    return {
        "u": (d, e, d, e + 1), "v": (d, e + 1, d, e), "w": (d, e, d, e), "delz": (d, e, d, e), "pt": (d, e, d, e),
        "delp": (d, e, d, e), "ps": (d, e, d, e), "phis": (d, e, d, e), "q_con": (d, e, d, e), "omga": (d, e, d, e),
        "ua": (d, e, d, e), "va": (d, e, d, e), "uc": (d, e + 1, d, e), "vc": (d, e, d, e + 1),
        "pe": (-1, n, -1, n), "peln": (0, n - 1, 0, n - 1), "pk": (0, n - 1, 0, n - 1), "pkz": (0, n - 1, 0, n - 1),
        "mfx": (0, n, 0, n - 1), "mfy": (0, n - 1, 0, n), "cx": (0, n, d, e), "cy": (d, e, 0, n),
        "diss_est": (d, e, d, e),
    }


def state_to_savepoint(state, s, n, ng=3):
    """Inverse of fv_dynamics_state for sub-domain s of a 1x1 layout: {savepoint name: array}
    in the FV3 Fortran sections (pe / peln with k in the middle)."""
    inv = {v: k for k, v in FV_DYNAMICS_FIELDS.items()}
    out = {}
    for name, (i0, i1, j0, j1) in _sections(n).items():
        if name not in state:
            continue
        a = state[name][s][:, j0 + ng:j1 + ng + 1, i0 + ng:i1 + ng + 1]   # (k, j, i)
        a = np.transpose(a, (2, 1, 0))                                     # (i, j, k)
        if name in ("pe", "peln"):
            a = np.transpose(a, (0, 2, 1))                                 # (i, k, j)
        if name in ("ps", "phis"):
            a = a[:, :, 0]
        out[inv[name]] = np.asfortranarray(a)
    if "q" in state:
        npz = state["delp"].shape[1]
        d, e = -3, n - 1 + 3
        for iq, t in enumerate(FV_DYNAMICS_TRACERS):
            if (iq + 1) * npz > state["q"].shape[1]:
                break
            a = state["q"][s][iq * npz:(iq + 1) * npz, d + ng:e + ng + 1, d + ng:e + ng + 1]
            out[t] = np.asfortranarray(np.transpose(a, (2, 1, 0)))
    return out
