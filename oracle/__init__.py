"""CPU oracle for the FV3 dycore hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / reported CPU baseline.  The product
(libgeos_gtfv3_interface.so) never calls into it and has no CPU fallback.

Parity status: **parity unpinned.**  The reference repository (GEOS-ESM/
geosongpu-ci) holds no implementation of the dycore numerics: c_sw, d_sw,
fv_tp_2d, the Riemann solvers and the vertical remap live in external repos
(GEOS fvdycore / pyFV3 on NDSL-GT4Py-DaCe, pinned at experiments.yaml:8-20 and
NDSL 2024.04.00, sw_stack/discover/sles15/src/2024.04.00/basics.sh:19) that are
absent here and not fetchable.  This oracle is an fp64 numpy restatement of the
published algorithms (Lin & Rood 1996; Lin 2004; Putman & Lin 2007; Harris &
Lin 2013; FV3 module structure: tp_core, sw_core, nh_core, fv_mapz,
fv_tracer2d, a2b_edge) with the FV3 operation order, pinned only by the
reference's own semantics it touches:
  * Fortran <-> Python layout rule reshape(reversed(dim)).transpose()
    (templates/data_conversion.py:141) and flatten(order="F") (:184),
  * the K-column KATs of dsl_patterns/*.py,
  * the CI tolerances (physics_standalone.py:132-144, hook.py.jinja2:58,69),
plus analytic known-answer tests (constant preservation, mass conservation,
remap identity, hydrostatic rest state) in tests/.

Array convention = the HBM layout: a[k, j+NG, i+NG] per sub-domain.
"""
NG = 3
