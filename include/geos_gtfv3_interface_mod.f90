! geos_gtfv3_interface_mod — the Fortran binding of libgeos_gtfv3_interface.so, i.e. the
! module the reference generates from example_def_dycore.yaml through
! interface.f90.jinja2:24-82 (bind(c) names geos_gtfv3_<fn>_c, interface.f90.jinja2:39;
! type map argument.py:54-86: int -> integer(c_int),value; float -> real(c_float),value;
! array_float -> real(c_float) dimension(*); MPI -> integer(c_int),value).  The fp64 twin
! geos_gtfv3_run_f64_f binds geos_gtfv3_run_f64_c with real(c_double) buffers.
module geos_gtfv3_interface_mod
  use iso_c_binding
  implicit none
  interface
    subroutine geos_gtfv3_init_f(comm, npx, npy, npz, ntiles, is, ie, js, je, &
                                 isd, ied, jsd, jed, bdt, nq_tot) &
        bind(c, name='geos_gtfv3_init_c')
      import c_int, c_float
      integer(c_int), value :: comm, npx, npy, npz, ntiles, is, ie, js, je, isd, ied, jsd, jed, nq_tot
      real(c_float), value :: bdt
    end subroutine
    subroutine geos_gtfv3_run_f(comm, npx, npy, npz, ntiles, is, ie, js, je, isd, ied, jsd, jed, &
                                bdt, nq_tot, ng, ptop, ks, layout_1, layout_2, adiabatic, &
                                ak, bk, u, v, w, delz, pt, delp, q, ps, pe, pk, peln, pkz, phis, &
                                q_con, omga, ua, va, uc, vc, mfx, mfy, cx, cy, diss_est) &
        bind(c, name='geos_gtfv3_run_c')
      import c_int, c_float
      integer(c_int), value :: comm, npx, npy, npz, ntiles, is, ie, js, je, isd, ied, jsd, jed
      integer(c_int), value :: nq_tot, ng, ks, layout_1, layout_2, adiabatic
      real(c_float), value :: bdt, ptop
      real(c_float), dimension(*) :: ak, bk, u, v, w, delz, pt, delp, q, ps, pe, pk, peln, pkz, phis, &
                                     q_con, omga, ua, va, uc, vc, mfx, mfy, cx, cy, diss_est
    end subroutine
    subroutine geos_gtfv3_run_f64_f(comm, npx, npy, npz, ntiles, is, ie, js, je, isd, ied, jsd, jed, &
                                    bdt, nq_tot, ng, ptop, ks, layout_1, layout_2, adiabatic, &
                                    ak, bk, u, v, w, delz, pt, delp, q, ps, pe, pk, peln, pkz, phis, &
                                    q_con, omga, ua, va, uc, vc, mfx, mfy, cx, cy, diss_est) &
        bind(c, name='geos_gtfv3_run_f64_c')
      import c_int, c_float, c_double
      integer(c_int), value :: comm, npx, npy, npz, ntiles, is, ie, js, je, isd, ied, jsd, jed
      integer(c_int), value :: nq_tot, ng, ks, layout_1, layout_2, adiabatic
      real(c_float), value :: bdt, ptop
      real(c_double), dimension(*) :: ak, bk, u, v, w, delz, pt, delp, q, ps, pe, pk, peln, pkz, phis, &
                                      q_con, omga, ua, va, uc, vc, mfx, mfy, cx, cy, diss_est
    end subroutine
    subroutine geos_gtfv3_finalize_f() bind(c, name='geos_gtfv3_finalize_c')
    end subroutine
  end interface
end module
