! Fortran caller of libgeos_gtfv3_interface.so through geos_gtfv3_interface_mod
! (include/geos_gtfv3_interface_mod.f90), the way FVdycoreCubed_GridComp calls the
! reference bridge: FV3-bounded real(c_float) arrays (SURVEY.md §8b) handed to
! geos_gtfv3_init_f / geos_gtfv3_run_f / geos_gtfv3_finalize_f, updated in place.
! All six tiles are held by this one process (GTFV3_BRIDGE_TILES_PER_RANK=6: trailing
! tile axis).  I/O: argv(1) = input stream file, argv(2) = output stream file:
!   int32 npx, npz, nq, ks, adiabatic | float32 ptop, bdt | the 26 run arrays in
!   argument order (each the FV3 section, column-major, tiles last)
! and the output file holds the 26 arrays after the call, same order.
program fortran_driver
  use iso_c_binding
  use geos_gtfv3_interface_mod
  implicit none
  integer, parameter :: nt = 6, ng = 3
  integer(c_int) :: npx, npz, nq, ks, adiabatic, n, is, ie, js, je, isd, ied, jsd, jed
  real(c_float) :: ptop, bdt
  real(c_float), allocatable :: ak(:), bk(:)
  real(c_float), allocatable, dimension(:,:,:,:) :: u, v, w, delz, pt, delp, q, ps, pe, pk, peln, pkz, &
      phis, q_con, omga, ua, va, uc, vc, mfx, mfy, cx, cy, diss_est
  character(len=512) :: fin, fout
  integer :: uin, uout

  call get_command_argument(1, fin)
  call get_command_argument(2, fout)
  open(newunit=uin, file=trim(fin), access='stream', form='unformatted', status='old')
  read(uin) npx, npz, nq, ks, adiabatic, ptop, bdt
  n = npx - 1
  is = 1; ie = n; js = 1; je = n
  isd = is - ng; ied = ie + ng; jsd = js - ng; jed = je + ng
  allocate(ak(npz + 1), bk(npz + 1))
  allocate(u(isd:ied, jsd:jed+1, npz, nt), v(isd:ied+1, jsd:jed, npz, nt))
  allocate(w(isd:ied, jsd:jed, npz, nt), delz(isd:ied, jsd:jed, npz, nt), pt(isd:ied, jsd:jed, npz, nt))
  allocate(delp(isd:ied, jsd:jed, npz, nt), q(isd:ied, jsd:jed, npz*nq, nt), ps(isd:ied, jsd:jed, 1, nt))
  allocate(pe(is-1:ie+1, npz+1, js-1:je+1, nt), pk(is:ie, js:je, npz+1, nt), peln(is:ie, npz+1, js:je, nt))
  allocate(pkz(is:ie, js:je, npz, nt), phis(isd:ied, jsd:jed, 1, nt), q_con(isd:ied, jsd:jed, npz, nt))
  allocate(omga(isd:ied, jsd:jed, npz, nt), ua(isd:ied, jsd:jed, npz, nt), va(isd:ied, jsd:jed, npz, nt))
  allocate(uc(isd:ied+1, jsd:jed, npz, nt), vc(isd:ied, jsd:jed+1, npz, nt))
  allocate(mfx(is:ie+1, js:je, npz, nt), mfy(is:ie, js:je+1, npz, nt))
  allocate(cx(is:ie+1, jsd:jed, npz, nt), cy(isd:ied, js:je+1, npz, nt), diss_est(isd:ied, jsd:jed, npz, nt))
  read(uin) ak, bk, u, v, w, delz, pt, delp, q, ps, pe, pk, peln, pkz, phis, q_con, omga, ua, va, uc, vc, &
            mfx, mfy, cx, cy, diss_est
  close(uin)

  call geos_gtfv3_init_f(0, npx, npx, npz, nt, is, ie, js, je, isd, ied, jsd, jed, bdt, nq)
  call geos_gtfv3_run_f(0, npx, npx, npz, nt, is, ie, js, je, isd, ied, jsd, jed, bdt, nq, ng, ptop, ks, &
                        1, 1, adiabatic, ak, bk, u, v, w, delz, pt, delp, q, ps, pe, pk, peln, pkz, phis, &
                        q_con, omga, ua, va, uc, vc, mfx, mfy, cx, cy, diss_est)
  call geos_gtfv3_finalize_f()

  open(newunit=uout, file=trim(fout), access='stream', form='unformatted', status='replace')
  write(uout) ak, bk, u, v, w, delz, pt, delp, q, ps, pe, pk, peln, pkz, phis, q_con, omga, ua, va, uc, vc, &
              mfx, mfy, cx, cy, diss_est
  close(uout)
  print '(a)', 'fortran_driver: geos_gtfv3 init/run/finalize done'
end program
