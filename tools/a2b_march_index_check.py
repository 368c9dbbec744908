# Host replica of a2b_march_k (csrc/nh.hip) address math: lists any access outside its plane.
# Found the pre-fix read of the row before the plane (prefetch row j < j0 with J == 1).
# host replica of a2b_march_k address math: report any access outside [0, plane) of its plane
import itertools
NG=3
def r8(x): return (x+7)//8*8
def run(N, nx, ny, subs, nk, seg=45, AM_OUT=61, AM_B=2):
    pitch=r8(nx+2*NG+1); nj=ny+2*NG+1; plane=pitch*nj
    nstrip=-(-(nx+1)//AM_OUT); nseg=-(-(ny+1)//seg)
    bad=[]
    for s,(io,jo) in enumerate(subs):
      for strip in range(nstrip):
        for sg in range(nseg):
          last0=max(nx+1-AM_OUT,0)
          a0=min(strip*AM_OUT,last0)
          a1=min((strip+1)*AM_OUT,last0) if strip+1<nstrip else nx+1
          j0=sg*seg; j1=min(j0+seg,ny+1)
          rlast=j1+1
          for lane in range(64):
            c=a0-2+lane; I=c+io
            cc=min(c,nx+NG); xo=cc+NG
            row_of=lambda r:(min(r,rlast)+NG)*pitch+xo
            dxs=-1 if I==1 else (1 if I==N-1 else 0)
            qy_col = I>=max(0,io-2) and I<=min(N-1,io+nx+1)
            out_lane = lane>=2 and lane<2+AM_OUT and c<a1
            icols = I>=max(1,io) and I<=min(N-1,io+nx) and c<=nx
            def chk(what,off,r):
                if off<0 or off>=plane: bad.append((what,s,strip,sg,lane,r,off,plane))
            def fetch(r):
                o=row_of(r); chk('q',o,r)
                j=r-2; oj=(max(min(j,rlast),-NG)+NG)*pitch+xo
                if dxs: chk('qo_x',oj+dxs,r)
                J=j+jo
                if not (j>=j0 and j<j1): pass
                elif J==1: chk('qo_y-',oj-pitch,r)
                elif J==N-1: chk('qo_y+',oj+pitch,r)
            r0=j0-NG
            for u in range(AM_B): fetch(r0+u)
            while r0<=rlast:
                for u in range(AM_B): fetch(r0+AM_B+u)
                for u in range(AM_B):
                    r=r0+u
                    if r>rlast: break
                    o=(r+NG)*pitch+xo
                    j=r-2
                    if j<j0: continue
                    J=j+jo
                    oj=o-2*pitch
                    if qy_col:
                        dl=[]
                        if J==0: dl=[1,0]
                        elif J==N: dl=[-2,-1]
                        elif J==1 or J==N-1: dl=[0,-1]
                        for dj in dl: chk('dya',oj+dj*pitch,r)
                    jrows = J>=max(1,jo) and J<=min(N-1,jo+ny) and j<=ny
                    if out_lane and icols and jrows and j<j1: chk('store',oj,r)
                r0+=AM_B
    return bad
for N,lx,ly in [(12,1,2),(12,1,1),(12,2,2),(24,2,2),(180,1,1),(180,2,2),(48,1,4),(12,1,4),(24,1,4)]:
    nx,ny=N//lx,N//ly
    subs=[(i*nx,j*ny) for j in range(ly) for i in range(lx)]
    b=run(N,nx,ny,subs,1)
    print(N,lx,ly,len(b),b[:3])
