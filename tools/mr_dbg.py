"""Debug helper: 4-rank loopback step, prints rank exceptions (daemon threads)."""
import importlib, sys, threading, time
sys.path.insert(0, '.')
import torch
print("torch gpu", torch.cuda.is_available(), flush=True)
import gtfv3_pkg
pkg = gtfv3_pkg.load()
state = importlib.import_module(pkg.__name__ + ".state")
nr, layout, npz = int(sys.argv[1]), (int(sys.argv[2]), int(sys.argv[3])), 10
ak, bk, ks = state.hybrid_levels(npz)
if len(sys.argv) > 4:
    ref = pkg.Domain(npx=13, npz=npz, nq=2, layout_x=layout[0], layout_y=layout[1])
    st = state.jablonowski_williamson(ref, ak, bk)
    ref.set_vertical(ak, bk, ks)
    for k, v in st.items():
        ref.upload(k, v)
    t0 = time.time(); ref.step(1); ref.sync(); print("ref step", round(time.time() - t0, 2), "s", flush=True)
doms = [pkg.Domain(r, nr, None, npx=13, npz=npz, nq=2, layout_x=layout[0], layout_y=layout[1], loopback=7)
        for r in range(nr)]
for d in doms:
    st = state.jablonowski_williamson(d, ak, bk)
    d.set_vertical(ak, bk, ks)
    for k, v in st.items():
        d.upload(k, v)
errs = {}
def work(r, d):
    try:
        d.step(1)
        errs[r] = "ok"
    except Exception as e:
        errs[r] = repr(e)
ts = [threading.Thread(target=work, args=(r, d), daemon=True) for r, d in enumerate(doms)]
for t in ts: t.start()
t0 = time.time()
while time.time() - t0 < 60 and any(t.is_alive() for t in ts):
    time.sleep(0.5)
print("status after", round(time.time() - t0, 1), "s:", errs, flush=True)
import os; os._exit(0)
