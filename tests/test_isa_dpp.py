"""ISA check of the block-scan kernels (no GPU needed): no DPP move may sit inside an
exec-masked region nested below the kernel's whole-wave early exit.

A DPP read of a lane that EXEC disables returns 0 (bound_ctrl), so a lane shift written in
an arm of a lane-divergent `?:` (blockscan.hpp: `b == 0 ? x : blk_prev(v)`) silently reads
zeros from the lanes the condition turns off -- the first build of riem_scan_k did this and
its pp / w solves were wrong by O(1).  This compiles riem.hip and the probe for gfx950 and
walks each scan kernel's ISA, counting `s_and_saveexec` / `s_or_b64 exec` nesting."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

HIPCC = "/opt/rocm/bin/hipcc"
CSRC = os.path.join(ROOT, "geosongpu-ci_amd", "csrc")


def _blocks(body):
    """basic blocks of a kernel's ISA: [(label, [instructions], [successor labels])]"""
    blocks, cur, name, n = [], [], "entry", 0
    for line in body.split("\n"):
        t = line.split(";")[0].strip()
        if not t:
            continue
        if t.endswith(":"):
            if cur or name == "entry":
                blocks.append([name, cur])
            name, cur = t[:-1], []
            continue
        cur.append(t)
        if t.startswith(("s_branch", "s_cbranch", "s_endpgm")):
            blocks.append([name, cur])
            n += 1
            name, cur = f"_ft{n}", []
    blocks.append([name, cur])
    out = []
    for i, (nm, ins) in enumerate(blocks):
        succ = []
        last = ins[-1] if ins else ""
        if last.startswith(("s_branch", "s_cbranch")):
            succ.append(last.split()[1])
        if not last.startswith(("s_branch", "s_endpgm")) and i + 1 < len(blocks):
            succ.append(blocks[i + 1][0])
        out.append((nm, ins, succ))
    return out


def _step(depth, t):
    if t.startswith("s_and_saveexec_b64"):
        return depth + 1
    if t.startswith("s_or_b64 exec, exec,"):
        return max(depth - 1, 0)
    return depth


def masked_dpp(asm, kernel_re, allowed=1):
    """DPP moves that can issue inside a lane-divergent region nested below the kernel's
    whole-wave early exit (`allowed` regions: 1 for riem_scan_k's `if (c0 >= ncol) return`,
    0 for the probe), by a dataflow pass over the kernel's basic blocks: each
    `s_and_saveexec_b64` opens a region, each `s_or_b64 exec, exec, ...` closes one (an else
    part, `s_andn2_saveexec_b64`, stays inside); at a join the deeper nesting wins (a loop
    re-saves exec at its latch and restores it at its header, so its body stays at the
    loop's level)."""
    out = {}
    for m in re.finditer(r"^(" + kernel_re + r"):", asm, re.M):
        body = asm[m.end():asm.index(".Lfunc_end", m.end())]
        blocks = _blocks(body)
        index = {nm: i for i, (nm, _, _) in enumerate(blocks)}
        depth_in = {0: 0}
        work = [0]
        while work:
            i = work.pop()
            dpt = depth_in[i]
            for t in blocks[i][1]:
                dpt = _step(dpt, t)
            for sname in blocks[i][2]:
                j = index.get(sname)
                if j is not None and (j not in depth_in or dpt > depth_in[j]):
                    depth_in[j] = dpt
                    work.append(j)
        bad = 0
        for i, (nm, ins, _) in enumerate(blocks):
            dpt = depth_in.get(i, 0)
            for t in ins:
                dpt = _step(dpt, t)
                if "_dpp" in t and dpt > allowed:
                    bad += 1
        out[m.group(1)] = bad
    return out


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src,kre,allowed", [(os.path.join(CSRC, "riem.hip"), r"_Z\S*riem_scan_k\S*", 1),
                                             (os.path.join(CSRC, "remap.hip"), r"_Z\S*remap_blk_k\S*", 1),
                                             (os.path.join(CSRC, "moist.hip"), r"_Z\S*mpdrv_blk_k\S*", 1),
                                             (os.path.join(ROOT, "tests", "native", "blockscan_probe.hip"),
                                              r"_Z5k_tri\S*", 0)])
def test_no_dpp_under_divergent_exec(tmp_path, src, kre, allowed):
    out = tmp_path / "k.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "-x", "hip",
                    "--cuda-device-only", "-S", src, "-o", str(out)], check=True, capture_output=True)
    found = masked_dpp(out.read_text(), kre, allowed)
    assert found, "no scan kernel found in the ISA"
    bad = {k: v for k, v in found.items() if v}
    assert not bad, f"DPP moves inside lane-divergent exec regions: {bad}"
