"""Host-side helpers of bench.py: kernel families for the roofline line (no GPU)."""
import bench


def test_family_strips_template_arguments():
    assert bench.family("(tp_march<6, true, false>)") == "tp_march"
    assert bench.family("(riem_blk_k<18, true>)") == "riem_blk_k"
    assert bench.family("remap_job_k") == "remap_job_k"


def test_families_sum_instantiations():
    ks = {"(tp_march<6, true, false>)": (4.0, 18, 10.0), "(tp_march<6, true, true>)": (5.0, 13, 20.0),
          "remap_job_k": (8.0, 1, 1.0)}
    fam = bench.families(ks)
    assert fam["tp_march"] == (9.0, 31, 30.0)
    assert max(fam.items(), key=lambda kv: kv[1][0])[0] == "tp_march"


def test_layouts_divide_subdomains():
    for n in (1, 2, 4, 8):
        lx, ly = bench.layout_for(n)
        assert (6 * lx * ly) % n == 0
