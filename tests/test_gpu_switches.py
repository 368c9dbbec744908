"""The tuning and diagnostic switches of INTEGRATION.md §4 change how the step is scheduled,
not what it computes: the same Jablonowski-Williamson state stepped twice in child processes,
once with the defaults and once with the switch, must agree on every prognostic field bit for
bit (tools/ab_bitwise.py, the check each round-6 fold was measured with)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SWITCHES = ["GTFV3_XCD=0", "GTFV3_LVB=0", "GTFV3_TP_SEG=20", "GTFV3_TRACER_NF=1", "GTFV3_THERMO_FUSED=0",
            "GTFV3_TRACER_FUSED=0", "GTFV3_KLOOP=0", "GTFV3_KLOOP=3", "GTFV3_STREAMS=0", "GTFV3_EDGE_SIDE=0",
            "GTFV3_EARLY_WINDS=0", "GTFV3_A2B_EDGE=0", "GTFV3_SYNC_LAUNCH=1"]


@pytest.mark.gpu
@pytest.mark.parametrize("switch", SWITCHES)
def test_switch_is_bit_identical(require_gpu, switch):
    # C24 L16 (25 x 25 corners per tile), two steps, 2x2 sub-domains per tile
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "ab_bitwise.py"), "-", switch, "25", "16", "2",
                        "2", "2"], cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, f"{switch}: the step differs from the defaults\n{r.stdout[-2000:]}{r.stderr[-2000:]}"
    assert "identical" in r.stdout
