"""The conv12 LDS bank model (tools/c12_lds_banks.py) against the PMC pass it explains: the
conflict cycles it predicts per 8 x 8 tile, times config 2's 12,288 tiles, equal the measured
SQ_LDS_BANK_CONFLICT of conv12 (profiles/r5z_traffic.json / r5f_traffic.json)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import c12_lds_banks as M  # noqa: E402
import pytest  # noqa: E402

PMC = os.path.join(ROOT, "profiles", "r5f_traffic.json")


@pytest.mark.skipif(not os.path.exists(PMC), reason="profiles/ not in this tree (GPU-box upload)")
def test_conv12_conflicts_match_pmc():
    rows = [M.stream_reads(), M.patch_reads(), M.halo_writes()]
    assert rows[0] == (3200, 3200)  # conv2's B-fragment reads: conflict-free
    extra = sum(c - i for c, i in rows)
    assert extra == 970
    with open(PMC) as f:
        pmc = json.load(f)["layers"]["conv2"]
    assert extra * 12288 == int(pmc["SQ_LDS_BANK_CONFLICT"])
