"""bench.py's PMC lookups (profiles/pmc_traffic.json): a leg at a lane count
the profile did not run reads nothing, never the 8,192-lane figure."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_pmc_lookup_is_per_lane_count():
    j = json.load(open(os.path.join(REPO, "profiles", "pmc_traffic.json")))
    v, src = bench._pmc("1ply_fused", "fused", "hbm_bytes_per_step")
    assert v == j["1ply_fused"]["fused"]["hbm_bytes_per_step"] and "[1ply_fused]" in src
    assert bench._pmc("1ply_fused", "fused", "hbm_bytes_per_step", lanes=1234) == (None, None)
    for leg, grp in (("1ply_fused", "fused"), ("2ply_k4", "mlp"), ("2ply_kall", "movegen")):
        key = f"l4096_{leg}"
        v, src = bench._pmc(leg, grp, "hbm_bytes_per_launch", lanes=4096)
        if key in j:
            assert j[key]["lanes"] == 4096
            assert v == j[key][grp]["hbm_bytes_per_launch"] and f"[{key}]" in src
        else:
            assert (v, src) == (None, None)
