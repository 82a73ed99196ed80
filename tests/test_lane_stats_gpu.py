"""The blend backward's lane-statistics instantiation
(gs_blend_backward_lane_stats, a diagnostic): it replays exactly what the
product kernel replays -- bit-identical partials and flags -- and its
counters are consistent: the histogram's and the per-workgroup sums agree,
and the lanes it finds contributing are the forward's contributing pairs
(the same decisions, replayed)."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


@pytest.mark.parametrize("config", ["C1", "C2"])
def test_lane_stats_consistent(pkg, cuda, config):
    import lane_stats
    r = lane_stats.run(config)
    assert r["same_partials"]
    h, per = r["hist"], r["per"]
    reps = int(h[0].sum())
    assert reps == int(h[1].sum()) == int(per[:, 0].sum()) > 0
    assert int((h[0] * np.arange(65)).sum()) == int(per[:, 2].sum())
    con = int((h[1] * np.arange(65)).sum())
    assert con == int(per[:, 3].sum()) == r["contributing_fwd"]
    assert int(per[:, 1].sum()) == int(h[0][32:].sum())
    md = lane_stats.model(r)
    assert 0 <= md["saved_replays_best_case"] <= md["tail_replays"]
