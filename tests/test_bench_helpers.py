"""bench.py helpers that shape the timed region and its report (CPU only)."""
import types

import bench


def test_pick_steps_per_graph_divides_the_timed_steps():
    for cap in (1, 50, 200):
        for steps in (1, 5, 20, 199, 200, 201, 300, 500, 997):
            s = bench.pick_steps_per_graph(steps, cap)
            assert 1 <= s <= max(1, min(steps, cap))
            assert steps % s == 0            # no single-step remainder replays
            if steps <= cap:
                assert s == steps             # one replay for the whole timed region
    assert bench.pick_steps_per_graph(300, 200) == 150
    assert bench.pick_steps_per_graph(997, 200) == 1   # a prime above the cap: per-step replays
    assert bench.pick_steps_per_graph(0, 200) == 1


def test_mlp2_launches_names_the_persistent_kernel_only_when_it_runs():
    pst = types.SimpleNamespace(pst_ok=True)
    one = types.SimpleNamespace(pst_ok=False)
    assert bench._mlp2_launches(pst, "", 150).startswith("1/150 (persistent run-ahead")
    assert bench._mlp2_launches(pst, "", 1) == "1 (run-ahead mlp2_bwd)"   # 1-step graphs: one-step kernel
    assert bench._mlp2_launches(one, ", x", 150) == "1 (run-ahead mlp2_bwd, x)"
    assert bench._mlp2_launches(object(), "", 20) == "1 (run-ahead mlp2_bwd)"
