"""Fair-time scheduler parity with the reference split/share rules."""
from idunno.runtime.scheduler import FairTimeScheduler, fair_share, split_range


def test_split_bankers_rounding_parity():
    # reference example: 400 images over 6 workers -> 67,67,66,67,66,67
    chunks = split_range(0, 399, 6)
    assert [e - s + 1 for s, e in chunks] == [67, 67, 66, 67, 66, 67]
    assert chunks[0][0] == 0 and chunks[-1][1] == 399
    for (s0, e0), (s1, e1) in zip(chunks, chunks[1:]):
        assert s1 == e0 + 1


def test_split_even_and_edge_cases():
    assert split_range(0, 399, 5) == [(0, 79), (80, 159), (160, 239), (240, 319), (320, 399)]
    assert split_range(10, 12, 8) == [(10, 10), (11, 11), (12, 12)]
    assert split_range(5, 4, 3) == []
    assert split_range(0, 9, 0) == []


def test_fair_share_slower_model_gets_more():
    # reference formula: each model gets the share of its own time
    t = {"alexnet": 6.0, "resnet18": 9.0}
    assert fair_share(t, "alexnet", 10, 10) == 4
    assert fair_share(t, "resnet18", 10, 10) == 6
    t = {"alexnet": 100.0, "resnet18": 100.0}
    assert fair_share(t, "alexnet", 10, 10) == 5 and fair_share(t, "resnet18", 10, 10) == 5
    assert fair_share({"alexnet": 1, "resnet18": 100}, "resnet18", 10, 3) == 3  # clamp to alive


def test_scheduler_assign_and_ema():
    s = FairTimeScheduler(budget=8, seed=1)
    alive = [f"rank{i}" for i in range(8)]
    s.active_jobs = {"resnet18"}
    a = s.assign("resnet18", 0, 399, alive)
    assert len(a) == 8 and sum(e - st + 1 for _, st, e in a) == 400
    assert len({w for w, _, _ in a}) == 8
    s.active_jobs = {"resnet18", "alexnet"}
    s.observe("alexnet", 6.0)
    s.observe("resnet18", 9.0)
    assert s.n_workers("resnet18", alive) > s.n_workers("alexnet", alive)
    s.observe("resnet18", 3.0)
    assert abs(s.avg_time["resnet18"] - (0.7 * 9 + 0.3 * 3)) < 1e-9
