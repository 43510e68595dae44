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


def test_partition_budget_below_model_count():
    """budget 1 with two active jobs used to raise ValueError."""
    from idunno.runtime.scheduler import partition

    ws = [f"rank{i}" for i in range(8)]
    p = partition({"alexnet": 1.0, "resnet18": 2.0}, ["alexnet", "resnet18"], ws, budget=1)
    assert p == {"alexnet": ["rank0"], "resnet18": ["rank0"]}
    p = partition({"a": 1, "b": 1, "c": 1}, ["a", "b", "c"], ws[:2], budget=8)
    assert sorted(len(v) for v in p.values()) == [1, 1, 1]
    s = FairTimeScheduler(budget=1, seed=0)
    s.active_jobs = {"alexnet"}
    plan = s.assign("resnet18", 0, 399, ws)
    assert [(w, st, e) for w, st, e in plan] == [("rank0", 0, 399)]


def test_subsets_fixed_under_ema_jitter():
    """Between query boundaries the split never moves, whatever the EMA does;
    it is recomputed when a job starts / ends or a worker dies, and re-planned
    at a query boundary."""
    import random

    s = FairTimeScheduler(budget=8, seed=0)
    ws = [f"rank{i}" for i in range(8)]
    both = {"alexnet", "resnet18"}
    first = s.subsets(both, ws)                       # no measurements: equal split
    assert [len(first["alexnet"]), len(first["resnet18"])] == [4, 4]
    s.observe("alexnet", 3.0)                         # first measurements: the next boundary re-plans
    s.observe("resnet18", 5.0)
    assert s.subsets(both, ws) == first
    p0 = s.subsets(both, ws, boundary=True)
    assert (len(p0["alexnet"]), len(p0["resnet18"])) == (3, 5)      # slower model gets more
    assert set(p0["alexnet"]).isdisjoint(p0["resnet18"])
    rng = random.Random(7)
    for _ in range(200):                              # EMA jitter: +-60 %
        s.observe("alexnet", 3.0 * rng.uniform(0.4, 1.6))
        s.observe("resnet18", 5.0 * rng.uniform(0.4, 1.6))
        assert s.subsets(both, ws) == p0
        for m in both:                                # and every query lands on its subset
            s.active_jobs = both
            plan = s.assign(m, 0, 399, ws)
            assert [w for w, _, _ in plan] == p0[m]
    # a worker failure re-partitions over the survivors
    p1 = s.subsets(both, ws[:7])
    assert sum(len(v) for v in p1.values()) == 7 and set(p1["alexnet"]).isdisjoint(p1["resnet18"])
    # a job alone takes every GPU
    s.active_jobs = {"resnet18"}
    assert len(s.assign("resnet18", 0, 399, ws)) == 8


def test_adopted_averages_count_as_measurements():
    s = FairTimeScheduler(budget=8)
    s.adopt({"alexnet": 2.0, "resnet18": 6.0})
    p = s.subsets({"alexnet", "resnet18"}, [f"r{i}" for i in range(8)])
    assert (len(p["alexnet"]), len(p["resnet18"])) == (2, 6)


def test_split_follows_ema_only_at_query_boundaries():
    """with fake EMA drift, the fair-time split
    moves (5/5 -> 4/6 like report Fig 2) only at a query boundary (a job's next
    query being planned; ``drained`` is the old keyword), and the two jobs'
    subsets never overlap -- before, at, or after the move."""
    s = FairTimeScheduler(budget=10, seed=0)
    ws = [f"rank{i}" for i in range(10)]
    both = {"alexnet", "resnet18"}
    s.adopt({"alexnet": 5.0, "resnet18": 5.0})
    sizes = lambda p: (len(p["alexnet"]), len(p["resnet18"]))      # noqa: E731
    p0 = s.subsets(both, ws)
    assert sizes(p0) == (5, 5)
    # EMA drifts: resnet18 slows to 6/4 of alexnet's time -> exact share 4 / 6
    for _ in range(30):
        s.observe("alexnet", 4.0)
        s.observe("resnet18", 6.0)
        assert s.subsets(both, ws, drained=False) == p0             # queries in flight: frozen
    p1 = s.subsets(both, ws, drained=True)                           # drained boundary: moves
    assert sizes(p1) == (4, 6) and s.repartitions == 1
    assert set(p1["alexnet"]).isdisjoint(p1["resnet18"])
    assert sorted(p1["alexnet"] + p1["resnet18"]) == sorted(ws)
    # kept afterwards while queries run, and assign() lands on the new subsets
    s.active_jobs = both
    for m in both:
        assert [w for w, _, _ in s.assign(m, 0, 399, ws)] == p1[m]
    # jitter inside the hysteresis band never re-splits, drained or not
    import random
    rng = random.Random(3)
    for _ in range(100):
        s.observe("alexnet", 4.0 * rng.uniform(0.97, 1.03))
        s.observe("resnet18", 6.0 * rng.uniform(0.97, 1.03))
        assert s.subsets(both, ws, drained=rng.random() < 0.5) == p1
    assert s.repartitions == 1
    # drift back: follows again only once drained
    for _ in range(30):
        s.observe("alexnet", 5.0)
        s.observe("resnet18", 5.0)
    assert s.subsets(both, ws) == p1
    p2 = s.assign("alexnet", 0, 399, ws, drained=True)
    assert len(p2) == 5 and s.repartitions == 2



def test_chunk_time_fit_is_independent_of_the_split():
    """chunks of one model cut 3 or 5 ways have different
    per-image times (fixed cost per chunk); the fitted full-query time must be
    the same whichever way the queries were cut."""
    from idunno.runtime.scheduler import ChunkTimeFit

    a, b, B = 0.002, 0.0001, 400           # 2 ms per chunk + 0.1 ms per image
    f = ChunkTimeFit()
    for n in (133, 134, 133):
        f.add(n, a + b * n)
    per_image_only = f.full(B)             # one chunk size: per-image fallback, includes a's share
    assert abs(per_image_only / ((a / 133 + b) * B) - 1) < 1e-3
    for n in (80, 80, 80, 133, 80):
        f.add(n, a + b * n)
    assert abs(f.full(B) - (a + b * B)) < 1e-6
    # a per-image time that changed together with the chunk size is not a fixed cost
    g = ChunkTimeFit()
    for _ in range(5):
        g.add(167, 167 * 100e-6)
    for _ in range(2):
        g.add(100, 100 * 160e-6)
    assert g.full(500) > 500 * 100e-6      # never below the old regime's per-image time


def test_boundary_hand_over_waits_for_the_donors_chunks():
    """A worker moving between jobs joins the receiver only once the donor's
    chunks on it are done; meanwhile it is in neither subset."""
    s = FairTimeScheduler(budget=8, seed=0)
    ws = [f"r{i}" for i in range(8)]
    both = {"alexnet", "resnet18"}
    s.adopt({"alexnet": 1.0, "resnet18": 1.0})
    p0 = s.subsets(both, ws)
    assert (len(p0["alexnet"]), len(p0["resnet18"])) == (4, 4)
    s.adopt({"alexnet": 1.0, "resnet18": 3.0})         # exact share 2 / 6
    busy = {w: {"alexnet"} for w in p0["alexnet"]}
    p1 = s.subsets(both, ws, boundary=True, busy=busy)
    assert len(p1["alexnet"]) == 2 and len(p1["resnet18"]) == 4     # two workers in hand-over
    assert s.moves_deferred == 2
    left = set(ws) - set(p1["alexnet"]) - set(p1["resnet18"])
    assert left <= set(p0["alexnet"]) and len(left) == 2
    # still busy with alexnet: nothing moves; once free they join resnet18
    assert s.subsets(both, ws, boundary=True, busy=busy) == p1
    p2 = s.subsets(both, ws, boundary=True, busy={w: {"alexnet"} for w in p1["alexnet"]})
    assert len(p2["alexnet"]) == 2 and len(p2["resnet18"]) == 6 and left <= set(p2["resnet18"])
    assert set(p2["alexnet"]).isdisjoint(p2["resnet18"])
    # busy=None (round path): hand over at once
    s.adopt({"alexnet": 3.0, "resnet18": 1.0})
    p3 = s.subsets(both, ws, boundary=True)
    assert (len(p3["alexnet"]), len(p3["resnet18"])) == (6, 2)
