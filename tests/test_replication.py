"""Standby replication by sequence-numbered deltas (VERDICT r1
item 6): the mirror built from deltas equals the one built from snapshots,
gaps / truncation force a snapshot, and coordinator cost per query stays flat
over 100k queries (finished queries leave the open-query index)."""
import random
import time

import numpy as np

from idunno.runtime.jobstate import JobState


def _drive(js: JobState, rng: random.Random, nq: int, workers=("a", "b", "c", "d")):
    for _ in range(nq):
        m = rng.choice(["resnet18", "alexnet"])
        q = js.new_query_number(m)
        s = rng.randrange(0, 10000)
        n = rng.randint(1, 4)
        chunks = [(workers[i % len(workers)], s + 100 * i, s + 100 * i + 99) for i in range(n)]
        js.assign(m, q, chunks)
        for w, a, b in chunks:
            r = rng.random()
            if r < 0.1:
                js.reassign(w, "e", (m, q, a, b))
            elif r < 0.9:
                js.record_result(m, q, w, a, b, np.zeros(b - a + 1, np.int32), np.ones(b - a + 1, np.float32))


def _view(js: JobState):
    return (sorted((k, sorted(v)) for k, v in js.worker_set.items()),
            sorted((k, sorted(v)) for k, v in js.working_vm_set.items()),
            dict(js.next_qnum), sorted(js.pending()))


def _strip_times(view):
    ws, vm, nq, pend = view
    ws = [(k, [e[:4] for e in v]) for k, v in ws]
    return ws, vm, nq, [p[:5] for p in pend]


def test_deltas_reproduce_the_coordinator_tables():
    rng = random.Random(1)
    coord, mirror = JobState(), JobState()
    mirror.restore(coord.snapshot(include_results=False), keep_results=True)
    for _ in range(20):
        _drive(coord, rng, 25)
        d = coord.deltas_since(mirror.mirror_seq)
        assert d is not None
        assert mirror.apply_deltas(d)
        assert mirror.mirror_seq == coord.seq
    assert _strip_times(_view(mirror)) == _strip_times(_view(coord))
    # the same from a late full snapshot
    snap = JobState()
    snap.restore(coord.snapshot(include_results=False), keep_results=True)
    assert _strip_times(_view(snap)) == _strip_times(_view(coord))
    # re-applying old entries is harmless
    assert mirror.apply_deltas(coord.deltas_since(0) or [])
    assert _strip_times(_view(mirror)) == _strip_times(_view(coord))


def test_gap_and_truncation_force_a_snapshot():
    coord, mirror = JobState(), JobState()
    coord.log_cap = 50
    rng = random.Random(2)
    _drive(coord, rng, 5)
    d = coord.deltas_since(0)
    assert mirror.apply_deltas(d[:3])
    assert not mirror.apply_deltas(d[5:])          # entries 4..5 missing: gap
    _drive(coord, rng, 200)                         # log truncated far past the mirror
    assert coord.deltas_since(mirror.mirror_seq) is None
    mirror.restore(coord.snapshot(include_results=False), keep_results=True)
    assert mirror.mirror_seq == coord.seq
    assert coord.deltas_since(mirror.mirror_seq) == []


def test_coordinator_cost_flat_over_100k_queries():
    """submit (assign + pending scan) and ingest per query must not grow with
    history: the last 10k of 100k queries cost about what the first 10k did."""
    js = JobState()
    js.log_cap = 20_000

    def batch(n):
        t0 = time.perf_counter()
        for _ in range(n):
            q = js.new_query_number("resnet18")
            js.assign("resnet18", q, [("a", q * 400, q * 400 + 199), ("b", q * 400 + 200, q * 400 + 399)])
            js.pending()                                # what submit_query scans
            js.range_submitted("resnet18", q * 400, q * 400 + 399)
            for w, s, e in (("a", q * 400, q * 400 + 199), ("b", q * 400 + 200, q * 400 + 399)):
                js.record_result("resnet18", q, w, s, e, np.zeros(200, np.int32), np.ones(200, np.float32))
        return (time.perf_counter() - t0) / n

    # best of 5 windows of 2k queries at each end: the check is about growth with
    # history, not about a busy host's scheduling spikes
    first = min(batch(2_000) for _ in range(5))
    batch(80_000)
    last = min(batch(2_000) for _ in range(5))
    assert js.pending_count() == 0 and js.images_done("resnet18") == 100_000 * 400
    assert last < 2.0 * first + 20e-6, f"per-query cost grew: {first * 1e6:.1f} -> {last * 1e6:.1f} us"
    # a push after one more query carries a handful of entries, not the history
    seq = js.seq
    q = js.new_query_number("resnet18")
    js.assign("resnet18", q, [("a", 0, 9)])
    assert len(js.deltas_since(seq)) == 2


def test_bulk_round_ingest_matches_per_chunk_and_replicates():
    """record_results (one collective round of one query, bulk path) leaves the
    same tables as per-chunk record_result, and its single 'results' log op
    brings a standby to the same state; duplicates / partial overlaps fall back
    to the per-chunk path."""
    import numpy as np

    from idunno.runtime.jobstate import JobState

    a, b, standby = JobState(), JobState(), JobState()
    W, B = 8, 50
    cls, prob = np.arange(B, dtype=np.int32), np.full(B, 0.25, np.float32)
    for q in range(1, 6):
        plan = [(f"node{r:02d}", q * 1000 + r * B, q * 1000 + (r + 1) * B - 1) for r in range(W)]
        for st in (a, b):
            st.assign("resnet18", q, plan, now=1.0)
        recs = [("resnet18", q, w, s, e, cls, prob) for w, s, e in plan]
        assert a.record_results(recs, now=2.0) == W
        for r in recs:
            b.record_result(*r, now=2.0)
    # a duplicate round and a round overlapping finished images: per-chunk path, nothing new
    assert a.record_results(recs, now=3.0) == 0
    sa, sb = a.snapshot(), b.snapshot()
    for k in sa:
        if k != "seq":
            assert sa[k] == sb[k], k
    assert a.inference_result_list() == b.inference_result_list()
    assert any(op == "results" for _, op, _ in a._log)
    assert standby.apply_deltas(a.deltas_since(0))
    assert standby.pending_count() == 0 and standby.cq() == a.cq() and standby.cvm() == a.cvm()


def test_bulk_and_per_chunk_same_c2_without_configured_batchsize():
    """a model with no configured batch size gets the same c2 window
    (per-chunk time) whether a round takes the bulk or the per-chunk path."""
    import numpy as np

    from idunno.runtime.jobstate import JobState

    a, b = (JobState(batchsize={}, clock=lambda: 5.0) for _ in range(2))
    sizes = [30, 50, 20, 70]
    for q in range(1, 4):
        plan, s0 = [], q * 1000
        for r, n in enumerate(sizes):
            plan.append((f"node{r:02d}", s0, s0 + n - 1))
            s0 += n
        for st in (a, b):
            st.assign("vgg", q, plan, now=float(q))
        recs = [("vgg", q, w, s, e, np.zeros(e - s + 1, np.int32), np.zeros(e - s + 1, np.float32))
                for w, s, e in plan]
        assert a.record_results(recs, now=q + 0.5) == len(plan)
        for r in recs:
            b.record_result(*r, now=q + 0.5)
    assert list(a._ptime_win["vgg"]) == list(b._ptime_win["vgg"])
    assert a.c2() == b.c2() and "average 0.5" in a.c2()
    sa, sb = a.snapshot(), b.snapshot()
    for k in sa:
        if k != "seq":
            assert sa[k] == sb[k], k


def test_whole_query_fast_path_and_bulk_fallback_agree():
    """A round answering every chunk of its query (in any order: the round lists
    members in group order, the plan has the scheduler's sampled order) takes the
    whole-query path (_whole_ok); partial rounds take the bulk path.  Both leave
    the tables per-chunk record_result leaves."""
    import numpy as np

    from idunno.runtime.jobstate import JobState

    W, B = 4, 25
    cls, prob = np.arange(B, dtype=np.int32), np.full(B, 0.5, np.float32)
    a, b = JobState(), JobState()
    for q in range(1, 4):
        plan = [(f"n{r}", q * 1000 + r * B, q * 1000 + (r + 1) * B - 1) for r in range(W)]
        for st in (a, b):
            st.assign("alexnet", q, plan, now=1.0)
        recs = [("alexnet", q, w, s, e, cls, prob) for w, s, e in plan]
        if q == 1:
            assert a._whole_ok(recs)
            assert a.record_results(recs, now=2.0) == W
        elif q == 2:
            rev = recs[::-1]
            assert a._whole_ok(rev) and a._bulk_ok(rev)
            assert a.record_results(rev, now=2.0) == W
        else:
            assert not a._whole_ok(recs[:2])
            assert a.record_results(recs[:2], now=2.0) == 2
            assert not a._whole_ok(recs[2:])      # half the query is already held
            assert a.record_results(recs[2:], now=2.0) == 2
        for r in (recs[::-1] if q == 2 else recs):     # same arrival order as a
            b.record_result(*r, now=2.0)
    sa, sb = a.snapshot(), b.snapshot()
    for k in sa:
        if k != "seq":
            assert sa[k] == sb[k], k
    assert a.inference_result_list() == b.inference_result_list()
    assert a.pending_count() == 0 and a.finished_queries["alexnet"] == 3
