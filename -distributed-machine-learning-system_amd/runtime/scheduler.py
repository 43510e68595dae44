"""Fair-time query scheduler.

Reference behaviour (mp4_machinelearning.py:497-539):
  * ratio = avg_time[alexnet] / avg_time[resnet18]
  * workers(alexnet)  = clamp(round(ratio / (ratio + 1) * budget), 0, alive)
    workers(resnet18) = clamp(round((1/ratio) / ((1/ratio) + 1) * budget), 0, alive)
    i.e. each model gets the budget share of *its own* time, so the slower
    model receives more workers;
  * workers are a random sample of the alive set;
  * the inclusive index range [start, end] is cut into contiguous chunks of
    round(remaining / remaining_workers) using Python's banker's rounding
    (400 over 6 workers -> 67, 67, 66, 67, 66, 67).

Deliberate fix: the per-model average query time is a measured
EMA that the coordinator updates on every finished chunk, instead of a
constant 100 s that is never written.
"""
from __future__ import annotations

import random
import threading
from dataclasses import dataclass, field


def split_range(start: int, end: int, n_workers: int) -> list[tuple[int, int]]:
    """Split inclusive [start, end] into ``n_workers`` contiguous inclusive chunks.

    Chunk length = round(remaining / remaining_workers) with round-half-even,
    which is the reference's split rule.  Empty chunks are dropped.
    """
    if end < start or n_workers <= 0:
        return []
    remaining = end - start + 1
    n = min(n_workers, remaining)
    out: list[tuple[int, int]] = []
    cur = start
    for k in range(n, 0, -1):
        ln = round(remaining / k)
        if k == 1:
            ln = remaining
        if ln <= 0:
            continue
        out.append((cur, cur + ln - 1))
        cur += ln
        remaining -= ln
    return out


def time_shares(avg_time: dict[str, float], models) -> dict[str, float]:
    """Each active model's share of the worker budget: t_i / sum(t) over the
    active models (the slower model gets more workers).  For the reference's
    two models this is its formula: ratio = t_a / t_r, share_a = ratio /
    (ratio + 1) = t_a / (t_a + t_r) (mp4_machinelearning.py:504-514).  Every
    model reads ITS OWN average (the reference only knew alexnet/resnet18)."""
    models = sorted(set(models))
    t = {m: max(float(avg_time.get(m, 1.0)), 1e-9) for m in models}
    tot = sum(t.values())
    return {m: t[m] / tot for m in models}


def fair_share(avg_time: dict[str, float], model: str, budget: int, alive: int,
               active=("alexnet", "resnet18")) -> int:
    """Workers for ``model`` under the fair-time rule over the ``active``
    models (default: the reference's pair), rounded half-even and clamped to
    the alive count like the reference."""
    active = set(active) | {model}
    n = round(time_shares(avg_time, active)[model] * budget)
    return int(max(0, min(n, alive)))


def partition(avg_time: dict[str, float], models, workers: list, budget: int) -> dict[str, list]:
    """Disjoint worker subsets for concurrently active models (space sharing).

    Sizes follow ``fair_share`` (at least one worker each), then are adjusted
    by largest remainder so they add up to min(budget, len(workers)) -- the
    reference's independent rounding can leave a worker idle or over-commit
    one.  Subsets are contiguous slices of ``workers`` in model-name order, so
    consecutive queries of one job land on the same GPUs and two jobs'
    queries never share one (they can run in the same collective round).
    With more models than workers, workers are shared round-robin."""
    models = sorted(set(models))
    workers = list(workers)
    if not models or not workers:
        return {m: [] for m in models}
    eff = max(1, min(budget, len(workers)))
    if len(models) > eff:
        # fewer budgeted workers than active models (more jobs than GPUs, or a
        # budget below the job count): the models share the eff workers
        # round-robin, one each
        return {m: [workers[i % eff]] for i, m in enumerate(models)}
    if len(models) == 1:
        return {models[0]: workers[:eff]}
    sh = time_shares(avg_time, models)
    exact = {m: sh[m] * eff for m in models}
    n = {m: max(1, round(exact[m])) for m in models}
    while sum(n.values()) > eff:
        m = max((m for m in models if n[m] > 1), key=lambda m: (n[m] - exact[m], m))
        n[m] -= 1
    while sum(n.values()) < eff:
        m = max(models, key=lambda m: (exact[m] - n[m], m))
        n[m] += 1
    out, i = {}, 0
    for m in models:
        out[m] = workers[i:i + n[m]]
        i += n[m]
    return out


class ChunkTimeFit:
    """A model's chunk compute time as ``t(n) = a + b*n`` (fixed per-chunk cost
    + per-image cost), fitted by exponentially-forgotten least squares over the
    observed (chunk size, seconds) pairs.

    Why: the fair-time rule needs each model's *query*
    time, but a chunk's per-image time falls as the chunk grows (the fixed
    launch / tail cost is spread over more images) and the chunk size is set by
    the split itself -- a model given more workers gets smaller chunks, looks
    slower per image and would be given still more workers.  ``full(B)`` = a +
    b*B, the time ONE worker needs for a whole B-image query, does not depend on
    how the current split cut it.  Until two clearly different chunk sizes have
    been seen the fit falls back to the per-image time scaled to B, and it does
    so too when the line claims more than half of a chunk's time is fixed cost:
    a per-image time that CHANGED (the model got slower) together with the chunk
    size fits such a line, and it would fade only as the old points are
    forgotten."""

    MAX_FIXED = 0.5                 # intercept / mean chunk time above which the line is not trusted

    def __init__(self, forget: float = 0.2):
        self.forget = forget
        self.w = self.sn = self.st = self.snn = self.snt = 0.0
        self.nmin = self.nmax = None

    def add(self, n: int, t: float, w: float = 1.0) -> None:
        """One point (n images, t seconds) of weight ``w``: w equal points at once
        (one round's members with the same chunk size) forget the past as w
        separate adds would."""
        k = (1.0 - self.forget) ** w
        self.w, self.sn, self.st = k * self.w + w, k * self.sn + w * n, k * self.st + w * t
        self.snn, self.snt = k * self.snn + w * n * n, k * self.snt + w * n * t

    def full(self, B: int) -> float | None:
        if self.w <= 0:
            return None
        mn, mt = self.sn / self.w, self.st / self.w
        var = self.snn / self.w - mn * mn
        if var > (0.1 * mn) ** 2:                 # chunk sizes spread by >10 %: fit the line
            b = (self.snt / self.w - mn * mt) / var
            a = mt - b * mn
            if b > 0 and 0 <= a <= self.MAX_FIXED * mt:
                return a + b * B
        return mt / max(mn, 1e-9) * B


@dataclass
class FairTimeScheduler:
    """Chooses workers and chunks for each query.

    ``budget`` is the reference's RATE_FACTOR (mp4_machinelearning.py:44); in a
    one-node deployment it is the number of GPUs shared by concurrent jobs.
    ``ema`` is the smoothing of the measured per-model time (A1 fix).
    """

    budget: int = 8
    ema: float = 0.3
    seed: int | None = None
    avg_time: dict = field(default_factory=lambda: {"alexnet": 1.0, "resnet18": 1.0})
    active_jobs: set = field(default_factory=set)
    hysteresis: float = 0.1          # workers past the rounding point before a re-split

    def __post_init__(self):
        self._rng = random.Random(self.seed)
        self._seen: set = set()
        self._part: dict = {}
        self._fits: dict = {}
        self._leaving: dict = {}     # worker -> (donor, receiver): handed over once the donor's chunks end
        self._lock = threading.Lock()
        self.repartitions = 0        # query-boundary re-splits of the current (active, workers) key
        self.moves_deferred = 0      # hand-overs that waited for the donor's chunks on the worker

    def effective_avg(self, models) -> dict[str, float]:
        """Per-model average query time for the split: a model with no
        measurement yet takes the mean of the measured ones (the constructor's
        placeholder 1.0 s against measured milliseconds would hand it nearly
        every GPU until its first result)."""
        seen = [self.avg_time[m] for m in self._seen if m in self.avg_time]
        fill = sum(seen) / len(seen) if seen else 1.0
        return {m: (self.avg_time[m] if m in self._seen else fill) for m in models}

    def target_sizes(self, active, workers: list) -> dict[str, int]:
        """Subset sizes the current averages prescribe (``partition``'s rule)."""
        return {m: len(v) for m, v in partition(self.effective_avg(active), active, list(workers),
                                                self.budget).items()}

    def subsets(self, active, workers: list, boundary: bool = False, busy: dict | None = None,
                drained: bool = False) -> dict[str, list]:
        """``partition`` of ``workers`` over the ``active`` models.

        A fresh split is computed when the active set (a job starts or ends) or
        the worker set (a failure / join) changes.  Otherwise the split is
        re-planned at every query BOUNDARY
        (``boundary``: a job's next query is being planned), like the
        reference, which re-plans every query from the current averages
        (mp4_machinelearning.py:501-521; report Fig 2: 5/5 -> 4/6): when some
        model's exact share (t_i / sum(t) x workers) is more than
        ``hysteresis`` workers past the half-way point of its current count,
        workers move from the models above their target to the ones below it.
        Each model keeps the workers it is not giving up, so its queries keep
        landing on the same GPUs.

        Subsets never overlap in-flight chunks: ``busy`` (worker -> models with
        chunks running there) marks a donor's worker that still runs the
        donor's chunks; it leaves the donor's subset at once (the donor's next
        queries no longer use it) and joins the receiver at the first boundary
        after those chunks finished.  ``busy=None`` (the collective round path:
        queued queries are re-split onto the new subsets before they are
        posted, and a round gives each member one row) hands workers over at
        once.  ``drained`` is the old name of ``boundary``."""
        boundary = boundary or drained
        active = frozenset(active)
        key = (active, tuple(workers))
        with self._lock:
            cur = self._part.get(key)
            if cur is None:
                cur = partition(self.effective_avg(active), active, list(workers), self.budget)
                self._part = {key: cur}
                self._leaving = {}
                self.repartitions = 0
            elif boundary and 1 < len(active) <= max(1, min(self.budget, len(workers))):
                new = {m: list(v) for m, v in cur.items()}
                changed = self._settle(new, busy)
                size = {m: len(new[m]) + sum(1 for _d, r in self._leaving.values() if r == m) for m in active}
                eff = max(1, min(self.budget, len(workers)))
                sh = time_shares(self.effective_avg(active), active)
                if any(abs(sh[m] * eff - size[m]) > 0.5 + self.hysteresis for m in active):
                    changed |= self._shift(new, size, self.target_sizes(active, workers), busy)
                if changed:
                    cur = new
                    self._part = {key: cur}
                    self.repartitions += 1
            return cur

    def _settle(self, cur: dict, busy: dict | None) -> bool:
        """Workers handed over while still busy with their donor's chunks join
        their receiver once those chunks are done."""
        moved = False
        for w, (donor, recv) in list(self._leaving.items()):
            if recv in cur and (busy is None or donor not in busy.get(w, ())):
                cur[recv].append(w)
                del self._leaving[w]
                moved = True
        return moved

    def _shift(self, cur: dict, size: dict, want: dict, busy: dict | None) -> bool:
        """Move workers from models above their target size to models below
        it: a donor's idle workers first (its last ones first, so slices stay
        contiguous when nothing is busy); a busy one goes through
        ``_leaving``."""
        need = [m for m in sorted(cur) for _ in range(max(0, want.get(m, 0) - size[m]))]
        moved = False
        for donor in sorted(cur, key=lambda m: (size[m] - want.get(m, 0), m), reverse=True):
            while need and cur[donor] and size[donor] > max(1, want.get(donor, 0)):
                cands = list(reversed(cur[donor]))
                free = [w for w in cands if busy is None or donor not in busy.get(w, ())]
                w = free[0] if free else cands[0]
                cur[donor].remove(w)
                size[donor] -= 1
                recv = need.pop(0)
                size[recv] += 1
                if free:
                    cur[recv].append(w)
                else:
                    self._leaving[w] = (donor, recv)
                    self.moves_deferred += 1
                moved = True
        return moved

    def observe(self, model: str, normalized_query_time: float) -> None:
        """Feed a measured full-query-equivalent time for ``model`` (EMA)."""
        if model not in self._seen:
            self.avg_time[model] = float(normalized_query_time)
            self._seen.add(model)
        else:
            old = self.avg_time[model]
            self.avg_time[model] = (1 - self.ema) * old + self.ema * float(normalized_query_time)

    def observe_chunks(self, model: str, points, batch: int) -> None:
        """``observe_chunk`` for several (n, seconds) points of one model (one
        collective round's members), with one refit."""
        fit = self._fits.setdefault(model, ChunkTimeFit())
        by_n = {}
        for n, sec in points:
            if n > 0 and sec > 0:
                a = by_n.get(n)
                by_n[n] = (sec, 1) if a is None else (a[0] + sec, a[1] + 1)
        for n, (tot, c) in by_n.items():          # equal chunk sizes: their mean, weighted
            fit.add(int(n), tot / c, c)
        t = fit.full(int(batch))
        if t is not None:
            self.avg_time[model] = t
            self._seen.add(model)

    def observe_chunk(self, model: str, n: int, seconds: float, batch: int) -> None:
        """One warm chunk of ``n`` images took ``seconds`` of compute: refit the
        model's chunk-time line and take its full-query time ``a + b*batch``
        (``ChunkTimeFit``) as the model's average.  Callers leave out cold
        chunks (a worker's first chunk of a model and chunk size: graph capture,
        kernel load), so they never seed the average."""
        if n <= 0 or seconds <= 0:
            return
        fit = self._fits.setdefault(model, ChunkTimeFit())
        fit.add(int(n), float(seconds))
        t = fit.full(int(batch))
        if t is not None:
            self.avg_time[model] = t
            self._seen.add(model)

    def adopt(self, avg_time: dict) -> None:
        """Take over measured averages (standby mirror, checkpoint restore):
        they count as measurements, not placeholders."""
        for m, v in avg_time.items():
            self.avg_time[m] = float(v)
            self._seen.add(m)

    def n_workers(self, model: str, alive: list) -> int:
        if len(self.active_jobs - {model}) == 0:
            # a single job owns the whole budget
            return max(1, min(self.budget, len(alive)))
        act = set(self.active_jobs) | {model}
        return max(1, fair_share(self.effective_avg(act), model, self.budget, len(alive), act))

    def assign(self, model: str, start: int, end: int, alive: list,
               n: int | None = None, shuffle: bool = True, drained: bool = False,
               boundary: bool = False, busy: dict | None = None) -> list[tuple]:
        """Returns [(worker, s, e), ...] for the inclusive query range.

        A single active job gets the whole budget (a random sample of the
        alive workers when the budget is smaller, as the reference samples,
        :520-521).  With several active jobs each gets its own disjoint,
        fair-time-sized subset (``partition``), so concurrent jobs share the
        node in space instead of queueing on the same GPUs; ``boundary`` (this
        is a job's next query) lets that split follow the measured averages
        (``subsets``)."""
        if not alive:
            return []
        active = set(self.active_jobs) | {model}
        if n is None and len(active) > 1:
            workers = self.subsets(active, list(alive), boundary=boundary or drained, busy=busy)[model]
        else:
            n = self.n_workers(model, alive) if n is None else max(1, min(n, len(alive)))
            workers = self._rng.sample(list(alive), n) if shuffle else list(alive)[:n]
        chunks = split_range(start, end, len(workers))
        return [(w, s, e) for w, (s, e) in zip(workers, chunks)]
