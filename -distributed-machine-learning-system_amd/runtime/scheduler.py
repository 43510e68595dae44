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
    hysteresis: float = 0.1          # workers past the rounding point before a drained re-split

    def __post_init__(self):
        self._rng = random.Random(self.seed)
        self._seen: set = set()
        self._part: dict = {}
        self.repartitions = 0        # drained-boundary re-splits of the current (active, workers) key

    def effective_avg(self, models) -> dict[str, float]:
        """Per-model average query time for the split: a model with no
        measurement yet takes the mean of the measured ones (the constructor's
        placeholder 1.0 s against measured milliseconds would hand it nearly
        every GPU until its first result)."""
        seen = [self.avg_time[m] for m in self._seen if m in self.avg_time]
        fill = sum(seen) / len(seen) if seen else 1.0
        return {m: (self.avg_time[m] if m in self._seen else fill) for m in models}

    def subsets(self, active, workers: list, drained: bool = False) -> dict[str, list]:
        """``partition`` of ``workers`` over the ``active`` models.

        The split is computed when the active set (a job starts or ends), the
        worker set (a failure / join) or the set of measured models changes,
        and kept while queries are in flight, so EMA jitter never moves a job's
        GPUs under its running queries (a moved subset would collide with the
        other job's in-flight chunks).  At a DRAINED query boundary (no query of
        any job in flight, ``drained``) it follows the measured averages again,
        like the reference, which re-plans every query from the current averages
        (mp4_machinelearning.py:501-521; report Fig 2: 5/5 -> 4/6): the split
        moves when some model's exact share (t_i / sum(t) x workers) is more than
        ``hysteresis`` workers past the half-way point of its current count."""
        active = frozenset(active)
        key = (active, tuple(workers), frozenset(self._seen & active))
        cur = self._part.get(key)
        if cur is None:
            cur = partition(self.effective_avg(active), active, list(workers), self.budget)
            self._part = {key: cur}
            self.repartitions = 0
        elif drained and len(active) > 1:
            avg = self.effective_avg(active)
            eff = max(1, min(self.budget, len(workers)))
            sh = time_shares(avg, active)
            moved = any(abs(sh[m] * eff - len(cur[m])) > 0.5 + self.hysteresis for m in active)
            if moved:
                new = partition(avg, active, list(workers), self.budget)
                if {m: len(v) for m, v in new.items()} != {m: len(v) for m, v in cur.items()}:
                    cur = new
                    self._part = {key: cur}
                    self.repartitions += 1
        return cur

    def observe(self, model: str, normalized_query_time: float) -> None:
        """Feed a measured full-query-equivalent time for ``model`` (EMA)."""
        if model not in self._seen:
            self.avg_time[model] = float(normalized_query_time)
            self._seen.add(model)
        else:
            old = self.avg_time[model]
            self.avg_time[model] = (1 - self.ema) * old + self.ema * float(normalized_query_time)

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
               n: int | None = None, shuffle: bool = True, drained: bool = False) -> list[tuple]:
        """Returns [(worker, s, e), ...] for the inclusive query range.

        A single active job gets the whole budget (a random sample of the
        alive workers when the budget is smaller, as the reference samples,
        :520-521).  With several active jobs each gets its own disjoint,
        fair-time-sized subset (``partition``), so concurrent jobs share the
        node in space instead of queueing on the same GPUs; ``drained`` (no
        query in flight) lets that split follow the measured averages."""
        if not alive:
            return []
        active = set(self.active_jobs) | {model}
        if n is None and len(active) > 1:
            workers = self.subsets(active, list(alive), drained=drained)[model]
        else:
            n = self.n_workers(model, alive) if n is None else max(1, min(n, len(alive)))
            workers = self._rng.sample(list(alive), n) if shuffle else list(alive)[:n]
        chunks = split_range(start, end, len(workers))
        return [(w, s, e) for w, (s, e) in zip(workers, chunks)]
