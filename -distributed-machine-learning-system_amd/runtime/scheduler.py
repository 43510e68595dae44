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


def fair_share(avg_time: dict[str, float], model: str, budget: int, alive: int) -> int:
    """Workers for ``model`` under the two-job fair-time rule."""
    ta = max(avg_time.get("alexnet", 1.0), 1e-9)
    tr = max(avg_time.get("resnet18", 1.0), 1e-9)
    ratio = ta / tr
    if model == "alexnet":
        n = round(ratio / (ratio + 1) * budget)
    else:
        inv = 1.0 / ratio
        n = round(inv / (inv + 1) * budget)
    return int(max(0, min(n, alive)))


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

    def __post_init__(self):
        self._rng = random.Random(self.seed)
        self._seen: set = set()

    def observe(self, model: str, normalized_query_time: float) -> None:
        """Feed a measured full-query-equivalent time for ``model`` (EMA)."""
        if model not in self._seen:
            self.avg_time[model] = float(normalized_query_time)
            self._seen.add(model)
        else:
            old = self.avg_time[model]
            self.avg_time[model] = (1 - self.ema) * old + self.ema * float(normalized_query_time)

    def n_workers(self, model: str, alive: list) -> int:
        if len(self.active_jobs - {model}) == 0:
            # a single job owns the whole budget
            return max(1, min(self.budget, len(alive)))
        return max(1, fair_share(self.avg_time, model, self.budget, len(alive)))

    def assign(self, model: str, start: int, end: int, alive: list,
               n: int | None = None, shuffle: bool = True) -> list[tuple]:
        """Returns [(worker, s, e), ...] for the inclusive query range."""
        if not alive:
            return []
        n = self.n_workers(model, alive) if n is None else max(1, min(n, len(alive)))
        workers = self._rng.sample(list(alive), n) if shuffle else list(alive)[:n]
        chunks = split_range(start, end, n)
        return [(w, s, e) for w, (s, e) in zip(workers, chunks)]
