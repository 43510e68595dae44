"""Coordinator job-state tables and the c1/c2/c4/cq/cvm views.

Table layouts are kept identical to the reference so the shell output and the
standby snapshot look the same (mp4_machinelearning.py:115-160):

  worker_set        {(model, qnum): [(worker, start, end, 'w'|'f', t_start, t_end), ...]}   (cq)
  working_vm_set    {worker: [(model, qnum, start, end), ...]}                              (cvm)
  inference_result_list {"<model> <qnum>": [str([(img, category, prob), ...]), ...]}      (c4 -> result.txt)
  query_processing_time_meta {model: [mean, q1, q2, q3, std]}                               (c2)

Deliberate fixes:
  A2  c1/c2 numbers are measured for *every* model (none synthesised from the other)
  A3  finished-image counts are end - start + 1
  A4  results are kept as arrays (class id int32, prob fp32) and rendered to
      the reference's string format lazily, so no 4 KB truncation exists
  A11 query numbers are coordinator-assigned
  A13 single writer: every mutation goes through this object under one lock,
      and result ingestion is idempotent by chunk key (model, qnum, start, end)
"""
from __future__ import annotations

import json
import time
from collections import defaultdict, deque
from dataclasses import dataclass

import numpy as np

from ..utils import racecheck

WINDOW_S = 30.0  # reference SLIDING_WINDOW_SECONDS * SLIDING_WINDOW_FACTOR (10 * 3)

DEFAULT_BATCHSIZE = {"resnet18": 400, "alexnet": 500, "resnet50": 1024, "resnet34": 400}


def class_names(n: int = 1000, path: str | None = None) -> list[str]:
    """ImageNet category names if a classes file is available, else synthetic.

    The reference downloads imagenet_classes.txt (alexnet_resnet.py:27-42);
    there is no network here, so a local file is optional."""
    import os

    cands = [path] if path else []
    cands.append(os.environ.get("IDUNNO_CLASSES", ""))
    for p in cands:
        if p and os.path.exists(p):
            with open(p) as f:
                names = [ln.strip() for ln in f if ln.strip()]
            if len(names) >= n:
                return names[:n]
    return [f"class_{i}" for i in range(n)]


@dataclass
class ChunkResult:
    start: int
    end: int
    cls: np.ndarray      # int32 [n]
    prob: np.ndarray     # float32 [n]
    worker: str

    def render(self, names: list[str]) -> str:
        tup = [(f"test_{self.start + i}.JPEG", names[int(c)] if 0 <= int(c) < len(names) else str(int(c)),
                float(p)) for i, (c, p) in enumerate(zip(self.cls.tolist(), self.prob.tolist()))]
        return str(tup)


def _add_interval(ivs: list, s: int, e: int) -> int:
    """Merge [s, e] into the sorted, disjoint interval list ``ivs`` (in place);
    returns how many of its integers were not already covered."""
    new = e - s + 1
    out, i = [], 0
    while i < len(ivs) and ivs[i][1] < s - 1:
        out.append(ivs[i])
        i += 1
    lo, hi = s, e
    while i < len(ivs) and ivs[i][0] <= e + 1:
        a, b = ivs[i]
        new -= max(0, min(b, e) - max(a, s) + 1)
        lo, hi = min(lo, a), max(hi, b)
        i += 1
    out.append([lo, hi])
    out.extend(ivs[i:])
    ivs[:] = out
    return new


class JobState:
    # tables the race detector watches (all mutated only under self.lock)
    _TABLES = ("worker_set", "working_vm_set", "results", "finished_images", "finished_queries",
               "next_qnum", "jobs", "query_latency", "query_submit_time")

    def __init__(self, batchsize: dict | None = None, clock=time.time, window_s: float = WINDOW_S,
                 names: list[str] | None = None):
        self.lock = racecheck.make_lock("jobstate", reentrant=True)
        self.clock = clock
        self.window_s = window_s
        self.batchsize = dict(DEFAULT_BATCHSIZE, **(batchsize or {}))
        self.names = names
        self.worker_set: dict = defaultdict(list)
        self.working_vm_set: dict = defaultdict(list)
        self.results: dict = defaultdict(list)          # "model q" -> [ChunkResult]
        self._done_keys: set = set()
        self._done_imgs: dict = defaultdict(list)       # (model, qnum) -> merged finished [s, e] ranges
        self.finished_images: dict = defaultdict(int)
        self.finished_queries: dict = defaultdict(int)
        self._rate_win: dict = defaultdict(deque)       # model -> (t_finish, n_images)
        self._ptime_win: dict = defaultdict(deque)      # model -> (t_finish, normalised query time)
        self.query_processing_time_meta: dict = {}
        self._c2_dirty: set = set()                     # models whose c2 stats are stale
        self.next_qnum: dict = defaultdict(int)
        self.seq = 0                                    # mutation counter (standby replication)
        self.query_submit_time: dict = {}
        self.query_latency: dict = defaultdict(list)    # model -> [end-to-end seconds]
        self.jobs: dict = {}                            # job id -> {model, start, end, next}
        racecheck.instrument(self, self._TABLES)

    # -- coordinator-side jobs (C28 variant), replicated to the standby ----------
    def add_job(self, model: str, start: int, end: int, bs: int | None = None) -> int:
        """Register a coordinator-side job and reserve the query numbers of all
        its batch-size queries up front (query k of the job is ``qbase + k``).
        A promoted standby that resumes the job from a lagging snapshot then
        re-issues a query the dead coordinator had already dispatched under the
        SAME number, and ``record_result``'s per-query image dedupe keeps the
        late results of the original dispatch from being counted twice."""
        bs = int(bs or self.batchsize.get(model, 1))
        with self.lock:
            jid = len(self.jobs) + 1
            nq = (int(end) - int(start)) // bs + 1
            qbase = self.next_qnum[model] + 1
            self.next_qnum[model] += nq
            self.jobs[jid] = {"model": model, "start": int(start), "end": int(end), "next": int(start),
                              "bs": bs, "qbase": qbase}
            self.seq += 1
            return jid

    def images_held(self, model: str, qnum, s: int, e: int) -> bool:
        """True if results for every image of [s, e] under (model, qnum) are held."""
        with self.lock:
            return any(a <= s and e <= b for a, b in self._done_imgs.get((model, qnum), []))

    def job_query_number(self, jid: int, s: int) -> int:
        with self.lock:
            j = self.jobs[jid]
            return j["qbase"] + (int(s) - j["start"]) // j["bs"]

    def advance_job(self, jid: int, nxt: int) -> None:
        with self.lock:
            self.jobs[jid]["next"] = int(nxt)
            self.seq += 1

    def unfinished_jobs(self) -> list[int]:
        with self.lock:
            return [j for j, v in self.jobs.items() if v["next"] <= v["end"]]

    def range_submitted(self, model: str, s: int, e: int) -> bool:
        """True if some query of ``model`` already covers exactly [s, e] chunks
        (used when a promoted standby resumes a job from a lagging snapshot)."""
        with self.lock:
            for (m, _q), ents in self.worker_set.items():
                if m == model and ents and min(x[1] for x in ents) == s and max(x[2] for x in ents) == e:
                    return True
            return False

    # -- ids --------------------------------------------------------------------
    def new_query_number(self, model: str) -> int:
        """Coordinator-assigned query number (fix A11; the reference counted on the client)."""
        with self.lock:
            self.next_qnum[model] += 1
            return self.next_qnum[model]

    # -- mutations --------------------------------------------------------------
    def assign(self, model: str, qnum, chunks, now: float | None = None) -> None:
        """Record a dispatched query: chunks = [(worker, start, end), ...]."""
        now = self.clock() if now is None else now
        with self.lock:
            key = (model, qnum)
            self.query_submit_time.setdefault(key, now)
            for w, s, e in chunks:
                self.worker_set[key].append((w, int(s), int(e), "w", now, now))
                self.working_vm_set[w].append((model, qnum, int(s), int(e)))
            self.seq += 1

    def record_result(self, model: str, qnum, worker: str, start: int, end: int, cls, prob,
                      now: float | None = None) -> bool:
        """Ingest one finished chunk.  Idempotent: returns False for duplicates
        (e.g. a re-dispatched chunk whose original worker also answered)."""
        now = self.clock() if now is None else now
        start, end = int(start), int(end)
        with self.lock:
            ck = (model, qnum, start, end)
            key = (model, qnum)
            entries = self.worker_set.get(key, [])
            was_done = bool(entries) and all(ent[3] == "f" for ent in entries)
            hit = None
            for i, ent in enumerate(entries):
                if ent[1] == start and ent[2] == end and ent[3] == "w":
                    hit = i
                    break
            t_start = now
            if hit is not None:
                w, s, e, _, t_start, _ = entries[hit]
                entries[hit] = (w, s, e, "f", t_start, now)
                try:
                    self.working_vm_set[w].remove((model, qnum, s, e))
                except ValueError:
                    pass
                if not self.working_vm_set[w]:
                    self.working_vm_set.pop(w, None)
            # a duplicate still closes a matching 'w' entry (a re-dispatch with the
            # same chunk boundaries as the answered original) before it is dropped
            dup = ck in self._done_keys
            self._done_keys.add(ck)
            if entries and not was_done and all(ent[3] == "f" for ent in entries):
                self.finished_queries[model] += 1
                t0 = self.query_submit_time.get(key)
                if t0 is not None:
                    self.query_latency[model].append(now - t0)
            # images of this query already answered under another chunk split
            # (re-dispatch after a failure / a resumed job) are not counted again
            n = 0 if dup else _add_interval(self._done_imgs[key], start, end)   # fix A3: end-start+1 when new
            if n == 0:
                self.seq += 1
                return False
            self.finished_images[model] += n
            self._rate_win[model].append((now, n))
            bs = self.batchsize.get(model, n)
            self._ptime_win[model].append((now, (now - t_start) / n * bs))
            self._expire(model, now)
            self._c2_dirty.add(model)   # stats recomputed when read (c2 / snapshot), not per chunk
            self.results[f"{model} {qnum}"].append(
                ChunkResult(start, end, np.asarray(cls, dtype=np.int32), np.asarray(prob, dtype=np.float32),
                            worker))
            self.seq += 1
            return True

    def reopen_unheld(self) -> int:
        """Chunks marked finished in the replicated tables whose images this
        node never received (their RESULT reached only the old coordinator)
        go back to 'w', so a promoted standby recomputes them instead of
        reporting a query done whose results it cannot show (c4)."""
        with self.lock:
            n = 0
            for (m, q), ents in self.worker_set.items():
                ivs = self._done_imgs.get((m, q), [])
                for i, (w, s, e, st, t0, t1) in enumerate(ents):
                    if st == "f" and not any(a <= s and e <= b for a, b in ivs):
                        ents[i] = (w, s, e, "w", t0, t1)
                        self.working_vm_set[w].append((m, q, s, e))
                        n += 1
            if n:
                self.seq += 1
            return n

    def chunks_of(self, worker: str) -> list[tuple]:
        with self.lock:
            return list(self.working_vm_set.get(worker, []))

    def reassign(self, failed: str, new_worker: str, chunk: tuple, now: float | None = None) -> None:
        """Move one in-flight chunk of a failed worker to ``new_worker``
        (reference transfer_failed_inference_work, mp4_machinelearning.py:706-760)."""
        now = self.clock() if now is None else now
        model, qnum, s, e = chunk
        with self.lock:
            key = (model, qnum)
            ents = self.worker_set.get(key, [])
            for i, ent in enumerate(ents):
                if ent[0] == failed and ent[1] == s and ent[2] == e and ent[3] == "w":
                    ents.pop(i)
                    break
            ents.append((new_worker, s, e, "w", now, now))
            try:
                self.working_vm_set[failed].remove(chunk)
            except (ValueError, KeyError):
                pass
            if not self.working_vm_set.get(failed):
                self.working_vm_set.pop(failed, None)
            self.working_vm_set[new_worker].append(chunk)
            self.seq += 1

    def pending(self) -> list[tuple]:
        """All chunks still marked 'w': [(model, qnum, worker, s, e, t_start)]."""
        with self.lock:
            out = []
            for (model, q), ents in self.worker_set.items():
                for w, s, e, st, t0, _ in ents:
                    if st == "w":
                        out.append((model, q, w, s, e, t0))
            return out

    # -- metrics ------------------------------------------------------------------
    def _expire(self, model: str, now: float) -> None:
        for win in (self._rate_win[model], self._ptime_win[model]):
            while win and now - win[0][0] > self.window_s:
                win.popleft()

    def _refresh_c2(self) -> None:
        """Recompute the c2 statistics of models that got results since the
        last read.  Ingest only marks them stale: a per-chunk O(window)
        percentile costs the coordinator ~0.1 ms per chunk, and on the 8-rank
        throughput path a 30 s window holds tens of thousands of chunks."""
        for m in list(self._c2_dirty):
            self._expire(m, self.clock())
            self._recompute_c2(m)
        self._c2_dirty.clear()

    def _recompute_c2(self, model: str) -> None:
        vals = [v for _, v in self._ptime_win[model]]
        if vals:
            a = np.asarray(vals, dtype=np.float64)
            self.query_processing_time_meta[model] = [float(a.mean()), float(np.percentile(a, 25)),
                                                      float(np.percentile(a, 50)),
                                                      float(np.percentile(a, 75)), float(a.std())]

    def images_done(self, model: str) -> int:
        with self.lock:
            return int(self.finished_images.get(model, 0))

    def summary(self) -> dict:
        """Consistent view for the ``summary`` stats request (one lock hold: the
        tables are appended to by the result-ingest threads meanwhile)."""
        with self.lock:
            return {"ok": True, "done": {m: self.images_done(m) for m in self.models()},
                    "pending": len(self.pending()),
                    "latency": {m: list(v) for m, v in self.query_latency.items()},
                    "finished_queries": dict(self.finished_queries)}

    def rates(self, model: str, now: float | None = None) -> dict:
        now = self.clock() if now is None else now
        with self.lock:
            self._expire(model, now)
            win = self._rate_win[model]
            imgs = sum(n for _, n in win)
            span = self.window_s
            if win:
                span = max(min(self.window_s, now - win[0][0]), 1e-9)
            ips = imgs / span if win else 0.0
            return {"images_per_s": ips, "queries_per_s": ips / self.batchsize.get(model, 1),
                    "finished_images": self.images_done(model),
                    "finished_queries": int(self.finished_queries.get(model, 0))}

    def models(self) -> list[str]:
        with self.lock:
            ms = set(self.finished_images) | {m for m, _ in self.worker_set}
            return sorted(ms) or ["resnet18", "alexnet"]

    # -- shell views ------------------------------------------------------------
    def c1(self) -> str:
        """Query rate + finished count per model, reference labels (:1257-1267)."""
        label = {"resnet18": "Resnet18", "alexnet": "AlexNet"}
        lines = []
        for m in self.models():
            r = self.rates(m)
            L = label.get(m, m)
            lines.append(f"{L} query rate is {r['images_per_s']}")
            lines.append(f"{L} finished inference is {r['finished_images']}")
            lines.append(f"{L} finished batchsize query rare is {r['queries_per_s']}")
        return "\n".join(lines)

    def c2(self) -> str:
        """Processing-time stats per model over the sliding window (:1232-1253)."""
        lines = []
        with self.lock:
            self._refresh_c2()
            for m, v in sorted(self.query_processing_time_meta.items()):
                lines += [f"model {m} processing time", f"average {v[0]}", f"q1 {v[1]}", f"q2 {v[2]}",
                          f"q3 {v[3]}", f"stddev {v[4]}"]
        return "\n".join(lines)

    def inference_result_list(self) -> dict:
        names = self.names or class_names()
        with self.lock:
            return {k: [c.render(names) for c in sorted(v, key=lambda c: c.start)]
                    for k, v in self.results.items()}

    def c4(self, path: str = "result.txt") -> str:
        d = self.inference_result_list()
        with open(path, "w") as f:
            f.write(json.dumps(d))
        return str(d)

    def cq(self) -> str:
        with self.lock:
            return str(dict(self.worker_set))

    def cvm(self) -> str:
        with self.lock:
            return str(dict(self.working_vm_set))

    # -- replication (hot standby) --------------------------------------------------
    def snapshot(self, include_results: bool = True) -> dict:
        """Structured, JSON/msgpack-able snapshot (fix A12: no raw str() dumps).

        The coordinator's periodic push to the standby omits results: workers
        send every RESULT to the standby directly."""
        with self.lock:
            self._refresh_c2()
            return {
                "seq": self.seq,
                "worker_set": [[list(k), [list(e) for e in v]] for k, v in self.worker_set.items()],
                "working_vm_set": {w: [list(c) for c in v] for w, v in self.working_vm_set.items()},
                "results": ({k: [[c.start, c.end, c.cls.tolist(), c.prob.tolist(), c.worker] for c in v]
                             for k, v in self.results.items()} if include_results else None),
                "finished_images": dict(self.finished_images),
                "finished_queries": dict(self.finished_queries),
                "next_qnum": dict(self.next_qnum),
                "meta": dict(self.query_processing_time_meta),
                "submit": [[list(k), t] for k, t in self.query_submit_time.items()],
                "jobs": [[j, v] for j, v in self.jobs.items()],
            }

    def restore(self, snap: dict, keep_results: bool = False) -> None:
        """Adopt a snapshot.  With ``keep_results`` (standby mirror) the locally
        received results and counters are kept and chunks already answered
        stay marked 'f' even if the snapshot predates their RESULT."""
        with self.lock:
            if snap["seq"] < self.seq and not keep_results:
                return
            self.seq = max(self.seq, snap["seq"])
            self.worker_set = defaultdict(list)
            for k, v in snap["worker_set"]:
                self.worker_set[(k[0], k[1])] = [tuple(e) for e in v]
            self.working_vm_set = defaultdict(list, {w: [tuple(c) for c in v]
                                                     for w, v in snap["working_vm_set"].items()})
            if snap.get("results") is not None:
                self.results = defaultdict(list)
                self._done_keys = set()
                self._done_imgs = defaultdict(list)
                for k, v in snap["results"].items():
                    model, q = k.rsplit(" ", 1)
                    qn = int(q) if q.lstrip("-").isdigit() else q
                    for s, e, c, p, w in v:
                        self.results[k].append(ChunkResult(s, e, np.asarray(c, np.int32),
                                                           np.asarray(p, np.float32), w))
                        self._done_keys.add((model, qn, s, e))
                        _add_interval(self._done_imgs[(model, qn)], s, e)
            if not keep_results:
                self.finished_images = defaultdict(int, snap["finished_images"])
                self.finished_queries = defaultdict(int, snap["finished_queries"])
            # reconcile: chunks we already hold a result for are finished
            for (model, q), ents in self.worker_set.items():
                for i, (w, s, e, st, t0, t1) in enumerate(ents):
                    if st == "w" and (model, q, s, e) in self._done_keys:
                        ents[i] = (w, s, e, "f", t0, t1)
                        try:
                            self.working_vm_set[w].remove((model, q, s, e))
                        except ValueError:
                            pass
            for w in [w for w, v in self.working_vm_set.items() if not v]:
                self.working_vm_set.pop(w)
            for m, n in snap["next_qnum"].items():
                self.next_qnum[m] = max(self.next_qnum.get(m, 0), n)
            self.query_processing_time_meta.update(snap["meta"])
            for k, t in snap.get("submit", []):
                self.query_submit_time.setdefault((k[0], k[1]), t)
            for j, v in snap.get("jobs", []):
                cur = self.jobs.get(j)
                if cur is None or v["next"] > cur["next"]:
                    self.jobs[j] = dict(v)
            racecheck.instrument(self, self._TABLES)
