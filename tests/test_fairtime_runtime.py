"""Fair-time split at runtime: two jobs
submitted together through the coordinator (``submit_job``, the reference's
two-tier variant), 8 nodes of a LocalCluster, executors whose per-image time
depends on the model.  The split the coordinator actually plans must follow the
measured averages while both jobs run -- the reference re-plans every query
from its averages (mp4_machinelearning.py:501-521) -- re-split when the ratio
flips, and never give one worker chunks of both jobs at once (after the start,
where the second job's first query lands on the first job's GPUs).

Times: AlexNet queries are 500 images, ResNet18 400 (report p.1).  At 100 / 200
us per image a full query takes 50 / 80 ms on one worker, so the reference
rule gives ResNet18 80/130 x 8 = 4.9 -> 5 workers and AlexNet 3; flipped to 160
/ 100 us per image (80 / 40 ms) it gives AlexNet 5.3 -> 5 and ResNet18 3."""
import threading
import time

from idunno.runtime.cluster import LocalCluster
from idunno.runtime.executor import FakeExecutor

FAST = dict(heartbeat_period_s=0.05, failure_timeout_s=2.0, metadata_period_s=0.2, rpc_timeout_s=5.0)


class ModelTimedExecutor(FakeExecutor):
    """FakeExecutor whose per-image time is per model (shared table, so the
    test can flip it for every node at once)."""

    def __init__(self, per_image: dict):
        super().__init__()
        self.per_image = per_image

    def run(self, model, images, start, end):
        time.sleep(self.per_image[model] * (end - start + 1))
        return super().run(model, images, start, end)


def _split(state, model, q):
    with state.lock:
        return len({w for w, *_ in state.worker_set.get((model, q), [])})


def _sizes(state, model):
    with state.lock:
        qs = sorted(q for (m, q) in state.worker_set if m == model)
        return [len({w for w, *_ in state.worker_set[(model, q)]}) for q in qs]


def test_split_follows_averages_while_both_jobs_run():
    per_image = {"alexnet": 100e-6, "resnet18": 200e-6}
    c = LocalCluster(num_nodes=8, executor_factory=lambda i: ModelTimedExecutor(per_image), **FAST).start()
    try:
        coord = c.coordinator()
        assert coord.sched.budget == 8 and len(coord.membership.alive()) == 8
        cl = c.client()
        Q = 40
        overlaps, stop = [], threading.Event()

        def monitor():
            # the coordinator's own chunk table: no worker may hold chunks of both jobs
            # once both are running (the first queries of the second job land on the
            # GPUs the first job was using alone: that start is not a re-split)
            while not stop.is_set():
                with coord.state.lock:
                    nq = {m: sum(1 for (mm, _q) in coord.state.worker_set if mm == m)
                          for m in ("alexnet", "resnet18")}
                if min(nq.values()) >= 4:
                    for w, ms in coord.state.busy_workers().items():
                        if len(ms) > 1:
                            overlaps.append((w, sorted(ms), nq))
                time.sleep(0.001)

        th = threading.Thread(target=monitor, daemon=True)
        th.start()
        cl.submit_job(0, 500 * Q - 1, "alexnet")
        cl.submit_job(0, 400 * Q - 1, "resnet18")
        # flip the ratio half-way through the AlexNet job
        deadline = time.monotonic() + 60
        while coord.state.images_done("alexnet") < 500 * Q // 2 and time.monotonic() < deadline:
            time.sleep(0.01)
        before = (_sizes(coord.state, "alexnet"), _sizes(coord.state, "resnet18"))
        per_image.update(alexnet=160e-6, resnet18=100e-6)
        # the split planned while BOTH jobs still run (at the very end one job is
        # alone and takes every GPU, as it should)
        while coord.state.images_done("alexnet") < 500 * Q * 85 // 100 and time.monotonic() < deadline:
            time.sleep(0.01)
        both_running = coord.state.active_models() == {"alexnet", "resnet18"}
        after = (_sizes(coord.state, "alexnet"), _sizes(coord.state, "resnet18"))
        s = cl.wait_idle(90, {"alexnet": 500 * Q, "resnet18": 400 * Q})
        stop.set()
        th.join(2)
        assert s["done"]["alexnet"] == 500 * Q and s["done"]["resnet18"] == 400 * Q, s
        a0, r0 = before
        a_all, r_all = after
        print("alexnet split per query:", _sizes(coord.state, "alexnet"))
        print("resnet18 split per query:", _sizes(coord.state, "resnet18"))
        print("averages:", coord.sched.avg_time, "re-splits:", coord.sched.repartitions,
              "deferred hand-overs:", coord.sched.moves_deferred)
        # converged to the reference rule's 3 / 5 before the flip ...
        assert a0[-3:] == [3, 3, 3] and r0[-3:] == [5, 5, 5], (a0, r0)
        # ... and to 5 / 3 after it, within a few queries
        assert both_running
        assert a_all[-3:] == [5, 5, 5] and r_all[-3:] == [3, 3, 3], (a_all, r_all)
        assert coord.sched.repartitions >= 2
        assert not overlaps, overlaps[:5]
        # the planned split agrees with the coordinator's own averages at the end
        t = coord.sched.avg_time
        assert t["alexnet"] > t["resnet18"]
    finally:
        c.stop()
