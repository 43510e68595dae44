"""Unit tests of the coordinator's round loop (``RoundPlane._serve``) with a
fake node: no process group, no sockets.

ADVICE r5 (high): rounds built from the queue and then lost to a failed
descriptor multicast (a member died: the usual worker-failover case) must fall
back to TCP JOBs for every live member's chunk -- before the fix they were in
neither ``inflight`` nor ``announced`` and were never re-sent."""
import threading

from idunno.config import ClusterConfig
from idunno.runtime.rounds import RoundPlane


class _Membership:
    def __init__(self, alive):
        self._alive = list(alive)

    def alive(self):
        return list(self._alive)

    def is_alive(self, m):
        return m in self._alive


class _State:
    def active_models(self):
        return {"resnet18"}

    def images_held(self, model, qnum, s, e):
        return False


class _Tracer:
    def instant(self, *a, **k):
        pass

    def span(self, *a, **k):
        import contextlib
        return contextlib.nullcontext()


class _Transport:
    def __init__(self, lost):
        self.lost = lost
        self.frames = []

    def multicast(self, members, msg):
        self.frames.append((list(members), msg))
        return list(self.lost)

    def send(self, m, msg):
        pass


class _Node:
    def __init__(self, members, alive, lost):
        self.name = members[0]
        self.alive_flag = True
        self.is_coordinator = True
        self.cfg = ClusterConfig()
        self.membership = _Membership(alive)
        self.state = _State()
        self.tracer = _Tracer()
        self.transport = _Transport(lost)
        self.jobs = []
        self.standby = members[-1]
        self.source = None

    def _send_job(self, w, model, qnum, s, e):
        self.jobs.append((w, model, qnum, s, e))


def test_failed_announce_falls_back_on_every_live_row():
    members = ["node00", "node01", "node02", "node03"]
    node = _Node(members, alive=["node00", "node01", "node03"], lost=["node02"])
    plane = RoundPlane(node, "cpu")
    g = plane.group
    g.pg = object()                               # "formed"; nothing is ever posted
    g.epoch, g.members, g.rank = 1, list(members), 0
    plane.healthy = True
    with plane.cv:
        plane.members = list(members)
    plans = []
    for q in range(3):
        plan = [(w, q * 400 + 100 * i, q * 400 + 100 * i + 99) for i, w in enumerate(members)]
        assert plane.try_enqueue("resnet18", q, plan)
        plans.append(plan)
    done = threading.Event()

    def run():
        plane._serve()
        done.set()

    th = threading.Thread(target=run, daemon=True)
    th.start()
    assert done.wait(10)
    assert node.transport.frames, "the rounds were announced"
    assert plane.rounds_failed == 1 and not g.formed
    # every live member's chunk of every query went out as a TCP JOB; the dead
    # member's chunks belong to the failure handler's re-dispatch
    want = sorted((w, "resnet18", q, s, e) for q, plan in enumerate(plans) for w, s, e in plan if w != "node02")
    assert sorted(node.jobs) == want
    assert plane._reform_at is not None           # and a re-form is scheduled
