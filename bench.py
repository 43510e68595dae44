#!/usr/bin/env python3
"""Headline benchmark: ResNet18 bs=400 image-classification queries on 1..8 MI355X.

Metric (BASELINE.json): images/sec for the whole node + p50 query latency,
ResNet18, 400 images per query per GPU, synthetic 224x224x3 uint8 images and
random-init weights (no datasets or checkpoints are reachable).

Precision: the reference classifies in fp32 (torchvision eager,
/root/reference/alexnet_resnet.py:17-22, 74-75), so the headline runs the
framework's fp32 path (``--fp32-impl``):
  * "split" (default): every conv (the fused stem, the residual stages) on
    fp32-accurate split fp16 -- each fp32 value carried as (hi, lo) halfs (22
    significant bits, 4 bytes like fp32), hi*hi + hi*lo + lo*hi summed in f32
    on the f16 MFMA -- and the FC on the f32-input MFMA;
  * "f32mfma": every conv / FC on v_mfma_f32_16x16x4_f32 (exact f32 products,
    f32 accumulate), 3x3 stride-1 convs by fused fp32 Winograd F(2x2,3x3).
Both are checked against the fp64 CPU module on the same weights, next to
torch fp32 itself (``max_rel_logit_err_vs_fp64``,
``torch_fp32_max_rel_logit_err_vs_fp64``, ``max_rel_logit_err_vs_torch_fp32``).
The other fp32 implementation and the fp16 path (f16 MFMA, f32 accumulate,
fp16 activations) are reported as extra keys.

The process the driver starts is a pure LAUNCHER: it never touches a GPU and
runs three phases of child processes (one per GPU), then prints ONE JSON line.

  1. headline ("raw round loop"): one *step* is one round of the cluster's
     query path, end to end -- the coordinator (rank 0) splits the round's
     image range over the ranks with the scheduler's split rule (reference
     mp4_machinelearning.py:523-536) and broadcasts the chunk descriptors
     (RCCL); every rank runs preprocess + the HIP forward + fused
     softmax-top1 on its chunk of its HBM-resident dataset replica (one
     hipGraph replay of hand-written gfx950 kernels, window start read on the
     device); top-1 (class, prob) pairs are gathered to the coordinator (RCCL),
     copied to host and recorded in the job-state tables.  Weak scaling (400
     images per GPU per step); strong scaling (ONE 400-image query split over
     the N ranks) as ``*_strong`` keys.
  2. system (``value_system``, ``p50_system_s``, ``two_job_*``,
     ``workers_per_query_*``): N node processes of the fault-tolerant runtime
     (membership + failure detector, coordinator on rank 0, hot standby on the
     last rank, RCCL rounds for N > 1).  The coordinator's client submits
     ResNet18 queries (same shape as the headline), then an AlexNet job and a
     ResNet18 job at the same time: the fair-time scheduler splits the GPUs
     between them and the round path runs both side by side (report Fig 2).
  3. coordinator failover (``coord_failover_*``): max(N, 2) node processes;
     mid-job the launcher SIGKILLs the coordinator process, the standby
     promotes itself, re-forms the collective group over the survivors and
     finishes the job (report Fig 5).
Phases 2-3 are bounded (``--extras-timeout``); if one fails its keys are null
and ``extras_error`` says why -- the headline is never lost to them.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
  Without torchrun env vars the launcher starts the N ranks itself (RCCL over
  127.0.0.1 rendezvous); under torchrun (RANK set) each torchrun process
  starts its own rank child, and rank 0's launcher runs phases 2-3 on all N
  GPUs after the headline.  Exits non-zero if a headline rank fails.
  --dry-run: gloo on the CPU with a fake forward (launcher / collectives /
  JSON contract without a GPU).  --system: phase 2 only (its own JSON line).
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import signal
import socket
import statistics
import subprocess
import sys
import tempfile
import time

BASELINE_IMG_PER_S = 41.0          # 400 img / 9.749 s (ResNet18, 5 workers)
BASELINE_P50_S = 9.749             # p50 ResNet18 400-image query latency
BASELINE_COORD_RECOVERY_S = 6.999  # coordinator failure, 1 undone query (report Fig 5)
BASELINE_WORKER_RECOVERY_S = {1: 5.725, 2: 8.661, 4: 13.425, 6: 19.125, 8: 26.751}   # report Fig 4
BASELINE_SECOND_JOB_S = {"alexnet_first": 41.159, "resnet18_first": 46.752}   # report Fig 3 medians
REF_WORKER_START_DELAY_S = 3.0     # reference sleep before every chunk (mp4_machinelearning.py:594)
METRIC = "images/sec (whole node) + p50 query latency, ResNet18 bs=400 at 1/2/4/8 GPU"
QUERY = 400                        # images per query (reference report p.1, ResNet18)
QUERY_ALEXNET = 500                # AlexNet query size (report p.1)
COMPUTE_F32 = ("f32-input MFMA (v_mfma_f32_16x16x4_f32), fp32 activations/weights, fp32 accumulate; "
               "3x3/s1 convs by fused fp32 Winograd F(2x2,3x3)")
COMPUTE_SPLIT = ("fp32-accurate: every conv (fused stem, residual stages) on split fp16 (each fp32 value as "
                 "hi+lo halfs, 22-bit significand, 4 bytes; hi*hi+hi*lo+lo*hi on v_mfma_f32_16x16x32_f16, "
                 "fp32 accumulate), FC on the f32-input MFMA; logits checked against fp64 next to torch fp32")
ROLE = "IDUNNO_BENCH_ROLE"


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "fp16"],
                    help="headline precision (fp32 = the reference's)")
    ap.add_argument("--fp32-impl", default="split", choices=["split", "f32mfma"],
                    help="fp32 kernels: split-fp16 (fp32-accurate) residual stages, or all f32-MFMA")
    ap.add_argument("--batch", type=int, default=400, help="images per GPU per weak-scaling step")
    ap.add_argument("--dataset-images", type=int, default=2000,
                    help="synthetic images replicated in every rank's HBM (grown to fit a round)")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraph replay")
    ap.add_argument("--rehearse-gloo", action="store_true",
                    help="N > 1 on a box with fewer GPUs: gloo collectives on GPU tensors, ranks share "
                         "cuda:(local_rank %% device_count) -- exercises the multi-rank GPU path, not RCCL")
    ap.add_argument("--rehearse-rccl", action="store_true",
                    help="N > 1 on a box with fewer GPUs over RCCL itself: every process gets its own "
                         "NCCL_HOSTID (RCCL then treats the ranks sharing a GPU as separate hosts and "
                         "connects them over its socket transport on loopback); ranks share "
                         "cuda:(local_rank %% device_count) -- the RCCL code paths of the N-GPU run, not xGMI")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="N > 1: keep the descriptor broadcast and result gather between the forwards "
                         "(default: double-buffered, overlapped with the next round's forward)")
    ap.add_argument("--host-wait", default="auto", choices=["auto", "spin", "poll"],
                    help="how rank host threads wait for the GPU: spin (HIP synchronize), or poll (event "
                         "query + sleep, at most 2 rounds queued ahead); auto = poll for N > 1 (N rank "
                         "processes plus their RCCL proxy threads must not spin every CPU of the box)")
    ap.add_argument("--no-extras", action="store_true", help="skip the strong-scaling / fp16 / numerics extras")
    ap.add_argument("--no-system", action="store_true", help="skip phases 2-3 (system + failover)")
    ap.add_argument("--node-phases", default="system,failover,worker",
                    help="node phases to run after the headline (comma list of system, failover, worker)")
    ap.add_argument("--extras-timeout", type=float, default=150.0,
                    help="seconds per system / failover phase (bounded: the driver gives the whole run 600 s)")
    ap.add_argument("--extras-budget", type=float, default=240.0,
                    help="seconds for all phases after the headline together; a phase that would start "
                         "past it is skipped (extras_skipped), so the headline line always comes out in time")
    ap.add_argument("--two-job-queries", type=int, default=10, help="queries per job in the two-job run")
    ap.add_argument("--ref-delay-queries", type=int, default=3,
                    help="queries timed with the reference's 3 s worker start delay (0: skip)")
    ap.add_argument("--sdfs-images", type=int, default=4000,
                    help="N=1 system phase: images put into SDFS as 500-image shards, then served cold and warm")
    ap.add_argument("--sdfs-trace", default=None, help="write the SDFS cold pass's H2D / forward GPU timeline "
                                                      "(chrome trace JSON) here")
    ap.add_argument("--failover-queries", type=int, default=12, help="queries of the job the failover kills into")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--dry-run", action="store_true", help="CPU + gloo + fake forward (launcher/contract test)")
    ap.add_argument("--fail-rank", type=int, default=-1, help="testing: this rank exits 3 after warmup")
    ap.add_argument("--launch-timeout", type=float, default=300.0,
                    help="seconds before the headline ranks are killed (headline + in-rank extras; the driver's "
                         "lease is 600 s for the whole run)")
    ap.add_argument("--rank-extras-budget", type=float, default=150.0,
                    help="seconds for the in-rank extras after the headline; an extra that would start past "
                         "it is skipped (rank_extras_skipped)")
    ap.add_argument("--fail-after-headline", type=int, default=-1,
                    help="testing: this rank exits 3 right after the headline is measured")
    ap.add_argument("--hang-in-extras", type=int, default=-1, help="testing: this rank hangs in the extras")
    ap.add_argument("--system", action="store_true", help="phase 2 only (see docstring)")
    ap.add_argument("--phase", default="system", choices=["system", "failover", "worker"], help=argparse.SUPPRESS)
    ap.add_argument("--detector", default="reference", choices=["reference", "tuned"], help=argparse.SUPPRESS)
    ap.add_argument("--kill-chunks", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--worker-kill-chunks", type=lambda v: [int(x) for x in v.split(",")], default=[1, 4, 8],
                    help="chunks in flight on the killed worker, one cluster per value (report Fig 4)")
    ap.add_argument("--work-dir", default=None, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# launcher (never initialises a GPU: children are started with subprocess,
# nothing is ever exec'd in place)
# ---------------------------------------------------------------------------

def _free_port() -> int:
    """A rendezvous port P such that P and the node phases' blocks P+200..+215
    (node listeners) and P+300..+399 (per-epoch TCPStores) are free, below the
    kernel's ephemeral range (32768+): an outgoing connection of the many node
    clients can then never take one of them between two phases."""
    import random

    rng = random.Random()
    for _ in range(200):
        p = rng.randrange(20000, 32768 - 400)
        try:
            for q in [p, *range(p + 200, p + 216), *range(p + 300, p + 400)]:
                with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
                    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
                    s.bind(("127.0.0.1", q))
        except OSError:
            continue
        return p
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _child_env(role: str, rank: int, world: int, port: int, local: int | None = None) -> dict:
    env = dict(os.environ)
    for k in ("TORCHELASTIC_USE_AGENT_STORE", "TORCHELASTIC_RUN_ID", "GROUP_RANK", "ROLE_RANK"):
        env.pop(k, None)
    env.update({ROLE: role, "RANK": str(rank), "LOCAL_RANK": str(rank if local is None else local),
                "WORLD_SIZE": str(world), "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(port)})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def _spawn(argv, env) -> subprocess.Popen:
    return subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                            stdin=subprocess.DEVNULL)


def _stop_all(procs, grace: float = 20.0) -> None:
    for p in procs:
        if p.poll() is None:
            p.terminate()
    end = time.time() + grace
    for p in procs:
        try:
            p.wait(timeout=max(0.1, end - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def _wait_all(procs, timeout: float, what: str, on_poll=None) -> int:
    """Wait for every child; the first non-zero exit (or the timeout) stops
    the others.  Returns 0, the failing code, or 124."""
    deadline = time.time() + timeout
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                print(f"bench: a {what} process exited with {rc}; stopping the others", file=sys.stderr, flush=True)
                break
            if all(c == 0 for c in codes):
                return 0
            if time.time() > deadline:
                print(f"bench: {what} processes timed out", file=sys.stderr, flush=True)
                rc = 124
                break
            if on_poll is not None:
                on_poll()
            time.sleep(0.1)
    finally:
        _stop_all(procs)
    return rc


def _read_json(path: str):
    try:
        with open(path) as f:
            return json.loads(f.read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError):
        return None


def _headline(a, argv, work: str) -> tuple[int, dict | None]:
    """Phase 1.  Self-launch: N rank children.  Under torchrun: this
    process's own rank child (the others are started by their torchrun peers)."""
    out = os.path.join(work, "headline.json")
    child = [x for x in argv]
    child += ["--json-out", out]
    if "RANK" in os.environ:
        rank, world = int(os.environ["RANK"]), int(os.environ.get("WORLD_SIZE", "1"))
        if world != a.gpus:
            print(json.dumps({"error": f"--gpus {a.gpus} but WORLD_SIZE={world}"}), flush=True)
            return 2, None
        # a port of its own (the torchrun agent store keeps MASTER_PORT)
        port = int(os.environ.get("MASTER_PORT", "29500")) + 11
        local = int(os.environ.get("LOCAL_RANK", str(rank)))
        procs = [_spawn(child, _child_env("rank", rank, world, port, local))]
    else:
        port = _free_port()
        procs = [_spawn(child, _child_env("rank", r, a.gpus, port)) for r in range(a.gpus)]
    rc = _wait_all(procs, a.launch_timeout, "rank")
    if "RANK" in os.environ and int(os.environ["RANK"]) != 0:
        head = _read_json(f"{out}.rank{os.environ['RANK']}")
        # another torchrun rank: its child leaves a marker once the headline is measured;
        # a failure after that is reported by rank 0's line, not by this exit code
        # (a non-zero exit would make torchrun tear down rank 0's launcher and its line)
        return (0 if rc and head is not None else rc), None
    head = _read_json(out)
    if rc and head is not None:
        # the headline was measured and written before a rank failed / hung in an extra
        head["extras_error"] = (head.get("extras_error", "") +
                                f"; headline ranks failed or timed out after the headline (rc={rc})").lstrip("; ")
        head["headline_ranks_rc"] = rc
    return rc, head


def _system_phase(a, work: str) -> dict:
    """Phase 2: the runtime with N node processes (single job + two jobs)."""
    out = os.path.join(work, "system.json")
    port = _free_port()
    argv = _phase_argv(a, "system", out, work)
    procs = [_spawn(argv, _child_env("node", r, a.gpus, port)) for r in range(a.gpus)]
    rc = _wait_all(procs, min(a.extras_timeout, getattr(a, "phase_deadline", float("inf")) - time.time()),
                   "system-node")
    d = _read_json(out)
    if d is None:
        return {"extras_error": f"system phase failed (rc={rc})"}
    return d


def _kill_phase(a, work: str, phase: str, tag: str, extra: list, driver: int) -> dict:
    """Phases 3-4: max(N, 2) node processes; the driving node writes a marker
    naming the rank to SIGKILL (the coordinator, or a worker holding chunks)
    and the launcher kills that process at once and stamps the time."""
    sub = os.path.join(work, tag)
    os.makedirs(sub, exist_ok=True)
    out = os.path.join(sub, "out.json")
    n = max(a.gpus, 2)
    port = _free_port()
    argv = _phase_argv(a, phase, out, sub) + extra
    procs = [_spawn(argv, _child_env("node", r, n, port, local=r % a.gpus)) for r in range(n)]
    marker, killed = os.path.join(sub, "kill_now"), os.path.join(sub, "killed_at")
    state = {"done": False}

    def poll():
        if not state["done"] and os.path.exists(marker):
            try:
                with open(marker) as f:
                    victim = int(f.read().strip() or "0")
            except (OSError, ValueError):
                return                                    # being written
            procs[victim].send_signal(signal.SIGKILL)
            t = time.time()
            with open(killed + ".tmp", "w") as f:
                f.write(repr(t))
            os.replace(killed + ".tmp", killed)
            state["done"] = True

    drv = procs[driver % n]
    t_phase = time.time()
    deadline = min(time.time() + a.extras_timeout, getattr(a, "phase_deadline", float("inf")))
    try:
        while time.time() < deadline:
            poll()
            if drv.poll() is not None:                     # the driver wrote its result and left
                break
            if any(p.poll() not in (None, 0, -signal.SIGKILL) for p in procs):
                break
            time.sleep(0.02)
    finally:
        _stop_all(procs)
    print(f"bench: {tag} phase {time.time() - t_phase:.1f} s (driver rc={drv.returncode})", file=sys.stderr,
          flush=True)
    d = _read_json(out)
    if d is None:
        return {"extras_error": f"{tag} phase failed (driver rc={drv.returncode})"}
    return d


def _failover_phase(a, work: str) -> dict:
    """Phase 3: SIGKILL the coordinator mid-job, timed by the standby.  First
    with the reference's detector (0.3 s ping / 2 s timeout,
    mp4_machinelearning.py:191-220, 845-851), then with the tuned one
    (0.1 s / 1 s) as ``coord_failover_tuned_*`` keys."""
    d = _kill_phase(a, work, "failover", "failover_ref", ["--detector", "reference"], driver=-1)
    if "extras_error" in d:
        return d
    if getattr(a, "phase_deadline", float("inf")) - time.time() < 20.0:
        return d                                          # out of extras budget: the reference-detector run only
    t = _kill_phase(a, work, "failover", "failover_tuned", ["--detector", "tuned"], driver=-1)
    if "extras_error" in t:
        d["extras_error"] = t["extras_error"]
        return d
    for k in ("coord_failover_recovery_s", "coord_failover_detect_s", "coord_failover_all_done_s",
              "coord_failover_images_exact", "coord_failover_failure_timeout_s", "coord_failover_heartbeat_s"):
        d[k.replace("coord_failover_", "coord_failover_tuned_")] = t.get(k)
    return d


def _worker_failover_phase(a, work: str) -> dict:
    """Phase 4 (report Fig 4): a worker paused while k of its chunks are in
    flight is SIGKILLed; the coordinator times detection (reference 0.3 s /
    2 s detector), re-dispatch to the survivors and the last re-run chunk's
    result, for k in 1, 4, 8 (one cluster per k)."""
    out = {}
    rec = {}
    for k in a.worker_kill_chunks:
        if getattr(a, "phase_deadline", float("inf")) - time.time() < 20.0:
            break                                         # out of extras budget: report what ran
        d = _kill_phase(a, work, "worker", f"worker_k{k}", ["--kill-chunks", str(k)], driver=0)
        if "extras_error" in d:
            if not rec:
                return d
            out["extras_error"] = d["extras_error"]         # report the k that ran, and the failure
            break
        rec[str(k)] = d
    if not rec:
        return {"extras_error": "worker failover: out of extras budget"}
    first = next(iter(rec.values()))
    out["worker_failover_recovery_s"] = {k: v["recovery_s"] for k, v in rec.items()}
    out["worker_failover_detect_s"] = {k: v["detect_s"] for k, v in rec.items()}
    out["worker_failover_chunks_on_victim"] = {k: v["chunks_on_victim"] for k, v in rec.items()}
    out["worker_failover_images_exact"] = all(v["images_exact"] for v in rec.values())
    out["worker_failover_nodes"] = first["nodes"]
    out["worker_failover_rounds"] = first["rounds"]
    out["worker_failover_survivor_world"] = {k: v.get("survivor_world") for k, v in rec.items()}
    out["worker_failover_failure_timeout_s"] = first["failure_timeout_s"]
    out["worker_failover_ref_s"] = {k: BASELINE_WORKER_RECOVERY_S.get(int(k)) for k in rec}
    return out


def _phase_argv(a, phase: str, out: str, work: str) -> list:
    argv = ["--gpus", str(a.gpus), "--steps", str(a.steps), "--warmup", str(a.warmup), "--model", a.model,
            "--worker-kill-chunks", ",".join(str(k) for k in a.worker_kill_chunks),
            "--dtype", a.dtype, "--fp32-impl", a.fp32_impl, "--batch", str(a.batch), "--seed", str(a.seed),
            "--two-job-queries", str(a.two_job_queries), "--failover-queries", str(a.failover_queries),
            "--ref-delay-queries", str(a.ref_delay_queries),
            "--sdfs-images", str(a.sdfs_images), *(["--sdfs-trace", a.sdfs_trace] if a.sdfs_trace else []),
            "--phase", phase, "--json-out", out, "--work-dir", work, "--launch-timeout", str(a.extras_timeout)]
    if a.dry_run:
        argv.append("--dry-run")
    if a.rehearse_gloo:
        argv.append("--rehearse-gloo")
    if a.rehearse_rccl:
        argv.append("--rehearse-rccl")
    return argv


def launcher(a, argv) -> int:
    work = tempfile.mkdtemp(prefix="idunno_bench_")
    try:
        if a.system:                                      # phase 2 only
            d = _system_phase(a, work)
            line = json.dumps(d)
            print(line, flush=True)
            if a.json_out:
                with open(a.json_out, "w") as f:
                    f.write(line + "\n")
            return 0 if "extras_error" not in d else 1
        rc, head = _headline(a, [x for x in argv if x not in ("--json-out",)], work)
        if head is None:
            if rc and ("RANK" not in os.environ or int(os.environ["RANK"]) == 0):
                print(json.dumps({"metric": METRIC, "value": None, "n_gpus": a.gpus, "steps": a.steps,
                                  "warmup": a.warmup, "higher_is_better": True,
                                  "error": f"headline ranks failed (rc={rc}) before the headline was measured"}),
                      flush=True)
            return rc                                     # 0 for a torchrun rank other than 0
        if not a.no_system and not rc:                    # (a failed headline rank: no node phases on that box)
            t0 = time.time()
            skipped = []
            want = set(a.node_phases.split(","))
            for key, name, fn in (("system", "system", _system_phase), ("failover", "failover", _failover_phase),
                                  ("worker", "worker failover", _worker_failover_phase)):
                if key not in want:
                    continue
                left = a.extras_budget - (time.time() - t0)
                if left < 20.0:
                    skipped.append(name)
                    continue
                a.phase_deadline = time.time() + left
                tp = time.time()
                try:
                    d = fn(a, work)
                except Exception as e:  # noqa: BLE001
                    d = {"extras_error": f"{name}: {type(e).__name__}: {e}"}
                head.setdefault("phase_wall_s", {})[name] = round(time.time() - tp, 1)
                err = d.pop("extras_error", None)
                if err:
                    head["extras_error"] = (head.get("extras_error", "") + "; " + err).lstrip("; ")
                head.update(d)
            head["extras_wall_s"] = round(time.time() - t0, 1)
            if skipped:
                head["extras_skipped"] = skipped
        line = json.dumps(head)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
        return 0
    finally:
        shutil.rmtree(work, ignore_errors=True)


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    role = os.environ.get(ROLE)
    if a.rehearse_rccl and role in ("rank", "node"):
        # before any RCCL communicator: a host id of this process's own (see --rehearse-rccl)
        os.environ["NCCL_HOSTID"] = f"idunno-rehearse-{os.getpid()}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    if (a.rehearse_rccl or a.rehearse_gloo) and role in ("rank", "node") and a.gpus > 4:
        # before the HIP runtime starts: N rank processes on ONE GPU with HIP's 4 hardware
        # queues each oversubscribe the card's queue slots, and the scheduler then
        # time-slices queues while RCCL kernels spin waiting for peers (VERDICT r5 item 1:
        # 8 ranks, gather 14.5 ms per round with 4 queues, 0.4 ms with 1,
        # profiles/r6_rehearse_n8.md).  One GPU per rank never shares its queues.
        os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("IDUNNO_REHEARSE_HW_QUEUES", "1")
    if role == "rank":
        return run_rank(a)
    if role == "node":
        return run_node(a)
    # strip a --json-out the caller gave: the launcher writes the merged line there
    clean, skip = [], False
    for x in argv:
        if skip:
            skip = False
            continue
        if x == "--json-out":
            skip = True
            continue
        if x.startswith("--json-out="):
            continue
        clean.append(x)
    return launcher(a, clean)


# ---------------------------------------------------------------------------
# phase 1: one headline rank
# ---------------------------------------------------------------------------

class FakeRunner:
    """--dry-run forward: class = global image index % 1000, prob 0.5."""

    def __init__(self, device):
        self.device = device

    def window(self, dataset, batch, start, packed):
        import torch

        def run():
            s = int(start.item())
            idx = torch.arange(s, s + batch, dtype=torch.int32)
            packed[:batch, 0].copy_(idx % 1000)
            packed[:batch, 1].copy_(torch.full((batch,), 0.5).view(torch.int32))
        return run


def run_rank(a) -> int:
    import numpy as np
    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from idunno.parallel.dataplane import QueryPlane, init_from_env
    from idunno.runtime.jobstate import JobState
    from idunno.runtime.scheduler import split_range

    if (a.rehearse_gloo or a.rehearse_rccl) and not a.dry_run:
        # rehearsal of the N > 1 path on a box with fewer GPUs than ranks (see --rehearse-gloo/-rccl)
        os.environ["LOCAL_RANK"] = str(int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
    t_rank0 = time.perf_counter()
    # collectives time out well inside the launcher's limit (a dead peer must not hang a rank
    # past it: the launcher then prints the line rank 0 already wrote)
    env = init_from_env(backend="gloo" if (a.dry_run or a.rehearse_gloo) else None, cpu=a.dry_run,
                        timeout_s=min(120.0, max(30.0, a.launch_timeout / 3)))
    if env.world != a.gpus:
        print(json.dumps({"error": f"--gpus {a.gpus} but WORLD_SIZE={env.world}"}), flush=True)
        return 2
    if not a.dry_run and env.device.type != "cuda":
        print(json.dumps({"error": "bench.py needs a GPU (MI355X); use --dry-run on CPU"}), flush=True)
        return 2
    gpu = env.device.type == "cuda"
    coord = env.rank == 0
    W = env.world
    B = a.batch
    strong_chunk = -(-QUERY // W)
    # every rank holds a replica of the synthetic dataset (SDFS replication
    # factor = world): any chunk of a query can be served by any rank
    D = max(a.dataset_images, (W + 1) * B)

    poll = a.host_wait == "poll" or (a.host_wait == "auto" and W > 1)

    def wait_ev(ev):
        """The host waits for a recorded event: HIP's synchronize spins a CPU; the
        poll mode sleeps between queries (N rank processes on a box whose CPU
        share the RCCL proxy threads need too)."""
        if ev is None:
            return
        if not poll:
            ev.synchronize()
            return
        while not ev.query():
            time.sleep(50e-6)

    def sync():
        if gpu:
            if poll:
                ev = torch.cuda.Event()
                ev.record()
                wait_ev(ev)
            torch.cuda.synchronize()

    def barrier():
        if env.distributed:
            dist.barrier()
        sync()

    if a.dry_run:
        dataset = None
    else:
        from idunno import ops
        dataset = ops.synth_images(a.seed + 1234, 0, D, env.device)

    plane = QueryPlane(env, coordinator=0, max_chunk=max(B, strong_chunk), nbuf=2)
    start_dev, send = plane.row_start(), plane.send_buffer
    model_id = 1 if a.model.startswith("resnet") else 0

    def make_run(runner, batch):
        if runner is None:
            r = FakeRunner(env.device).window(dataset, batch, start_dev, send)
            return lambda q: r()
        if a.no_graph:
            return lambda q: runner.forward(dataset, start_dev, batch, 0, send)
        _, run = runner.capture_window(dataset, batch, start=start_dev, start_offset=0, packed=send)
        return lambda q: run()

    def make_slot_runs(runner, batch):
        """Pipelined variant (N > 1): one captured forward per descriptor/result
        slot of the double-buffered plane, so round q+1's descriptor broadcast
        and round q's gather run on the RCCL stream under the other slot's
        forward."""
        runs = []
        for slot in range(2):
            st, pk = plane.row_start_slot(slot), plane.send_slot(slot)
            if runner is None:
                runs.append(FakeRunner(env.device).window(dataset, batch, st, pk))
            elif a.no_graph:
                runs.append(lambda st=st, pk=pk: runner.forward(dataset, st, batch, 0, pk))
            else:
                runs.append(runner.capture_window(dataset, batch, start=st, start_offset=0, packed=pk)[1])
        return lambda q: runs[q % 2]()

    def make_scatter_run(runner, batch, per_round):
        """M9 data variant: the images live only in the coordinator's HBM.
        Round q's chunks are scattered to the ranks (grouped P2P, RCCL over
        xGMI) into one of two receive buffers while round q-1 computes on the
        other; each rank's captured forward reads its receive buffer."""
        shape = (batch, 224, 224, 3) if not a.dry_run else (batch, 4, 4, 3)
        bufs = [torch.zeros(shape, dtype=torch.uint8, device=env.device) for _ in range(2)]
        src = dataset if not a.dry_run else (torch.zeros((D,) + shape[1:], dtype=torch.uint8) if coord else None)
        if runner is None:
            fakes = [FakeRunner(env.device).window(dataset, batch, start_dev, send) for _ in range(2)]
        else:
            fakes = []
            for b in bufs:
                st0, rep = runner.capture_window(b, batch, packed=send)
                st0.zero_()
                fakes.append(rep)
        posted = {}

        def chunks_of(q):
            off = (q * per_round) % (D - max(per_round, plane.max_chunk) + 1)
            return split_range(off, off + per_round - 1, W)

        def run(q):
            if q not in posted:
                posted[q] = plane.scatter_async(src, chunks_of(q), bufs[q % 2])
            # round q+1's scatter goes on the RCCL stream BEFORE round q's forward is
            # queued: it waits only for round q-1 (the last reader of its buffer)
            posted[q + 1] = plane.scatter_async(src, chunks_of(q + 1), bufs[(q + 1) % 2])
            plane.wait_scatter(posted.pop(q))
            fakes[q % 2]()

        def finish():
            for reqs in posted.values():
                plane.wait_scatter(reqs)
            posted.clear()
        return run, finish

    def record_round(state, res, tab, t1):
        """Coordinator: one gathered round (host int32 [W, max_chunk, 2]) into the job state."""
        cls_all, prob_all = res[:, :, 0], res[:, :, 1].view(np.float32)
        for r, row in enumerate(tab):
            n = row[3] - row[2] + 1
            state.record_result(a.model, row[1], f"rank{r}", row[2], row[3], cls_all[r, :n].copy(),
                                prob_all[r, :n].copy(), t1)

    def table_of(q, per_round):
        """Round q's chunks (one per rank) and descriptor rows."""
        off = (q * per_round) % (D - max(per_round, plane.max_chunk) + 1)
        chunks = split_range(off, off + per_round - 1, W)
        return chunks, [(model_id, q, s, e) for s, e in chunks]

    def fail_on_purpose(q, warmup):
        if a.fail_rank == env.rank and q == warmup:
            print(f"bench: rank {env.rank} failing on purpose (--fail-rank)", file=sys.stderr, flush=True)
            os._exit(3)

    def run_phases(step, drain, lat, steps, warmup, timing=None, cpu_stats=None):
        """Warmup rounds, then EXACTLY ``steps`` timed rounds (each rank's own
        region between a drain + barrier on both sides; the slowest rank's
        counts), then >= 5 unloaded rounds one at a time for the p50 latency.
        ``step(q, nxt)``: round q, with round q+1 to follow in this phase."""
        for q in range(warmup):
            step(q, q + 1 < warmup)
        drain()
        lat.clear()
        if timing is not None:
            timing[0] = True
        cg0 = _cgroup_cpu() if coord else None
        c_start = _proc_cpu_s()
        t_start = time.perf_counter()
        for q in range(warmup, warmup + steps):
            step(q, q + 1 < warmup + steps)
        drain()
        elapsed = time.perf_counter() - t_start
        cpu = _proc_cpu_s() - c_start
        cg1 = _cgroup_cpu() if coord else None
        if timing is not None:
            timing[0] = False
        per_rank, cpu_rank = [elapsed], [cpu]
        if env.distributed:
            t = torch.tensor([elapsed, cpu], dtype=torch.float64, device=env.device)
            outs = [torch.zeros_like(t) for _ in range(W)]
            dist.all_gather(outs, t)
            per_rank = [float(x[0].item()) for x in outs]
            cpu_rank = [float(x[1].item()) for x in outs]
            elapsed = max(per_rank)
        if cpu_stats is not None:
            cpu_stats[:] = [cpu_rank, _cgroup_delta(cg0, cg1, elapsed)]
        p50_loaded = statistics.median(lat) if lat else None
        lat.clear()
        for q in range(warmup + steps, warmup + steps + max(5, min(steps, 20))):
            step(q, False)
            drain()
        p50 = statistics.median(lat) if lat else None
        return elapsed, per_rank, p50_loaded, p50

    def measure(run, per_round: int, steps: int, warmup: int, label: str, pipelined: bool = False, runner=None):
        """Time `steps` pipelined rounds of `per_round` images (split over the
        ranks), then `unloaded` rounds one at a time for the p50 latency.

        ``pipelined`` (``run`` from ``make_slot_runs``): round q alternates
        between the plane's two slots; the broadcast of round q+1's
        descriptors is posted before round q's forward and round q's gather
        is waited for only after round q+1's forward is queued, so at N > 1
        neither collective sits between two forwards on the compute stream.
        Otherwise both collectives sit between the forwards (and the gather is
        timed: ``gather_us``)."""
        state = JobState() if coord else None
        host = [torch.empty(W, plane.max_chunk, 2, dtype=torch.int32, pin_memory=gpu) for _ in range(2)] \
            if coord else None
        lat, pending = [], []
        step, drain, gtimes, timing = (pipelined_round if pipelined else serial_round)(
            run, per_round, warmup, state, host, lat, pending)
        cpu_stats = []
        elapsed, per_rank, p50_loaded, p50 = run_phases(step, drain, lat, steps, warmup, timing, cpu_stats)
        g_us = ([1000.0 * g0.elapsed_time(g1) for g0, g1 in gtimes] if gpu else [1e6 * x for x in gtimes]) \
            if gtimes else []
        recorded = state.images_done(a.model) if coord else None
        return {"elapsed": elapsed, "ips": per_round * steps / elapsed, "p50": p50, "p50_loaded": p50_loaded,
                "recorded": recorded, "label": label,
                "rank_ms": [1000.0 * x / steps for x in per_rank],
                "cpu": cpu_stats,
                "gather_us": statistics.median(g_us) if g_us else None,
                "verified": verify(state, runner)}

    ahead = {}      # poll mode: round -> event after its forward (the host queues <= 2 rounds ahead)

    def throttle_before(q: int) -> None:
        if poll and gpu:
            wait_ev(ahead.pop(q - 2, None))

    def mark_after(q: int) -> None:
        if poll and gpu:
            ev = torch.cuda.Event()
            ev.record()
            ahead[q] = ev

    def serial_round(run, per_round, warmup, state, host, lat, pending):
        """Round q: descriptor broadcast, forward, gather, one after another on
        the compute stream; the coordinator copies the round to pinned memory
        and ingests the round before it."""
        gtimes = []            # (start, end) CUDA events / host seconds around each timed round's gather
        timing = [False]

        def ingest():
            ev, table, slot, t0 = pending.pop(0)
            wait_ev(ev)
            record_round(state, host[slot].numpy(), table, time.perf_counter())
            lat.append(time.perf_counter() - t0)

        def step(q: int, nxt: bool):
            t0 = time.perf_counter()
            throttle_before(q)
            table = None
            if coord:
                chunks, table = table_of(q, per_round)
                state.assign(a.model, q, [(f"rank{r}", s, e) for r, (s, e) in enumerate(chunks)], t0)
            plane.dispatch_device(table, slot=q)
            fail_on_purpose(q, warmup)
            run(q)
            if timing[0] and gpu:
                g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                g0.record()
                plane.gather(None, None)
                g1.record()
                gtimes.append((g0, g1))
            elif timing[0]:
                g0 = time.perf_counter()
                plane.gather(None, None)
                gtimes.append(time.perf_counter() - g0)
            else:
                plane.gather(None, None)
            mark_after(q)
            if coord:
                slot = q % 2
                host[slot].copy_(plane.gathered_all, non_blocking=gpu)
                ev = None
                if gpu:
                    ev = torch.cuda.Event()
                    ev.record()
                if pending:
                    ingest()
                pending.append((ev, table, slot, t0))

        def drain():
            if coord:
                while pending:
                    ingest()
            ahead.clear()
            barrier()
        return step, drain, gtimes, timing

    def pipelined_round(run, per_round, warmup, state, host, lat, pending):
        """Round q on slot q % 2 of the double-buffered plane (see ``measure``)."""
        posted, gathers, t0s, tables = {}, [], {}, {}

        def post(q):
            tab = None
            if coord:
                tables[q] = table_of(q, per_round)
                tab = tables[q][1]
            posted[q] = plane.post_dispatch(tab, slot=q % 2, hslot=q)

        def ingest():
            ev, q = pending.pop(0)
            wait_ev(ev)
            record_round(state, host[q % 2].numpy(), tables.pop(q)[1], time.perf_counter())
            lat.append(time.perf_counter() - t0s.pop(q))

        def finish_gather():
            """The compute stream waits for the oldest posted gather; the
            coordinator copies that round to the host and ingests the round
            before it (whose copy has had a forward's time to land)."""
            q, work = gathers.pop(0)
            plane.wait_work(work)
            if coord:
                host[q % 2].copy_(plane.gathered_slot(q % 2), non_blocking=gpu)
                ev = None
                if gpu:
                    ev = torch.cuda.Event()
                    ev.record()
                if pending:
                    ingest()
                pending.append((ev, q))

        def step(q: int, nxt: bool):
            t0s[q] = time.perf_counter()
            throttle_before(q)
            if q not in posted:
                post(q)
            if coord:
                chunks, _ = tables[q]
                state.assign(a.model, q, [(f"rank{r}", s, e) for r, (s, e) in enumerate(chunks)], t0s[q])
            if nxt:
                post(q + 1)          # RCCL stream: waits only for round q-1 (last reader of slot (q+1)%2)
            plane.wait_work(posted.pop(q))
            fail_on_purpose(q, warmup)
            run(q)
            if gathers:
                finish_gather()      # round q-1's gather ran under round q's forward
            gathers.append((q, plane.post_gather(q % 2)))
            mark_after(q)

        def drain():
            while gathers:
                finish_gather()
            if coord:
                while pending:
                    ingest()
            ahead.clear()
            barrier()
        return step, drain, [], None

    def verify(state, runner=None) -> bool | None:
        """Every recorded chunk holds the classes of ITS images, i.e. no slot
        mix-up between the descriptors, the forwards and the gathered rounds.
        --dry-run: all chunks against the fake forward (global index % 1000).
        GPU: the coordinator recomputes the last timed round's chunks of up to
        three ranks (its own, rank 1, the last) with an eager forward over the
        same images of its replica and compares classes (probabilities to 1e-6)."""
        if not coord:
            return None
        with state.lock:
            chunks = [c for v in state.results.values() for c in v]
        if a.dry_run:
            return bool(chunks) and all(
                np.array_equal(c.cls, np.arange(c.start, c.end + 1) % 1000) for c in chunks)
        if runner is None or not chunks:
            return None
        last = max(chunks, key=lambda c: c.start)
        key = next(k for k, v in state.results.items() if any(c is last for c in v))
        pick = {f"rank{r}" for r in {0, 1, W - 1}}
        ok = True
        for c in state.results[key]:
            if c.worker not in pick:
                continue
            n = c.end - c.start + 1
            st0 = torch.tensor([c.start], dtype=torch.int64, device=env.device)
            cls, prob = runner.forward(dataset, st0, n, 0)
            torch.cuda.synchronize()
            ok &= bool(np.array_equal(cls.cpu().numpy(), c.cls)) and \
                bool(np.allclose(prob.cpu().numpy(), c.prob, rtol=0, atol=1e-6))
        return ok

    # ---- headline: weak scaling at the headline precision --------------------
    runner = None
    if not a.dry_run:
        from idunno.models import HipRunner, build_program, program_flops
        runner = HipRunner(build_program(a.model, seed=a.seed, dtype=a.dtype), env.device)
        runner.split = a.fp32_impl == "split"
    pipe = W > 1 and not a.no_pipeline

    def make(r, batch):
        return make_slot_runs(r, batch) if pipe else make_run(r, batch)

    def progress(what: str) -> None:
        """One line per finished phase on stderr (rank 0): long multi-rank runs
        show where they are."""
        if coord:
            print(f"bench: rank 0 {what} ({time.perf_counter() - t_rank0:.1f} s)", file=sys.stderr, flush=True)

    progress("model ready")
    head = measure(make(runner, B), W * B, a.steps, a.warmup, "weak", pipelined=pipe, runner=runner)
    progress("headline measured")
    extras = {"pipelined_collectives": pipe}
    t_extras = time.perf_counter()
    skipped = []

    def emit() -> None:
        """Rank 0 writes the line as it stands (atomically): first right after the
        headline, then after every extra -- a rank that dies or hangs in an extra
        cannot take the headline with it (the launcher prints the last line).
        The other ranks write a marker that their headline is done."""
        if not a.json_out:
            return
        line = json.dumps(headline_line(a, W, B, head, extras, runner, env, dist, serial) if coord else
                          {"rank": env.rank, "headline_done": True})
        path = a.json_out if coord else f"{a.json_out}.rank{env.rank}"
        with open(path + ".tmp", "w") as f:
            f.write(line + "\n")
        os.replace(path + ".tmp", path)

    def budget_left(name: str) -> bool:
        ok = time.perf_counter() - t_extras < a.rank_extras_budget
        if not ok:
            skipped.append(name)
            extras["rank_extras_skipped"] = skipped
        return ok

    serial = None
    emit()
    if a.fail_after_headline == env.rank:
        print(f"bench: rank {env.rank} failing after the headline on purpose", file=sys.stderr, flush=True)
        os._exit(3)
    if a.hang_in_extras == env.rank:
        print(f"bench: rank {env.rank} hanging in the extras on purpose", file=sys.stderr, flush=True)
        time.sleep(3600)
    if pipe and budget_left("serial collectives"):
        # the same rounds with the broadcast and gather between the forwards on the
        # compute stream: what the pipelining saves, and the gather's own time
        serial = measure(make_run(runner, B), W * B, a.steps, a.warmup, "weak-serial")
        extras.update({"value_serial_collectives": round(serial["ips"], 2),
                       "ms_per_step_serial_collectives": round(1000 * serial["elapsed"] / a.steps, 4)})
        emit()
    if not a.no_extras:
        if budget_left("strong scaling"):
            # strong scaling: ONE 400-image query split over the W ranks
            strong = measure(make(runner, strong_chunk), QUERY, a.steps, a.warmup, "strong", pipelined=pipe)
            progress("strong scaling measured")
            extras.update({
                "images_per_s_strong": round(strong["ips"], 2),
                "p50_query_latency_strong_s": round(strong["p50"], 6) if strong["p50"] else None,
                "strong_chunk_per_gpu": strong_chunk,
            })
            emit()
        if not a.dry_run and budget_left("other precision"):
            other = "fp16" if a.dtype == "fp32" else "fp32"
            r2 = HipRunner(build_program(a.model, seed=a.seed, dtype=other), env.device)
            m2 = measure(make_run(r2, B), W * B, a.steps, a.warmup, other)
            extras.update({f"value_{other}": round(m2["ips"], 2),
                           f"ms_per_step_{other}": round(1000 * m2["elapsed"] / a.steps, 4),
                           f"p50_query_latency_{other}_s": round(m2["p50"], 6) if m2["p50"] else None})
            del r2
            progress(f"{other} measured")
            emit()
        if not a.dry_run and a.dtype == "fp32" and budget_left("other fp32 kernels"):
            alt = "f32mfma" if a.fp32_impl == "split" else "split"
            runner.split = alt == "split"
            m3 = measure(make_run(runner, B), W * B, a.steps, a.warmup, alt)
            runner.split = a.fp32_impl == "split"
            extras.update({f"value_fp32_{alt}": round(m3["ips"], 2),
                           f"ms_per_step_fp32_{alt}": round(1000 * m3["elapsed"] / a.steps, 4)})
            emit()
        if not a.dry_run and budget_left("numerics"):
            if coord:
                extras.update(numerics_check(runner, a, env.device))
            progress("numerics checked")
            emit()
        if not a.dry_run and W == 1 and a.model == "resnet18" and a.dtype == "fp32" and budget_left("b50"):
            extras.update(b50_extra(a, env, runner, dataset))
            progress("b50 forward measured")
            emit()
        if not a.dry_run and W == 1 and a.model == "resnet18" and budget_left("alexnet"):
            extras.update(alexnet_extra(a, env))
            progress("alexnet measured")
            emit()
        if not a.dry_run and W == 1 and a.model == "resnet18" and budget_left("resnet50"):
            extras.update(resnet50_extra(a, env, make_run))
            progress("resnet50 measured")
            emit()
        if W > 1 and not a.rehearse_gloo and budget_left("scatter"):
            # last and bounded: the only extra whose collective never ran on RCCL before round 5
            # (a rehearsal skips it: gloo moves GPU tensors point-to-point through the host)
            # M9 data variant: images only in the coordinator's HBM,
            # scattered every round over RCCL (bucketed over the peers), double-buffered
            srun, sfinish = make_scatter_run(runner, B, W * B)
            sc = measure(srun, W * B, a.steps, a.warmup, "scatter")
            sfinish()
            extras.update({"images_per_s_scatter": round(sc["ips"], 2),
                           "ms_per_step_scatter": round(1000 * sc["elapsed"] / a.steps, 4),
                           "scatter_mb_per_round": round((W - 1) * B * 150528 / 1e6, 1)})
            emit()
    extras["rank_extras_wall_s"] = round(time.perf_counter() - t_extras, 1)
    emit()
    if env.distributed:
        dist.barrier()
        dist.destroy_process_group()
    return 0





def _proc_cpu_s() -> float:
    """CPU seconds of this process, every thread (RCCL proxy, watchdog) included."""
    import resource

    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime + r.ru_stime


def _cgroup_cpu() -> dict | None:
    """cgroup v2 CPU accounting of the container (every rank of this box):
    usage and CFS-quota throttling counters, plus the quota itself."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            st = {k: int(v) for k, v in (ln.split() for ln in f if ln.strip())}
    except (OSError, ValueError):
        return None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        st["quota_cpus"] = None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        st["quota_cpus"] = None
    return st


def _cgroup_delta(c0, c1, wall: float) -> dict:
    if not c0 or not c1:
        return {}
    d = {"cgroup_cpus_used": round((c1.get("usage_usec", 0) - c0.get("usage_usec", 0)) / 1e6 / wall, 2),
         "cgroup_quota_cpus": c1.get("quota_cpus")}
    if "nr_throttled" in c1:
        d["cgroup_throttled_periods"] = c1["nr_throttled"] - c0.get("nr_throttled", 0)
        d["cgroup_throttled_ms"] = round((c1.get("throttled_usec", 0) - c0.get("throttled_usec", 0)) / 1e3, 1)
    return d


def _cpu_keys(head: dict, a) -> dict:
    """Host CPU use of the timed headline region: every rank process's CPU
    seconds per wall second (summed), and the container cgroup's usage and
    quota throttling.  At N ranks on ONE box (rehearsals) the ranks and their
    RCCL proxy threads share the box's CPU share."""
    st = head.get("cpu") or []
    if not st:
        return {}
    cpu_rank, cg = st
    wall = head["elapsed"]
    mode = a.host_wait if a.host_wait != "auto" else ("poll" if a.gpus > 1 else "spin")
    hwq = os.environ.get("GPU_MAX_HW_QUEUES")
    return {"host_wait": mode, **({"gpu_max_hw_queues": int(hwq)} if hwq and hwq.isdigit() else {}), "host_cpus_used_by_ranks": round(sum(cpu_rank) / wall, 2),
            "host_cpu_per_rank_max": round(max(cpu_rank) / wall, 2), **cg}


def headline_line(a, W, B, head, extras, runner, env, dist, serial) -> dict:
    """The bench line (rank 0) from the headline measurement and the extras so far."""
    import torch

    ips = head["ips"]
    p50 = head["p50"]
    headline = a.model == "resnet18" and B == QUERY
    out = {
        "metric": METRIC if headline else
        f"images/sec (whole node) + p50 query latency, {a.model} bs={B} at {W} GPU",
        "value": round(ips, 2),
        "unit": "images/sec",
        "n_gpus": W,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(1000 * head["elapsed"] / a.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(ips / BASELINE_IMG_PER_S, 2) if headline else None,
        "dtype": "fp32" if a.dry_run else a.dtype,
        "data": "synthetic uint8 224x224x3 images (dataset replicated in every GPU's HBM), random-init weights",
        "config": {"model": a.model, "global_batch": W * B, "seq_len": None, "image_hw": 224,
                   "batch_per_gpu": B, "parallelism": f"dp{W}", "graph": not a.no_graph,
                   "fp32_impl": a.fp32_impl if a.dtype == "fp32" else None,
                   "compute": (COMPUTE_SPLIT if a.fp32_impl == "split" else COMPUTE_F32) if a.dtype == "fp32" else
                   "f16 MFMA, fp16 activations, fp32 accumulate",
                   "dry_run": a.dry_run},
        "p50_query_latency_s": round(p50, 6) if p50 else None,
        "p50_query_latency_loaded_s": round(head["p50_loaded"], 6) if head["p50_loaded"] else None,
        "p50_vs_baseline_speedup": round(BASELINE_P50_S / p50, 1) if p50 and headline else None,
        "results_recorded": head["recorded"],
        **({"results_verified": head["verified"]} if head["verified"] is not None else {}),
        # readiness keys: the collective the timed rounds ran on, read from the
        # live process group, the per-rank spread of the step time and the gather's own time
        "comm_backend": (dist.get_backend() if env.distributed else "none (single rank: no collective)"),
        "comm_world": dist.get_world_size() if env.distributed else 1,
        "rccl": bool(env.distributed and dist.get_backend() == "nccl" and torch.version.hip is not None),
        "ms_per_step_rank_min": round(min(head["rank_ms"]), 4),
        "ms_per_step_rank_max": round(max(head["rank_ms"]), 4),
        "gather_us_per_round": (round(serial["gather_us"], 1) if serial and serial["gather_us"] is not None else
                                round(head["gather_us"], 1) if head["gather_us"] is not None else None),
        **_cpu_keys(head, a),
        **extras,
    }
    if runner is not None:
        from idunno.models import program_flops

        out["model_tflops"] = round(program_flops(runner.p) * ips / 1e12, 2)
    return out


def _round_extra(a, env, model: str, batch: int, dtype: str, split: bool, model_id: int, seed_off: int):
    """One model's round loop on this GPU (descriptor, hipGraph replay of the
    forward, top-1 to the host, job-state ingest) at ``batch`` images per step:
    (images/s, ms per step, results recorded)."""
    import torch

    from idunno import ops
    from idunno.models import HipRunner, build_program
    from idunno.parallel.dataplane import QueryPlane
    from idunno.runtime.jobstate import JobState

    ds = ops.synth_images(a.seed + seed_off, 0, 2 * batch, env.device)
    r = HipRunner(build_program(model, seed=a.seed, dtype=dtype), env.device)
    r.split = split
    plane = QueryPlane(env, coordinator=0, max_chunk=batch, nbuf=1)
    _, run = r.capture_window(ds, batch, start=plane.row_start(), start_offset=0, packed=plane.send_buffer)
    state = JobState()
    host = torch.empty(1, batch, 2, dtype=torch.int32, pin_memory=True)

    def step(q):
        off = (q % 2) * batch
        state.assign(model, q, [("rank0", off, off + batch - 1)], time.perf_counter())
        plane.dispatch_device([(model_id, q, off, off + batch - 1)], slot=q)
        run()
        plane.gather(None, None)
        host.copy_(plane.gathered_all)
        state.record_result(model, q, "rank0", off, off + batch - 1, host[0, :, 0].numpy().copy(),
                            host[0, :, 1].view(torch.float32).numpy().copy(), time.perf_counter())

    steps = max(5, min(a.steps, 20))
    for q in range(3):
        step(q)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for q in range(3, 3 + steps):
        step(q)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    recorded = state.images_done(model)
    r.close()
    return batch * steps / el, 1000 * el / steps, recorded


def resnet50_extra(a, env, make_run) -> dict:
    """BASELINE config 5 (ResNet50 bs=1024 fp16) as extra keys of the default line."""
    ips, ms, rec = _round_extra(a, env, "resnet50", 1024, "fp16", False, 2, 99)
    return {"value_resnet50_fp16": round(ips, 2), "ms_per_step_resnet50_fp16": round(ms, 4),
            "resnet50_batch": 1024, "resnet50_results_recorded": rec}


def alexnet_extra(a, env) -> dict:
    """BASELINE config 3's other job (AlexNet, 500-image queries, report p.1) at the
    headline's precision: fp32 via split fp16 (reference alexnet_resnet.py:17-18)."""
    ips, ms, rec = _round_extra(a, env, "alexnet", QUERY_ALEXNET, "fp32", True, 0, 77)
    return {"value_alexnet_b500": round(ips, 2), "ms_per_step_alexnet_b500": round(ms, 4),
            "alexnet_precision": "fp32 (split fp16)", "alexnet_results_recorded": rec}


def b50_extra(a, env, runner, dataset) -> dict:
    """The per-GPU compute of the north-star strong-scaling query: one 400-image
    ResNet18 query over 8 GPUs is a 50-image forward per GPU (reference
    mp4_machinelearning.py:523-536 chunks a query over its workers).  The
    headline runner's split-fp32 hipGraph at B=50, replayed back to back
    between two events (the graph reads its window start on the device)."""
    import torch

    Bs = 50
    st = torch.zeros(1, dtype=torch.int64, device=env.device)
    buf = torch.zeros(Bs, 2, dtype=torch.int32, device=env.device)
    _, run = runner.capture_window(dataset, Bs, start=st, start_offset=0, packed=buf)
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    iters = 200
    e0.record()
    for _ in range(iters):
        run()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / iters
    return {"ms_per_forward_b50": round(ms, 4), "images_per_s_b50": round(Bs / ms * 1e3, 1),
            "b50_precision": "fp32 (split fp16)" if runner.split else "fp32 (f32 MFMA)"}

# ---------------------------------------------------------------------------
# phases 2-3: one node process of the fault-tolerant runtime
# ---------------------------------------------------------------------------

def run_node(a) -> int:
    """One node of the --system / failover measurement (see the docstring)."""
    import torch

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from idunno.config import ClusterConfig
    from idunno.runtime.data import ResidentSource
    from idunno.runtime.executor import FakeExecutor, HipExecutor
    from idunno.runtime.node import Node
    from idunno.runtime.transport import TcpTransport

    if os.environ.get("IDUNNO_BENCH_STACKS"):
        # debugging a stuck phase: every node process dumps all its threads' stacks
        # to stderr every IDUNNO_BENCH_STACKS seconds
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["IDUNNO_BENCH_STACKS"]), repeat=True)
    rank = int(os.environ.get("RANK", "0"))
    n = int(os.environ.get("WORLD_SIZE", "1"))           # node processes (failover: >= 2)
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    gpu = not a.dry_run and torch.cuda.is_available()
    if not a.dry_run and not gpu:
        print(json.dumps({"error": "bench.py phases 2-3 need a GPU (MI355X); use --dry-run on CPU"}), flush=True)
        return 2
    if gpu and (a.rehearse_gloo or a.rehearse_rccl):
        local %= max(1, torch.cuda.device_count())       # N nodes on fewer GPUs (gloo / RCCL-socket rounds)
    dev = torch.device("cuda", local) if gpu else torch.device("cpu")
    if gpu:
        torch.cuda.set_device(dev)
    W = a.gpus
    B = a.batch
    base = int(os.environ.get("MASTER_PORT", "29500")) + 200
    tmp = tempfile.mkdtemp(prefix=f"idunno_bench_r{rank}_")
    # rounds need one GPU per node process (RCCL for n > 1, a one-member group at n = 1);
    # the 1-GPU failover puts 2 nodes on GPU 0 (TCP path)
    rounds = n <= W
    cfg = ClusterConfig(num_nodes=n, base_port=base, store_root=tmp, collective_rounds=rounds, dtype=a.dtype,
                        fp32_impl=a.fp32_impl, max_chunk=max(2048, B), rpc_timeout_s=60.0, worker_budget=W,
                        dataset_size=10 ** 9, collective_port_offset=100,
                        batch_size={"resnet18": QUERY * W, "alexnet": QUERY_ALEXNET * W, a.model: B * W},
                        collective_backend="gloo" if a.rehearse_gloo else "")
    if a.phase in ("failover", "worker"):
        # reference detector: 0.3 s ping period, 2 s timeout (mp4_machinelearning.py:191-220, 845-851);
        # tuned: 0.1 s / 1 s
        if a.detector == "tuned":
            cfg.update(heartbeat_period_s=0.1, failure_timeout_s=1.0, metadata_period_s=0.2)
        else:
            cfg.update(heartbeat_period_s=0.3, failure_timeout_s=2.0, metadata_period_s=0.2)
    if os.environ.get("IDUNNO_BENCH_LOG_DIR"):
        # node logs of every phase kept (debugging a rehearsal): <dir>/<phase tag>/nodeNN.log
        cfg.update(log_dir=os.path.join(os.environ["IDUNNO_BENCH_LOG_DIR"],
                                        os.path.basename((a.work_dir or a.phase).rstrip("/"))))
    name = cfg.node_name(rank)
    ex = FakeExecutor() if a.dry_run else HipExecutor(dev, seed=a.seed, dtype=a.dtype, fp32_impl=a.fp32_impl)
    if not a.dry_run and (a.rehearse_gloo or a.rehearse_rccl) and n > max(1, torch.cuda.device_count()):
        # node processes sharing one GPU: free cached activation blocks of retired chunk
        # sizes early (executor._capture), or eight caches fill the card's 288 GB
        ex.trim_slack_bytes = 2 << 30
    node = Node(cfg, name, TcpTransport(name, cfg.address, cfg.address(name)), ex)
    node.source = None
    if not a.dry_run:
        # the dataset resident in HBM as in the raw loop: the system phase's query
        # ranges generated once before any clock starts (rounds read them in place)
        src = ResidentSource(cfg.data_seed, dev)
        if a.phase == "system" and not os.environ.get("IDUNNO_BENCH_NO_RESIDENT"):
            share = -(-n // max(1, torch.cuda.device_count())) if (a.rehearse_gloo or a.rehearse_rccl) else 1
            want = W * B * (a.warmup + a.steps + max(5, min(a.steps, 20)) + 2)
            src.make_resident(min(want, (32 << 30) // (224 * 224 * 3) // max(1, share)))
        node.source = src
    if not a.dry_run:
        ex.warmup(a.model, B)                           # capture before any clock starts
    if rank != 0:
        _wait_port(cfg.address(cfg.coordinator_name), 120)   # the coordinator listens first
    node.start(join=True)
    driver = (rank == n - 1) if a.phase == "failover" else (rank == 0)
    if not driver:
        t_end = time.time() + a.launch_timeout
        while node.alive_flag and time.time() < t_end:
            time.sleep(0.2)
        node.stop()
        return 0
    try:
        if a.phase == "system":
            res = _drive_system(a, node, W, B)
        elif a.phase == "failover":
            res = _drive_failover(a, node, n)
        else:
            res = _drive_worker_failover(a, node, n)
        with open(a.json_out + ".tmp", "w") as f:
            f.write(json.dumps(res) + "\n")
        os.replace(a.json_out + ".tmp", a.json_out)
        return 0
    finally:
        from idunno.runtime.messages import Type

        if node.rounds is not None and node.is_coordinator:
            node.rounds.release()                       # members leave the epoch cleanly
        for m in node.membership.alive():
            if m != node.name:
                node.transport.send(m, {"t": Type.KILL})
        time.sleep(0.2)
        node.stop()


def _wait_port(addr, timeout: float) -> None:
    end = time.time() + timeout
    while time.time() < end:
        try:
            socket.create_connection(addr, timeout=0.2).close()
            return
        except OSError:
            time.sleep(0.05)


def _wait_progress(node, pred, timeout: float) -> bool:
    """Wait until ``pred()`` holds, woken by the node's result-ingest
    notifications (``Node._progress``), not by polling."""
    end = time.monotonic() + timeout
    with node._progress:
        while not pred():
            left = end - time.monotonic()
            if left <= 0:
                return bool(pred())
            node._progress.wait(min(left, 0.05))
    return True


def _cluster_ready(node, n: int, timeout: float = 120.0) -> None:
    from idunno.runtime.transport import wait_for

    assert wait_for(lambda: len(node.membership.alive()) == n, timeout), node.membership.table()
    if node.cfg.collective_rounds and node.is_coordinator:
        # formed AND healthy: queries submitted before the plane is marked healthy take the TCP path
        assert wait_for(lambda: node.rounds.group.formed and node.rounds.healthy
                        and len(node.rounds.group.members) == n, timeout)


def _drive_system(a, node, W: int, B: int) -> dict:
    """Coordinator (rank 0): single-job throughput + p50, then two concurrent
    jobs under the fair-time split."""
    from idunno.runtime.client import Client
    from idunno.runtime.transport import wait_for

    _cluster_ready(node, W)
    cl = Client(node)
    st = node.state
    per_q = W * B
    nxt = [0]

    def submit(k, size=per_q):
        for _ in range(k):
            s0 = nxt[0]
            nxt[0] += size
            cl.submit(a.model, s0, s0 + size - 1)

    def wait_done(target, timeout=300):
        # block on the coordinator's progress condition (notified per ingested round)
        # instead of polling: a 1 ms polling thread competes with the round driver
        # for the interpreter lock
        return _wait_progress(node, lambda: st.images_done(a.model) >= target and st.pending_count() == 0, timeout)

    submit(a.warmup)
    assert wait_done(nxt[0]), st.summary()
    lat0 = len(st.query_latency[a.model])
    ra = node.rounds.stats() if node.rounds is not None else None
    import torch

    dev = node.device if node.device is not None else None
    gpu_node = dev is not None and torch.device(dev).type == "cuda"
    ms0 = torch.cuda.memory_stats(dev) if gpu_node else {}
    t_wall0 = time.time()
    t0 = time.perf_counter()
    submit(a.steps)
    assert wait_done(nxt[0]), st.summary()
    elapsed = time.perf_counter() - t0
    rb = node.rounds.stats() if node.rounds is not None else None
    loaded = sorted(st.query_latency[a.model][lat0:])
    lat1 = len(st.query_latency[a.model])
    for _ in range(max(5, min(a.steps, 20))):   # unloaded: one query at a time
        submit(1)
        assert wait_done(nxt[0])
    unloaded = sorted(st.query_latency[a.model][lat1:])
    ips = per_q * a.steps / elapsed
    p50 = unloaded[len(unloaded) // 2]
    out = {"value_system": round(ips, 2), "ms_per_step_system": round(1000 * elapsed / a.steps, 4),
           "p50_system_s": round(p50, 6),
           "p50_system_loaded_s": round(loaded[len(loaded) // 2], 6) if loaded else None,
           # the loaded p50 is over `steps` queries submitted at once: a query's
           # latency includes the queue ahead of it
           "system_loaded_queue_depth": a.steps,
           "system_path": ("client -> coordinator Node (membership, hot standby) -> fair-time split -> "
                           + (("RCCL rounds" if W > 1 else "pipelined rounds (one-member group)")
                              if node.rounds is not None else "local JOB queue")
                           + " -> job-state ingest"),
           "system_results_recorded": st.images_done(a.model)}
    if ra is not None and rb["rounds_done"] > ra["rounds_done"]:
        # the coordinator's own host work per round (plan, post, ingest; not the gather wait)
        nr = rb["rounds_done"] - ra["rounds_done"]
        out["system_host_ms_per_round"] = round(1000 * (rb["host_s"] - ra["host_s"]) / nr, 4)
        out["system_host_cpu_ms_per_round"] = round(1000 * (rb["host_cpu_s"] - ra["host_cpu_s"]) / nr, 4)
        out["system_host_wait_ms_per_round"] = round(1000 * (rb["host_wait_s"] - ra["host_wait_s"]) / nr, 4)
        out["system_rounds"] = nr
        out["system_host_post_ms_per_round"] = round(1000 * (rb["host_post_s"] - ra["host_post_s"]) / nr, 4)
        out["system_launch_cpu_ms"] = round(1000 * (rb["launch_cpu_s"] - ra["launch_cpu_s"]) / nr, 4)
        if gpu_node:
            ms1 = torch.cuda.memory_stats(dev)
            for k in ("num_device_alloc", "num_device_free", "num_alloc_retries", "num_sync_all_streams"):
                out[f"system_alloc_{k}"] = ms1.get(k, 0) - ms0.get(k, 0)
        # where the coordinator's own chunk spends its host time (tracer spans of the timed rounds)
        with node.tracer.lock:
            evs = [e for e in node.tracer.events if e[0] == "X" and e[2] >= t_wall0]
        for nm in ("round.stage", "round.launch"):
            d = [e[3] for e in evs if e[1] == nm]
            if d:
                out[f"system_{nm.replace('.', '_')}_ms"] = round(1000 * statistics.mean(d), 4)
        out["system_host_send_ms_per_round"] = round(1000 * (rb["host_send_s"] - ra["host_send_s"]) / nr, 4)
        out["system_host_release_ms_per_round"] = round(1000 * (rb["host_release_s"] - ra["host_release_s"]) / nr, 4)

    # strong scaling (the north star's p50): ONE 400-image query split over the W
    # members, one at a time (p50), then `steps` of them queued at once (images/s);
    # two untimed queries first capture the graphs of the chunk size
    submit(2, QUERY)
    assert wait_done(nxt[0])
    ls0 = len(st.query_latency[a.model])
    for _ in range(max(5, min(a.steps, 20))):
        submit(1, QUERY)
        assert wait_done(nxt[0])
    strong = sorted(st.query_latency[a.model][ls0:])
    t0 = time.perf_counter()
    submit(a.steps, QUERY)
    assert wait_done(nxt[0]), st.summary()
    el_strong = time.perf_counter() - t0
    out.update({"p50_system_strong_s": round(strong[len(strong) // 2], 6),
                "images_per_s_system_strong": round(QUERY * a.steps / el_strong, 2),
                "system_strong_chunk_per_gpu": -(-QUERY // W)})

    if W == 1 and a.sdfs_images > 0:
        out.update(_sdfs_pass(a, node, per_q))

    # two concurrent jobs: AlexNet + ResNet18 (report Fig 2), coordinator-side jobs
    bs = {"alexnet": QUERY_ALEXNET * W, "resnet18": QUERY * W}
    done = {m: st.images_done(m) for m in bs}
    base_img = [10 ** 7]

    def two_jobs(q: int):
        qn0 = {m: st.next_qnum[m] for m in bs}
        t = time.perf_counter()
        for m in ("alexnet", "resnet18"):
            cl.submit_job(base_img[0], base_img[0] + q * bs[m] - 1, m)
            done[m] += q * bs[m]
        base_img[0] += 10 ** 6
        ok = _wait_progress(node, lambda: all(st.images_done(m) >= done[m] for m in bs) and st.pending_count() == 0,
                            300)
        assert ok, st.summary()
        return time.perf_counter() - t, qn0

    two_jobs(2)                                  # warm: graphs for the split sizes, EMAs settle
    r0 = node.rounds.stats() if node.rounds is not None else {}
    wall, qn0 = two_jobs(a.two_job_queries)
    r1 = node.rounds.stats() if node.rounds is not None else {}
    imgs = a.two_job_queries * sum(bs.values())
    per = {}
    with st.lock:
        for m in bs:
            ws = []
            for q in range(qn0[m] + 1, st.next_qnum[m] + 1):
                ents = st.worker_set.get((m, q), [])
                if ents:
                    ws.append(len({e[0] for e in ents}))
            per[m] = ws
            lat = st.query_latency[m][-a.two_job_queries:]
            out[f"two_job_p50_{m}_s"] = round(statistics.median(lat), 6) if lat else None
    out.update({"two_job_images_per_s": round(imgs / wall, 2), "two_job_wall_s": round(wall, 4),
                "two_job_queries_per_job": a.two_job_queries,
                "two_job_query_images": bs,
                "workers_per_query_alexnet": per["alexnet"], "workers_per_query_resnet18": per["resnet18"],
                "two_job_mixed_rounds": (r1.get("mixed_rounds", 0) - r0.get("mixed_rounds", 0)) if r1 else None,
                # worker split of every round that ran both jobs (disjoint by construction: one row
                # per member), counted over the timed jobs: one entry = the split never moved
                "two_job_mixed_splits": {k: v - r0.get("mixed_splits", {}).get(k, 0)
                                         for k, v in r1.get("mixed_splits", {}).items()
                                         if v > r0.get("mixed_splits", {}).get(k, 0)} if r1 else None,
                "sched_avg_time_s": {m: round(v, 6) for m, v in node.sched.avg_time.items()},
                # every mixed round of the timed jobs: [seq, split, the averages the scheduler held
                # when the round was posted, the exact fair-time shares they give]
                "two_job_split_log": r1.get("mixed_log", [])[
                    -max(0, min(24, r1.get("mixed_rounds", 0) - r0.get("mixed_rounds", 0))):] if r1 and
                    r1.get("mixed_rounds", 0) > r0.get("mixed_rounds", 0) else [] if r1 else None})

    # time to start a second job (report Fig 3: 40-42 s AlexNet first, 45-49 s ResNet18 first): job A
    # runs; job B is submitted; until B's first query has finished
    def second_job(first: str, second: str, q: int = 4) -> float:
        fq = {m: st.finished_queries.get(m, 0) for m in bs}
        cl.submit_job(base_img[0], base_img[0] + q * bs[first] - 1, first)
        done[first] += q * bs[first]
        assert _wait_progress(node, lambda: st.finished_queries.get(first, 0) > fq[first], 120), st.summary()
        t = time.perf_counter()
        cl.submit_job(base_img[0] + 5 * 10 ** 5, base_img[0] + 5 * 10 ** 5 + q * bs[second] - 1, second)
        done[second] += q * bs[second]
        assert _wait_progress(node, lambda: st.finished_queries.get(second, 0) > fq[second], 120), st.summary()
        dt = time.perf_counter() - t
        base_img[0] += 10 ** 6
        assert _wait_progress(node, lambda: all(st.images_done(m) >= done[m] for m in bs) and st.pending_count() == 0,
                              300), st.summary()
        return dt

    sj = {"alexnet_first": second_job("alexnet", "resnet18"), "resnet18_first": second_job("resnet18", "alexnet")}
    out["second_job_start_s"] = {k: round(v, 4) for k, v in sj.items()}
    out["second_job_start_ref_s"] = BASELINE_SECOND_JOB_S

    # like-for-like latency ("numbers also reported with those sleeps
    # enabled"): the reference sleeps 3 s before every chunk (mp4_machinelearning.py:594);
    # with that delay on the coordinator's own chunk every query waits for it
    if a.ref_delay_queries > 0:
        delay0 = node.cfg.worker_start_delay_s
        node.cfg.worker_start_delay_s = REF_WORKER_START_DELAY_S
        lat = []
        try:
            for i in range(a.ref_delay_queries):
                d0 = st.images_done(a.model)
                q0 = base_img[0] + i * per_q
                t = time.perf_counter()
                node.submit_query(a.model, q0, q0 + per_q - 1)
                assert _wait_progress(node, lambda: st.images_done(a.model) >= d0 + per_q and st.pending_count() == 0,
                                      60), st.summary()
                lat.append(time.perf_counter() - t)
        finally:
            node.cfg.worker_start_delay_s = delay0
        base_img[0] += 10 ** 6
        out.update({"p50_query_latency_ref_delay_s": round(statistics.median(lat), 4),
                    "ref_worker_start_delay_s": REF_WORKER_START_DELAY_S,
                    "p50_query_latency_ref_delay_vs_baseline": round(BASELINE_P50_S / statistics.median(lat), 2)})
    grp = node.rounds.group.describe() if node.rounds is not None else {}
    out["system_comm_backend"] = grp.get("backend", "tcp (no collective)")
    out["system_comm_world"] = grp.get("world", 1)
    return out


def _timeline_overlap(tl: list) -> tuple[float, list]:
    """Fraction of the H2D staging time (side stream) that ran while a forward
    (private compute stream) was executing, from the recorded CUDA events, and
    the intervals as (kind, start ms, end ms, n) on one clock."""
    if not tl:
        return 0.0, []
    ref = tl[0][1]
    iv = [(k, ref.elapsed_time(e0), ref.elapsed_time(e1), n) for k, e0, e1, n in tl]
    fw = sorted((t0, t1) for k, t0, t1, _ in iv if k == "fwd")
    tot = ov = 0.0
    for k, t0, t1, _ in iv:
        if k != "h2d":
            continue
        tot += t1 - t0
        ov += sum(max(0.0, min(t1, f1) - max(t0, f0)) for f0, f1 in fw)
    return (ov / tot if tot > 0 else 0.0), iv


def _sdfs_pass(a, node, per_q: int) -> dict:
    """SDFS -> HBM on the measured path: the synthetic
    dataset is put into SDFS as 500-image uint8 shards, then the same ResNet18
    queries are served from ``SdfsSource`` -- cold (every shard read from the
    node's SDFS store and staged host -> HBM through pinned ping-pong buffers
    on a side stream while the previous round computes) and warm (HBM-cached
    shards).  Reference: images are read from local disk per image,
    alexnet_resnet.py:24,49."""
    import torch

    from idunno.runtime.data import SdfsSource, put_synthetic_dataset

    st, cfg = node.state, node.cfg
    n_img = max(per_q, a.sdfs_images // per_q * per_q)
    t = time.perf_counter()
    shards = put_synthetic_dataset(node.sdfs, n_img, cfg.data_seed, shard_images=500)
    put_s = time.perf_counter() - t
    keep = node.source
    src = SdfsSource(node.sdfs, node.device if node.device is not None else "cpu", shard_images=500,
                     peer_copy=False, readahead=4,
                     stage_streams=int(os.environ.get("IDUNNO_BENCH_STAGE_STREAMS", "1")))
    gpu = src.device.type == "cuda"
    node.source = src
    out = {}
    try:
        def run_pass(label):
            done0 = st.images_done(a.model)
            t0 = time.perf_counter()
            for q0 in range(0, n_img, per_q):
                node.submit_query(a.model, q0, q0 + per_q - 1)
            assert _wait_progress(node, lambda: st.images_done(a.model) >= done0 + n_img and st.pending_count() == 0,
                                  300), st.summary()
            return time.perf_counter() - t0

        tl = [] if gpu else None
        for sg in src.stagers:
            sg.timeline = tl
        node.gpu_timeline = tl
        b0 = sum(sg.bytes_staged for sg in src.stagers)
        r0 = sum(sg.native_read_s for sg in src.stagers)
        w0 = sum(sg.native_wait_s for sg in src.stagers)
        src.tracer = node.tracer
        th0 = time.time()
        cold = run_pass("cold")
        th1 = time.time()
        src.tracer = None
        node.gpu_timeline = None
        for sg in src.stagers:
            sg.timeline = None
        staged = sum(sg.bytes_staged for sg in src.stagers) - b0
        read_s = sum(sg.native_read_s for sg in src.stagers) - r0
        dma_wait_s = sum(sg.native_wait_s for sg in src.stagers) - w0
        if gpu:
            torch.cuda.synchronize(src.device)
        ovl, iv = _timeline_overlap(tl) if gpu else (None, [])
        warm = run_pass("warm")
        # wall time with at least one H2D in flight (the union: stagers overlap each other)
        h2d_ms, end = 0.0, float("-inf")
        for t0, t1 in sorted((t0, t1) for k, t0, t1, _ in iv if k == "h2d"):
            if t1 > end:
                h2d_ms += t1 - max(t0, end)
                end = t1
        out = {"value_system_sdfs_cold": round(n_img / cold, 2), "value_system_sdfs_warm": round(n_img / warm, 2),
               "sdfs_cold_to_warm": round(warm / cold, 4), "sdfs_images": n_img, "sdfs_shards": shards,
               "sdfs_put_gb_per_s": round(n_img * 150528 / put_s / 1e9, 3),
               "sdfs_bytes_staged": staged,
               "sdfs_host_read_gb_per_s": round(staged / read_s / 1e9, 2) if read_s > 0 else None,
               "sdfs_stager_dma_wait_ms": round(dma_wait_s * 1e3, 2),
               "hbm_stage_gb_per_s": round(staged / (h2d_ms * 1e-3) / 1e9, 2) if h2d_ms > 0 else None,
               "sdfs_h2d_overlap_frac": round(ovl, 4) if ovl is not None else None,
               "sdfs_local_file_reads": src.local_reads, "sdfs_readahead_hits": src.readahead_hits,
               "sdfs_path": "SDFS store (local replica file) -> parallel preadv into pinned ping-pong buffers -> "
                            f"hipMemcpyAsync on {src.nstage} side stream(s) -> HBM shard cache -> rounds (4-shard readahead)"}
        if a.sdfs_trace and iv:
            ev = [{"name": k, "ph": "X", "ts": 1000.0 * t0, "dur": 1000.0 * (t1 - t0), "pid": 0,
                   "tid": 1 if k == "h2d" else 0, "args": {"n": n}} for k, t0, t1, n in iv]
            # host spans of the cold pass (node thread activity: query submit, chunk staging
            # waits, launches, SDFS fetches), on their own clock (pid 1)
            ev += [dict(e, pid=1, ts=e["ts"] - th0 * 1e6) for e in node.tracer.export()
                   if e["ph"] in ("X", "i") and th0 * 1e6 <= e["ts"] <= th1 * 1e6]
            with open(a.sdfs_trace, "w") as f:
                json.dump({"traceEvents": ev, "displayTimeUnit": "ms"}, f)
    finally:
        node.source = keep
        node.gpu_timeline = None
    return out


def _drive_failover(a, node, n: int) -> dict:
    """Standby (last node): submit a job, let the launcher SIGKILL the
    coordinator mid-job, time the promotion and the restored service."""
    from idunno.runtime.client import Client
    from idunno.runtime.transport import wait_for

    _cluster_ready(node, n)
    if node.cfg.collective_rounds:
        wait_for(lambda: False, 1.0)             # let the coordinator's epoch settle
    cl = Client(node)
    st = node.state
    model = "resnet18"
    bs = node.cfg.batch_for(model)
    Q = a.failover_queries
    total = Q * bs
    promoted = {}
    node.membership.on_master_change.append(
        lambda new, ep: promoted.setdefault("t", time.time()) if new == node.name else None)
    cl.submit_job(0, total - 1, model)
    # kill once a few queries have finished at the standby (mirrored results)
    assert wait_for(lambda: st.images_done(model) >= min(2, Q - 1) * bs, 120, 0.002), st.summary()
    done_at_kill = st.images_done(model)
    work = a.work_dir or tempfile.gettempdir()
    with open(os.path.join(work, "kill_now.tmp"), "w") as f:
        f.write("0")                                  # the coordinator's rank
    os.replace(os.path.join(work, "kill_now.tmp"), os.path.join(work, "kill_now"))
    killed = os.path.join(work, "killed_at")
    assert wait_for(lambda: os.path.exists(killed), 30, 0.001), "launcher did not kill the coordinator"
    with open(killed) as f:
        t_kill = float(f.read())
    assert wait_for(lambda: "t" in promoted and node.is_coordinator, 60, 0.001), "standby did not promote"
    base_done = st.images_done(model)
    t_prom = promoted["t"]
    wait_for(lambda: st.images_done(model) > base_done or st.images_done(model) >= total, 60, 0.001)
    t_restored = time.time()
    ok = wait_for(lambda: st.images_done(model) >= total and st.pending_count() == 0, 120, 0.002)
    t_all = time.time()
    rec = max(0.0, t_restored - t_kill)
    survivor = {}
    if node.rounds is not None:
        # the epoch this node formed as the new coordinator (not the old one it was a member of)
        g = node.rounds.group
        wait_for(lambda: g.formed and g.members[:1] == [node.name], 15, 0.01)
        survivor = g.describe() if g.members[:1] == [node.name] else {}
    return {"coord_failover_recovery_s": round(rec, 4),
            "coord_failover_detect_s": round(t_prom - t_kill, 4),
            "coord_failover_all_done_s": round(t_all - t_kill, 4),
            "coord_failover_undone_queries": Q - done_at_kill // bs,
            "coord_failover_images_exact": bool(ok and st.images_done(model) == total),
            "coord_failover_nodes": n, "coord_failover_failure_timeout_s": node.cfg.failure_timeout_s,
            "coord_failover_heartbeat_s": node.cfg.heartbeat_period_s,
            "coord_failover_vs_baseline_speedup": round(BASELINE_COORD_RECOVERY_S / rec, 1) if rec > 0 else None,
            "coord_failover_rounds": bool(node.cfg.collective_rounds),
            # the epoch the promoted standby formed over the survivors (RCCL at N >= 2)
            "coord_failover_survivor_world": survivor.get("world"),
            "coord_failover_survivor_backend": survivor.get("backend")}


def _drive_worker_failover(a, node, n: int) -> dict:
    """Coordinator (rank 0): pause a worker (fault-injection delay), submit k
    queries so k of its chunks are in flight, have the launcher SIGKILL it,
    then time the detection, the re-dispatch and the last result (report
    Fig 4: "3 s + n * send time", 5.7 s for 1 task ... 26.8 s for 8)."""
    from idunno.runtime.client import Client
    from idunno.runtime.messages import Type
    from idunno.runtime.transport import wait_for

    _cluster_ready(node, n)
    cfg = node.cfg
    victim_rank = 1 if n >= 3 else n - 1          # a worker; the standby only when there is no other
    victim = cfg.node_name(victim_rank)
    cl = Client(node)
    st = node.state
    model = a.model
    k = a.kill_chunks
    detected = {}
    node.membership.on_failure.insert(0, lambda nd: detected.setdefault(nd, time.time()))   # before re-dispatch
    # the victim stalls before each chunk: its chunks pile up as in-flight work
    assert node.transport.send(victim, {"t": Type.KILL, "mode": "delay", "seconds": 600.0})
    node.sched.budget = n                             # every query spans every node, the victim included
    per_q = cfg.batch_for(model)
    base = 5 * 10 ** 7
    for i in range(k):
        cl.submit(model, base + i * per_q, base + (i + 1) * per_q - 1)
    assert wait_for(lambda: len(st.chunks_of(victim)) >= k, 30, 0.002), st.cvm()
    time.sleep(0.2)                                   # the others' chunks of these queries finish
    held = len(st.chunks_of(victim))
    work = a.work_dir or tempfile.gettempdir()
    with open(os.path.join(work, "kill_now.tmp"), "w") as f:
        f.write(str(victim_rank))
    os.replace(os.path.join(work, "kill_now.tmp"), os.path.join(work, "kill_now"))
    killed = os.path.join(work, "killed_at")
    assert wait_for(lambda: os.path.exists(killed), 30, 0.001), "launcher did not kill the worker"
    with open(killed) as f:
        t_kill = float(f.read())
    total = k * per_q
    ok = wait_for(lambda: st.images_done(model) >= total and st.pending_count() == 0, 120, 0.002)
    t_done = time.time()
    survivor = {}
    if node.rounds is not None:
        wait_for(lambda: node.rounds.group.formed and node.rounds.group.world == n - 1, 15, 0.01)
        survivor = node.rounds.group.describe()
    return {"recovery_s": round(t_done - t_kill, 4),
            "detect_s": round(detected[victim] - t_kill, 4) if victim in detected else None,
            "chunks_on_victim": held, "images_exact": bool(ok and st.images_done(model) == total),
            "nodes": n, "rounds": bool(cfg.collective_rounds), "survivor_world": survivor.get("world"),
            "survivor_backend": survivor.get("backend"), "failure_timeout_s": cfg.failure_timeout_s}


def numerics_check(runner, a, device, n: int = 8) -> dict:
    """Max |logit - oracle| / max |oracle| of the benchmarked program on n
    images against the plain PyTorch fp32 module with the same weights."""
    import torch

    from idunno.models import reference as ref

    m = ref.build(ref.canonical(a.model), seed=a.seed).eval().to(device)
    from idunno import ops

    img = ops.synth_images(a.seed + 99, 0, n, device)
    with torch.no_grad():
        want = m(ref.preprocess_u8(img)).float()
        got = runner.logits(img).float()
        # fp64 oracle on the CPU (same weights): the error torch fp32 itself makes is the yardstick
        x64 = ref.preprocess_u8(img.cpu()).double()
        want64 = m.cpu().double()(x64)
    err = ((got - want).abs().max() / want.abs().max()).item()
    agree = (got.argmax(1) == want.argmax(1)).float().mean().item()
    s64 = want64.abs().max()
    err64 = ((got.cpu().double() - want64).abs().max() / s64).item()
    t64 = ((want.cpu().double() - want64).abs().max() / s64).item()
    return {"max_rel_logit_err_vs_torch_fp32": float(f"{err:.3g}"), "top1_agreement_vs_torch_fp32": agree,
            "max_rel_logit_err_vs_fp64": float(f"{err64:.3g}"),
            "torch_fp32_max_rel_logit_err_vs_fp64": float(f"{t64:.3g}")}


if __name__ == "__main__":
    sys.exit(main())
