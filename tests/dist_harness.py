"""Spawned-rank harness for the multi-process tests (gloo on CPU, gloo / nccl on the GPU box).

``run_ranks(target, world, args)`` starts ``world`` spawned processes, each running
``target(rank, world, *args)`` inside an initialised process group, and returns the ranks' results in
rank order.  It is built around the two ways a spawned-rank test can fail for reasons that are not
the code under test:

* **Results travel by value.**  A torch tensor put on a ``torch.multiprocessing`` queue is a handle
  into the SENDER's shared memory; the receiver maps it while unpickling, through a socket the sender
  serves.  A rank that has already left (its barrier and ``destroy_process_group`` take milliseconds)
  cannot serve it, and ``q.get`` raises ``ConnectionRefusedError`` / ``FileNotFoundError`` in the
  parent — a race the parent loses whenever it is slow to read (a loaded CPU suite) and more often the
  more ranks there are.  This was the round-5 world-4 failure of ``test_grad_exchange_gloo_world2``
  (reproduced by delaying the parent's first ``q.get`` by 8 s: ``FileNotFoundError`` in
  ``multiprocessing/connection.py``).  Every tensor in a result is converted to a numpy array (pickled
  by value) before it is queued.
* **No port is picked in advance.**  The rendezvous is a ``FileStore`` in a fresh temporary directory
  (``init_method="file://..."``), so there is no bind / close / reuse window for another socket to
  take the port.

Every rank reports ``(rank, "ok", result)`` or ``(rank, "error", traceback)``; the parent collects
all reports (up to a deadline), and on any error, missing report or non-zero exit code raises one
AssertionError that lists every rank's status, traceback and exit code.
"""
import datetime
import os
import queue as _queue
import shutil
import sys
import tempfile
import time
import traceback

import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def to_value(obj):
    """Tensors (nested in tuples / lists / dicts) -> numpy arrays, so the result pickles by value."""
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu().numpy().copy()
    if isinstance(obj, dict):
        return {k: to_value(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(to_value(v) for v in obj)
    return obj


def _rank_main(target, rank, world, init_file, backend, args, q, threads):
    if REPO not in sys.path:
        sys.path.insert(0, REPO)
    import torch.distributed as dist
    torch.set_num_threads(threads)
    try:
        dist.init_process_group(backend, init_method="file://" + init_file, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=180))
    except BaseException:
        q.put((rank, "error", "init_process_group failed:\n" + traceback.format_exc()))
        return
    try:
        res = to_value(target(rank, world, *args))
        q.put((rank, "ok", res))
    except BaseException:
        q.put((rank, "error", traceback.format_exc()))
        q.close()
        q.join_thread()   # the report is in the pipe before the process ends
        # the other ranks may be blocked in a collective with this one: leave without the barrier
        os._exit(3)
    dist.barrier()
    dist.destroy_process_group()


def run_ranks(target, world, args=(), timeout=240, backend="gloo", threads=1):
    """Run target(rank, world, *args) on `world` spawned ranks; return their results in rank order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    tmp = tempfile.mkdtemp(prefix="vst_pg_")
    init_file = os.path.join(tmp, "store")
    procs = [ctx.Process(target=_rank_main, args=(target, r, world, init_file, backend, args, q, threads))
             for r in range(world)]
    try:
        for p in procs:
            p.start()
        reports = {}
        deadline = time.monotonic() + timeout
        while len(reports) < world:
            left = deadline - time.monotonic()
            if left <= 0:
                break
            try:
                rank, status, payload = q.get(timeout=min(left, 5.0))
            except _queue.Empty:
                if all(p.exitcode is not None for p in procs):
                    break   # every rank has ended and the queue stayed empty: some died without reporting
                continue
            reports[rank] = (status, payload)
        # ranks that reported ok leave after their barrier; after an error the rest may be stuck in it
        grace = 60.0 if len(reports) == world and all(st == "ok" for st, _ in reports.values()) else 5.0
        end = time.monotonic() + grace
        for p in procs:
            p.join(timeout=max(0.1, end - time.monotonic()))
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
        bad = [r for r in range(world) if r not in reports or reports[r][0] != "ok"] + \
              [r for r, p in enumerate(procs) if p.exitcode != 0]
        if bad:
            lines = ["%d-rank run failed; per rank:" % world]
            for r in range(world):
                st, payload = reports.get(r, ("no report", ""))
                lines.append("--- rank %d: %s, exit code %s" % (r, st, procs[r].exitcode))
                if st != "ok":
                    lines.append(str(payload))
            raise AssertionError("\n".join(lines))
        return [reports[r][1] for r in range(world)]
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
