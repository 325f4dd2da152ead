"""Multi-process rank harness for the N > 1 tests (gloo on the CPU, or the
one-GPU rehearsal): no port to race for, bounded waits, no orphans.

  * rendezvous through a FileStore in the test's tmp dir
    (init_method="file://..."), not a MASTER_PORT picked by binding port 0
    and releasing it -- that port can be taken (EADDRINUSE) before rank 0's
    TCPStore listens on it;
  * init_process_group(timeout=...) bounds every collective;
  * ranks are daemon processes, terminated and joined in a `finally`, so a
    rank blocked in a rendezvous never holds the interpreter at exit;
  * every rank reports (rank, ok, payload) on one queue -- a rank that raises
    anywhere (before the rendezvous included) fails the test at once with its
    traceback, without waiting for the others' timeouts.

`fn(rank, world, *args)` runs in each rank after init_process_group; rank 0's
return value (picklable) is returned to the test.
"""
from __future__ import annotations

import os
import queue
import time
import traceback


def _entry(fn, rank, world, store, backend, timeout_s, args, q, before):
    try:
        from datetime import timedelta

        if before is not None:
            before(rank, world)

        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend, init_method=f"file://{store}", rank=rank, world_size=world,
                                timeout=timedelta(seconds=timeout_s))
        res = fn(rank, world, *args)
    except BaseException:  # noqa: BLE001 -- reported to the parent, which fails the test
        q.put((rank, False, traceback.format_exc()))
        # no orderly teardown after a failure: destroy_process_group could
        # wait on peers that wait on this rank; the parent reaps the rest
        q.close()
        q.join_thread()
        os._exit(1)
    q.put((rank, True, res if rank == 0 else None))
    dist.destroy_process_group()


def run(fn, world, tmp_path, args=(), backend="gloo", timeout=120.0, init_timeout=60.0, before=None):
    """Run fn(rank, world, *args) in `world` spawned processes (after
    before(rank, world), if given, ahead of the rendezvous); return rank 0's
    result.  Raises RuntimeError with the failing rank's traceback as soon
    as any rank fails, TimeoutError after `timeout` s; every child is gone
    when this returns or raises."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = os.path.join(str(tmp_path), f"store_{os.getpid()}_{time.monotonic_ns()}")
    procs = [ctx.Process(target=_entry, args=(fn, r, world, store, backend, init_timeout, args, q, before), daemon=True)
             for r in range(world)]
    try:
        for p in procs:
            p.start()
        deadline = time.monotonic() + timeout
        done, result = set(), None
        while len(done) < world:
            left = deadline - time.monotonic()
            if left <= 0:
                raise TimeoutError(f"ranks {sorted(set(range(world)) - done)} did not finish in {timeout} s")
            try:
                r, ok, payload = q.get(timeout=min(left, 1.0))
            except queue.Empty:
                dead = [i for i, p in enumerate(procs) if i not in done and p.exitcode not in (None, 0)]
                if dead:
                    raise RuntimeError(f"rank {dead[0]} died (exit code {procs[dead[0]].exitcode}) "
                                       "without reporting")
                continue
            if not ok:
                raise RuntimeError(f"rank {r} failed:\n{payload}")
            done.add(r)
            if r == 0:
                result = payload
        for p in procs:
            p.join(timeout=30)
        return result
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
                p.join(timeout=5)
        q.close()
        q.join_thread()
