"""Helpers for the multi-process GPU tests: a worker that hangs (a collective or the RCCL bootstrap
that never returns) must fail its test within a bounded time instead of blocking the GPU suite.
Workers arm faulthandler to dump their stacks and exit after `seconds`; the parent polls the result
queue against a deadline of its own and kills what is left."""
import queue
import sys
import time

import pytest


def watchdog(seconds=150):
    import faulthandler
    faulthandler.dump_traceback_later(seconds, exit=True, file=sys.stderr)


def collect(procs, q, n, deadline=170):
    """n results from the workers' queue; fails (killing the workers) once a worker died without its
    result or the deadline passed, then joins them all (exit codes left to the caller, which checks
    the results first: a worker's traceback travels in its result)"""
    out, t_end = [], time.monotonic() + deadline
    while len(out) < n:
        try:
            out.append(q.get(timeout=5))
        except queue.Empty:
            dead = [p.exitcode for p in procs if not p.is_alive() and p.exitcode != 0]
            if dead or time.monotonic() > t_end:
                for p in procs:
                    if p.is_alive():
                        p.kill()
                pytest.fail(f"worker(s) {'exited with ' + str(dead) if dead else 'timed out'} after {len(out)} "
                            f"of {n} results (stacks, if any, in the captured stderr)")
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
            pytest.fail("worker did not exit after sending its result")
    return out
