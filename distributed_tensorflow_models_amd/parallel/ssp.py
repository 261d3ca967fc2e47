"""SSP: stale-synchronous parallel staleness clock (reference inception/ssp_manager.py:14-58,
inception/imagenet_inception_ssp.py:81-89,193).

The reference runs a Thrift ``CheckStaleness`` service on PS task 0 (port 8000) whose handler
mutates a shared list from W server threads without a lock and busy-waits inside the RPC.  Here
the clock is W integer keys in the c10d TCPStore (atomic set/get, already running for the
process group): after every local step a worker publishes its step and blocks *client side*
while ``step > min(all steps) + max_staleness``.  The slowest worker never waits, so the protocol
cannot deadlock; the bound holds by construction (tests/test_dist_cpu.py checks it).
"""
import time

from . import process_group as pg


class StalenessClock:
    def __init__(self, max_staleness=5, store=None, rank=None, world=None, run_id="0", poll_s=0.002,
                 timeout_s=3600.0, log_fn=None, read_only=False):
        """``read_only``: an observer (the debug CLI) - publishes nothing, cannot tick."""
        if store is None:
            from .asp import _default_store
            store = _default_store()
        self.store = store
        self.rank = pg.rank() if rank is None else rank
        self.world = pg.world_size() if world is None else world
        self.s = int(max_staleness)
        self.prefix = "dtm_ssp/%s/clock/" % run_id
        self.poll_s, self.timeout_s = poll_s, timeout_s
        self.log_fn = log_fn
        self.waited_s = 0.0
        self.max_observed_gap = 0
        self.read_only = bool(read_only)
        if not self.read_only:
            self.store.set(self.prefix + str(self.rank), "0")

    def _keys(self):
        return [self.prefix + str(r) for r in range(self.world)]

    def steps(self):
        keys = self._keys()
        self.store.wait(keys)
        mg = getattr(self.store, "multi_get", None)
        vals = mg(keys) if mg is not None else [self.store.get(k) for k in keys]
        return [int(v) for v in vals]

    def tick(self, local_step):
        """check_staleness(task_index, local_step): publish, then wait until within the bound."""
        if self.read_only:
            raise RuntimeError("StalenessClock: a read-only observer cannot tick")
        self.store.set(self.prefix + str(self.rank), str(int(local_step)))
        t0 = time.time()
        warned = False
        while True:
            st = self.steps()
            gap = local_step - min(st)
            if gap <= self.s:
                self.max_observed_gap = max(self.max_observed_gap, max(st) - min(st))
                break
            if not warned and self.log_fn is not None:
                self.log_fn("worker %d too fast: step %d > min %d + %d" % (self.rank, local_step, min(st), self.s))
                warned = True
            if time.time() - t0 > self.timeout_s:
                raise TimeoutError("SSP wait exceeded %.0fs (a worker died?)" % self.timeout_s)
            time.sleep(self.poll_s)
        self.waited_s += time.time() - t0
        return min(st)

    def finish(self, final_step=None):
        """Release waiters when this worker stops (publish a step that never blocks anyone)."""
        if self.read_only:
            return
        self.store.set(self.prefix + str(self.rank), str(1 << 40))


class SspManager:
    """Compatibility factory for the reference's ``SspManager(num_of_replicas, max_stale)``
    (inception/ssp_manager.py: Thrift ``CheckStaleness`` server on PS 0 + per-worker clients).
    There is no server process here: the "server" is the c10d store every rank already shares,
    and a client's ``check_staleness(task_index, local_step)`` is ``StalenessClock.tick``."""

    def __init__(self, num_of_replicas, max_stale=5, run_id="0"):
        self.world, self.max_stale, self.run_id = int(num_of_replicas), int(max_stale), run_id
        self._clock = None

    def create_rpc_server(self, host=None):
        return self  # nothing to serve; kept so reference-style call sites still work

    def serve(self):
        return None

    def create_rpc_client(self, host=None):
        return self

    def check_staleness(self, task_index, local_step):
        if self._clock is None:
            self._clock = StalenessClock(self.max_stale, rank=task_index, world=self.world, run_id=self.run_id)
        return self._clock.tick(local_step)


def main():  # debug CLI (replaces CheckStaleness-remote): print the clock of a running job
    import argparse
    import datetime

    import torch.distributed as dist
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=29500)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--run-id", default="0")
    a = ap.parse_args()
    st = dist.TCPStore(a.host, a.port, is_master=False, timeout=datetime.timedelta(seconds=10))
    c = StalenessClock(store=st, rank=-1, world=a.world, run_id=a.run_id, read_only=True)
    print(c.steps())


if __name__ == "__main__":
    main()
