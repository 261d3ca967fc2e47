"""Per-rank heartbeat files and the launcher's hang detector.

The reference has no failure detector: a hung worker leaves the others blocked inside the PS
queues (or, here, an RCCL collective) until a timeout measured in tens of minutes.  Every worker
touches ``<dir>/rank_<r>`` after each training step (at most once per ``min_interval_s``; one
small file write, never on the GPU path), and the launcher treats a rank whose heartbeat is older
than ``--hang_timeout`` seconds as hung: the whole job is stopped and, with ``--max_restarts``,
restarted from the latest checkpoint - the same path as a crashed rank.
"""
import os
import time

ENV_DIR = "DTM_HEARTBEAT_DIR"


class Heartbeat:
    def __init__(self, rank, directory=None, min_interval_s=1.0):
        self.dir = directory if directory is not None else os.environ.get(ENV_DIR, "")
        self.path = os.path.join(self.dir, "rank_%d" % rank) if self.dir else None
        self.min_interval_s = min_interval_s
        self._last = 0.0
        if self.path:
            os.makedirs(self.dir, exist_ok=True)
            self.beat(-1, force=True)

    def beat(self, step, force=False):
        if not self.path:
            return
        now = time.time()
        if not force and now - self._last < self.min_interval_s:
            return
        self._last = now
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            f.write("%d %.3f %d\n" % (step, now, os.getpid()))
        os.replace(tmp, self.path)  # atomic: the monitor never reads a half-written file


def read(directory, rank):
    """(step, unix time) of rank's last heartbeat, or None."""
    try:
        with open(os.path.join(directory, "rank_%d" % rank)) as f:
            s, t, _ = f.read().split()
        return int(s), float(t)
    except (OSError, ValueError):
        return None


def stale_ranks(directory, nranks, timeout_s, started_at, now=None):
    """Ranks whose last heartbeat (or, before the first one, the job start) is older than timeout."""
    now = time.time() if now is None else now
    out = []
    for r in range(nranks):
        hb = read(directory, r)
        last = hb[1] if hb is not None else started_at
        if now - last > timeout_s:
            out.append(r)
    return out


def clear(directory):
    if directory and os.path.isdir(directory):
        for n in os.listdir(directory):
            if n.startswith("rank_"):
                try:
                    os.remove(os.path.join(directory, n))
                except OSError:
                    pass
