"""Per-parameter step-1 gradient table: W ranks (same batch) vs 1 rank, in backward order.

  python tools/dp_grad_diag.py resnet_v1_50 DTM_DISABLE=sibling_group [--no-overlap] [--world 2] [--steps 1]

Two gloo ranks share the one GPU of a test box (RCCL refuses two ranks on one device); deterministic
reductions make a correct run bit-exact, so any non-zero row is a real data-parallel defect.  The first
non-zero row in BACKWARD order is where it originates (step 1: nothing has fed back through the update yet).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_tensorflow_models_amd.utils import dp_check  # noqa: E402
from distributed_tensorflow_models_amd.utils.testing import run_workers  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model")
    ap.add_argument("knobs", nargs="*")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--show", type=int, default=12)
    a = ap.parse_args()
    knobs = dict(k.split("=", 1) for k in a.knobs)
    ov = not a.no_overlap
    single = run_workers(dp_check.grad_worker, 1, a.model, knobs, 2.0, ov, a.steps)[0]
    multi = run_workers(dp_check.grad_worker, a.world, a.model, knobs, 2.0, ov, a.steps)
    print("model %s knobs %s overlap %s world %d: buckets %d launched %d compact %d sibling_merged %d "
          "writes_checked %d unreported %s" % (a.model, knobs, ov, a.world, multi[0]["buckets"], multi[0]["launched"],
                                               multi[0]["compact"], multi[0]["sibling_merged"],
                                               multi[0]["writes_checked"], multi[0]["unreported"][:4]))
    ok = True
    for st in range(a.steps):
        rows = dp_check.compare(multi[0], single, st)
        bad = [r for r in rows if r[1] > 0]
        print("step %d: %d / %d tensors differ (max rel %.3g)" % (st + 1, len(bad), len(rows),
                                                                 max([r[1] for r in rows] or [0])))
        for name, rel, mx in bad[:a.show]:
            print("   %-70s rel %.3e  max abs %.3e" % (name, rel, mx))
        ok &= not bad
    rep = all(bool((m["params"] == multi[0]["params"]).all()) for m in multi)
    print("replicas identical: %s" % rep)
    print("RESULT %s" % ("EXACT" if ok and rep else "MISMATCH"))


if __name__ == "__main__":
    main()
