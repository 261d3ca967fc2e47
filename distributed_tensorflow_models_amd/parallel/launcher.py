"""Single-node launcher (replaces reference train.sh / clear.sh).

The reference ssh-launched one PS process per ``$ps`` host and one worker per ``$workers`` host and
started the evaluator on worker 0 after ``sleep 20`` with the GPU hidden (train.sh:29-61);
``clear.sh`` ran ``pkill python`` everywhere.  Here one worker process is started per MI355X on this
node (``RANK``/``LOCAL_RANK``/``WORLD_SIZE``/``MASTER_ADDR=127.0.0.1``/``MASTER_PORT``), there are no
PS processes (parameters live on the GPUs), the optional evaluator is started after ``--eval_delay``
seconds, logs go to ``<log_dir>/worker_<i>.log`` / ``model_eval.log``, and the PIDs are recorded
in ``<log_dir>/pids`` so ``--stop`` ends exactly those processes (never a name pattern).

  python -m distributed_tensorflow_models_amd.parallel.launcher --model vgg --mode bsp --nproc 8
  python -m distributed_tensorflow_models_amd.parallel.launcher --stop --log_dir runs/vgg_bsp
"""
import argparse
import os
import signal
import socket
import subprocess
import sys
import time

from ..utils import heartbeat as hbmod

PKG = "distributed_tensorflow_models_amd.trainers"

# (model, mode) -> trainer module; model -> eval module (train.sh:29-61 path conventions)
TRAINERS = {
    ("cnn", "bsp"): "cifar10_cnn_bsp",
    ("alexnet", "bsp"): "cifar10_alexnet_bsp",
    ("vgg", "bsp"): "cifar10_vgg_bsp",
    ("vgg", "asp"): "cifar10_vgg_asp",
    ("resnet", "bsp"): "cifar10_resnet_bsp",
    ("cifarnet", "bsp"): "cifar10_cifarnet_bsp",
    ("inception", "bsp"): "imagenet_inception_bsp",
    ("inception", "asp"): "imagenet_inception_asp",
    ("inception", "ssp"): "imagenet_inception_ssp",
    ("resnet50", "bsp"): "imagenet_resnet50_bsp",
    ("lenet", "bsp"): "mnist_lenet_bsp",
    ("mobilenet", "bsp"): "mobilenet_v1_train",
}
EVALS = {"cnn": "cifar10_cnn_eval", "alexnet": "cifar10_alexnet_eval", "vgg": "cifar10_vgg_eval",
         "resnet": "cifar10_resnet_eval", "cifarnet": "cifar10_cifarnet_eval",
         "inception": "imagenet_inception_eval", "mobilenet": "mobilenet_v1_eval"}


def resolve(model, mode):
    if (model, mode) in TRAINERS:
        return TRAINERS[(model, mode)], []
    # every CIFAR/ImageNet trainer runs in any sync mode through --sync_mode (MI355X extension)
    for (m, _md), mod in TRAINERS.items():
        if m == model:
            return mod, ["--sync_mode=%s" % mode]
    raise SystemExit("unknown model %r (known: %s)" % (model, sorted({m for m, _ in TRAINERS})))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gpu_count():
    v = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    if v is not None:
        return len([x for x in v.split(",") if x])
    try:
        import torch
        return torch.cuda.device_count()  # does not initialise HIP on this image
    except Exception:
        return 0


def build_commands(model, mode, nproc, extra, port, eval_=True, hb_dir=None):
    mod, mode_args = resolve(model, mode)
    env_base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(nproc),
                    DTM_RUN_ID=str(port))
    if hb_dir:
        env_base[hbmod.ENV_DIR] = hb_dir
    env_base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmds = []
    for r in range(nproc):
        env = dict(env_base, RANK=str(r), LOCAL_RANK=str(r))
        cmds.append(("worker_%d" % r, [sys.executable, "-m", "%s.%s" % (PKG, mod)] + mode_args + list(extra), env))
    ev = None
    if eval_ and model in EVALS:
        env = dict(os.environ)
        env["HIP_VISIBLE_DEVICES"] = ""  # evaluator on the host, like the reference (train.sh:58)
        ev = ("model_eval", [sys.executable, "-m", "%s.%s" % (PKG, EVALS[model])] +
              [a for a in extra if a.startswith(("--data_dir", "--train_dir"))], env)
        ev = (ev[0], [a.replace("--train_dir", "--checkpoint_dir") for a in ev[1]], ev[2])
    return cmds, ev


def _start(cmds, log_dir, pf, attempt):
    procs = []
    for name, cmd, env in cmds:
        out = open(os.path.join(log_dir, name + ".log"), "a" if attempt else "w")
        if attempt:
            out.write("\n==== restart %d ====\n" % attempt)
            out.flush()
        p = subprocess.Popen(cmd, env=env, stdout=out, stderr=subprocess.STDOUT, start_new_session=True)
        procs.append(p)
        pf.write("%d\n" % p.pid)
        pf.flush()
    return procs


def _kill_group(p, sig=signal.SIGTERM):
    try:
        os.killpg(p.pid, sig)
    except (ProcessLookupError, PermissionError):
        pass


HANG_EXIT = 124  # exit code reported for a job stopped by the hang detector (as timeout(1) does)


def _stop_all(procs, poll_s, grace_s):
    for p in procs:
        if p.poll() is None:
            _kill_group(p)
    t0 = time.time()
    while any(p.poll() is None for p in procs) and time.time() - t0 < grace_s:
        time.sleep(poll_s)
    for p in procs:
        if p.poll() is None:
            _kill_group(p, signal.SIGKILL)
            p.wait()


def _supervise(procs, poll_s=0.2, grace_s=10.0, hb_dir=None, hang_timeout=0.0):
    """Wait for all ranks; when one fails, stop the rest (a dead peer would otherwise leave the
    survivors blocked in a collective until its timeout).  With ``hang_timeout`` > 0 a rank whose
    heartbeat is older than that is treated as failed too (a hung rank never exits by itself).
    Returns the first non-zero exit code (HANG_EXIT for a detected hang)."""
    started = time.time()
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            _stop_all(procs, poll_s, grace_s)
            return bad[0]
        if all(c is not None for c in codes):
            return 0
        if hang_timeout > 0 and hb_dir:
            live = [r for r, c in enumerate(codes) if c is None]
            stale = [r for r in hbmod.stale_ranks(hb_dir, len(procs), hang_timeout, started) if r in live]
            if stale:
                print("launcher: rank(s) %s sent no heartbeat for %.0f s - treating the job as hung"
                      % (stale, hang_timeout), flush=True)
                _stop_all(procs, poll_s, grace_s)
                return HANG_EXIT
        time.sleep(poll_s)


def launch(model, mode, nproc, extra, log_dir, eval_=False, eval_delay=20.0, wait=True, port=None,
           max_restarts=0, hang_timeout=0.0):
    """Start ``nproc`` ranks (+ evaluator); with ``max_restarts`` > 0 a failed (or, with
    ``hang_timeout`` > 0, hung) job is restarted (fresh rendezvous port) and resumes from the latest
    checkpoint in its train_dir."""
    os.makedirs(log_dir, exist_ok=True)
    hb_dir = os.path.join(log_dir, "heartbeat")
    evp = None
    attempt = 0
    with open(os.path.join(log_dir, "pids"), "w") as pf:
        while True:
            hbmod.clear(hb_dir)
            cmds, ev = build_commands(model, mode, nproc, extra, port or free_port(), eval_, hb_dir)
            # a restart must resume, so never pass --fresh again
            if attempt:
                cmds = [(n, [a for a in c if a not in ("--fresh", "--fresh=true", "--fresh=True")],
                         dict(e, DTM_ATTEMPT=str(attempt))) for n, c, e in cmds]
            procs = _start(cmds, log_dir, pf, attempt)
            if ev is not None and evp is None:
                time.sleep(eval_delay)
                out = open(os.path.join(log_dir, ev[0] + ".log"), "w")
                evp = subprocess.Popen(ev[1], env=ev[2], stdout=out, stderr=subprocess.STDOUT,
                                       start_new_session=True)
                pf.write("%d\n" % evp.pid)
                pf.flush()
            if not wait:
                return procs
            rc = _supervise(procs, hb_dir=hb_dir, hang_timeout=hang_timeout)
            if rc == 0 or attempt >= max_restarts:
                break
            attempt += 1
            print("launcher: job failed (exit %s); restart %d/%d" % (rc, attempt, max_restarts), flush=True)
    if evp is not None:
        _kill_group(evp)
    return rc


def stop(log_dir):
    """clear.sh replacement: signal exactly the recorded process groups."""
    path = os.path.join(log_dir, "pids")
    if not os.path.exists(path):
        return 0
    n = 0
    for line in open(path):
        line = line.strip()
        if not line:
            continue
        try:
            os.killpg(int(line), signal.SIGTERM)
            n += 1
        except (ProcessLookupError, PermissionError):
            pass
    os.remove(path)
    return n


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--model", default="")
    ap.add_argument("--mode", default="bsp")
    ap.add_argument("--nproc", type=int, default=0, help="ranks (default: visible GPUs, min 1)")
    ap.add_argument("--log_dir", default="")
    ap.add_argument("--eval", action="store_true", help="also start the evaluator (train.sh:57-59)")
    ap.add_argument("--eval_delay", type=float, default=20.0)
    ap.add_argument("--stop", action="store_true")
    ap.add_argument("--max_restarts", type=int, default=0, help="restart a failed job and resume")
    ap.add_argument("--hang_timeout", type=float, default=0.0,
                    help="seconds without a rank heartbeat before the job counts as hung (0 = off)")
    ap.add_argument("--dry_run", action="store_true")
    a, extra = ap.parse_known_args(argv)
    if extra and extra[0] == "--":
        extra = extra[1:]
    log_dir = a.log_dir or os.path.join("runs", "%s_%s" % (a.model, a.mode))
    if a.stop:
        print("stopped %d process groups" % stop(log_dir))
        return 0
    if not a.model:
        ap.error("please specify model and sync mode (bsp, asp, ssp)!")
    nproc = a.nproc or max(_gpu_count(), 1)
    if a.dry_run:
        cmds, ev = build_commands(a.model, a.mode, nproc, extra, 29500, a.eval)
        for name, cmd, env in cmds + ([ev] if ev else []):
            print("%s: RANK=%s WORLD_SIZE=%s %s" % (name, env.get("RANK", "-"), env.get("WORLD_SIZE", "-"),
                                                   " ".join(cmd)))
        return 0
    return launch(a.model, a.mode, nproc, extra, log_dir, a.eval, a.eval_delay, max_restarts=a.max_restarts,
                  hang_timeout=a.hang_timeout)


if __name__ == "__main__":
    sys.exit(main())
