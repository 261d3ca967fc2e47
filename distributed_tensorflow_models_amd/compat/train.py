"""``tf.train`` facade: cluster/server, schedules, optimizers, SyncReplicas, EMA, Supervisor, Saver.

This is an API surface over the MI355X runtime, not a graph runtime:
  * ClusterSpec / Server map the reference's ``--ps_hosts/--worker_hosts/--job_name/--task_id``
     onto a torch.distributed process group (RCCL for GPU tensors, gloo on CPU);
    ``ps`` processes have nothing to serve in BSP (gradients are all-reduced) and return from
    ``join()`` immediately; in ASP/SSP the parameter shards live on the worker ranks (C10/C14).
  * optimizers are configuration records consumed by the fused multi-tensor kernel (ops.optim);
  * SyncReplicasOptimizer selects BSP (bucketed all-reduce) semantics (C9);
  * Supervisor = chief init-or-restore from logdir + periodic checkpoints at step boundaries (C7).
"""
import math
import os
import time

import torch

from ..ckpt.saver import (Saver, checkpoint_exists, get_checkpoint_state,  # noqa: F401
                          latest_checkpoint)
from . import logging

# ---------------------------------------------------------------------------------------------
# cluster


class ClusterSpec:
    def __init__(self, cluster):
        self._cluster = {k: list(v) for k, v in cluster.items()}

    def job_tasks(self, job):
        return list(self._cluster.get(job, []))

    def num_tasks(self, job):
        return len(self._cluster.get(job, []))

    def as_dict(self):
        return dict(self._cluster)

    @property
    def jobs(self):
        return list(self._cluster)


class Server:
    """Starts this process' role.  For ``worker`` it initialises the process group: rank =
    task_index, world = #workers, rendezvous at the first worker host (port + 1000)."""

    def __init__(self, cluster, job_name="worker", task_index=0, protocol="grpc", config=None, start=True):
        if isinstance(cluster, dict):
            cluster = ClusterSpec(cluster)
        self.cluster, self.job_name, self.task_index, self.protocol = cluster, job_name, task_index, protocol
        self.target = "dtm://%s/%d" % (job_name, task_index)
        if job_name == "worker" and start:
            from ..parallel import process_group
            workers = cluster.job_tasks("worker")
            if len(workers) > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1:
                host, port = (workers[0].split(":") + ["22223"])[:2] if workers else ("127.0.0.1", "22223")
                process_group.init(rank=task_index, world_size=max(len(workers), 1), master_addr=host,
                                   master_port=int(port) + 1000)

    def join(self):
        logging.info("ps task %d: parameters are owned by worker ranks on the MI355X runtime; nothing to serve",
                     self.task_index)


# ---------------------------------------------------------------------------------------------
# schedules


def exponential_decay(learning_rate, global_step, decay_steps, decay_rate, staircase=False, name=None):
    """lr * rate^(step/decay_steps) (floor when staircase) -- SURVEY.md C19."""
    step = int(global_step.item() if torch.is_tensor(global_step) else global_step)
    p = step / float(decay_steps)
    if staircase:
        p = math.floor(p)
    return learning_rate * decay_rate ** p


class ExponentialDecay:
    """Schedule object (callable on the step) with the same semantics."""

    def __init__(self, learning_rate, decay_steps, decay_rate, staircase=True):
        self.lr, self.steps, self.rate, self.staircase = learning_rate, decay_steps, decay_rate, staircase

    def __call__(self, step):
        return exponential_decay(self.lr, step, self.steps, self.rate, self.staircase)


def get_or_create_global_step(device=None):
    return torch.zeros((), dtype=torch.int64, device=device)


# ---------------------------------------------------------------------------------------------
# optimizers (records for the fused kernel)


class Optimizer:
    kind = None

    def __init__(self, learning_rate, **kw):
        self.learning_rate = learning_rate
        self.kw = kw

    def config(self):
        d = dict(optimizer=self.kind, lr=self.learning_rate)
        d.update(self.kw)
        return d


class GradientDescentOptimizer(Optimizer):
    kind = "sgd"


class MomentumOptimizer(Optimizer):
    kind = "momentum"

    def __init__(self, learning_rate, momentum, use_nesterov=False):
        if use_nesterov:
            raise NotImplementedError("use_nesterov=True (reference never uses it)")
        super().__init__(learning_rate, momentum=momentum)


class RMSPropOptimizer(Optimizer):
    kind = "rmsprop"

    def __init__(self, learning_rate, decay=0.9, momentum=0.0, epsilon=1e-10):
        super().__init__(learning_rate, rho=decay, momentum=momentum, epsilon=epsilon)


class SyncReplicasOptimizer:
    """BSP wrapper: gradients of all replicas are averaged before one update (C9).  With
    replicas_to_aggregate == total_num_replicas (every reference call site) this is exactly a
    synchronous all-reduce; backup workers (aggregate < total) are not supported (C11)."""

    def __init__(self, opt, replicas_to_aggregate, total_num_replicas=None, variable_averages=None,
                 variables_to_average=None):
        if total_num_replicas is not None and replicas_to_aggregate != total_num_replicas:
            raise NotImplementedError("backup workers (replicas_to_aggregate < total_num_replicas)")
        self.opt = opt
        self.replicas = replicas_to_aggregate
        self.variable_averages = variable_averages

    def config(self):
        d = self.opt.config()
        d["sync_mode"] = "bsp"
        if self.variable_averages is not None:
            d["ema_decay"] = self.variable_averages.decay
        return d

    def get_chief_queue_runner(self):
        return None

    def get_init_tokens_op(self, num_tokens=-1):
        return None


class ExponentialMovingAverage:
    """Shadow variables <v>/ExponentialMovingAverage, decay min(decay, (1+n)/(10+n)) (C22)."""

    def __init__(self, decay, num_updates=None, zero_debias=False, name="ExponentialMovingAverage"):
        self.decay = decay
        self.num_updates = num_updates

    def effective_decay(self, n):
        return min(self.decay, (1.0 + n) / (10.0 + n)) if n is not None else self.decay


def replica_device_setter(ps_tasks=0, ps_device="/job:ps", worker_device="/job:worker", cluster=None):
    """Round-robin placement strings of variables over ps tasks (C14).  On this runtime the result
    is used as the owner map of the ASP/SSP sharded parameter store."""
    if cluster is not None:
        ps_tasks = ClusterSpec(cluster).num_tasks("ps") if isinstance(cluster, dict) else cluster.num_tasks("ps")
    state = {"next": 0}

    def device_fn(var_name=None):
        if ps_tasks <= 0:
            return worker_device
        t = state["next"] % ps_tasks
        state["next"] += 1
        return "%s/task:%d/cpu:0" % (ps_device, t)

    device_fn.ps_tasks = ps_tasks
    return device_fn


# ---------------------------------------------------------------------------------------------
# Supervisor


class Supervisor:
    """Chief init-or-restore from ``logdir``, then checkpoints every ``save_model_secs`` at step
    boundaries (the reference's background saver thread, without racing parameter updates)."""

    def __init__(self, is_chief=True, logdir=None, saver=None, global_step=None, save_model_secs=600,
                 recovery_wait_secs=1, init_op=None, summary_op=None, max_to_keep=5):
        self.is_chief, self.logdir, self.saver = is_chief, logdir, saver
        self.global_step = global_step
        self.save_model_secs = save_model_secs
        self.recovery_wait_secs = recovery_wait_secs
        self._last_save = time.time()
        self.restored_from = None

    def prepare_or_wait_for_session(self, target=None, broadcast_fn=None):
        """Restore the latest checkpoint in logdir (if any); non-chief ranks receive the chief's
        parameters through ``broadcast_fn`` (a collective), replacing the reference's 1-s polling."""
        if self.logdir and self.saver is not None and self.is_chief:
            path = latest_checkpoint(self.logdir)
            if path:
                self.saver.restore(path)
                self.saver.recover_last_checkpoints(self.logdir)
                self.restored_from = path
                logging.info("restored %s", path)
        if broadcast_fn is not None:
            broadcast_fn()
        return self

    def save_path(self):
        return os.path.join(self.logdir, "model.ckpt")

    def maybe_save(self, step, force=False, async_=True):
        """Periodic saves are asynchronous (pinned-host snapshot + writer thread); a forced (final)
        save is synchronous and also drains any save still in flight."""
        if not (self.is_chief and self.logdir and self.saver is not None):
            return None
        if force or (self.save_model_secs and time.time() - self._last_save >= self.save_model_secs):
            self._last_save = time.time()
            use_async = async_ and not force and hasattr(self.saver, "wait")
            path = self.saver.save(self.save_path(), global_step=step, async_=use_async) if use_async else \
                self.saver.save(self.save_path(), global_step=step)
            if force and hasattr(self.saver, "wait"):
                self.saver.wait()
            return path
        return None

    def should_stop(self):
        return False

    def stop(self):
        pass
