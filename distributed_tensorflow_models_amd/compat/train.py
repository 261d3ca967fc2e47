"""``tf.train`` facade: cluster/server, schedules, optimizers, SyncReplicas, EMA, Supervisor, Saver.

This is an API surface over the MI355X runtime, not a graph runtime:
  * ClusterSpec / Server map the reference's ``--ps_hosts/--worker_hosts/--job_name/--task_id``
     onto a torch.distributed process group (RCCL for GPU tensors, gloo on CPU);
    ``ps`` processes have nothing to serve in BSP (gradients are all-reduced) and return from
    ``join()`` immediately; in ASP/SSP the parameter shards live on the worker ranks (C10/C14).
  * optimizers build the training step: ``opt.minimize(loss_fn, model, global_step)`` (or
    compute_gradients + apply_gradients) returns a ``TrainOp`` over engine.TrainStep (fused
    multi-tensor update, ops.optim) or the ASP parameter store;
  * SyncReplicasOptimizer selects BSP (bucketed all-reduce) semantics (C9), with the EMA of
    ``variables_to_average`` (C22);
  * Supervisor = chief init-or-restore from logdir + periodic checkpoints at step boundaries (C7);
    ``prepare_or_wait_for_session`` returns a ``Session`` whose ``run([train_op, "loss", gs])`` steps.
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
    """lr * rate^(step/decay_steps) (floor when staircase) -- SURVEY.md C19.

    With an int step this is the value.  With the global-step TENSOR (the reference's call shape,
    alexnet/cifar10_alexnet_bsp.py:72-76) it returns a ``DecayedLearningRate`` bound to that tensor:
    the optimizer re-evaluates it at every step, as the TF graph op does."""
    if torch.is_tensor(global_step):
        return DecayedLearningRate(ExponentialDecay(learning_rate, decay_steps, decay_rate, staircase), global_step)
    step = int(global_step)
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


class DecayedLearningRate:
    """A schedule bound to a global-step tensor: ``float(lr)`` = the value at the tensor's current step,
    ``lr(step)`` = the value at ``step``."""

    def __init__(self, schedule, global_step):
        self.schedule, self.global_step = schedule, global_step

    def __call__(self, step=None):
        return float(self.schedule(int(self.global_step) if step is None else step))

    def __float__(self):
        return self()


def get_or_create_global_step(device=None):
    return torch.zeros((), dtype=torch.int64, device=device)


def global_step(sess, global_step_tensor):
    """tf.train.global_step(sess, gs): the current value as an int."""
    return int(global_step_tensor)


# ---------------------------------------------------------------------------------------------
# optimizers (records for the fused kernel)


class GradientsAndVars:
    """What ``compute_gradients`` returns on this runtime: the loss function and the model whose
    trainable variables it differentiates (there is no symbolic gradient list - gradients are
    produced by backward into the flat all-reduce buffer).  ``scale(w)`` is the reference's per-worker
    batch-size hook (grads * batch_size / FLAGS.batch_size)."""

    def __init__(self, loss, model, scale=1.0):
        self.loss, self.model, self.weight = loss, model, float(scale)

    def scale(self, w):
        return GradientsAndVars(self.loss, self.model, self.weight * float(w))


class Optimizer:
    kind = None

    def __init__(self, learning_rate, **kw):
        self.learning_rate = learning_rate
        self.kw = kw

    def config(self):
        d = dict(optimizer=self.kind, lr=self.learning_rate)
        d.update(self.kw)
        return d

    # ---- graph-building API (consumed: these build the MI355X training step) ------------------
    def compute_gradients(self, loss, model=None, var_list=None):
        """``loss``: callable(logits, labels) -> scalar loss (the graph the reference builds after the
        network); ``model``: the network (nn.Module from models/ or nets_factory)."""
        if model is None:
            raise ValueError("compute_gradients needs the model whose variables the loss depends on")
        return GradientsAndVars(loss, model)

    def apply_gradients(self, grads_and_vars, global_step=None, name=None, **kw):
        return TrainOp(self, grads_and_vars, global_step, **kw)

    def minimize(self, loss, model=None, global_step=None, var_list=None, **kw):
        return self.apply_gradients(self.compute_gradients(loss, model), global_step=global_step, **kw)


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
        self.variables_to_average = variables_to_average

    def config(self):
        d = self.opt.config()
        d["sync_mode"] = "bsp"
        if self.variable_averages is not None:
            d["ema_decay"] = self.variable_averages.decay
        return d

    def compute_gradients(self, loss, model=None, var_list=None):
        return self.opt.compute_gradients(loss, model, var_list)

    def apply_gradients(self, grads_and_vars, global_step=None, name=None, **kw):
        return TrainOp(self, grads_and_vars, global_step, **kw)

    def minimize(self, loss, model=None, global_step=None, var_list=None, **kw):
        return self.apply_gradients(self.compute_gradients(loss, model), global_step=global_step, **kw)

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
        self._stop = False

    def prepare_or_wait_for_session(self, target=None, broadcast_fn=None, config=None):
        """Restore the latest checkpoint in logdir (if any) and return a ``Session``.  Every rank restores
        the same checkpoint file in BSP (identical replicas, no broadcast needed); ``broadcast_fn`` (a
        collective) lets non-chief ranks receive the chief's values instead, replacing the reference's
        1-s polling of an initialised PS."""
        op = _DEFAULT_GRAPH["train_op"]
        restore_here = self.is_chief or (op is not None and op.mode == "bsp")
        if self.logdir and self.saver is not None and restore_here:
            path = latest_checkpoint(self.logdir) if os.path.isdir(self.logdir) else None
            if path:
                self.saver.restore(path)
                if self.is_chief:
                    self.saver.recover_last_checkpoints(self.logdir)
                self.restored_from = path
                logging.info("restored %s", path)
                if op is not None:
                    op.restored()
        if broadcast_fn is not None:
            broadcast_fn()
        self._last_save = time.time()
        return Session(self)

    def start_queue_runners(self, sess=None, queue_runners=None):
        """Input threads start with the pipeline objects themselves; the BSP chief queue runner does not
        exist (the all-reduce replaces it).  Returns the (empty) thread list."""
        return []

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
        return self._stop

    def request_stop(self, ex=None):
        self._stop = True

    def stop(self):
        """End of training: a final (synchronous) checkpoint by the chief, as Supervisor.stop() does."""
        if self._stop:
            return
        self._stop = True
        op = _DEFAULT_GRAPH["train_op"]
        if op is not None:
            op.finish()
        if self.global_step is not None:
            self.maybe_save(int(self.global_step), force=True)
        if op is not None:
            op.close()


# ---------------------------------------------------------------------------------------------
# the training "graph": optimizer record + loss + model -> the MI355X training step


def trainable_variables(model):
    """tf.trainable_variables() of a model: its trainable parameters, in creation order."""
    return [p for p in model.parameters() if p.requires_grad]


def moving_average_variables(model):
    """tf.moving_average_variables(): the BN moving statistics (slim BN puts them there)."""
    from ..engine import moving_average_buffers
    return moving_average_buffers(model)


_DEFAULT_GRAPH = {"train_op": None}


class TrainOp:
    """The result of ``opt.minimize`` / ``opt.apply_gradients``: one training step per ``Session.run``.

    Built from the optimizer records exactly as the reference wires them
    (alexnet/cifar10_alexnet_bsp.py:72-94, inception/imagenet_inception_bsp.py:123-157):
      * ``SyncReplicasOptimizer(opt, W, W, variable_averages=ema)`` -> BSP: ``engine.TrainStep``
        (bucketed all-reduce of the mean gradient, fused update, EMA of ``variables_to_average``);
      * a plain optimizer with more than one worker -> ASP (reference vgg/cifar10_vgg_asp.py,
        inception/imagenet_inception_asp.py): owner-sharded ``parallel.asp.ParamStore`` + ``ASPTrainStep``;
      * one worker -> the same TrainStep on one rank.
    ``weight_decay``: the reference's ``wd * add_n(l2_loss(v) for v in trainable_variables())`` term,
    applied as the identical coupled gradient term inside the fused optimizer (an explicit L2 term in
    the loss callable works too, through autograd, just slower).  The learning rate may be a float or
    the ``DecayedLearningRate`` returned by ``exponential_decay(lr, global_step_tensor, ...)``."""

    def __init__(self, optimizer, grads, global_step=None, weight_decay=None, bucket_mb=32.0, label_smoothing=0.0,
                 input_fn=None):
        from ..engine import TrainStep
        from ..parallel import process_group as pg
        sync = isinstance(optimizer, SyncReplicasOptimizer)
        base = optimizer.opt if sync else optimizer
        ema = optimizer.variable_averages if sync else getattr(optimizer, "variable_averages", None)
        self.model, self.loss, self.global_step = grads.model, grads.loss, global_step
        self.input_fn = input_fn
        self.world = pg.world_size()
        self.mode = "bsp" if (sync or self.world == 1) else "asp"
        lr = base.learning_rate
        sched = lr if callable(lr) else None
        lr0 = float(lr(0) if isinstance(lr, DecayedLearningRate) else lr)
        if isinstance(lr, DecayedLearningRate):
            sched = lr.schedule  # evaluated at the engine's own step counter
        kw = base.config()
        kw.pop("optimizer", None), kw.pop("lr", None)
        if weight_decay is not None:
            for p in trainable_variables(self.model):
                p.weight_decay = float(weight_decay)
        avg = getattr(optimizer, "variables_to_average", None)
        if self.world > 1:  # the chief's initial values everywhere (reference: chief init_op, workers wait)
            pg.broadcast_tensors([p for p in self.model.parameters()] + list(self.model.buffers()))
        if self.mode == "bsp":
            ema_buffers = True
            if avg is not None:
                ids = {id(t) for t in avg}
                ema_buffers = any(id(b) in ids for b in moving_average_variables(self.model))
            self.step = TrainStep(self.model, optimizer=base.kind, lr=lr0, lr_schedule=sched, bucket_mb=bucket_mb,
                                  label_smoothing=label_smoothing, batch_weight=grads.weight,
                                  ema_decay=ema.decay if ema is not None else None, ema_buffers=ema_buffers,
                                  momentum=kw.get("momentum", 0.9), rho=kw.get("rho", 0.9),
                                  epsilon=kw.get("epsilon", 1e-10))
            self.step.loss_fn = self._loss
            self.store = None
        else:
            from ..engine import prepare_compute_copies
            from ..parallel.asp import ASPTrainStep, ParamStore
            prepare_compute_copies(self.model)
            self.store = ParamStore(list(self.model.parameters()), base.kind, lr0, kw.get("momentum", 0.9),
                                    kw.get("rho", 0.9), kw.get("epsilon", 1e-10),
                                    run_id=os.environ.get("DTM_RUN_ID", "facade"),
                                    buffers=moving_average_variables(self.model))
            self.step = ASPTrainStep(self.model, self._loss_weighted(grads.weight), self.store, sched)
        _DEFAULT_GRAPH["train_op"] = self

    def _loss(self, out, labels):
        loss = self.loss(out, labels)
        w = self.step.batch_weight if hasattr(self.step, "batch_weight") else 1.0
        return loss * w if w != 1.0 else loss

    def _loss_weighted(self, w):
        def fn(out, labels):
            loss = self.loss(out, labels)
            return loss * w if w != 1.0 else loss
        return fn

    def run(self, images, labels):
        """One training step; returns (loss tensor, global step after the step)."""
        if self.mode == "bsp":
            loss = self.step(images, labels)
            gs = self.step.global_step
        else:
            loss, gs = self.step(images, labels)
        if self.global_step is not None:
            self.global_step.fill_(int(gs))
        return loss, gs

    def variables(self, prefix="", partitions=None):
        """Every variable a tf.train.Saver() of this graph saves (weights, BN statistics, optimizer slots,
        EMA shadows, global step) with its TF name."""
        from ..ckpt.saver import model_variables
        opt = self.step.opt if self.mode == "bsp" else None
        vs = model_variables(self.model, opt, self.global_step, prefix=prefix, partitions=partitions,
                             store=self.store)
        return vs

    def finish(self):
        """End of training: ASP replicas pull the final shared parameters (what the chief saves)."""
        if self.store is not None:
            self.store.pull()

    def close(self):
        if self.store is not None:  # owners keep their shards alive until every worker is done
            from ..parallel.asp import wait_all_done
            wait_all_done(self.store.store, self.world, self.store.run_id)
            self.store.close()
            self.store = None
        elif self.mode == "bsp":
            self.step.dp.close()

    def restored(self):
        """After a restore: the engine's counters and compute copies follow the restored tensors."""
        from ..ops.nn import invalidate_weight_copies
        invalidate_weight_copies(self.model.parameters())
        if self.mode == "bsp" and self.global_step is not None:
            self.step.global_step = int(self.global_step)
            self.step.opt.num_updates = int(self.global_step)


class Saver:
    """tf.train.Saver facade: ``Saver()`` (no var_list) saves every variable of the default graph (the
    last built TrainOp), resolved when first used, like TF's global-variables default."""

    def __init__(self, var_list=None, max_to_keep=5, prefix="", partitions=None):
        from ..ckpt import saver as _saver
        self._impl = _saver.Saver(var_list, max_to_keep=max_to_keep) if var_list is not None else None
        self._max_to_keep, self._prefix, self._partitions = max_to_keep, prefix, partitions

    def _resolve(self):
        if self._impl is None:
            from ..ckpt import saver as _saver
            op = _DEFAULT_GRAPH["train_op"]
            if op is None:
                raise ValueError("Saver(): no variables (build the train op first)")
            self._impl = _saver.Saver(op.variables(self._prefix, self._partitions), max_to_keep=self._max_to_keep)
        return self._impl

    def __getattr__(self, name):  # save / restore / wait / recover_last_checkpoints
        return getattr(self._resolve(), name)


class Session:
    """``sess.run(fetches, feed_dict)`` over TrainOps and tensors.  ``fetches``: a TrainOp (-> its loss
    as a float), a tensor (-> its value: the global step as an int), or a list / tuple of them, as in
    ``sess.run([train_op, loss, global_step], feed_dict=...)``; the string ``"loss"`` fetches the loss of
    the train op run in the same call.  ``feed_dict``: {"images": x, "labels": y} (or the train op's
    ``input_fn`` supplies the batch); ``{"batch_size": n}`` uses the first n examples and weights the
    gradient by n / the fed batch's size (the reference's per-step batch placeholder, C15)."""

    def __init__(self, supervisor=None):
        self.sv = supervisor

    def run(self, fetches, feed_dict=None):
        single = not isinstance(fetches, (list, tuple))
        fl = [fetches] if single else list(fetches)
        feed = dict(feed_dict or {})
        results, loss = {}, None
        for i, f in enumerate(fl):
            if isinstance(f, TrainOp):
                x, y = feed.get("images"), feed.get("labels")
                if x is None:
                    if f.input_fn is None:
                        raise ValueError("feed images/labels or build the train op with input_fn")
                    x, y = f.input_fn()
                n = feed.get("batch_size")
                if n is not None and int(n) < x.shape[0]:
                    w = int(n) / float(x.shape[0])
                    x, y = x[:int(n)], y[:int(n)]
                    if f.mode == "bsp":
                        saved = f.step.batch_weight
                        f.step.batch_weight = saved * w
                        try:
                            loss, gs = f.run(x, y)
                        finally:
                            f.step.batch_weight = saved
                    else:
                        loss, gs = f.run(x, y)
                else:
                    loss, gs = f.run(x, y)
                if self.sv is not None:
                    self.sv.maybe_save(int(gs))
                results[i] = float(loss)
        for i, f in enumerate(fl):
            if i in results:
                continue
            if isinstance(f, str) and f == "loss":
                results[i] = float(loss) if loss is not None else float("nan")
            elif torch.is_tensor(f):
                results[i] = int(f) if (f.dim() == 0 and not f.is_floating_point()) else f.detach().cpu().numpy()
            else:
                results[i] = f
        out = [results[i] for i in range(len(fl))]
        return out[0] if single else out

    def close(self):
        if self.sv is not None:
            self.sv.stop()
