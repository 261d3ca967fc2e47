"""tf.train.Saver-compatible checkpointing.

* files: ``<dir>/model.ckpt-<global_step>.index`` / ``.data-00000-of-00001`` (TensorBundle V2) plus
  the text ``checkpoint`` state file (``model_checkpoint_path`` / ``all_model_checkpoint_paths``)
  that evaluators poll (reference cnn/cifar10_eval.py:72-80, inception/inception_eval.py:68-81);
* TF variable names and layouts: conv kernels are exported HWIO ([R,S,C,K]) from the internal
  [K,R,S,C]; optimizer slots ``<v>/Momentum``, ``<v>/RMSProp``, ``<v>/RMSProp_1``; EMA shadows
  ``<v>/ExponentialMovingAverage``; ``global_step`` int64;
* ``max_to_keep`` retention; writes are atomic (tempstate + rename in the native writer);
* the ``.meta`` GraphDef is not produced (there is no TF graph) - documented deviation.
"""
import os
import re
import threading

import numpy as np
import torch

from .bundle import DT_BFLOAT16, BundleReader, partition_axis0, write_bundle


class TFVar:
    """One checkpoint variable.  ``partitions``: the variable lives under a partitioned variable_scope
    (tf.fixed_size_partitioner(P, axis=0), reference alexnet/cifar10_alexnet_bsp.py:50-51,
    vgg/cifar10_vgg_bsp.py:52-53) and is written as P axis-0 slices of its TF-layout tensor."""
    __slots__ = ("name", "tensor", "layout", "partitions")

    def __init__(self, name, tensor, layout=None, partitions=None):
        self.name, self.tensor, self.layout, self.partitions = name, tensor, layout, partitions

    def _wrap(self, arr, tf_dtype=None):
        if self.partitions and arr.ndim >= 1:
            return partition_axis0(arr, self.partitions, tf_dtype)
        return (arr, tf_dtype) if tf_dtype is not None else arr

    def export(self):
        t = self.tensor.detach()
        if self.layout == "KRSC->HWIO":
            t = t.permute(1, 2, 3, 0)
        if t.dtype == torch.bfloat16:
            return self._wrap(t.contiguous().view(torch.int16).cpu().numpy().view(np.uint16), DT_BFLOAT16)
        return self._wrap(t.contiguous().cpu().numpy())

    def load(self, arr):
        t = torch.from_numpy(np.require(arr, requirements="C"))
        if self.layout == "KRSC->HWIO":
            t = t.permute(3, 0, 1, 2)
        if tuple(t.shape) != tuple(self.tensor.shape):
            raise ValueError("shape mismatch for %s: ckpt %s vs var %s" % (self.name, tuple(t.shape),
                                                                         tuple(self.tensor.shape)))
        with torch.no_grad():
            if self.tensor.dtype == torch.bfloat16 and t.dtype == torch.int16:
                t = t.view(torch.bfloat16)
            self.tensor.copy_(t.to(self.tensor.dtype))


def model_variables(model, optimizer=None, global_step=None, include_slots=True, prefix="", partitions=None,
                    store=None):
    """Collect TFVar records for a model built from models.layers (+ optimizer slots / EMA).

    prefix: the trainer's variable_scope ('partitioned_space/', 'root/'); partitions: P of its
    fixed_size_partitioner (slots of a partitioned variable are partitioned like it, as TF's
    slot_creator does); store: an ASP/SSP ParamStore whose owner shards hold the optimizer slots."""
    from ..models.layers import tf_variables
    out = []
    by_param = {}
    for name, t, layout, _trainable in tf_variables(model):
        v = TFVar(prefix + name, t, layout, partitions)
        out.append(v)
        by_param[id(t)] = v
    if optimizer is not None and include_slots:
        for p in optimizer.params:
            base = by_param.get(id(p))
            if base is None:
                continue
            st = optimizer.state[p]
            if optimizer.kind == "momentum":
                out.append(TFVar(base.name + "/Momentum", st["s1"], base.layout, partitions))
            elif optimizer.kind == "rmsprop":
                out.append(TFVar(base.name + "/RMSProp", st["s2"], base.layout, partitions))
                out.append(TFVar(base.name + "/RMSProp_1", st["s1"], base.layout, partitions))
            if "ema" in st:
                out.append(TFVar(base.name + "/ExponentialMovingAverage", st["ema"], base.layout, partitions))
        for b, shadow in getattr(optimizer, "buffer_shadows", lambda: [])():
            base = by_param.get(id(b))
            if base is not None:
                out.append(TFVar(base.name + "/ExponentialMovingAverage", shadow, base.layout, partitions))
    if store is not None and include_slots:
        # ASP / SSP: the slots live in the owner shards (every rank maps every shard)
        for i, p in enumerate(store.params):
            base = by_param.get(id(p))
            if base is None:
                continue
            sh = store.shards[i]
            if store.kind == "momentum":
                out.append(TFVar(base.name + "/Momentum", sh["s1"], base.layout, partitions))
            elif store.kind == "rmsprop":
                out.append(TFVar(base.name + "/RMSProp", sh["s2"], base.layout, partitions))
                out.append(TFVar(base.name + "/RMSProp_1", sh["s1"], base.layout, partitions))
    if global_step is not None:
        out.append(TFVar("global_step", global_step))
    return out


class CheckpointState:
    def __init__(self, model_checkpoint_path, all_model_checkpoint_paths):
        self.model_checkpoint_path = model_checkpoint_path
        self.all_model_checkpoint_paths = list(all_model_checkpoint_paths)

    def __repr__(self):
        return "CheckpointState(%r, %r)" % (self.model_checkpoint_path, self.all_model_checkpoint_paths)


def _state_path(d):
    return os.path.join(d, "checkpoint")


def get_checkpoint_state(checkpoint_dir, latest_filename="checkpoint"):
    path = os.path.join(checkpoint_dir, latest_filename)
    if not os.path.exists(path):
        return None
    cur, allp = None, []
    for line in open(path):
        m = re.match(r'\s*(\w+)\s*:\s*"(.*)"\s*$', line)
        if not m:
            continue
        key, val = m.group(1), m.group(2)
        if not os.path.isabs(val):
            val = os.path.join(checkpoint_dir, val)
        if key == "model_checkpoint_path":
            cur = val
        elif key == "all_model_checkpoint_paths":
            allp.append(val)
    if cur is None:
        return None
    return CheckpointState(cur, allp or [cur])


def latest_checkpoint(checkpoint_dir):
    st = get_checkpoint_state(checkpoint_dir)
    if st is None:
        return None
    if os.path.exists(st.model_checkpoint_path + ".index"):
        return st.model_checkpoint_path
    return None


def checkpoint_exists(prefix):
    return os.path.exists(prefix + ".index")


def step_from_path(path):
    """Eval scripts parse global_step from the suffix (reference cnn/cifar10_eval.py:77-80)."""
    return int(path.split("/")[-1].split("-")[-1])


def _write_state(d, current, allp):
    tmp = _state_path(d) + ".tmp"
    with open(tmp, "w") as f:
        f.write('model_checkpoint_path: "%s"\n' % os.path.basename(current))
        for p in allp:
            f.write('all_model_checkpoint_paths: "%s"\n' % os.path.basename(p))
    os.replace(tmp, _state_path(d))


class Saver:
    """Subset of tf.train.Saver: save / restore / last_checkpoints / max_to_keep."""

    def __init__(self, var_list, max_to_keep=5):
        if isinstance(var_list, dict):
            var_list = [TFVar(k, v) if not isinstance(v, TFVar) else v for k, v in var_list.items()]
        self.vars = list(var_list)
        names = [v.name for v in self.vars]
        if len(set(names)) != len(names):
            dup = sorted({n for n in names if names.count(n) > 1})
            raise ValueError("duplicate variable names: %s" % dup[:5])
        self.max_to_keep = max_to_keep
        self.last_checkpoints = []
        self._thread = None
        self._error = None

    def _snapshot(self):
        """Device -> pinned host copies of every variable (HWIO transpose done on the device), queued
        on the current stream; returns (arrays-producer, event)."""
        host = []
        for v in self.vars:
            t = v.tensor.detach()
            if v.layout == "KRSC->HWIO":
                t = t.permute(1, 2, 3, 0)
            t = t.contiguous()
            if t.is_cuda:
                h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                h.copy_(t, non_blocking=True)
            else:
                h = t.clone()
            host.append((v.name, h))
        ev = None
        if any(v.tensor.is_cuda for v in self.vars):
            ev = torch.cuda.Event()
            ev.record()

        def arrays():
            from .bundle import DT_BFLOAT16
            out = {}
            for v, (name, h) in zip(self.vars, host):
                if h.dtype == torch.bfloat16:
                    out[name] = v._wrap(h.view(torch.int16).numpy().view(np.uint16), DT_BFLOAT16)
                else:
                    out[name] = v._wrap(h.numpy())
            return out
        return arrays, ev

    def wait(self):
        """Block until an in-flight asynchronous save has been written."""
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        if self._error is not None:
            err, self._error = self._error, None
            raise err

    def save(self, save_path, global_step=None, write_state=True, async_=False):
        """Write ``<save_path>-<global_step>``.  With ``async_`` the variables are snapshotted to
        pinned host memory on the device stream and the bundle is written by a background thread,
        so the training loop continues immediately (at most one save in flight)."""
        if global_step is not None:
            step = int(global_step.item() if torch.is_tensor(global_step) else global_step)
            prefix = "%s-%d" % (save_path, step)
        else:
            prefix = save_path
        d = os.path.dirname(prefix) or "."
        os.makedirs(d, exist_ok=True)
        self.wait()
        if async_:
            arrays, ev = self._snapshot()

            def run():
                try:
                    if ev is not None:
                        ev.synchronize()
                    write_bundle(prefix, arrays())
                    self._finish_save(prefix, d, write_state)
                except Exception as e:  # surfaced by the next wait()/save()
                    self._error = e
            self._thread = threading.Thread(target=run, name="ckpt-writer", daemon=True)
            self._thread.start()
            return prefix
        write_bundle(prefix, {v.name: v.export() for v in self.vars})
        self._finish_save(prefix, d, write_state)
        return prefix

    def _finish_save(self, prefix, d, write_state):
        if prefix in self.last_checkpoints:
            self.last_checkpoints.remove(prefix)
        self.last_checkpoints.append(prefix)
        if self.max_to_keep and len(self.last_checkpoints) > self.max_to_keep:
            old = self.last_checkpoints.pop(0)
            for f in os.listdir(d):
                full = os.path.join(d, f)
                if full.startswith(old + ".index") or full.startswith(old + ".data-") or full == old + ".meta":
                    os.remove(full)
        if write_state:
            _write_state(d, prefix, self.last_checkpoints)

    def restore(self, save_path, strict=True):
        r = BundleReader(save_path)
        missing = []
        try:
            for v in self.vars:
                if r.has_tensor(v.name):
                    v.load(r.get_tensor(v.name))
                else:
                    missing.append(v.name)
        finally:
            r.close()
        if missing and strict:
            raise KeyError("variables missing from %s: %s" % (save_path, missing[:10]))
        return missing

    def recover_last_checkpoints(self, checkpoint_dir):
        st = get_checkpoint_state(checkpoint_dir)
        if st is not None:
            self.last_checkpoints = [p for p in st.all_model_checkpoint_paths if checkpoint_exists(p)]


def ema_variables_to_restore(variables):
    """Map shadow names -> model vars (tf.train.ExponentialMovingAverage.variables_to_restore):
    evaluation loads ``<v>/ExponentialMovingAverage`` into ``v``."""
    return [TFVar(v.name + "/ExponentialMovingAverage", v.tensor, v.layout) for v in variables]
