"""GPU ImageNet input pipeline (reference inception/image_processing.py:
batch_inputs / image_preprocessing with num_readers reader threads and num_preprocess_threads
preprocessing threads).

MI355X-native split of the work:
  * host: TFRecord readers (threads) -> JPEG decode on a thread pool (PIL releases the GIL while it
    decodes) -> per-image random parameters (``imagenet.sample_params``: distorted bounding box,
    resize method = thread id % 4, flip, colour factors and ordering = thread id % 2, with thread id =
    the example's slot % num_preprocess_threads) -> a background assembler packs each batch into a
    pinned ragged uint8 buffer + a parameter table (two batches ahead);
  * device: one H2D copy per batch and two HIP kernels (``dtm_imagenet_prep``, csrc/kernels/image.hip):
    crop + TF-1 legacy resample + flip + colour distortion + clip + [-1, 1], written straight into
    the bf16 NHWC batch the model consumes.  The host oracle of the same math is
    ``imagenet.preprocess_with_params`` (tests/test_data_gpu.py).
"""
import ctypes
import queue
import random
import threading
from concurrent.futures import CancelledError, ThreadPoolExecutor

import numpy as np
import torch

from ..ops import _lib
from . import imagenet
from .tfrecord import tf_record_iterator

PARAM_FIELDS = ("src_off", "h", "w", "y0", "x0", "ch", "cw", "method", "flip", "color", "ordering",
                "bright", "sat", "hue", "contrast")
_PARAM_DT = np.dtype([("src_off", "<i8"), ("h", "<i4"), ("w", "<i4"), ("y0", "<i4"), ("x0", "<i4"),
                      ("ch", "<i4"), ("cw", "<i4"), ("method", "<i4"), ("flip", "<i4"), ("color", "<i4"),
                      ("ordering", "<i4"), ("bright", "<f4"), ("sat", "<f4"), ("hue", "<f4"),
                      ("contrast", "<f4")])


def _decode_chunk(tasks):
    """Decode worker (thread or spawned process): [(serialized Example, thread id, seed, train)] ->
    [(HxWx3 uint8, label, preprocessing parameters)].  The parameters are drawn here, from a per-image
    seed the assembler assigned in submission order, so the stream is reproducible for a given seed
    and the assembler thread does no per-image sampling."""
    out = []
    for rec, tid, seed, train in tasks:
        try:
            data, label, bbox, _ = imagenet.parse_example_proto(rec)
            img = imagenet._decode_jpeg(data)
            p = imagenet.sample_params(img.shape[0], img.shape[1], bbox, np.random.RandomState(seed), tid, train)
        except Exception as e:  # corrupt / undecodable record: skipped (and counted) by the assembler
            out.append((None, repr(e), None))
            continue
        out.append((img, label, p))
    return out


def param_table(images, params):
    """-> structured parameter table (src_off from the images' byte sizes), built in one numpy call."""
    offs = np.cumsum([0] + [im.nbytes for im in images])
    rows = [(int(offs[i]), im.shape[0], im.shape[1]) + tuple(p[k] for k in PARAM_FIELDS[3:])
            for i, (im, p) in enumerate(zip(images, params))]
    return np.array(rows, _PARAM_DT), int(offs[-1])


def pack_batch(images, params, out=None):
    """-> (uint8 ragged buffer, structured parameter table) for a list of HxWx3 uint8 images.  ``out``
    (optional) = a uint8 array of at least the total size to pack into (e.g. a pinned host tensor's
    numpy view): the copies are plain contiguous numpy copies, which run without the GIL."""
    tab, total = param_table(images, params)
    buf = out[:total] if out is not None else np.empty(total, np.uint8)
    for i, im in enumerate(images):
        o = int(tab[i]["src_off"])
        np.copyto(buf[o:o + im.nbytes], np.ascontiguousarray(im, np.uint8).reshape(-1))
    return buf, tab


def gpu_preprocess(images, params, size, device, out_dtype=torch.bfloat16):
    """Run the HIP preprocessing on host-decoded images with given parameters -> [B, size, size, 3]."""
    L = _lib.lib()
    assert L.dtm_prep_params_bytes() == _PARAM_DT.itemsize
    buf, tab = pack_batch(images, params)
    return _launch(torch.from_numpy(buf), torch.from_numpy(tab.view(np.uint8)), len(images), size, device,
                   out_dtype)


def _launch(buf_cpu, tab_cpu, B, size, device, out_dtype, stage=None):
    L = _lib.lib()
    src = buf_cpu.to(device, non_blocking=True)
    tab = tab_cpu.to(device, non_blocking=True)
    if stage is None or stage.numel() < B * size * size * 3:
        stage = torch.empty(B * size * size * 3, device=device, dtype=torch.float32)
    sums = torch.empty(B * 3, device=device, dtype=torch.float32)
    out = torch.empty((B, size, size, 3), device=device, dtype=out_dtype)
    rc = L.dtm_imagenet_prep(_lib.ptr(src), _lib.ptr(tab), _lib.ptr(stage), _lib.ptr(sums), _lib.ptr(out),
                             int(out_dtype == torch.bfloat16), B, size, _lib.stream_ptr())
    if rc != 0:
        raise RuntimeError("dtm_imagenet_prep failed (%d)" % rc)
    return out, stage


class GPUBatchInputs:
    """Drop-in for ``imagenet.BatchInputs`` producing device batches ([B,S,S,3] bf16, [B] int64)."""

    def __init__(self, dataset, batch_size, train=True, image_size=299, num_preprocess_threads=4, num_readers=4,
                 num_decoders=8, seed=0, device="cuda", shuffle_buffer=1024, prefetch=2, decode_processes=None):
        self.files = dataset.data_files()
        self.B, self.S, self.train = batch_size, image_size, train
        self.device = torch.device(device)
        self.nthreads = max(1, num_preprocess_threads)
        self.records = queue.Queue(maxsize=shuffle_buffer)
        self.ready = queue.Queue(maxsize=max(1, prefetch))
        self.stop = threading.Event()
        self.bad_records = 0
        self.ndec = max(1, num_decoders)
        # decoders: processes (spawned - never forked from a process holding a HIP context) by default;
        # a thread pool is GIL-bound in PIL's Python-level JPEG header parsing and the Example parse
        # (DTM_DECODE_PROCESSES=0 or decode_processes=False selects threads)
        if decode_processes is None:
            import os
            decode_processes = os.environ.get("DTM_DECODE_PROCESSES", "1") != "0" and self.ndec > 1
        self.chunk = 8 if decode_processes else 1  # records per task (fewer IPC round trips)
        if decode_processes:
            import multiprocessing
            from concurrent.futures import ProcessPoolExecutor
            self.pool = ProcessPoolExecutor(max_workers=self.ndec, mp_context=multiprocessing.get_context("spawn"))
        else:
            self.pool = ThreadPoolExecutor(max_workers=self.ndec)
        self.rng = np.random.RandomState(seed)
        self.slot = 0
        self.pin = self.device.type == "cuda" and torch.cuda.is_available()
        self.threads = []
        for r in range(num_readers):
            t = threading.Thread(target=self._read, args=(r, num_readers, seed + r), daemon=True)
            t.start()
            self.threads.append(t)
        t = threading.Thread(target=self._assemble, daemon=True)
        t.start()
        self.threads.append(t)
        self._stage = None
        self.images_done = 0

    def _read(self, rid, n, seed):
        rng = random.Random(seed)
        files = self.files[rid::n] or self.files
        while not self.stop.is_set():
            if self.train:
                rng.shuffle(files)
            for f in files:
                try:
                    for rec in tf_record_iterator(f):
                        while not self.stop.is_set():
                            try:
                                self.records.put(rec, timeout=0.5)
                                break
                            except queue.Full:
                                continue
                        if self.stop.is_set():
                            return
                except Exception as e:  # unreadable record file: next_batch raises it
                    self._fail("reading %s: %r" % (f, e))
                    return
            # eval loops too (string_input_producer without num_epochs, reference
            # image_processing.py:444-452): repeated eval_once calls on one pipeline never starve

    @staticmethod
    def _decode(rec):
        img, label, _p = _decode_chunk([(rec, 0, 0, False)])[0]
        return img, label

    def _host_buffer(self, nbytes):
        """Pinned (device runs) host staging buffer of at least ``nbytes``, as (tensor, numpy view)."""
        t = torch.empty(max(nbytes, 1), dtype=torch.uint8, pin_memory=self.pin)
        return t, t.numpy()

    def _assemble(self):
        """Decodes stream through the pool (the next batch's JPEGs decode while this one is packed);
        this thread only samples the per-image parameters (one RNG, deterministic order), builds the
        parameter table in one numpy call and copies the pixels straight into a fresh pinned buffer
        (GIL-free numpy copies) - no per-batch pool barrier, no pin_memory() copy."""
        from collections import deque
        pending, done = deque(), deque()
        depth = (self.B + 2 * self.ndec * self.chunk) // self.chunk + 1  # tasks in flight: a batch + look-ahead
        while not self.stop.is_set():
            while len(pending) < depth and not self.stop.is_set():
                tasks = []
                while len(tasks) < self.chunk and not self.stop.is_set():
                    try:
                        rec = self.records.get(timeout=0.5)
                    except queue.Empty:
                        break
                    # the reference's per-thread resize method / colour ordering: thread id = slot % threads
                    tasks.append((rec, self.slot % self.nthreads, int(self.rng.randint(2 ** 31 - 1)), self.train))
                    self.slot += 1
                if not tasks:
                    break
                pending.append(self.pool.submit(_decode_chunk, tasks))
            while pending and len(done) < self.B:
                try:
                    for d in pending.popleft().result():
                        if d[0] is None:
                            self.bad_records += 1
                            imagenet._log_bad_record(d[1], self.bad_records)
                        else:
                            done.append(d)
                except CancelledError:  # close() cancelled the queued decodes
                    return
                except Exception as e:  # e.g. BrokenProcessPool: a decoder process died
                    self._fail("decoder: %r" % (e,))
                    return
            if len(done) < self.B:
                continue
            dec = [done.popleft() for _ in range(self.B)]
            imgs = [d[0] for d in dec]
            labels = [d[1] for d in dec]
            params = [d[2] for d in dec]
            tab, total = param_table(imgs, params)
            bt, view = self._host_buffer(total)
            for i, im in enumerate(imgs):
                o = int(tab[i]["src_off"])
                np.copyto(view[o:o + im.nbytes], im.reshape(-1))
            tt = torch.from_numpy(tab.view(np.uint8))
            lab = torch.tensor(labels, dtype=torch.int64)
            if self.pin:
                tt, lab = tt.pin_memory(), lab.pin_memory()
            while not self.stop.is_set():
                try:
                    self.ready.put((bt, tt, lab), timeout=0.5)
                    break
                except queue.Full:
                    continue

    def _fail(self, msg):
        """A pipeline thread died: hand the error to the consumer (no silent hang in next_batch)."""
        while not self.stop.is_set():
            try:
                self.ready.put(imagenet._PipelineError(msg), timeout=0.5)
                return
            except queue.Full:
                continue

    def next_batch(self):
        item = self.ready.get()
        if isinstance(item, imagenet._PipelineError):
            self.ready.put(item)  # every later call fails the same way
            raise RuntimeError("ImageNet input pipeline failed: %s" % item.msg)
        bt, tt, lab = item
        x, self._stage = _launch(bt, tt, self.B, self.S, self.device, torch.bfloat16, self._stage)
        self.images_done += self.B
        return x, lab.to(self.device, non_blocking=True)

    def close(self):
        self.stop.set()
        self.pool.shutdown(wait=False, cancel_futures=True)


def distorted_inputs(dataset, batch_size, num_preprocess_threads=4, image_size=299, **kw):
    return GPUBatchInputs(dataset, batch_size, True, image_size, num_preprocess_threads, **kw)


def inputs(dataset, batch_size, num_preprocess_threads=4, image_size=299, **kw):
    return GPUBatchInputs(dataset, batch_size, False, image_size, num_preprocess_threads, num_readers=1, **kw)
