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


_COEF_SCRATCH = {}
_SCAN_SCRATCH = {}


def _decode_chunk(tasks, split=False):
    """Decode worker (thread or spawned process): [(serialized Example, thread id, seed, train)] ->
    [(HxWx3 uint8 or None, label, preprocessing parameters, coefficients or None)].  The parameters are
    drawn here, from a per-image seed the assembler assigned in submission order, so the stream is
    reproducible for a given seed and the assembler thread does no per-image sampling.

    ``split`` (decode mode): 0 = full PIL decode here; 1 = only the entropy decode runs here (data/jpeg.py, ~2x
    cheaper than a full PIL decode), the item carries (JpegInfo bytes, int16 coefficients) and the device finishes
    the decode bit-exactly; 2 = only the marker parse + byte unstuffing runs here (~30x cheaper than the entropy
    decode), the item carries (JpegInfo + JpegScan bytes, unstuffed stream) and the device does the rest, Huffman
    decode included.  Files outside the decoders' subset (progressive, CMYK, ...) are decoded by PIL as before."""
    out = []
    for rec, tid, seed, train in tasks:
        try:
            img, label, p, coef = _decode_one(rec, tid, seed, train, split, copy=True)
        except Exception as e:  # corrupt / undecodable record: skipped (and counted) by the assembler
            out.append((None, repr(e), None, None))
            continue
        out.append((img, label, p, coef))
    return out


def _decode_one(rec, tid, seed, train, split, copy=True):
    """One record -> (pixels or None, label, parameters, (JpegInfo bytes, int16 coefficients) or None).
    ``copy=False``: the coefficients are a view of this thread's scratch (valid until its next call)."""
    data, label, bbox, _ = imagenet.parse_example_proto(rec)
    coef = img = None
    if split == 2:
        from . import jpeg
        key = threading.get_ident()
        st = _SCAN_SCRATCH.get(key)
        if st is None or st[0].size < len(data) + jpeg.STREAM_PAD:
            st = _SCAN_SCRATCH[key] = (np.empty(max(1 << 22, len(data) + jpeg.STREAM_PAD), np.uint8),
                                       np.empty(1 << 14, np.int32))
        coef = jpeg.scan_item(data, *st)
        if coef is not None:
            info = np.frombuffer(coef[0], jpeg.INFO_DT, count=1)[0]
            h, w = int(info["height"]), int(info["width"])
    elif split:
        from . import jpeg
        key = threading.get_ident()
        buf = _COEF_SCRATCH.get(key)
        if buf is None:
            buf = _COEF_SCRATCH[key] = np.empty(1 << 21, np.int16)
        r = jpeg.huffman_decode(data, buf)
        if r is not None:
            info, cf = r
            coef = (info.tobytes(), cf.copy() if copy else cf)
            h, w = int(info["height"]), int(info["width"])
    if coef is None:
        img = imagenet._decode_jpeg(data)
        h, w = img.shape[0], img.shape[1]
    p = imagenet.sample_params(h, w, bbox, _SeedRng(seed), tid, train)
    return img, label, p, coef


class _SeedRng(random.Random):
    """Per-image RNG with the numpy RandomState draw interface sample_params uses (randint with an
    exclusive high, uniform): seeding Python's Mersenne Twister costs ~16 us vs RandomState's ~150 us,
    which was half of the per-image parameter sampling."""

    def randint(self, a, b=None):
        if b is None:
            a, b = 0, a
        return self.randrange(a, b)


# ---- decoder processes that read their own shards and hand results over in shared memory ------------
_ALIGN = 64


def _shm_worker(wid, nworkers, files, seed, split, train, nthreads, shm_name, nslots, slot_bytes, per_slot, free_q,
                done_q, stop):
    """Decoder process: reads its share of the TFRecord files (round-robin, reshuffled every epoch in
    training - the reference's num_readers readers), decodes (split or full), samples the per-image
    parameters, and packs results into free slots of its shared-memory ring; only small metadata
    (offsets, JpegInfo bytes, labels, parameters) crosses the queue - no pixel / coefficient pickling."""
    import queue as _q
    from multiprocessing import shared_memory
    shm = shared_memory.SharedMemory(name=shm_name)
    try:
        ring = np.ndarray((nslots * slot_bytes,), np.uint8, buffer=shm.buf)
        mine = files[wid::nworkers] or files[wid % len(files)::len(files)]
        rrng = random.Random(seed * 7919 + wid)
        prng = np.random.RandomState((seed * 1000003 + wid) % (2 ** 31))
        count, slot, meta, off = 0, None, [], 0

        def flush():
            nonlocal slot, meta, off
            if slot is not None and meta:
                done_q.put((wid, slot, meta))
                slot, meta, off = None, [], 0

        while not stop.is_set():
            if train:
                rrng.shuffle(mine)
            for f in mine:
                for rec in tf_record_iterator(f):
                    if stop.is_set():
                        return
                    while slot is None:
                        try:
                            slot = free_q.get(timeout=0.5)
                        except _q.Empty:
                            if stop.is_set():
                                return
                    tid, s = count % nthreads, int(prng.randint(2 ** 31 - 1))
                    count += 1
                    try:
                        img, label, p, coef = _decode_one(rec, tid, s, train, split, copy=False)
                    except Exception as e:
                        meta.append(("bad", repr(e)))
                        continue
                    pay = coef[1].view(np.uint8) if coef is not None else img.reshape(-1)
                    if pay.nbytes > slot_bytes:  # oversized image: pickled instead
                        meta.append(("inline", coef[0] if coef else None, pay.copy(), label, p,
                                     None if coef else img.shape))
                    else:
                        if off + pay.nbytes > slot_bytes:
                            flush()
                            while slot is None:
                                try:
                                    slot = free_q.get(timeout=0.5)
                                except _q.Empty:
                                    if stop.is_set():
                                        return
                        o = slot * slot_bytes + off
                        np.copyto(ring[o:o + pay.nbytes], pay)
                        meta.append(("shm", coef[0] if coef else None, off, pay.nbytes, label, p,
                                     None if coef else img.shape))
                        off += (pay.nbytes + _ALIGN - 1) // _ALIGN * _ALIGN
                    if len(meta) >= per_slot:
                        flush()
            flush()
    except Exception as e:  # a dying worker reports instead of starving the consumer
        try:
            done_q.put(("error", repr(e)))
        except Exception:
            pass
    finally:
        del ring
        shm.close()


class _ShmDecoders:
    """N decoder processes, each with a ring of shared-memory slots (see _shm_worker)."""

    def __init__(self, files, n, seed, split, train, nthreads, nslots=None, slot_mb=24, per_slot=16, batch=0):
        import multiprocessing as mp
        from multiprocessing import shared_memory
        ctx = mp.get_context("spawn")  # never fork a process that may hold a HIP context
        # enough slots that a batch normally fits in what the workers own with one slot each left to fill
        # (the assembler's copy-out under pressure, detach_worker, covers the rest: large images fill a slot
        # with fewer than per_slot items)
        if nslots is None:
            nslots = max(6, -(-int(batch) // max(1, n * per_slot)) + 2)
        self.n, self.nslots, self.slot_bytes = n, nslots, int(slot_mb * (1 << 20))
        self.stop = ctx.Event()
        self.done_q = ctx.Queue()
        self.free_q, self.shm, self.rings, self.procs = [], [], [], []
        for w in range(n):
            shm = shared_memory.SharedMemory(create=True, size=nslots * self.slot_bytes)
            self.shm.append(shm)
            self.rings.append(np.ndarray((nslots * self.slot_bytes,), np.uint8, buffer=shm.buf))
            q = ctx.Queue()
            for sl in range(nslots):
                q.put(sl)
            self.free_q.append(q)
        for w in range(n):
            p = ctx.Process(target=_shm_worker, args=(w, n, list(files), seed, split, train, nthreads, self.shm[w].name,
                                                      nslots, self.slot_bytes, per_slot, self.free_q[w], self.done_q,
                                                      self.stop), daemon=True)
            p.start()
            self.procs.append(p)
        self.refs = {}
        self.detached = 0  # items copied out of shared memory under slot pressure (detach_worker)

    def items(self, msg):
        """(wid, slot, meta) -> decoded items in the pool format, views into the slot (release after use)."""
        from . import jpeg
        wid, slot, meta = msg
        ring = self.rings[wid]
        out = []
        for m in meta:
            if m[0] == "bad":
                out.append((None, m[1], None, None, None))
                continue
            if m[0] == "inline":
                _k, info, pay, label, p, shape = m
            else:
                _k, info, o, nb, label, p, shape = m
                b = slot * self.slot_bytes + o
                pay = ring[b:b + nb]
            if info is not None:  # (device-decode items carry JpegInfo + JpegScan and the raw stream bytes)
                item = (None, label, p, (info, pay if len(info) > jpeg.INFO_DT.itemsize else pay.view(np.int16)))
            else:
                item = (pay.reshape(shape), label, p, None)
            out.append(item + ((wid, slot) if m[0] == "shm" else None,))
        n_shm = sum(1 for m in meta if m[0] == "shm")
        if n_shm:
            self.refs[(wid, slot)] = n_shm
        else:
            self.free_q[wid].put(slot)
        return out

    def release(self, key):
        if key is None:
            return
        self.refs[key] -= 1
        if self.refs[key] == 0:
            del self.refs[key]
            self.free_q[key[0]].put(key[1])

    def held(self, wid):
        """Slots of worker ``wid`` the assembler still holds items in."""
        return sum(1 for k in self.refs if k[0] == wid)

    def detach_worker(self, items, wid):
        """Copy the payloads of ``items`` (a mutable sequence of pool-format items) that live in worker wid's
        slots out of shared memory and release those slots.  Called when the assembler holds all but one of
        a worker's slots: a worker with no free slot blocks, and if the batch still needs its items the
        pipeline would stall for good (large images, or a batch larger than the slots can hold)."""
        for i, d in enumerate(items):
            key = d[4]
            if key is None or key[0] != wid:
                continue
            px = d[0].copy() if d[0] is not None else None
            coef = (d[3][0], d[3][1].copy()) if d[3] is not None else None
            items[i] = (px, d[1], d[2], coef, None)
            self.release(key)
            self.detached += 1

    def close(self):
        self.stop.set()
        for p in self.procs:
            p.join(timeout=5)
            if p.is_alive():
                p.terminate()
        self.rings = []
        for shm in self.shm:
            try:
                shm.close()
                shm.unlink()
            except Exception:
                pass


def _item_hw(d):
    """(height, width) of a decoded item (pixels or split coefficients)."""
    if d[0] is not None:
        return d[0].shape[0], d[0].shape[1]
    from . import jpeg
    info = np.frombuffer(d[3][0], jpeg.INFO_DT, count=1)[0]
    return int(info["height"]), int(info["width"])


def param_table(images, params, hw=None):
    """-> structured parameter table (src_off from the images' byte sizes), built in one numpy call.
    ``hw``: [(h, w)] instead of ``images`` (split-decoded items: their pixels only exist on the device)."""
    hw = hw if hw is not None else [(im.shape[0], im.shape[1]) for im in images]
    offs = np.cumsum([0] + [h * w * 3 for h, w in hw])
    rows = [(int(offs[i]), h, w) + tuple(p[k] for k in PARAM_FIELDS[3:])
            for i, ((h, w), p) in enumerate(zip(hw, params))]
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
                 num_decoders=8, seed=0, device="cuda", shuffle_buffer=1024, prefetch=2, decode_processes=None,
                 split_decode=None, shm_kw=None):
        self.files = dataset.data_files()
        # split JPEG decode (host Huffman + device IDCT / colour, data/jpeg.py; bit-exact with PIL): opt-in
        # (DTM_SPLIT_DECODE=1).  Measured on one MI355X box with 16 decoder processes
        # (profiles/r3/r3_imagenet_pipeline_split_vs_full.log): full host decode 12.2-13.6k img/s, split
        # 9.7-10.3k - with the shared-memory decoder processes the host decode is no longer the bottleneck,
        # and the split path's larger per-batch table work in the assembler thread costs more than it saves.
        # DTM_SPLIT_DECODE=2 / split_decode="device": the device decode (host marker parse + unstuffing only,
        # data/jpeg.py scan_prep; Huffman decode, IDCT and colour as HIP kernels)
        if split_decode is None:
            import os
            env = os.environ.get("DTM_SPLIT_DECODE", "0")
            split_decode = {"1": 1, "2": 2, "device": 2}.get(env, 0) if torch.device(device).type == "cuda" else 0
        self.split = {"full": 0, "split": 1, "device": 2}.get(split_decode, split_decode)
        self.split = int(self.split)  # 0 full host decode, 1 host Huffman + device IDCT, 2 device decode
        self.decode_errors = 0  # device-decoded images whose entropy-coded data was corrupt
        self._status = []
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
        self.rng = np.random.RandomState(seed)
        self.slot = 0
        self.pin = self.device.type == "cuda" and torch.cuda.is_available()
        self.threads = []
        self.workers = self.pool = None
        if decode_processes:
            # decoder processes read their own shards and return results through shared memory (the
            # record / pixel pickling of a process pool capped the pipeline at ~4k img/s per box)
            self.workers = _ShmDecoders(self.files, self.ndec, seed, self.split, train, self.nthreads,
                                        batch=batch_size, **(shm_kw or {}))
            t = threading.Thread(target=self._assemble_shm, daemon=True)
            t.start()
            self.threads.append(t)
            self._stage = None
            self.images_done = 0
            return
        self.pool = ThreadPoolExecutor(max_workers=self.ndec)
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
        img, label, _p, _c = _decode_chunk([(rec, 0, 0, False)])[0]
        return img, label

    def _host_buffer(self, nbytes):
        """Pinned (device runs) host staging buffer of at least ``nbytes``, as (tensor, numpy view)."""
        t = torch.empty(max(nbytes, 1), dtype=torch.uint8, pin_memory=self.pin)
        return t, t.numpy()

    def _assemble(self):
        try:
            self._assemble_loop()
        except Exception as e:  # anything else that kills the assembler surfaces in next_batch
            self._fail("assembler: %r" % (e,))

    def _assemble_loop(self):
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
                pending.append(self.pool.submit(_decode_chunk, tasks, self.split))
            while pending and len(done) < self.B:
                try:
                    for d in pending.popleft().result():
                        if d[0] is None and d[3] is None:
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
            labels = [d[1] for d in dec]
            params = [d[2] for d in dec]
            lab = torch.tensor(labels, dtype=torch.int64)
            if any(d[3] is not None for d in dec):
                item = self._pack_split(dec, params)
            else:
                imgs = [d[0] for d in dec]
                tab, total = param_table(imgs, params)
                bt, view = self._host_buffer(total)
                for i, im in enumerate(imgs):
                    o = int(tab[i]["src_off"])
                    np.copyto(view[o:o + im.nbytes], im.reshape(-1))
                item = (bt, torch.from_numpy(tab.view(np.uint8)), None)
            bt, tt, split = item
            if self.pin:
                tt, lab = tt.pin_memory(), lab.pin_memory()
            while not self.stop.is_set():
                try:
                    self.ready.put((bt, tt, lab, split), timeout=0.5)
                    break
                except queue.Full:
                    continue

    def _assemble_shm(self):
        try:
            self._assemble_shm_loop()
        except Exception as e:
            self._fail("assembler: %r" % (e,))

    def _assemble_shm_loop(self):
        """Batches from the decoder processes' shared-memory slots: B items -> pinned batch buffers (one
        copy out of shared memory), then the slots go back to their workers."""
        from collections import deque
        W = self.workers
        done = deque()
        while not self.stop.is_set():
            while len(done) < self.B and not self.stop.is_set():
                try:
                    msg = W.done_q.get(timeout=0.5)
                except queue.Empty:
                    continue
                if msg[0] == "error":
                    self._fail("decoder process: %s" % (msg[1],))
                    return
                for d in W.items(msg):
                    if d[0] is None and d[3] is None:
                        self.bad_records += 1
                        imagenet._log_bad_record(d[1], self.bad_records)
                        W.release(d[4])
                    else:
                        done.append(d)
                if len(done) < self.B and W.held(msg[0]) >= W.nslots - 1:
                    # the worker is down to its last slot while the batch still needs more items: copy this
                    # worker's pending items out of shared memory so it can keep decoding (no deadlock)
                    W.detach_worker(done, msg[0])
            if len(done) < self.B:
                continue
            dec = [done.popleft() for _ in range(self.B)]
            params = [d[2] for d in dec]
            lab = torch.tensor([d[1] for d in dec], dtype=torch.int64)
            if any(d[3] is not None for d in dec):
                bt, tt, split = self._pack_split(dec, params)
            else:
                imgs = [d[0] for d in dec]
                tab, total = param_table(imgs, params)
                bt, view = self._host_buffer(total)
                for i, im in enumerate(imgs):
                    o = int(tab[i]["src_off"])
                    np.copyto(view[o:o + im.nbytes], im.reshape(-1))
                tt, split = torch.from_numpy(tab.view(np.uint8)), None
            for d in dec:  # payloads copied out of shared memory: slots back to their workers
                W.release(d[4])
            if self.pin:
                tt, lab = tt.pin_memory(), lab.pin_memory()
            while not self.stop.is_set():
                try:
                    self.ready.put((bt, tt, lab, split), timeout=0.5)
                    break
                except queue.Full:
                    continue

    def _pack_split(self, dec, params):
        """Batch of split-decoded items (+ any PIL-decoded fallbacks): one pinned int16 coefficient buffer
        and the JpegDesc table for the device decode, whose RGB outputs land at the parameter table's
        src_off offsets; fallback pixels go in a small pinned buffer of their own (copied to their
        src_off on the device)."""
        from . import jpeg
        hw = [_item_hw(d) for d in dec]
        tab, total = param_table(None, params, hw)
        split_idx = [i for i, d in enumerate(dec) if d[3] is not None]
        if len(dec[split_idx[0]][3][0]) > jpeg.INFO_DT.itemsize:  # device decode items
            batch = jpeg.DeviceBatch([jpeg.unpack_scan_item(*dec[i][3]) for i in split_idx],
                                     rgb_offs=tab["src_off"][split_idx], rgb_bytes=int(total), pin=self.pin)
            return batch, torch.from_numpy(tab.view(np.uint8)), ("device", self._fallbacks(dec, tab), int(total),
                                                                len(split_idx))
        infos = [np.frombuffer(dec[i][3][0], jpeg.INFO_DT)[0] for i in split_idx]
        descs, ncoef, nplane, _nrgb, maxb, maxp = jpeg.batch_table(infos)
        descs["rgb_off"] = tab["src_off"][split_idx]
        coefs = torch.empty(max(ncoef, 8), dtype=torch.int16, pin_memory=self.pin)
        cv = coefs.numpy()
        for j, i in enumerate(split_idx):
            cf = dec[i][3][1]
            b = int(descs[j]["coef_base"])
            np.copyto(cv[b:b + cf.size], cf)
        fb = self._fallbacks(dec, tab)
        dt = torch.from_numpy(descs.view(np.uint8))
        if self.pin:
            dt = dt.pin_memory()
        return coefs, torch.from_numpy(tab.view(np.uint8)), (dt, len(split_idx), int(maxb), int(maxp), int(nplane),
                                                            int(total), fb)

    def _fallbacks(self, dec, tab):
        """PIL-decoded items of a split / device batch: (pinned pixel buffer, [(rgb offset, buffer offset, bytes)])
        or None."""
        falls = [(int(tab[i]["src_off"]), dec[i][0]) for i in range(len(dec)) if dec[i][3] is None]
        if not falls:
            return None
        fb_t, fv = self._host_buffer(sum(im.nbytes for _o, im in falls))
        off, lst = 0, []
        for o, im in falls:
            np.copyto(fv[off:off + im.nbytes], im.reshape(-1))
            lst.append((o, off, im.nbytes))
            off += im.nbytes
        return fb_t, lst

    def _check_status(self, block=False):
        """Count the corrupt images of device-decoded batches whose status copy has landed (no sync)."""
        keep = []
        for host, ev in self._status:
            if block or ev.query():
                ev.synchronize()
                bad = int((host < 0).sum())
                if bad:
                    self.decode_errors += bad
                    import logging
                    logging.getLogger("distributed_tensorflow_models_amd").warning(
                        "input pipeline: %d device-decoded image(s) had corrupt entropy-coded data (%d so far)",
                        bad, self.decode_errors)
            else:
                keep.append((host, ev))
        self._status = keep

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
        bt, tt, lab, split = item
        if split is not None:
            bt = self._device_decode(bt, split)
        x, self._stage = _launch(bt, tt, self.B, self.S, self.device, torch.bfloat16, self._stage)
        self.images_done += self.B
        return x, lab.to(self.device, non_blocking=True)

    def _device_decode(self, coefs, split):
        """IDCT + upsampling + colour of the batch's split items on the device -> the RGB ragged buffer
        (device) that the preprocessing kernel reads; fallback (PIL) pixels are copied into their slots."""
        if split[0] == "device":  # coefs: the jpeg.DeviceBatch
            _k, fb, total, n = split
            rgb = torch.empty(max(total, 1), dtype=torch.uint8, device=self.device)
            if n:
                rgb, status = coefs.launch(self.device, rgb=rgb)
                host = torch.empty(n, dtype=torch.int32, pin_memory=self.pin)
                host.copy_(status, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                self._check_status()
                self._status.append((host, ev))
        else:
            dt, n, maxb, maxp, nplane, total, fb = split
            rgb = self._coef_decode(coefs, dt, n, maxb, maxp, nplane, total)
        if fb is not None:
            fb_t, lst = fb
            src = fb_t.to(self.device, non_blocking=True)
            for o, so, nb in lst:
                rgb[o:o + nb].copy_(src[so:so + nb])
        return rgb

    def _coef_decode(self, coefs, dt, n, maxb, maxp, nplane, total):
        L = _lib.lib()
        rgb = torch.empty(max(total, 1), dtype=torch.uint8, device=self.device)
        if n:
            cd = coefs.to(self.device, non_blocking=True)
            dd = dt.to(self.device, non_blocking=True)
            planes = torch.empty(max(nplane, 8), dtype=torch.uint8, device=self.device)
            rc = L.dtm_jpeg_decode_gpu(_lib.ptr(cd), _lib.ptr(dd), n, maxb, maxp, _lib.ptr(planes), _lib.ptr(rgb),
                                       _lib.stream_ptr())
            if rc != 0:
                raise RuntimeError("dtm_jpeg_decode_gpu failed (%d)" % rc)
        return rgb

    def close(self):
        self.stop.set()
        if self.pool is not None:
            self.pool.shutdown(wait=False, cancel_futures=True)
        if self.workers is not None:
            for t in self.threads:
                t.join(timeout=2)
            self.workers.close()


def distorted_inputs(dataset, batch_size, num_preprocess_threads=4, image_size=299, **kw):
    return GPUBatchInputs(dataset, batch_size, True, image_size, num_preprocess_threads, **kw)


def inputs(dataset, batch_size, num_preprocess_threads=4, image_size=299, **kw):
    return GPUBatchInputs(dataset, batch_size, False, image_size, num_preprocess_threads, num_readers=1, **kw)
