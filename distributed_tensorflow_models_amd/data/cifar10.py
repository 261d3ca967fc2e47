"""CIFAR-10 input pipeline (reference */cifar10_input.py).

Host side: the native C++ reader loads ``data_batch_{1..5}.bin`` / ``test_batch.bin`` (1 label byte +
3072 CHW bytes) into an HWC table and a worker thread fills a ring of pinned batches
(replacing FixedLengthRecordReader + 16-thread tf.train.batch).  Device side: one HIP kernel per
batch does random crop (``IMAGE_SIZE`` 24 for the cnn trainer, 32 elsewhere), flip, brightness
(+-63), contrast [0.2, 1.8] and per_image_standardization (``distorted_inputs``), or the central
crop/pad + standardization of ``inputs`` (eval).  Without the binary files a deterministic synthetic
CIFAR stand-in of the same shape is used (there is no network access to download them).
"""
import ctypes
import os

import numpy as np
import torch

NUM_CLASSES = 10
NUM_EXAMPLES_PER_EPOCH_FOR_TRAIN = 50000
NUM_EXAMPLES_PER_EPOCH_FOR_EVAL = 10000
DATA_URL = "https://www.cs.toronto.edu/~kriz/cifar-10-binary.tar.gz"


def data_files(data_dir, eval_data=False):
    d = os.path.join(data_dir, "cifar-10-batches-bin")
    if not os.path.isdir(d):
        d = data_dir
    names = ["test_batch.bin"] if eval_data else ["data_batch_%d.bin" % i for i in range(1, 6)]
    return [os.path.join(d, n) for n in names]


def maybe_download_and_extract(data_dir):
    """Reference cifar10.py:394-411.  No network here: only checks for pre-placed files."""
    files = data_files(data_dir)
    if all(os.path.exists(f) for f in files):
        return True
    tgz = os.path.join(data_dir, "cifar-10-binary.tar.gz")
    if os.path.exists(tgz):
        import tarfile
        with tarfile.open(tgz) as t:
            t.extractall(data_dir, filter="data")
        return True
    return False


class AugParams(ctypes.Structure):
    _fields_ = [("oy", ctypes.c_int), ("ox", ctypes.c_int), ("flip", ctypes.c_int), ("brightness", ctypes.c_float),
                ("contrast", ctypes.c_float), ("pad0", ctypes.c_float)]


def augment(images_u8, out_size, distort=True, rng=None, dtype=torch.bfloat16):
    """images_u8: [B,H,W,3] uint8 (device).  Returns [B,S,S,3] standardized images."""
    B, H, W, C = images_u8.shape
    rng = rng or np.random
    p = np.zeros((B, 6), dtype=np.float32)
    pi = p.view(np.int32)
    if distort:
        pi[:, 0] = rng.randint(0, H - out_size + 1, B)
        pi[:, 1] = rng.randint(0, W - out_size + 1, B)
        pi[:, 2] = rng.randint(0, 2, B)
        p[:, 3] = rng.uniform(-63, 63, B)
        p[:, 4] = rng.uniform(0.2, 1.8, B)
    else:  # central crop / pad (resize_image_with_crop_or_pad)
        pi[:, 0] = (H - out_size) // 2
        pi[:, 1] = (W - out_size) // 2
        p[:, 4] = 1.0
    dev = images_u8.device
    if dev.type == "cuda":
        from ..ops import _lib
        L = _lib.lib()
        if not hasattr(L, "_aug_sig"):
            L.dtm_augment.restype = ctypes.c_int
            L.dtm_augment.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p] + \
                [ctypes.c_int] * 6 + [ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
            L._aug_sig = True
        params = torch.from_numpy(p.view(np.uint8).reshape(-1).copy()).to(dev, non_blocking=True)
        out = torch.empty(B, out_size, out_size, C, device=dev, dtype=dtype)
        rc = L.dtm_augment(_lib.ptr(images_u8.contiguous()), _lib.ptr(out), int(dtype == torch.bfloat16),
                           _lib.ptr(params), B, H, W, C, out_size, 1, 1.0, 0.0, _lib.stream_ptr())
        if rc == 0:
            return out
    return _augment_torch(images_u8, out_size, p, dtype)


def _augment_torch(images_u8, S, p, dtype):
    """Reference (CPU) implementation of the same transform, used as the numerics oracle."""
    B, H, W, C = images_u8.shape
    pi = p.view(np.int32)
    out = torch.zeros(B, S, S, C)
    x = images_u8.float().cpu()
    for b in range(B):
        oy, ox, fl = int(pi[b, 0]), int(pi[b, 1]), int(pi[b, 2])
        img = torch.zeros(S, S, C)
        ys, xs = max(0, oy), max(0, ox)
        ye, xe = min(H, oy + S), min(W, ox + S)
        img[ys - oy:ye - oy, xs - ox:xe - ox] = x[b, ys:ye, xs:xe]
        if fl:
            img = img.flip(1)
        img = img + float(p[b, 3])
        c = float(p[b, 4])
        if c != 1.0:
            m = img.mean((0, 1), keepdim=True)
            img = (img - m) * c + m
        n = img.numel()
        mean = img.mean()
        std = img.var(unbiased=False).sqrt()
        img = (img - mean) / max(float(std), 1.0 / n ** 0.5)
        out[b] = img
    return out.to(images_u8.device).to(dtype)


class Cifar10Input:
    """distorted_inputs(batch) / inputs(eval) with a native prefetching reader."""

    def __init__(self, data_dir, batch_size, image_size=32, eval_data=False, device="cpu", shuffle=True, seed=0,
                 nslots=4, synthetic_if_missing=True):
        self.batch_size, self.image_size, self.eval_data = batch_size, image_size, eval_data
        self.device = torch.device(device)
        self.rng = np.random.RandomState(seed)
        files = data_files(data_dir or "", eval_data)
        self.native = None
        self.synthetic = False
        if all(os.path.exists(f) for f in files):
            from ..utils.native import rt
            L = rt()
            h = L.dtm_cifar_table_open("\n".join(files).encode(), 1)
            if not h:
                raise IOError("failed to read CIFAR files %s" % files)
            self.L, self.h = L, h
            self.size = L.dtm_cifar_table_size(h)
            pin = torch.cuda.is_available()
            self.img_slots = torch.empty(nslots * batch_size * 3072, dtype=torch.uint8)
            self.lab_slots = torch.empty(nslots * batch_size, dtype=torch.int32)
            if pin:
                self.img_slots = self.img_slots.pin_memory()
                self.lab_slots = self.lab_slots.pin_memory()
            L.dtm_loader_start(h, batch_size, nslots, ctypes.c_void_p(self.img_slots.data_ptr()),
                               ctypes.c_void_p(self.lab_slots.data_ptr()), int(shuffle and not eval_data), seed)
            self.native = True
        elif synthetic_if_missing:
            self.synthetic = True
            g = torch.Generator().manual_seed(seed)
            n = 1024
            self.syn_images = torch.randint(0, 256, (n, 32, 32, 3), generator=g, dtype=torch.uint8)
            self.syn_labels = torch.randint(0, NUM_CLASSES, (n,), generator=g)
            self.size = n
            self._cursor = 0
        else:
            raise IOError("CIFAR-10 binary files not found under %s" % data_dir)

    def _raw_batch(self):
        B = self.batch_size
        if self.native:
            s = self.L.dtm_loader_next(self.h)
            img = self.img_slots[s * B * 3072:(s + 1) * B * 3072].view(B, 32, 32, 3)
            lab = self.lab_slots[s * B:(s + 1) * B]
            img_d = img.to(self.device, non_blocking=True)
            lab_d = lab.to(self.device, non_blocking=True).long()
            if self.device.type == "cuda":
                torch.cuda.current_stream().synchronize()
            else:
                img_d, lab_d = img_d.clone(), lab_d.clone()
            self.L.dtm_loader_release(self.h, s)
            return img_d, lab_d
        idx = torch.arange(self._cursor, self._cursor + B) % self.size
        self._cursor = (self._cursor + B) % self.size
        return self.syn_images[idx].to(self.device), self.syn_labels[idx].to(self.device)

    def next_batch(self):
        img, lab = self._raw_batch()
        dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        return augment(img, self.image_size, distort=not self.eval_data, rng=self.rng, dtype=dtype), lab

    def close(self):
        if self.native:
            self.L.dtm_cifar_table_close(self.h)
            self.native = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def distorted_inputs(data_dir, batch_size, image_size=32, device="cpu", **kw):
    return Cifar10Input(data_dir, batch_size, image_size, False, device, **kw)


def inputs(eval_data, data_dir, batch_size, image_size=32, device="cpu", **kw):
    return Cifar10Input(data_dir, batch_size, image_size, bool(eval_data), device, shuffle=False, **kw)
