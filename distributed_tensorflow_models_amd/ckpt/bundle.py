"""TensorFlow V2 checkpoint (TensorBundle) I/O on top of the native C++ reader/writer.

``write_bundle(prefix, {name: ndarray})`` produces ``<prefix>.index`` + ``<prefix>.data-00000-of-00001``
exactly as ``tf.train.Saver`` (V2) lays them out; ``BundleReader`` reads any V2 bundle (multi-shard
supported).  Partitioned variables (``tf.fixed_size_partitioner`` under the reference's
``partitioned_space`` / ``root`` variable scopes, e.g. alexnet/cifar10_alexnet_bsp.py:50-51) are written
as TF's BundleWriter::AddSlice does - a full-tensor entry listing its slices plus one entry per slice
under an OrderedCode slice key (``Sliced``, ``partition_axis0``) - and reassembled on read.
"""
import ctypes

import numpy as np

from ..utils.native import rt

# tensorflow/core/framework/types.proto
DT = {np.dtype("float32"): 1, np.dtype("float64"): 2, np.dtype("int32"): 3, np.dtype("uint8"): 4,
      np.dtype("int16"): 5, np.dtype("int8"): 6, np.dtype("int64"): 9, np.dtype("bool"): 10,
      np.dtype("float16"): 19, np.dtype("uint16"): 17}
DT_BFLOAT16 = 14
NP = {v: k for k, v in DT.items()}


class Sliced:
    """A partitioned variable: full shape + [(starts, lengths, array)] boxes (length -1 = full extent)."""
    __slots__ = ("full_shape", "slices", "tf_dtype")

    def __init__(self, full_shape, slices, tf_dtype=None):
        self.full_shape, self.slices, self.tf_dtype = tuple(int(d) for d in full_shape), list(slices), tf_dtype


def partition_sizes(dim, num_shards):
    """tf.fixed_size_partitioner(num_shards, axis) + variable_scope._iter_slices: min(num_shards, dim)
    parts, the first dim % parts of them one element longer."""
    n = max(1, min(int(num_shards), int(dim)))
    base, extra = divmod(int(dim), n)
    return [base + (1 if i < extra else 0) for i in range(n)]


def partition_axis0(a, num_shards, tf_dtype=None):
    """Slice a (non-scalar) array along axis 0 the way a partitioned variable_scope stores it; every
    dim of each slice spec is explicit (TF's SaveSliceInfo.spec), so even one shard is a sliced entry."""
    a = np.require(a, requirements="C")
    slices, off = [], 0
    for n in partition_sizes(a.shape[0], num_shards):
        starts = [off] + [0] * (a.ndim - 1)
        lengths = [n] + list(a.shape[1:])
        slices.append((starts, lengths, a[off:off + n]))
        off += n
    return Sliced(a.shape, slices, tf_dtype)


def write_bundle(prefix, tensors):
    """tensors: dict name -> numpy array (or (array, tf_dtype) for bfloat16 stored as uint16, or Sliced)."""
    L = rt()
    h = L.dtm_bundle_writer_new(prefix.encode())
    if not h:
        raise IOError("cannot open checkpoint for writing: %s" % prefix)
    try:
        for name, a in tensors.items():
            if isinstance(a, Sliced):
                nd = len(a.full_shape)
                full = (ctypes.c_int64 * max(1, nd))(*a.full_shape)
                for starts, lengths, arr in a.slices:
                    arr = np.require(arr, requirements="C")
                    dt = a.tf_dtype if a.tf_dtype is not None else DT[arr.dtype]
                    st = (ctypes.c_int64 * max(1, nd))(*starts)
                    ln = (ctypes.c_int64 * max(1, nd))(*lengths)
                    rc = L.dtm_bundle_writer_add_slice(h, name.encode(), dt, full, nd, st, ln,
                                                       arr.ctypes.data_as(ctypes.c_void_p), arr.nbytes)
                    if rc != 0:
                        raise IOError("write failed for slice of %s (%d)" % (name, rc))
                continue
            tf_dtype = None
            if isinstance(a, tuple):
                a, tf_dtype = a
            a = np.require(a, requirements="C")  # keeps 0-d arrays 0-d (ascontiguousarray does not)
            dt = tf_dtype if tf_dtype is not None else DT[a.dtype]
            shape = (ctypes.c_int64 * max(1, a.ndim))(*a.shape)
            rc = L.dtm_bundle_writer_add(h, name.encode(), dt, shape, a.ndim, a.ctypes.data_as(ctypes.c_void_p),
                                         a.nbytes)
            if rc != 0:
                raise IOError("write failed for %s" % name)
    finally:
        rc = L.dtm_bundle_writer_finish(h)
    if rc != 0:
        raise IOError("checkpoint finalize failed (%d) for %s" % (rc, prefix))


class BundleReader:
    def __init__(self, prefix):
        self.L = rt()
        self.h = self.L.dtm_bundle_reader_open(prefix.encode())
        if not self.h:
            raise IOError("cannot open checkpoint %s (missing or corrupt .index)" % prefix)
        self.index = {}
        self.sliced = set()  # partitioned variables (reassembled from their slices by get_tensor)
        n = self.L.dtm_bundle_reader_num(self.h)
        for i in range(n):
            name = self.L.dtm_bundle_reader_name(self.h, i).decode()
            dt, nd, sl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
            shp = (ctypes.c_int64 * 8)()
            nb = ctypes.c_int64()
            self.L.dtm_bundle_reader_info2(self.h, i, ctypes.byref(dt), shp, ctypes.byref(nd), ctypes.byref(nb),
                                           ctypes.byref(sl))
            self.index[name] = (i, dt.value, tuple(shp[:nd.value]), nb.value)
            if sl.value:
                self.sliced.add(name)

    def close(self):
        if self.h:
            self.L.dtm_bundle_reader_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def names(self):
        return sorted(self.index)

    def get_variable_to_shape_map(self):
        return {k: list(v[2]) for k, v in self.index.items()}

    def get_variable_to_dtype_map(self):
        return {k: v[1] for k, v in self.index.items()}

    def has_tensor(self, name):
        return name in self.index

    def get_tensor(self, name):
        i, dt, shape, nb = self.index[name]
        if dt == DT_BFLOAT16:
            npdt = np.dtype("uint16")
        else:
            npdt = NP[dt]
        out = np.empty(shape, dtype=npdt)
        if out.nbytes != nb:
            raise IOError("size mismatch for %s" % name)
        rc = self.L.dtm_bundle_reader_read(self.h, i, out.ctypes.data_as(ctypes.c_void_p), nb)
        if rc == -2:
            raise IOError("crc32c mismatch reading %s" % name)
        if rc == -4:
            raise IOError("partitioned variable %s: slices missing or not tiling the tensor" % name)
        if rc != 0:
            raise IOError("read failed (%d) for %s" % (rc, name))
        return out
