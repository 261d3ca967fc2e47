"""TFRecord files and tf.train.Example protos without TensorFlow.

Framing (length, masked crc32c) is done by the native runtime (csrc/runtime/data_io.cpp); the
Example proto (Features map<string, Feature{bytes_list|float_list|int64_list}>) is encoded and
decoded here with a minimal protobuf wire-format codec.
"""
import ctypes
import struct

from ..utils.native import rt


# ---- protobuf wire helpers ----------------------------------------------------------------------
def _varint(n):
    out = bytearray()
    n &= (1 << 64) - 1
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def _read_varint(b, i):
    r = s = 0
    while True:
        c = b[i]
        i += 1
        r |= (c & 0x7F) << s
        if not c & 0x80:
            return r, i
        s += 7


def _ld(field, payload):
    return _varint((field << 3) | 2) + _varint(len(payload)) + payload


def encode_example(features):
    """features: {name: bytes | str | [bytes] | int | [int] | float | [float]}"""
    entries = b""
    for key, v in features.items():
        if isinstance(v, (bytes, str)):
            v = [v]
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            v = [v]
        v = list(v)
        if v and isinstance(v[0], (bytes, str)):
            inner = b"".join(_ld(1, x.encode() if isinstance(x, str) else x) for x in v)
            feat = _ld(1, inner)
        elif v and isinstance(v[0], float):
            packed = struct.pack("<%df" % len(v), *v)
            feat = _ld(2, _ld(1, packed))
        else:
            packed = b"".join(_varint(int(x)) for x in v)
            feat = _ld(3, _ld(1, packed))
        entry = _ld(1, key.encode()) + _ld(2, feat)
        entries += _ld(1, entry)
    return _ld(1, entries)


def _parse_list(b, kind):
    out = []
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        f, wt = key >> 3, key & 7
        if f != 1:
            raise ValueError("bad list field")
        if wt == 2:
            ln, i = _read_varint(b, i)
            chunk = b[i:i + ln]
            i += ln
            if kind == 1:
                out.append(bytes(chunk))
            elif kind == 2:
                out.extend(struct.unpack("<%df" % (ln // 4), chunk))
            else:
                j = 0
                while j < ln:
                    v, j = _read_varint(chunk, j)
                    out.append(v - (1 << 64) if v >= (1 << 63) else v)
        elif wt == 0:
            v, i = _read_varint(b, i)
            out.append(v - (1 << 64) if v >= (1 << 63) else v)
        elif wt == 5:
            out.append(struct.unpack_from("<f", b, i)[0])
            i += 4
    return out


def decode_example(data):
    """-> {name: list of bytes / floats / ints}"""
    b = memoryview(data)
    res = {}
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        ln, i = _read_varint(b, i)
        if key >> 3 != 1:
            i += ln
            continue
        feats, end = b[i:i + ln], ln
        i += ln
        j = 0
        while j < end:
            k2, j = _read_varint(feats, j)
            l2, j = _read_varint(feats, j)
            entry = feats[j:j + l2]
            j += l2
            name, fv, e = None, None, 0
            while e < len(entry):
                k3, e = _read_varint(entry, e)
                l3, e = _read_varint(entry, e)
                if k3 >> 3 == 1:
                    name = bytes(entry[e:e + l3]).decode()
                elif k3 >> 3 == 2:
                    fv = entry[e:e + l3]
                e += l3
            vals = []
            if fv is not None and len(fv):
                k4, q = _read_varint(fv, 0)
                l4, q = _read_varint(fv, q)
                vals = _parse_list(fv[q:q + l4], k4 >> 3)
            res[name] = vals
    return res


# ---- record files -------------------------------------------------------------------------------
class TFRecordWriter:
    def __init__(self, path):
        self.L = rt()
        self.h = self.L.dtm_tfrecord_writer_open(path.encode())
        if not self.h:
            raise IOError("cannot open %s" % path)

    def write(self, record: bytes):
        buf = ctypes.create_string_buffer(record, len(record))
        if self.L.dtm_tfrecord_write(self.h, buf, len(record)) != 0:
            raise IOError("write failed")

    def close(self):
        if self.h:
            self.L.dtm_tfrecord_writer_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def tf_record_iterator(path, verify=True):
    L = rt()
    h = L.dtm_tfrecord_reader_open(path.encode(), int(verify))
    if not h:
        raise IOError("cannot open %s" % path)
    try:
        p = ctypes.c_void_p()
        while True:
            n = L.dtm_tfrecord_next(h, ctypes.byref(p))
            if n == -1:
                return
            if n < 0:
                raise IOError("corrupt record in %s" % path)
            yield ctypes.string_at(p, n)
    finally:
        L.dtm_tfrecord_reader_close(h)
