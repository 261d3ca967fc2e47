"""ctypes binding of the host C++ runtime ``_native/libdtm_runtime.so`` (no GPU needed)."""
import ctypes
import os

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNTIME_PATH = os.path.join(_HERE, "_native", "libdtm_runtime.so")
_rt = None

_P, _I, _L, _C = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_char_p
_SIGS = {
    "dtm_crc32c": (ctypes.c_uint32, [_P, ctypes.c_size_t]),
    "dtm_crc32c_masked": (ctypes.c_uint32, [_P, ctypes.c_size_t]),
    "dtm_bundle_writer_new": (_P, [_C]),
    "dtm_bundle_writer_add": (_I, [_P, _C, _I, ctypes.POINTER(ctypes.c_int64), _I, _P, _L]),
    "dtm_bundle_writer_add_slice": (_I, [_P, _C, _I, ctypes.POINTER(ctypes.c_int64), _I,
                                        ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64), _P, _L]),
    "dtm_bundle_writer_finish": (_I, [_P]),
    "dtm_bundle_reader_info2": (_I, [_P, _I, ctypes.POINTER(_I), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(_I),
                                     ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(_I)]),
    "dtm_bundle_reader_open": (_P, [_C]),
    "dtm_bundle_reader_num": (_I, [_P]),
    "dtm_bundle_reader_name": (_C, [_P, _I]),
    "dtm_bundle_reader_info": (_I, [_P, _I, ctypes.POINTER(_I), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(_I),
                                    ctypes.POINTER(ctypes.c_int64)]),
    "dtm_bundle_reader_read": (_I, [_P, _I, _P, _L]),
    "dtm_bundle_reader_close": (None, [_P]),
    "dtm_tfrecord_writer_open": (_P, [_C]),
    "dtm_tfrecord_write": (_I, [_P, _P, _L]),
    "dtm_tfrecord_writer_close": (_I, [_P]),
    "dtm_tfrecord_reader_open": (_P, [_C, _I]),
    "dtm_tfrecord_next": (_L, [_P, ctypes.POINTER(ctypes.c_void_p)]),
    "dtm_tfrecord_reader_close": (None, [_P]),
    "dtm_cifar_table_open": (_P, [_C, _I]),
    "dtm_cifar_table_size": (_L, [_P]),
    "dtm_cifar_table_get": (_I, [_P, _L, _I, _P, _P]),
    "dtm_loader_start": (_I, [_P, _I, _I, _P, _P, _I, ctypes.c_uint64]),
    "dtm_loader_next": (_I, [_P]),
    "dtm_loader_release": (None, [_P, _I]),
    "dtm_cifar_table_close": (None, [_P]),
}


def rt():
    global _rt
    if _rt is None:
        if not os.path.exists(RUNTIME_PATH):
            raise RuntimeError("native runtime %s missing: run `python tools/build_native.py`" % RUNTIME_PATH)
        L = ctypes.CDLL(RUNTIME_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _rt = L
    return _rt


def crc32c(data: bytes, masked=False):
    L = rt()
    buf = ctypes.create_string_buffer(data, len(data))
    return (L.dtm_crc32c_masked if masked else L.dtm_crc32c)(buf, len(data))
