"""TensorBundle V2 checkpoints + Saver facade (CPU)."""
import os
import struct

import numpy as np
import pytest
import torch

from distributed_tensorflow_models_amd.ckpt import saver as S
from distributed_tensorflow_models_amd.ckpt.bundle import BundleReader, write_bundle
from distributed_tensorflow_models_amd.utils.native import crc32c


def test_crc32c_known_vector():
    assert crc32c(b"123456789") == 0xE3069283
    assert crc32c(b"") == 0


def _varint(b, i):
    r, s = 0, 0
    while True:
        c = b[i]
        i += 1
        r |= (c & 0x7F) << s
        s += 7
        if not c & 0x80:
            return r, i


def _parse_block(b):
    n = struct.unpack_from("<I", b, len(b) - 4)[0]
    end = len(b) - 4 - 4 * n
    i, key, out = 0, b"", []
    while i < end:
        sh, i = _varint(b, i)
        ns, i = _varint(b, i)
        vl, i = _varint(b, i)
        key = key[:sh] + b[i:i + ns]
        i += ns
        out.append((key, b[i:i + vl]))
        i += vl
    return out


def test_index_is_a_leveldb_table(tmp_path):
    """Independent pure-python SSTable walk of the .index we write (format check)."""
    prefix = str(tmp_path / "m.ckpt-1")
    tensors = {"b/w": np.arange(6, dtype=np.float32).reshape(2, 3), "a": np.array(7, dtype=np.int64)}
    for i in range(40):  # force several data blocks
        tensors["layer_%03d/weights" % i] = np.random.rand(3, 3).astype(np.float32)
    write_bundle(prefix, tensors)
    data = open(prefix + ".index", "rb").read()
    footer = data[-48:]
    assert struct.unpack_from("<Q", footer, 40)[0] == 0xDB4775248B80FB57
    i = 0
    _moff, i = _varint(footer, i)
    _msz, i = _varint(footer, i)
    ioff, i = _varint(footer, i)
    isz, i = _varint(footer, i)
    index = _parse_block(data[ioff:ioff + isz])
    keys = []
    for _k, handle in index:
        off, j = _varint(handle, 0)
        sz, j = _varint(handle, j)
        assert data[off + sz] == 0  # uncompressed
        keys += [k for k, _ in _parse_block(data[off:off + sz])]
    assert keys[0] == b""  # header entry first
    assert keys[1:] == sorted(k.encode() for k in tensors)
    assert os.path.getsize(prefix + ".data-00000-of-00001") == sum(a.nbytes for a in tensors.values())


def test_bundle_roundtrip(tmp_path):
    prefix = str(tmp_path / "model.ckpt-5")
    src = {"conv1/weights": np.random.rand(7, 7, 3, 64).astype(np.float32),
           "global_step": np.array(5, dtype=np.int64),
           "x/int": np.arange(10, dtype=np.int32), "h": np.random.rand(4).astype(np.float16)}
    write_bundle(prefix, src)
    r = BundleReader(prefix)
    assert set(r.names()) == set(src)
    for k, v in src.items():
        got = r.get_tensor(k)
        assert got.dtype == v.dtype and got.shape == v.shape
        np.testing.assert_array_equal(got, v)
    r.close()


def test_bundle_detects_corruption(tmp_path):
    prefix = str(tmp_path / "c")
    write_bundle(prefix, {"v": np.ones(1000, np.float32)})
    p = prefix + ".data-00000-of-00001"
    b = bytearray(open(p, "rb").read())
    b[100] ^= 0xFF
    open(p, "wb").write(bytes(b))
    r = BundleReader(prefix)
    with pytest.raises(IOError):
        r.get_tensor("v")


def test_saver_state_file_and_retention(tmp_path):
    w = torch.randn(8, 3, 3, 4)
    b = torch.randn(8)
    gs = torch.tensor(0, dtype=torch.int64)
    vars_ = [S.TFVar("conv/weights", w, "KRSC->HWIO"), S.TFVar("conv/biases", b), S.TFVar("global_step", gs)]
    sv = S.Saver(vars_, max_to_keep=2)
    d = str(tmp_path)
    for step in (10, 20, 30):
        gs.fill_(step)
        sv.save(os.path.join(d, "model.ckpt"), global_step=step)
    st = S.get_checkpoint_state(d)
    assert st.model_checkpoint_path.endswith("model.ckpt-30")
    assert [os.path.basename(p) for p in st.all_model_checkpoint_paths] == ["model.ckpt-20", "model.ckpt-30"]
    assert not os.path.exists(os.path.join(d, "model.ckpt-10.index"))
    assert S.step_from_path(S.latest_checkpoint(d)) == 30
    # HWIO export
    r = BundleReader(S.latest_checkpoint(d))
    assert r.get_variable_to_shape_map()["conv/weights"] == [3, 3, 4, 8]
    np.testing.assert_allclose(r.get_tensor("conv/weights"), w.permute(1, 2, 3, 0).numpy())
    r.close()
    # restore into fresh tensors
    w2, b2, g2 = torch.zeros_like(w), torch.zeros_like(b), torch.tensor(0, dtype=torch.int64)
    S.Saver([S.TFVar("conv/weights", w2, "KRSC->HWIO"), S.TFVar("conv/biases", b2),
             S.TFVar("global_step", g2)]).restore(S.latest_checkpoint(d))
    assert torch.equal(w2, w) and torch.equal(b2, b) and int(g2) == 30


def test_async_save_matches_sync(tmp_path):
    import torch
    from distributed_tensorflow_models_amd.ckpt.bundle import BundleReader
    from distributed_tensorflow_models_amd.ckpt.saver import Saver, TFVar
    w = torch.randn(8, 3, 3, 4)
    b = torch.randn(8).to(torch.bfloat16)
    gs = torch.tensor(7, dtype=torch.int64)
    vs = [TFVar("conv/weights", w, "KRSC->HWIO"), TFVar("conv/biases", b), TFVar("global_step", gs)]
    s1, s2 = Saver(vs), Saver(vs)
    p1 = s1.save(str(tmp_path / "a" / "model.ckpt"), global_step=gs)
    p2 = s2.save(str(tmp_path / "b" / "model.ckpt"), global_step=gs, async_=True)
    w.add_(1.0)          # mutate after the snapshot: the async checkpoint must hold the old values
    s2.wait()
    r1, r2 = BundleReader(p1), BundleReader(p2)
    for n in ("conv/weights", "conv/biases", "global_step"):
        np.testing.assert_array_equal(r1.get_tensor(n), r2.get_tensor(n))
    assert (tmp_path / "b" / "checkpoint").exists()


def test_partitioned_variables_roundtrip(tmp_path):
    """fixed_size_partitioner(P, axis=0) layout: min(P, dim0) slices (the first dim0 % P one longer),
    a data-less full entry listing them, OrderedCode slice keys; the reader reassembles."""
    from distributed_tensorflow_models_amd.ckpt.bundle import (BundleReader, partition_axis0, partition_sizes,
                                                                write_bundle)
    assert partition_sizes(11, 3) == [4, 4, 3] and partition_sizes(2, 5) == [1, 1] and partition_sizes(64, 1) == [64]
    rng = np.random.RandomState(0)
    w = rng.randn(11, 11, 3, 64).astype(np.float32)
    b = rng.randn(64).astype(np.float32)
    big = rng.randn(200, 70).astype(np.float32)  # slice offsets >= 64: multi-byte signed OrderedCode
    p = str(tmp_path / "model.ckpt-7")
    write_bundle(p, {"partitioned_space/alexnet_v2/conv1/weights": partition_axis0(w, 3),
                     "partitioned_space/alexnet_v2/conv1/biases": partition_axis0(b, 1),
                     "root/vgg_16/fc6/weights": partition_axis0(big, 4),
                     "partitioned_space/Variable": np.array(7, np.int64)})
    r = BundleReader(p)
    assert r.names() == ["partitioned_space/Variable", "partitioned_space/alexnet_v2/conv1/biases",
                         "partitioned_space/alexnet_v2/conv1/weights", "root/vgg_16/fc6/weights"]
    assert r.sliced == {"partitioned_space/alexnet_v2/conv1/biases", "partitioned_space/alexnet_v2/conv1/weights",
                        "root/vgg_16/fc6/weights"}
    assert r.get_variable_to_shape_map()["partitioned_space/alexnet_v2/conv1/weights"] == [11, 11, 3, 64]
    np.testing.assert_array_equal(r.get_tensor("partitioned_space/alexnet_v2/conv1/weights"), w)
    np.testing.assert_array_equal(r.get_tensor("partitioned_space/alexnet_v2/conv1/biases"), b)
    np.testing.assert_array_equal(r.get_tensor("root/vgg_16/fc6/weights"), big)
    assert int(r.get_tensor("partitioned_space/Variable")) == 7


def _table_keys(path):
    data = open(path, "rb").read()
    footer = data[-48:]
    i = 0
    _moff, i = _varint(footer, i)
    _msz, i = _varint(footer, i)
    ioff, i = _varint(footer, i)
    isz, i = _varint(footer, i)
    keys = []
    for _k, handle in _parse_block(data[ioff:ioff + isz]):
        off, j = _varint(handle, 0)
        sz, j = _varint(handle, j)
        keys += [k for k, _ in _parse_block(data[off:off + sz])]
    return keys


def test_ordered_code_slice_key_encoding(tmp_path):
    """The slice entry keys are checkpoint::EncodeTensorNameSlice strings: byte 0 (NumIncreasing 0), the
    escaped name + 0x00 0x01, the rank, then (start, length) per dim as SignedNumIncreasing
    (x < 64: one byte 0x80 ^ x; 64 <= x < 8192: two bytes, header 0xc0)."""
    from distributed_tensorflow_models_amd.ckpt.bundle import partition_axis0, write_bundle
    p = str(tmp_path / "k")
    write_bundle(p, {"v": partition_axis0(np.zeros((100, 3), np.float32), 2)})
    keys = _table_keys(p + ".index")
    head = b"\x00" + b"v\x00\x01" + b"\x01\x02"
    assert keys == [b"", head + bytes([0x80, 0x80 ^ 50, 0x80, 0x80 ^ 3]),   # dim0 (0, 50), dim1 (0, 3)
                    head + bytes([0x80 ^ 50, 0x80 ^ 50, 0x80, 0x80 ^ 3]), b"v"]  # dim0 (50, 50)
    # 100 = 0b1100100 (7 bits) -> two bytes 0xc0 | 0x00, 0x64 (rank 1 = NumIncreasing bytes 01 01)
    write_bundle(p + "2", {"w": partition_axis0(np.zeros((300,), np.float32), 3)})
    keys = _table_keys(p + "2.index")
    assert b"\x00w\x00\x01\x01\x01" + bytes([0xc0, 0x64, 0xc0, 0x64]) in keys  # slice 1: start 100, len 100


def test_saver_partitioned_vars_and_slots(tmp_path):
    """TFVar(partitions=P): the variable and its slots are written as sliced entries and restore."""
    import torch
    from distributed_tensorflow_models_amd.ckpt.bundle import BundleReader
    from distributed_tensorflow_models_amd.ckpt.saver import Saver, TFVar
    w = torch.randn(64, 5, 5, 3)  # internal KRSC -> TF HWIO [5, 5, 3, 64], partitioned along 5
    m = torch.randn(64, 5, 5, 3)
    vs = [TFVar("root/conv/weights", w, "KRSC->HWIO", 2), TFVar("root/conv/weights/Momentum", m, "KRSC->HWIO", 2),
          TFVar("root/Variable", torch.tensor(3, dtype=torch.int64))]
    s = Saver(vs)
    s.save(str(tmp_path / "model.ckpt"), global_step=3)
    r = BundleReader(str(tmp_path / "model.ckpt-3"))
    assert r.sliced == {"root/conv/weights", "root/conv/weights/Momentum"}
    np.testing.assert_array_equal(r.get_tensor("root/conv/weights"), w.permute(1, 2, 3, 0).numpy())
    w2, m2 = torch.zeros_like(w), torch.zeros_like(m)
    Saver([TFVar("root/conv/weights", w2, "KRSC->HWIO"), TFVar("root/conv/weights/Momentum", m2, "KRSC->HWIO")]
          ).restore(str(tmp_path / "model.ckpt-3"))
    assert torch.equal(w2, w) and torch.equal(m2, m)
