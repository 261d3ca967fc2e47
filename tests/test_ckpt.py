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
