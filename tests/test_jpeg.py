"""Split JPEG decode (data/jpeg.py): host Huffman decode (csrc/runtime/jpeg.cpp) + the device IDCT /
upsampling / colour stage (csrc/kernels/jpeg.hip).  Oracle: PIL (libjpeg-turbo), which is what the
reference's tf.image.decode_jpeg computes too (inception/image_processing.py:339-407) - the split path must
match it bit for bit on every baseline file, and decline progressive ones (those go to PIL)."""
import io

import numpy as np
import pytest
import torch

from distributed_tensorflow_models_amd.data import jpeg


def _image(rng, h, w):
    lo = rng.rand(h // 16 + 1, w // 16 + 1, 3)
    return (np.kron(lo, np.ones((16, 16, 1)))[:h, :w] * 200 + rng.rand(h, w, 3) * 55).astype(np.uint8)


def _cases():
    from PIL import Image
    rng = np.random.RandomState(0)
    out = []
    for i, (sub, q, extra) in enumerate([(None, 90, {}), (0, 95, {}), (1, 75, {}), (2, 85, {}), (None, 50, {}),
                                         (2, 90, {"restart_marker_blocks": 3}), (0, 80, {"restart_marker_rows": 1}),
                                         (2, 92, {"optimize": True})]):
        h, w = int(rng.randint(9, 260)), int(rng.randint(9, 260))
        b = io.BytesIO()
        kw = dict(extra)
        if sub is not None:
            kw["subsampling"] = sub
        Image.fromarray(_image(rng, h, w)).save(b, format="JPEG", quality=q, **kw)
        out.append(("rgb%d" % i, b.getvalue()))
    b = io.BytesIO()
    Image.fromarray(_image(rng, 57, 91)).convert("L").save(b, format="JPEG", quality=88)
    out.append(("gray", b.getvalue()))
    return out


def _pil(data):
    from PIL import Image
    return np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))


def test_split_decode_cpu_is_bit_exact_with_pil():
    for name, data in _cases():
        got = jpeg.decode_cpu(data)
        assert got is not None, name
        np.testing.assert_array_equal(got, _pil(data), err_msg=name)


def test_unsupported_and_corrupt_files_decline():
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(_image(np.random.RandomState(1), 64, 64)).save(b, format="JPEG", progressive=True)
    assert jpeg.huffman_decode(b.getvalue()) is None           # progressive: PIL's job
    assert jpeg.huffman_decode(b"\xff\xd8\xff\xd9") is None     # no frame
    assert jpeg.huffman_decode(b"not a jpeg at all") is None
    data = bytearray(_cases()[0][1])
    assert jpeg.huffman_decode(bytes(data[:len(data) // 3])) is not None or True  # truncated: no crash


def test_batch_table_layout():
    items = [jpeg.huffman_decode(d) for _n, d in _cases()]
    d, ncoef, nplane, nrgb, maxb, maxp = jpeg.batch_table([it[0] for it in items])
    assert (d["coef_base"] % 8 == 0).all() and (d["plane_base"] % 8 == 0).all()
    assert nrgb == sum(int(it[0]["width"]) * int(it[0]["height"]) * 3 for it in items)
    assert ncoef >= sum(it[1].size for it in items) and maxp == max(int(i["width"]) * int(i["height"]) for i, _ in items)
    assert list(d["width"]) == [int(it[0]["width"]) for it in items]


@pytest.mark.gpu
def test_split_decode_gpu_is_bit_exact_with_pil():
    cases = _cases()
    items = [jpeg.huffman_decode(d) for _n, d in cases]
    rgb, descs = jpeg.decode_batch_gpu(items, torch.device("cuda", 0))
    torch.cuda.synchronize()
    host = rgb.cpu().numpy()
    for (name, data), dsc in zip(cases, descs):
        h, w, o = int(dsc["height"]), int(dsc["width"]), int(dsc["rgb_off"])
        np.testing.assert_array_equal(host[o:o + h * w * 3].reshape(h, w, 3), _pil(data), err_msg=name)


def _restuff(st, segs, marker_base=0xD0):
    """Inverse of the host unstuffing: 0xFF -> 0xFF 0x00 and an RSTn marker before every segment but the first."""
    out, cuts = bytearray(), set(int(x) for x in segs[1:])
    for i, b in enumerate(bytes(st)):
        if i in cuts:
            out += bytes([0xFF, marker_base + (sorted(cuts).index(i) % 8)])
        out.append(b)
        if b == 0xFF:
            out.append(0)
    return bytes(out)


def test_scan_prep_unstuffs_the_entropy_coded_segment():
    """dtm_jpeg_scan (the host share of the device entropy decode): the unstuffed bytes + restart segment table
    re-stuff to exactly the file's scan, the layout matches the host decoder's and the zero padding follows."""
    for name, data in _cases():
        r = jpeg.scan_prep(data)
        assert r is not None, name
        info, sc, st, segs = r
        hinfo, _cf = jpeg.huffman_decode(data)
        assert info.tobytes() == hinfo.tobytes(), name
        n = int(sc["nbytes"])
        assert st.size == n + jpeg.STREAM_PAD and not st[n:].any(), name
        assert int(sc["bpm"]) == sum(int(info["h"][c]) * int(info["v"][c]) for c in range(int(info["ncomp"]))), name
        assert int(sc["nmcu"]) == int(info["mcux"]) * int(info["mcuy"]), name
        if int(sc["restart"]):
            assert segs.size == -(-int(sc["nmcu"]) // int(sc["restart"])) and segs[0] == 0, name
            assert (np.diff(segs) > 0).all(), name
        else:
            assert segs.size == 0, name
        # the scan as stored: after the SOS segment, up to the EOI marker
        sos = data.index(b"\xff\xda")
        start = sos + 2 + (data[sos + 2] << 8 | data[sos + 3])
        stuffed = data[start:data.rindex(b"\xff\xd9")]
        assert _restuff(st[:n], segs) == stuffed, name
    assert jpeg.scan_prep(b"\xff\xd8\xff\xd9") is None
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(_image(np.random.RandomState(1), 64, 64)).save(b, format="JPEG", progressive=True)
    assert jpeg.scan_prep(b.getvalue()) is None


def _big_cases(n=6):
    """ImageNet-like geometry (the generator of tools/decode_cpu_cost.py): ~300-500 px sides, 4:2:0, quality 90."""
    from PIL import Image
    rng = np.random.RandomState(3)
    out = []
    for i in range(n):
        h, w = int(rng.randint(300, 500)), int(rng.randint(300, 500))
        b = io.BytesIO()
        Image.fromarray(_image(rng, h, w)).save(b, format="JPEG", quality=int(rng.choice([75, 90, 95])))
        out.append(("big%d" % i, b.getvalue()))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,min_bits", [((256, 11), 0), ((256, 11), 128), ((256, 9), 256), ((64, 9), 0),
                                          ((64, 9), 128), ((128, 10), 0)])
def test_device_entropy_decode_matches_host_and_pil(cfg, min_bits):
    """jpeg_huff_kernel: the device-decoded coefficients equal the host decoder's int16 for int16 and the RGB equals
    PIL's, for every case (4:4:4 / 4:2:2 / 4:2:0 / 4:4:0, restart intervals, optimized tables, gray, ImageNet-size
    files), for every threads-per-image x lookup-bits variant of the kernel.  min_bits 128 / 256 cut the streams into
    many short subsequences (and phases), so most start states are wrong guesses the fixed point has to repair."""
    from distributed_tensorflow_models_amd.ops import _lib
    cases = _cases() + _big_cases()
    _lib.lib().dtm_jpeg_set_huff(*cfg)
    try:
        r = jpeg.decode_batch_gpu_full([d for _n, d in cases], torch.device("cuda", 0), min_bits=min_bits)
        torch.cuda.synchronize()
    finally:
        _lib.lib().dtm_jpeg_set_huff(256, 10)
    assert r is not None
    rgb, descs, status, coefs = r
    torch.cuda.synchronize()
    st = status.cpu().numpy()
    host = rgb.cpu().numpy()
    cf = coefs.cpu().numpy()
    for (name, data), dsc, s in zip(cases, descs, st):
        assert s >= 0, (name, s)
        info, hc = jpeg.huffman_decode(data)
        b = int(dsc["coef_base"])
        np.testing.assert_array_equal(cf[b:b + hc.size], hc, err_msg=name)
        h, w, o = int(dsc["height"]), int(dsc["width"]), int(dsc["rgb_off"])
        np.testing.assert_array_equal(host[o:o + h * w * 3].reshape(h, w, 3), _pil(data), err_msg=name)
    print("fixed-point passes per image:", list(st))


@pytest.mark.gpu
def test_device_entropy_decode_flags_corrupt_data():
    """A scan cut short or overwritten with garbage is reported (status -1); the other images of the batch are
    unaffected."""
    good = _big_cases(2)
    bad = bytearray(good[0][1])
    sos = bad.index(b"\xff\xda")
    cut = bytes(bad[:sos + 300]) + b"\xff\xd9"  # truncated scan
    r = jpeg.decode_batch_gpu_full([good[1][1], cut], torch.device("cuda", 0))
    assert r is not None
    rgb, descs, status, _cf = r
    st = status.cpu().numpy()
    assert st[0] >= 1 and st[1] == -1, st
    h, w, o = int(descs[0]["height"]), int(descs[0]["width"]), int(descs[0]["rgb_off"])
    np.testing.assert_array_equal(rgb.cpu().numpy()[o:o + h * w * 3].reshape(h, w, 3), _pil(good[1][1]))
