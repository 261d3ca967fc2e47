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
