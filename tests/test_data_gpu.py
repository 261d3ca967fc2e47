"""GPU ImageNet preprocessing (csrc/kernels/image.hip dtm_imagenet_prep) against the host oracle
(data/imagenet.preprocess_with_params) with identical per-image parameters; the GPU batch pipeline
from TFRecord shards."""
import io

import numpy as np
import pytest
import torch

from distributed_tensorflow_models_amd.data import imagenet
from distributed_tensorflow_models_amd.data import imagenet_gpu as G

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("train", [True, False])
@pytest.mark.parametrize("size", [299, 37])
def test_gpu_preprocess_matches_oracle(train, size):
    rng = np.random.RandomState(3)
    shapes = [(375, 500), (333, 250), (120, 90), (64, 300), (500, 400), (41, 33), (299, 299), (480, 640)]
    imgs = [(rng.rand(h, w, 3) * 255).astype(np.uint8) for h, w in shapes]
    params = []
    for i, im in enumerate(imgs):
        bbox = np.array([[0.1, 0.2, 0.9, 0.8]], np.float32) if i % 2 else None
        params.append(imagenet.sample_params(im.shape[0], im.shape[1], bbox, rng, i, train))  # all 4 methods
    out, _ = G.gpu_preprocess(imgs, params, size, torch.device("cuda"), torch.float32)
    torch.cuda.synchronize()
    for i, (im, p) in enumerate(zip(imgs, params)):
        want = imagenet.preprocess_with_params(im, size, p)
        got = out[i].cpu().numpy()
        err = np.abs(got - want)
        # float32 device math vs float64 host math; HSV sector changes at exact ties may flip a few pixels
        assert np.mean(err) < 2e-4 and np.quantile(err, 0.999) < 5e-3, (i, p, err.max())


def test_gpu_batch_inputs_from_tfrecords(tmp_path):
    from PIL import Image

    from distributed_tensorflow_models_amd.data.tfrecord import TFRecordWriter, encode_example
    out = tmp_path / "data"
    out.mkdir()
    rng = np.random.RandomState(0)
    with TFRecordWriter(str(out / "train-00000-of-00001")) as w:
        for i in range(24):
            b = io.BytesIO()
            Image.fromarray((rng.rand(50 + i, 70, 3) * 255).astype(np.uint8)).save(b, format="JPEG")
            w.write(encode_example({"image/encoded": b.getvalue(), "image/class/label": i % 5 + 1,
                                    "image/object/bbox/xmin": [0.1], "image/object/bbox/ymin": [0.1],
                                    "image/object/bbox/xmax": [0.9], "image/object/bbox/ymax": [0.9]}))
    ds = imagenet.ImagenetData("train", str(out))
    bi = G.distorted_inputs(ds, 8, num_preprocess_threads=4, image_size=64, num_readers=1, num_decoders=2)
    x, y = bi.next_batch()
    x2, _ = bi.next_batch()
    bi.close()
    assert x.is_cuda and x.dtype == torch.bfloat16 and tuple(x.shape) == (8, 64, 64, 3)
    assert float(x.float().min()) >= -1.0 and float(x.float().max()) <= 1.0
    assert set(y.tolist()) <= set(range(1, 6)) and not torch.equal(x, x2)


def test_split_decode_pipeline_matches_full_decode(tmp_path):
    """Device batches through the split JPEG decode (host Huffman + HIP IDCT / upsampling / colour) and through the
    device decode (host marker parse only + HIP Huffman / IDCT / colour, split_decode=2) equal the full host-decode
    pipeline's (same seeds -> same crops and colour parameters), including a
    progressive file that takes the PIL fallback inside a split batch.  (The decoded pixels are bit-exact -
    tests/test_jpeg.py; the preprocessing's per-image contrast mean is an fp32 atomic sum, so the bf16
    batches agree to rounding.)"""
    from PIL import Image

    from distributed_tensorflow_models_amd.data.tfrecord import TFRecordWriter, encode_example
    out = tmp_path / "d"
    out.mkdir()
    rng = np.random.RandomState(5)
    with TFRecordWriter(str(out / "train-00000-of-00001")) as w:
        for i in range(16):
            b = io.BytesIO()
            img = (rng.rand(40 + 7 * i, 60 + 5 * i, 3) * 255).astype(np.uint8)
            Image.fromarray(img).save(b, format="JPEG", quality=80 + i, progressive=(i == 5),
                                      subsampling=[0, 1, 2][i % 3])
            w.write(encode_example({"image/encoded": b.getvalue(), "image/class/label": i + 1,
                                    "image/object/bbox/xmin": [0.05], "image/object/bbox/ymin": [0.1],
                                    "image/object/bbox/xmax": [0.9], "image/object/bbox/ymax": [0.95]}))
    ds = imagenet.ImagenetData("train", str(out))
    res = []
    for split in (False, True, 2):
        bi = G.GPUBatchInputs(ds, 8, train=True, image_size=64, num_readers=1, num_decoders=2, seed=11, device="cuda",
                              decode_processes=False, shuffle_buffer=32, split_decode=split)
        try:
            res.append([bi.next_batch() for _ in range(2)])
        finally:
            bi.close()
    torch.cuda.synchronize()
    for other in res[1:]:
        for (x0, y0), (x1, y1) in zip(res[0], other):
            assert torch.equal(y0, y1)
            torch.testing.assert_close(x0.float(), x1.float(), rtol=0, atol=1e-2)
            assert (x0 != x1).float().mean().item() < 0.01
