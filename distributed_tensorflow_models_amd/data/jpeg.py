"""Split JPEG decoding, bit-exact with libjpeg(-turbo)'s default decompression (the reference's
tf.image.decode_jpeg, inception/image_processing.py:339-407, and PIL both use it).  Two splits:

* host Huffman (csrc/runtime/jpeg.cpp) + device IDCT / upsampling / colour (csrc/kernels/jpeg.hip):
  ``huffman_decode(data)`` -> (JpegInfo numpy record, int16 coefficients) or None when the file is outside
  the supported subset (progressive, CMYK, ...: decode those with PIL).  ``pixels_cpu`` is the host form of
  the device stage (the oracle of the HIP kernel); ``decode_batch_gpu`` runs the device stage for a batch.
* everything past the marker parse on the device: ``scan_prep(data)`` walks the markers and unstuffs the
  entropy-coded bytes on the host (no bit-level work); ``decode_batch_gpu_full`` Huffman-decodes the batch with
  jpeg_huff_kernel (one workgroup per image, self-synchronising subsequence decode) and runs the same IDCT /
  colour stage.
"""
import ctypes

import numpy as np

from ..utils import native

# mirror of struct JpegInfo (csrc/runtime/jpeg.cpp)
INFO_DT = np.dtype([("width", "<i4"), ("height", "<i4"), ("ncomp", "<i4"), ("hmax", "<i4"), ("vmax", "<i4"),
                    ("mcux", "<i4"), ("mcuy", "<i4"), ("h", "<i4", 3), ("v", "<i4", 3), ("bw", "<i4", 3),
                    ("bh", "<i4", 3), ("coef_off", "<i4", 3), ("coef_count", "<i4"), ("qt", "<u2", (3, 64))])

UNSUPPORTED, CORRUPT, TOO_SMALL = -2, -1, -3

# mirror of struct JpegScan (csrc/runtime/jpeg.cpp, csrc/kernels/jpeg.hip)
SCAN_DT = np.dtype([("nbytes", "<i4"), ("nseg", "<i4"), ("restart", "<i4"), ("ncomp", "<i4"), ("bpm", "<i4"),
                    ("mcux", "<i4"), ("nmcu", "<i4"), ("nslot", "<i4"), ("bcomp", "<i4", 12), ("bdy", "<i4", 12),
                    ("bdx", "<i4", 12), ("h", "<i4", 3), ("v", "<i4", 3), ("bw", "<i4", 3), ("coef_off", "<i4", 3),
                    ("dc_slot", "<i4", 3), ("ac_slot", "<i4", 3), ("slot_dc", "<i4", 4), ("counts", "u1", (4, 16)),
                    ("vals", "u1", (4, 256))])
STREAM_PAD = 32  # zero bytes after every image's unstuffed stream


def _rt():
    L = native.rt()
    if not getattr(L, "_jpeg_bound", False):
        L.dtm_jpeg_decode.restype = ctypes.c_int
        L.dtm_jpeg_decode.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
        L.dtm_jpeg_pixels.restype = ctypes.c_int
        L.dtm_jpeg_pixels.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.dtm_jpeg_info_bytes.restype = ctypes.c_int
        assert L.dtm_jpeg_info_bytes() == INFO_DT.itemsize, (L.dtm_jpeg_info_bytes(), INFO_DT.itemsize)
        L.dtm_jpeg_scan.restype = ctypes.c_int
        L.dtm_jpeg_scan.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_long, ctypes.c_void_p, ctypes.c_long]
        L.dtm_jpeg_scan_bytes.restype = ctypes.c_int
        assert L.dtm_jpeg_scan_bytes() == SCAN_DT.itemsize, (L.dtm_jpeg_scan_bytes(), SCAN_DT.itemsize)
        L._jpeg_bound = True
    return L


def huffman_decode(data, out=None):
    """Entropy-decode one JPEG.  ``out``: optional int16 array to decode into (its prefix is used).
    Returns (info, coefs view) or None if unsupported / corrupt (the caller falls back to PIL)."""
    L = _rt()
    info = np.zeros(1, INFO_DT)
    buf = np.frombuffer(data, np.uint8)
    if out is None:
        out = np.empty(1 << 20, np.int16)
    rc = L.dtm_jpeg_decode(buf.ctypes.data, buf.size, info.ctypes.data, out.ctypes.data, out.size)
    if rc == TOO_SMALL:
        out = np.empty(int(info["coef_count"][0]), np.int16)
        rc = L.dtm_jpeg_decode(buf.ctypes.data, buf.size, info.ctypes.data, out.ctypes.data, out.size)
    if rc != 0:
        return None
    return info[0], out[:int(info["coef_count"][0])]


def plane_bytes(info):
    return int(sum(int(info["bw"][c]) * 8 * int(info["bh"][c]) * 8 for c in range(int(info["ncomp"]))))


def pixels_cpu(info, coefs):
    """Host form of the device stage: islow IDCT + fancy upsampling + YCbCr -> RGB -> HxWx3 uint8."""
    L = _rt()
    inf = np.array([info], INFO_DT)
    scratch = np.empty(plane_bytes(info), np.uint8)
    rgb = np.empty((int(info["height"]), int(info["width"]), 3), np.uint8)
    coefs = np.ascontiguousarray(coefs, np.int16)
    L.dtm_jpeg_pixels(coefs.ctypes.data, inf.ctypes.data, scratch.ctypes.data, rgb.ctypes.data)
    return rgb


def decode_cpu(data):
    """Full host decode through the split path (None if unsupported)."""
    r = huffman_decode(data)
    if r is None:
        return None
    return pixels_cpu(*r)


# ---- device stage ------------------------------------------------------------------------------------
# mirror of struct JpegDesc (csrc/kernels/jpeg.hip)
DESC_DT = np.dtype([("coef_base", "<i8"), ("plane_base", "<i8"), ("rgb_off", "<i8"), ("width", "<i4"),
                    ("height", "<i4"), ("ncomp", "<i4"), ("hmax", "<i4"), ("vmax", "<i4"), ("h", "<i4", 3),
                    ("v", "<i4", 3), ("bw", "<i4", 3), ("bh", "<i4", 3), ("coef_off", "<i4", 3), ("nblocks", "<i4"),
                    ("pad", "<i4"), ("qt", "<u2", (3, 64))])


def batch_table(infos):
    """Descriptor table + buffer sizes for a batch of decoded headers: (descs, coef int16 count, plane bytes,
    rgb bytes, max blocks, max pixels).  Coefficient bases are 8-int16 aligned, plane bases 8-byte aligned."""
    n = len(infos)
    d = np.zeros(n, DESC_DT)
    coef = plane = rgb = 0
    maxb = maxp = 0
    for i, inf in enumerate(infos):
        for f in ("width", "height", "ncomp", "hmax", "vmax", "h", "v", "bw", "bh", "coef_off"):
            d[i][f] = inf[f]
        d[i]["qt"] = inf["qt"]
        nc = int(inf["ncomp"])
        nb = int(sum(int(inf["bw"][c]) * int(inf["bh"][c]) for c in range(nc)))
        d[i]["nblocks"] = nb
        d[i]["coef_base"] = coef
        d[i]["plane_base"] = plane
        d[i]["rgb_off"] = rgb
        coef += (int(inf["coef_count"]) + 7) // 8 * 8
        plane += (plane_bytes(inf) + 7) // 8 * 8
        npx = int(inf["width"]) * int(inf["height"])
        rgb += npx * 3
        maxb, maxp = max(maxb, nb), max(maxp, npx)
    return d, coef, plane, rgb, maxb, maxp


def decode_batch_gpu(items, device, stream=None):
    """[(info, coefs)] -> (device uint8 RGB ragged buffer, descriptor table): image i is the HxWx3 block at
    descs[i]['rgb_off'].  Coefficients travel as one H2D copy; two HIP launches decode the batch."""
    import torch

    from ..ops import _lib
    L = _lib.lib()
    assert L.dtm_jpeg_desc_bytes() == DESC_DT.itemsize, (L.dtm_jpeg_desc_bytes(), DESC_DT.itemsize)
    infos = [it[0] for it in items]
    d, ncoef, nplane, nrgb, maxb, maxp = batch_table(infos)
    host = torch.empty(max(ncoef, 8), dtype=torch.int16, pin_memory=True)
    hv = host.numpy()
    for (inf, cf), base in zip(items, d["coef_base"]):
        hv[int(base):int(base) + cf.size] = cf
    coefs = host.to(device, non_blocking=True)
    descs = torch.from_numpy(d.view(np.uint8)).to(device, non_blocking=True)
    planes = torch.empty(max(nplane, 8), dtype=torch.uint8, device=device)
    rgb = torch.empty(max(nrgb, 1), dtype=torch.uint8, device=device)
    rc = L.dtm_jpeg_decode_gpu(_lib.ptr(coefs), _lib.ptr(descs), len(items), int(maxb), int(maxp), _lib.ptr(planes),
                               _lib.ptr(rgb), _lib.stream_ptr())
    if rc != 0:
        raise RuntimeError("dtm_jpeg_decode_gpu failed (%d)" % rc)
    return rgb, d


# ---- device entropy decode -----------------------------------------------------------------------------
# mirror of struct HuffDesc (csrc/kernels/jpeg.hip)
HUFF_DESC_DT = np.dtype([("stream_off", "<i8"), ("coef_base", "<i8"), ("coef_count", "<i4"), ("seg_off", "<i4"),
                         ("min_bits", "<i4"), ("pad", "<i4"), ("s", SCAN_DT)])


def scan_prep(data, stream=None, segs=None):
    """Host share of the device entropy decode: marker parse + byte unstuffing.  ``stream`` / ``segs``: optional
    uint8 / int32 scratch to write into (their prefix is used).  Returns (JpegInfo, JpegScan, unstuffed bytes +
    STREAM_PAD zeros, restart segment offsets) - views of the scratch - or None (unsupported / corrupt: the host
    decoders take the file)."""
    L = _rt()
    info = np.zeros(1, INFO_DT)
    sc = np.zeros(1, SCAN_DT)
    buf = np.frombuffer(data, np.uint8)
    if stream is None or stream.size < buf.size + STREAM_PAD:
        stream = np.empty(buf.size + STREAM_PAD, np.uint8)
    if segs is None:
        segs = np.empty(64, np.int32)
    rc = L.dtm_jpeg_scan(buf.ctypes.data, buf.size, info.ctypes.data, sc.ctypes.data, stream.ctypes.data,
                         stream.size, segs.ctypes.data, segs.size)
    if rc == TOO_SMALL:
        segs = np.empty(max(1, int(sc["nseg"][0])), np.int32)
        rc = L.dtm_jpeg_scan(buf.ctypes.data, buf.size, info.ctypes.data, sc.ctypes.data, stream.ctypes.data,
                             stream.size, segs.ctypes.data, segs.size)
    if rc != 0:
        return None
    n = int(sc["nbytes"][0])
    return info[0], sc[0], stream[:n + STREAM_PAD], segs[:int(sc["nseg"][0])]


HDR_SCAN_BYTES = INFO_DT.itemsize + SCAN_DT.itemsize


def scan_item(data, stream=None, segs=None):
    """scan_prep packed for the input pipeline: (JpegInfo + JpegScan bytes, one uint8 payload = the unstuffed
    stream, 4-byte aligned, then the restart segment table) or None."""
    r = scan_prep(data, stream, segs)
    if r is None:
        return None
    info, sc, st, sg = r
    a = (st.size + 3) // 4 * 4
    pay = np.zeros(a + 4 * sg.size, np.uint8)
    pay[:st.size] = st
    pay[a:].view(np.int32)[:] = sg
    return info.tobytes() + sc.tobytes(), pay


def unpack_scan_item(hdr, pay):
    """Inverse of scan_item -> (JpegInfo, JpegScan, stream bytes, segments): scan_prep's result."""
    info = np.frombuffer(hdr, INFO_DT, count=1)[0]
    sc = np.frombuffer(hdr, SCAN_DT, count=1, offset=INFO_DT.itemsize)[0]
    n = int(sc["nbytes"]) + STREAM_PAD
    a = (n + 3) // 4 * 4
    return info, sc, pay[:n], pay[a:a + 4 * int(sc["nseg"])].view(np.int32)


def huff_batch_table(scans, descs, min_bits=0):
    """Entropy-decode descriptors for a batch prepared by scan_prep: [(JpegScan, stream bytes, segments)] and the
    JpegDesc table of the same images (batch_table) -> (HuffDesc table, stream bytes, segment count).  Streams are
    16-byte aligned."""
    n = len(scans)
    h = np.zeros(n, HUFF_DESC_DT)
    off = nseg = 0
    for i, (sc, st, sg) in enumerate(scans):
        h[i]["s"] = sc
        h[i]["stream_off"] = off
        h[i]["coef_base"] = descs[i]["coef_base"]
        nb = int(descs[i]["nblocks"]) * 64
        h[i]["coef_count"] = nb
        h[i]["seg_off"] = nseg
        h[i]["min_bits"] = min_bits
        off += (st.size + 15) // 16 * 16  # (16-byte aligned: the kernel stages subsequences with 16-byte loads)
        nseg += sg.size
    return h, off, nseg


class DeviceBatch:
    """A batch prepared by scan_prep for the device decode: the pinned host staging (unstuffed streams, restart
    segment table, HuffDesc / JpegDesc tables) and, after ``launch``, the device buffers.  ``rgb_offs``: where each
    image's HxWx3 output goes in the RGB buffer (default: packed in order); ``rgb_bytes``: that buffer's size."""

    def __init__(self, preps, min_bits=0, rgb_offs=None, rgb_bytes=None, pin=True):
        import torch
        d, ncoef, nplane, nrgb, maxb, maxp = batch_table([p[0] for p in preps])
        if rgb_offs is not None:
            d["rgb_off"] = rgb_offs
        h, nbytes, nseg = huff_batch_table([p[1:] for p in preps], d, min_bits)
        self.n, self.ncoef, self.nplane, self.maxb, self.maxp = len(preps), ncoef, nplane, int(maxb), int(maxp)
        self.nrgb = nrgb if rgb_bytes is None else rgb_bytes
        self.descs = d
        self.stream = torch.empty(max(nbytes, 16) + max(nseg, 1) * 4, dtype=torch.uint8, pin_memory=pin)
        hv = self.stream.numpy()
        self.seg_byte_off = max(nbytes, 16)
        segs = hv[self.seg_byte_off:].view(np.int32)
        for (_inf, _sc, st, sg), hd in zip(preps, h):
            o = int(hd["stream_off"])
            hv[o:o + st.size] = st
            segs[int(hd["seg_off"]):int(hd["seg_off"]) + sg.size] = sg
        self.tables = torch.from_numpy(np.concatenate([h.view(np.uint8), d.view(np.uint8)]))
        if pin:
            self.tables = self.tables.pin_memory()
        self.hbytes = h.nbytes

    def launch(self, device, stream_ptr=None, rgb=None):
        """Upload + jpeg_huff_kernel + jpeg_idct_kernel + jpeg_color_kernel on the current (or the given) stream.
        Returns (device RGB buffer, device int32 status per image: fixed-point passes, 0 = restart segments, -1 =
        corrupt data)."""
        import torch

        from ..ops import _lib
        L = _lib.lib()
        assert L.dtm_jpeg_huff_desc_bytes() == HUFF_DESC_DT.itemsize, (L.dtm_jpeg_huff_desc_bytes(),
                                                                       HUFF_DESC_DT.itemsize)
        ds = self.stream.to(device, non_blocking=True)
        dt = self.tables.to(device, non_blocking=True)
        coefs = torch.empty(max(self.ncoef, 8), dtype=torch.int16, device=device)
        status = torch.empty(self.n, dtype=torch.int32, device=device)
        planes = torch.empty(max(self.nplane, 8), dtype=torch.uint8, device=device)
        if rgb is None:
            rgb = torch.empty(max(self.nrgb, 1), dtype=torch.uint8, device=device)
        sp = _lib.stream_ptr() if stream_ptr is None else stream_ptr
        rc = L.dtm_jpeg_huff_gpu(_lib.ptr(ds), _lib.ptr(ds[self.seg_byte_off:]), _lib.ptr(dt), self.n,
                                 _lib.ptr(coefs), _lib.ptr(status), sp)
        if rc == 0:
            rc = L.dtm_jpeg_decode_gpu(_lib.ptr(coefs), _lib.ptr(dt[self.hbytes:]), self.n, self.maxb, self.maxp,
                                       _lib.ptr(planes), _lib.ptr(rgb), sp)
        if rc != 0:
            raise RuntimeError("device JPEG decode failed (%d)" % rc)
        self.coefs = coefs  # (kept for tests: the entropy decoder's output)
        return rgb, status


def decode_batch_gpu_full(datas, device, min_bits=0, stream=None):
    """Device decode of a batch of JPEG files (bytes): host marker parse + unstuffing, then jpeg_huff_kernel +
    jpeg_idct_kernel + jpeg_color_kernel.  Returns (device uint8 RGB ragged buffer, JpegDesc table, per-image
    status: passes of the subsequence fixed point, 0 for restart-segment images, -1 corrupt, device coefficients)
    - or None when scan_prep declines a file (the caller decodes those on the host)."""
    preps = [scan_prep(d) for d in datas]
    if any(p is None for p in preps):
        return None
    b = DeviceBatch(preps, min_bits)
    rgb, status = b.launch(device, stream)
    return rgb, b.descs, status, b.coefs
