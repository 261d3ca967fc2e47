"""TF padding / output-size arithmetic (NHWC).

TF 'SAME' padding is asymmetric: the extra pad goes bottom/right (SURVEY.md §2.6 notes;
reference vgg/nets/resnet_utils.py:77-122 uses explicit symmetric pads + VALID instead).
"""
from dataclasses import dataclass


def _pair(v):
    if isinstance(v, (tuple, list)):
        return int(v[0]), int(v[1])
    return int(v), int(v)


@dataclass(frozen=True)
class ConvGeom:
    N: int
    H: int
    W: int
    C: int
    K: int
    R: int
    S: int
    P: int
    Q: int
    stride: int
    pad_h: int
    pad_w: int
    pad_b: int  # bottom pad (informational / CPU path)
    pad_r: int
    dilation: int = 1

    def as_desc(self, ConvDesc):
        return ConvDesc(self.N, self.H, self.W, self.C, self.K, self.R, self.S, self.P, self.Q,
                        self.stride, self.pad_h, self.pad_w)


def same_pads(size, k, stride, dilation=1):
    keff = (k - 1) * dilation + 1
    out = -(-size // stride)
    total = max((out - 1) * stride + keff - size, 0)
    return out, total // 2, total - total // 2


def explicit_pads(padding):
    """int | (ph, pw) symmetric | ((top, bottom), (left, right)) -> (top, bottom, left, right).
    The asymmetric form is resnet_utils.conv2d_same with an even kernel (tf.pad [beg, end] then VALID;
    reference vgg/nets/resnet_utils.py:77-122): the extra row / column goes bottom / right."""
    if isinstance(padding, (tuple, list)) and len(padding) == 2 and isinstance(padding[0], (tuple, list)):
        (pt, pb), (pl, pr) = padding
        return int(pt), int(pb), int(pl), int(pr)
    ph, pw = _pair(padding)
    return ph, ph, pw, pw


def conv_geom(x_shape, k_shape, stride=1, padding="SAME", dilation=1):
    """x_shape NHWC, k_shape (K, R, S, C). padding: 'SAME' | 'VALID' | int | (ph, pw) symmetric |
    ((top, bottom), (left, right)) explicit.  The kernels take the top/left pad and the output size;
    bottom/right padding is the zero fill of out-of-range taps."""
    N, H, W, C = x_shape
    K, R, S, C2 = k_shape
    if C2 != C:
        raise ValueError("channel mismatch: input %d vs kernel %d" % (C, C2))
    sh, sw = _pair(stride)
    if sh != sw:
        raise ValueError("only square strides are supported")
    if isinstance(padding, str):
        p = padding.upper()
        if p == "SAME":
            P, pt, pb = same_pads(H, R, sh, dilation)
            Q, pl, pr = same_pads(W, S, sw, dilation)
        elif p == "VALID":
            P = (H - ((R - 1) * dilation + 1)) // sh + 1
            Q = (W - ((S - 1) * dilation + 1)) // sw + 1
            pt = pb = pl = pr = 0
        else:
            raise ValueError(padding)
    else:
        pt, pb, pl, pr = explicit_pads(padding)
        P = (H + pt + pb - ((R - 1) * dilation + 1)) // sh + 1
        Q = (W + pl + pr - ((S - 1) * dilation + 1)) // sw + 1
    if P <= 0 or Q <= 0:
        raise ValueError("non-positive conv output %dx%d for input %dx%d kernel %dx%d" % (P, Q, H, W, R, S))
    return ConvGeom(N, H, W, C, K, R, S, P, Q, sh, pt, pl, pb, pr, dilation)


@dataclass(frozen=True)
class PoolGeom:
    N: int
    H: int
    W: int
    C: int
    P: int
    Q: int
    KH: int
    KW: int
    SH: int
    SW: int
    PH: int
    PW: int
    PB: int
    PR: int

    def as_args(self, PoolArgs):
        return PoolArgs(self.N, self.H, self.W, self.C, self.P, self.Q, self.KH, self.KW, self.SH, self.SW,
                        self.PH, self.PW)


def pool_geom(x_shape, kernel, stride, padding="VALID"):
    N, H, W, C = x_shape
    kh, kw = _pair(kernel)
    sh, sw = _pair(stride)
    if isinstance(padding, str) and padding.upper() == "SAME":
        P, pt, pb = same_pads(H, kh, sh)
        Q, pl, pr = same_pads(W, kw, sw)
    elif isinstance(padding, str) and padding.upper() == "VALID":
        P = (H - kh) // sh + 1
        Q = (W - kw) // sw + 1
        pt = pb = pl = pr = 0
    else:
        ph, pw = _pair(padding)
        pt = pb = ph
        pl = pr = pw
        P = (H + 2 * ph - kh) // sh + 1
        Q = (W + 2 * pw - kw) // sw + 1
    return PoolGeom(N, H, W, C, P, Q, kh, kw, sh, sw, pt, pl, pb, pr)


def live_taps(g):
    """Kernel rows [r0, r1) / cols [s0, s1) that touch at least one real input pixel for some output.

    Taps outside fall on zero padding for EVERY output pixel (e.g. VGG-16's fc6 as a 7x7 'SAME'
    conv over a 1x1 map in the CIFAR geometry: only the centre tap is live), so the conv equals the
    conv with the kernel cropped to the live window and the paddings reduced to match."""
    st = g.stride
    r0 = max(0, g.pad_h - (g.P - 1) * st)
    r1 = min(g.R - 1, g.H - 1 + g.pad_h) + 1
    s0 = max(0, g.pad_w - (g.Q - 1) * st)
    s1 = min(g.S - 1, g.W - 1 + g.pad_w) + 1
    return r0, r1, s0, s1


def cropped_geom(g, r0, r1, s0, s1):
    return ConvGeom(g.N, g.H, g.W, g.C, g.K, r1 - r0, s1 - s0, g.P, g.Q, g.stride, g.pad_h - r0, g.pad_w - s0,
                    g.pad_b - (g.R - r1), g.pad_r - (g.S - s1), g.dilation)
