"""Inception-v3 in the bundled *old* TF-Slim (reference inception/slim/inception_model.py:54-358,
wrapper inception/inception_model.py:49-96) - the model of the inception_{bsp,asp,ssp} trainers.

Checkpoint layout is reproduced exactly (golden: inception/slim/collections_test.py:35-117):
no top-level prefix, default op scopes uniquified per variable scope ('Conv', 'Conv_1', ...),
conv = weights + BatchNorm{beta, moving_mean, moving_variance} (scale=False: no gamma), aux head
'aux_logits/{proj,Conv,FC}', classifier 'logits/logits/{weights,biases}'.
Defaults (inception_v3_parameters): weight decay 4e-5 on conv+fc weights, conv stddev 0.1,
BN decay 0.9997 eps 1e-3 (biased moving variance - tf.nn.moments path), dropout keep 0.8.
Returns (logits, aux_logits) in training mode; the trainer weights the aux loss by 0.4.
"""
import torch

from ..ops import nn as F
from ..ops import fused as _fused
from ..ops.fused import concat_channels
from .layers import BatchNorm, Conv2d, Dropout, FullyConnected, Layer, fused_enabled


class _Scope:
    """old-slim default scope names: ops.conv2d -> 'Conv', 'Conv_1', ... inside one variable scope."""

    def __init__(self, prefix):
        self.prefix = prefix
        self.counts = {}

    def name(self, scope, default):
        if scope is not None:
            return self.prefix + scope
        n = self.counts.get(default, 0)
        self.counts[default] = n + 1
        return self.prefix + (default if n == 0 else "%s_%d" % (default, n))


class InceptionV3Slim(Layer):
    default_image_size = 299

    def __init__(self, num_classes=1001, dropout_keep_prob=0.8, weight_decay=0.00004, stddev=0.1,
                 batch_norm_decay=0.9997, batch_norm_epsilon=0.001, scope=""):
        super().__init__(scope)
        self._bn = dict(decay=batch_norm_decay, epsilon=batch_norm_epsilon, scale=False, bessel=False)
        self._wd, self._std = weight_decay, stddev
        self.layers = torch.nn.ModuleDict()
        self.plan = []
        self.num_classes = num_classes
        c = self._stem(scope)
        for name, width in (("mixed_35x35x256a", 32), ("mixed_35x35x288a", 64), ("mixed_35x35x288b", 64)):
            c = self._mixed35(scope + name, c, width)
        c = self._mixed17a(scope + "mixed_17x17x768a", c)
        for name, w in (("mixed_17x17x768b", 128), ("mixed_17x17x768c", 160), ("mixed_17x17x768d", 160),
                        ("mixed_17x17x768e", 192)):
            c = self._mixed17(scope + name, c, w)
        # aux head
        sc = _Scope(scope + "aux_logits/")
        self.aux_proj = self._conv(sc.name("proj", "Conv"), c, 128, 1)
        self.aux_conv = self._conv(sc.name(None, "Conv"), 128, 768, 5, padding="VALID", stddev=0.01)
        self.aux_fc = FullyConnected(sc.name(None, "FC"), 768, num_classes, None, None, True, weight_decay,
                                     ("truncated_normal", 0.001), 0.0)
        c = self._mixed17_1280(scope + "mixed_17x17x1280a", c)
        c = self._mixed8(scope + "mixed_8x8x2048a", c)
        c = self._mixed8(scope + "mixed_8x8x2048b", c)
        self.dropout = Dropout(scope + "logits/dropout", dropout_keep_prob)
        self.fc = FullyConnected(scope + "logits/logits", c, num_classes, None, None, True, weight_decay,
                                 ("truncated_normal", 0.01), 0.0)

    # ---- builders -------------------------------------------------------------------------------
    def _conv(self, name, cin, cout, k, stride=1, padding="SAME", stddev=None):
        c = Conv2d(name, cin, cout, k, stride, padding, "relu", dict(self._bn), False, self._wd,
                   ("truncated_normal", self._std if stddev is None else stddev))
        self.layers[name.replace("/", "__") or "root"] = c
        return c

    def _stem(self, scope):
        sc = _Scope(scope)
        self.stem = [self._conv(sc.name("conv0", "Conv"), 3, 32, 3, 2, "VALID"),
                     self._conv(sc.name("conv1", "Conv"), 32, 32, 3, 1, "VALID"),
                     self._conv(sc.name("conv2", "Conv"), 32, 64, 3, 1, "SAME"),
                     "pool1",
                     self._conv(sc.name("conv3", "Conv"), 64, 80, 1, 1, "VALID"),
                     self._conv(sc.name("conv4", "Conv"), 80, 192, 3, 1, "VALID"),
                     "pool2"]
        return 192

    def _mixed35(self, s, cin, pool_w):
        b = {}
        b["branch1x1"] = [self._conv(_Scope(s + "/branch1x1/").name(None, "Conv"), cin, 64, 1)]
        sc = _Scope(s + "/branch5x5/")
        b["branch5x5"] = [self._conv(sc.name(None, "Conv"), cin, 48, 1), self._conv(sc.name(None, "Conv"), 48, 64, 5)]
        sc = _Scope(s + "/branch3x3dbl/")
        b["branch3x3dbl"] = [self._conv(sc.name(None, "Conv"), cin, 64, 1), self._conv(sc.name(None, "Conv"), 64, 96, 3),
                             self._conv(sc.name(None, "Conv"), 96, 96, 3)]
        b["branch_pool"] = ["avg3", self._conv(_Scope(s + "/branch_pool/").name(None, "Conv"), cin, pool_w, 1)]
        self.plan.append((s, "cat", [b["branch1x1"], b["branch5x5"], b["branch3x3dbl"], b["branch_pool"]]))
        return 64 + 64 + 96 + pool_w

    def _mixed17a(self, s, cin):
        br3 = [self._conv(_Scope(s + "/branch3x3/").name(None, "Conv"), cin, 384, 3, 2, "VALID")]
        sc = _Scope(s + "/branch3x3dbl/")
        dbl = [self._conv(sc.name(None, "Conv"), cin, 64, 1), self._conv(sc.name(None, "Conv"), 64, 96, 3),
               self._conv(sc.name(None, "Conv"), 96, 96, 3, 2, "VALID")]
        self.plan.append((s, "cat", [br3, dbl, ["max3s2"]]))
        return 384 + 96 + cin

    def _mixed17(self, s, cin, w):
        b1 = [self._conv(_Scope(s + "/branch1x1/").name(None, "Conv"), cin, 192, 1)]
        sc = _Scope(s + "/branch7x7/")
        b7 = [self._conv(sc.name(None, "Conv"), cin, w, 1), self._conv(sc.name(None, "Conv"), w, w, (1, 7)),
              self._conv(sc.name(None, "Conv"), w, 192, (7, 1))]
        sc = _Scope(s + "/branch7x7dbl/")
        b7d = [self._conv(sc.name(None, "Conv"), cin, w, 1), self._conv(sc.name(None, "Conv"), w, w, (7, 1)),
               self._conv(sc.name(None, "Conv"), w, w, (1, 7)), self._conv(sc.name(None, "Conv"), w, w, (7, 1)),
               self._conv(sc.name(None, "Conv"), w, 192, (1, 7))]
        bp = ["avg3", self._conv(_Scope(s + "/branch_pool/").name(None, "Conv"), cin, 192, 1)]
        self.plan.append((s, "cat", [b1, b7, b7d, bp]))
        if s.endswith("mixed_17x17x768e"):
            self.plan.append((s, "aux", None))
        return 768

    def _mixed17_1280(self, s, cin):
        sc = _Scope(s + "/branch3x3/")
        b3 = [self._conv(sc.name(None, "Conv"), cin, 192, 1), self._conv(sc.name(None, "Conv"), 192, 320, 3, 2, "VALID")]
        sc = _Scope(s + "/branch7x7x3/")
        b7 = [self._conv(sc.name(None, "Conv"), cin, 192, 1), self._conv(sc.name(None, "Conv"), 192, 192, (1, 7)),
              self._conv(sc.name(None, "Conv"), 192, 192, (7, 1)),
              self._conv(sc.name(None, "Conv"), 192, 192, 3, 2, "VALID")]
        self.plan.append((s, "cat", [b3, b7, ["max3s2"]]))
        return 320 + 192 + cin

    def _mixed8(self, s, cin):
        b1 = [self._conv(_Scope(s + "/branch1x1/").name(None, "Conv"), cin, 320, 1)]
        sc = _Scope(s + "/branch3x3/")
        b3 = [self._conv(sc.name(None, "Conv"), cin, 384, 1),
              ("split", self._conv(sc.name(None, "Conv"), 384, 384, (1, 3)), self._conv(sc.name(None, "Conv"), 384, 384, (3, 1)))]
        sc = _Scope(s + "/branch3x3dbl/")
        b3d = [self._conv(sc.name(None, "Conv"), cin, 448, 1), self._conv(sc.name(None, "Conv"), 448, 384, 3),
               ("split", self._conv(sc.name(None, "Conv"), 384, 384, (1, 3)),
                self._conv(sc.name(None, "Conv"), 384, 384, (3, 1)))]
        bp = ["avg3", self._conv(_Scope(s + "/branch_pool/").name(None, "Conv"), cin, 192, 1)]
        self.plan.append((s, "cat", [b1, b3, b3d, bp]))
        return 320 + 768 + 768 + 192

    # ---- merged branch heads ----------------------------------------------------------------------
    @staticmethod
    def _sibling_heads(branches):
        """The branches' first convs that join the block's sibling group, in call order, as (weight, BatchNorm or
        None): a 1x1 stride-1 conv+BN at the branch start, and the commuted pool branch's 1x1 conv (no BN on its
        output: the BN follows the pool).  None when fewer than two."""
        heads = []
        for b in branches:
            op = b[0]
            if isinstance(op, Conv2d) and op.kh == 1 and op.kw == 1 and op.stride == 1 and op.bn is not None:
                heads.append((op.weights, op.bn))
            elif (op == "avg3" and len(b) > 1 and isinstance(b[1], Conv2d) and b[1].kh == 1 and b[1].kw == 1 and
                  b[1].stride == 1 and b[1].bn is not None and _fused.pool_commute_enabled()):
                heads.append((b[1].weights, None))
        return heads if len(heads) >= 2 else None

    def sibling_weight_groups(self):
        """Weight groups whose bf16 compute copies live side by side in one buffer (engine.prepare_compute_copies),
        so a mixed block's merged head conv reads its concatenated weights without a copy."""
        return [[w for w, _bn in h] for _n, kind, branches in self.plan if kind == "cat"
                for h in [self._sibling_heads(branches)] if h]

    # ---- forward --------------------------------------------------------------------------------
    @staticmethod
    def _run(branch, x, training):
        skip = False
        for i, op in enumerate(branch):
            if skip:
                skip = False
                continue
            # a pooling branch reads the block input alongside the branch convs: it joins their
            # gradient hand-off (its backward runs first and stashes; the last conv folds the stash)
            if op == "avg3":
                nxt = branch[i + 1] if i + 1 < len(branch) else None
                if (isinstance(nxt, Conv2d) and nxt.kh == 1 and nxt.kw == 1 and nxt.stride == 1 and
                        nxt.bn is not None and nxt.activation == "relu" and _fused.pool_commute_enabled() and
                        getattr(x, "is_cuda", False) and fused_enabled()):
                    # conv -> pool -> BN: the pool runs over the conv's output channels (ops.fused)
                    x = _fused.conv_avgpool_bn(x, nxt.weights, nxt.bn, training, relu=True)
                    skip = True
                    continue
                x = F.avg_pool(x, 3, 1, "SAME", grad_handoff=True)
            elif op == "max3s2":
                x = F.max_pool(x, 3, 2, "VALID", grad_handoff=True)
            elif isinstance(op, tuple):
                # a 'split' pair ends the branch with two channel parts
                return [op[1](x, training), op[2](x, training)]
            else:
                x = op(x, training)
        return [x]

    STEM_END_POINTS = ("conv0", "conv1", "conv2", "pool1", "conv3", "conv4", "pool2")

    def run_stem(self, x, training=True, end_points=None):
        net = x
        for op, name in zip(self.stem, self.STEM_END_POINTS):
            net = F.max_pool(net, 3, 2, "VALID") if isinstance(op, str) else op(net, training)
            if end_points is not None:
                end_points[name] = net
        return net

    def run_block(self, branches, net, training=True):
        """One mixed block: branch outputs written straight into their channel slices (zero-copy concat); the
        branches' first 1x1 conv+BNs on the block input share one forward (one conv + one finalize) and one
        backward (ops.fused.sibling_group)."""
        with _fused.sibling_group(net, training, heads=self._sibling_heads(branches)):
            parts = [p for b in branches for p in self._run(b, net, training)]
        return concat_channels(parts)

    def run_aux(self, net, training=True):
        # (a tail consumer of the Mixed_6e output: its gradient is added into the one Mixed_7a's backward returns)
        a = F.avg_pool(net, 5, 3, "VALID", grad_tail=True)
        a = self.aux_conv(self.aux_proj(a, training), training)
        return self.aux_fc(_t(a).reshape(a.shape[0], -1), training)

    def run_logits(self, net, training=True):
        k = net.shape[1]
        if _t(net).is_cuda:
            # the whole-map VALID average pool = the global mean (its kernel: one block per 256 channels and image
            # instead of one lane per output chunk, 128 blocks for the 8x8x2048 map; bf16 as the pool would store)
            net = F.global_avg_pool(net, out_bf16=True)
        else:
            net = F.avg_pool(net, (k, net.shape[2]), 1, "VALID")
        net = self.dropout(_t(net).reshape(net.shape[0], -1), training)
        return self.fc(net, training)

    def forward(self, x, training=True, end_points=None):
        # end points as the reference names them (inception/slim/inception_model.py:88-331)
        net = self.run_stem(x, training, end_points)
        aux = None
        for name, kind, branches in self.plan:
            if kind == "aux":
                aux = self.run_aux(net, training)
                if end_points is not None:
                    end_points["aux_logits"] = aux
                continue
            net = self.run_block(branches, net, training)
            if end_points is not None:
                end_points[name] = net
        logits = self.run_logits(net, training)
        if end_points is not None:
            end_points["logits"] = logits
            end_points["predictions"] = torch.softmax(logits.float(), -1)
        if training:
            return logits, aux
        return logits


def _t(x):
    from ..ops.lazy import as_tensor
    return as_tensor(x)


def inference(num_classes=1001, for_training=True, **kw):
    """inception/inception_model.py:inference equivalent (returns the module)."""
    return InceptionV3Slim(num_classes=num_classes, **kw)


BN_CLS = BatchNorm  # re-export for tests
