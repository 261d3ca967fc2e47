import sys, torch
sys.path.insert(0, "/root/repo")
from distributed_tensorflow_models_amd.engine import TrainStep
from distributed_tensorflow_models_amd.models import nets_factory
from distributed_tensorflow_models_amd.ops import _lib
import distributed_tensorflow_models_amd.ops.nn as nnm
model = sys.argv[1]
from bench import PRESETS
S, ncls, B0, opt, extra = PRESETS[model]
torch.manual_seed(0)
kw = {"fc_conv_padding": "SAME"} if model == "vgg_16" else {}
net = nets_factory.build(model, num_classes=ncls, **kw).cuda()
step = TrainStep(net, optimizer=opt, lr=0.01, momentum=0.9, **extra)
x = torch.randn(8, S, S, 3, device="cuda").to(torch.bfloat16)
y = torch.randint(0, ncls, (8,), device="cuda")
L = _lib.lib()
calls = []
orig = nnm.weight_flipped
def wf(w, K, R, S_, C, dec=None):
    c = getattr(w, "_flip" if dec is None else "_flipdec", None)
    fresh = c is not None and c[0] == nnm.WEIGHT_VERSION[0] and c[1].shape == (C, R, S_, K) and c[2] == dec
    if not fresh:
        calls.append((tuple(w.shape), type(w).__name__, dec, None if c is None else (c[0], nnm.WEIGHT_VERSION[0], tuple(c[1].shape), c[2])))
    return orig(w, K, R, S_, C, dec)
nnm.weight_flipped = wf
import distributed_tensorflow_models_amd.ops.fused as fm
fm.weight_flipped = wf
for i in range(4):
    calls.clear()
    step(x, y)
    torch.cuda.synchronize()
    print("step", i, "refresh misses:", len(calls))
for c in calls: print(c)
