"""Probe: eager PyTorch-ROCm (MIOpen/hipBLASLt) ResNet-50 v1 (slim geometry) bf16 step time.
Used only to size the target for the hand-written kernel path."""
import time, torch, torch.nn as nn, torch.nn.functional as F, json, sys
torch.backends.cudnn.benchmark = True
dev = 'cuda'
class Bott(nn.Module):
    def __init__(s, cin, depth, bd, stride):
        super().__init__()
        s.stride = stride
        s.short = None if cin == depth else nn.Sequential(nn.Conv2d(cin, depth, 1, bias=False), nn.BatchNorm2d(depth))
        s.c1 = nn.Conv2d(cin, bd, 1, bias=False); s.b1 = nn.BatchNorm2d(bd)
        s.c2 = nn.Conv2d(bd, bd, 3, stride, 1, bias=False); s.b2 = nn.BatchNorm2d(bd)
        s.c3 = nn.Conv2d(bd, depth, 1, bias=False); s.b3 = nn.BatchNorm2d(depth)
    def forward(s, x):
        sc = x[:, :, ::s.stride, ::s.stride] if s.short is None else s.short(x)
        y = F.relu(s.b1(s.c1(x))); y = F.relu(s.b2(s.c2(y))); y = s.b3(s.c3(y))
        return F.relu(y + sc)
class R50(nn.Module):
    def __init__(s):
        super().__init__()
        s.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(), nn.MaxPool2d(3, 2, 1))
        L = []; cin = 64
        for d, n, st in [(64, 3, 2), (128, 4, 2), (256, 6, 2), (512, 3, 1)]:
            for i in range(n):
                L.append(Bott(cin, d * 4, d, st if i == n - 1 else 1)); cin = d * 4
        s.blocks = nn.Sequential(*L); s.fc = nn.Linear(2048, 1000)
    def forward(s, x):
        return s.fc(s.blocks(s.stem(x)).mean((2, 3)))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
res = {}
for mode in ['autocast_cl']:
    m = R50().to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(B, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (B,), device=dev)
    def step():
        with torch.autocast('cuda', dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        opt.zero_grad(set_to_none=True); loss.backward(); opt.step()
    for _ in range(8): step()
    torch.cuda.synchronize(); t = time.time(); n = 20
    for _ in range(n): step()
    torch.cuda.synchronize(); dt = (time.time() - t) / n
    res[mode] = {'ms': dt * 1e3, 'img_s': B / dt}
    print(mode, res[mode], flush=True)
# conv microbench fwd/bwd per shape (bf16 NHWC)
shapes = [(56,64,64,3,1),(56,64,64,3,2),(28,128,128,3,1),(14,256,256,3,1),(7,512,512,3,1),(56,64,256,1,1),(56,256,64,1,1),(28,512,128,1,1),(14,1024,256,1,1),(7,2048,512,1,1),(224,3,64,7,2)]
for H,C,K,R,S in shapes:
    x = torch.randn(B, C, H, H, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last).requires_grad_()
    w = torch.randn(K, C, R, R, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last).requires_grad_()
    pad = R // 2
    def f(): return F.conv2d(x, w, None, S, pad)
    y = f(); g = torch.randn_like(y)
    for _ in range(3): f()
    torch.cuda.synchronize(); t = time.time()
    for _ in range(10): f()
    torch.cuda.synchronize(); tf = (time.time() - t) / 10
    for _ in range(2): torch.autograd.grad(f(), (x, w), g)
    torch.cuda.synchronize(); t = time.time()
    for _ in range(10): torch.autograd.grad(f(), (x, w), g)
    torch.cuda.synchronize(); tb = (time.time() - t) / 10 - tf
    Ho = y.shape[2]; fl = 2 * B * Ho * Ho * K * C * R * R
    print(f'conv H{H} C{C} K{K} R{R} S{S}: fwd {tf*1e3:.3f}ms {fl/tf/1e12:.0f}TF  bwd {tb*1e3:.3f}ms {2*fl/tb/1e12:.0f}TF', flush=True)
