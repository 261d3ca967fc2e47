import copy, os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_models_amd.models.resnet_v1 import ResNetV1
def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()
for dtype in ["bf16", "fp32cpu_bf16in"]:
    torch.manual_seed(0)
    net_cpu = ResNetV1(blocks=[(16, 2, 2), (32, 2, 1)], num_classes=10, scope="r")
    net_gpu = copy.deepcopy(net_cpu).cuda()
    x = torch.randn(16, 32, 32, 3).to(torch.bfloat16).float()
    lab = torch.randint(0, 10, (16,))
    ep_c, ep_g = {}, {}
    out_c = net_cpu(x, training=True, end_points=ep_c)
    torch.nn.functional.cross_entropy(out_c.float(), lab).backward()
    out_g = net_gpu(x.cuda().to(torch.bfloat16), training=True, end_points=ep_g)
    torch.nn.functional.cross_entropy(out_g.float(), lab.cuda()).backward()
    torch.cuda.synchronize()
    print("out", rel(out_g, out_c))
    for k in ep_c:
        if torch.is_tensor(ep_c[k]) and torch.is_tensor(ep_g.get(k)):
            print("  ep", k, round(rel(ep_g[k], ep_c[k]), 4))
    pc = dict(net_cpu.named_parameters())
    for n, p in net_gpu.named_parameters():
        print(" ", n, round(rel(p.grad, pc[n].grad), 4))
    break
