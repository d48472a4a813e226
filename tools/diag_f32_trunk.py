"""Per-parameter gradient error of the fp32 HIP ResNet-18 trunk and of the fp32 CPU
oracle, both against the float64 oracle (diagnostic; run on the GPU box)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from greedy_multimodal_learning_amd.resnet import resnet18  # noqa: E402
from oracle.resnet_ref import resnet18 as resnet18_ref  # noqa: E402


def err(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max()) / (float(b.abs().max()) + 1e-30)


torch.manual_seed(0)
ref = resnet18_ref(num_classes=40).double()
r32 = resnet18_ref(num_classes=40)
r32.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
net = resnet18(num_classes=40)
net.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
net = net.cuda()
g = torch.Generator().manual_seed(11)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4
S = int(sys.argv[2]) if len(sys.argv) > 2 else 64
x = torch.randn(N, 3, S, S, generator=g)
out, o32, oref = net(x.cuda()), r32(x), ref(x.double())
print("logits err hip", err(out, oref), "cpu32", err(o32, oref))
gy = torch.randn(oref.shape, generator=g)
out.backward(gy.cuda())
o32.backward(gy)
oref.backward(gy.double())
rp, p32 = dict(ref.named_parameters()), dict(r32.named_parameters())
rows = [(err(p.grad, rp[n].grad), err(p32[n].grad, rp[n].grad), n) for n, p in net.named_parameters()]
for e, e32, n in sorted(rows, reverse=True)[:25]:
    print(f"{n:40s} hip {e:.3e}  cpu32 {e32:.3e}")


def feats(m, x):
    x = m.maxpool(m.bn1(m.conv1(x), relu=True)) if hasattr(m.bn1, "num_features") and "GM" in type(m.bn1).__name__ \
        else m.maxpool(m.relu(m.bn1(m.conv1(x))))
    return m.layer4(m.layer3(m.layer2(m.layer1(x))))


for m in (net, ref):
    for p in m.parameters():
        p.grad = None
xs = (x.cuda(), x.double())
fs = []
for m, xx in ((net, xs[0]), (ref, xs[1])):
    f = feats(m, xx)
    f.retain_grad()
    o = m.fc(torch.flatten(m.avgpool(f), 1))
    o.backward(gy.to(o.device, o.dtype))
    fs.append(f)
print("features err", err(fs[0], fs[1]), "dfeat err", err(fs[0].grad, fs[1].grad),
      "strides", fs[0].grad.stride(), fs[0].grad.is_contiguous())
print("bn2.bias", err(net.layer4[1].bn2.bias.grad, ref.layer4[1].bn2.bias.grad))
# the last BN's bias gradient is sum(dy * [y > 0]) over the map
mask = (fs[1] > 0).double()
print("sum dz ref", float((fs[1].grad * mask).sum((0, 2, 3)).abs().max()),
      "direct from hip f/grad", err((fs[0].grad.double() * (fs[0] > 0).double()).sum((0, 2, 3)),
                                    (fs[1].grad * mask).sum((0, 2, 3))))
