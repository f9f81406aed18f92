"""pyprof walk-through on a LeNet-style net (reference apex/pyprof/examples/lenet.py,
user_annotation/resnet.py).

    cd /tmp && rocprofv3 --kernel-trace --marker-trace --hip-runtime-trace --output-format csv \\
        -d /tmp/pyprof_out -- python3 /root/repo/examples/pyprof/lenet.py
    python -m apex.pyprof.parse /tmp/pyprof_out > /tmp/parsed.txt
    python -m apex.pyprof.prof -c idx,dir,layer,op,kernel,params,sil,tc,flops,bytes -w 200 /tmp/parsed.txt
    python -m apex.pyprof.prof --summary op /tmp/parsed.txt

Every torch op (forward AND backward), every nn.Module forward and every apex multi-tensor op is
a marker range; ``pyprof.layer`` adds user layer names; ``pyprof.wrap`` annotates a custom
function."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))  # uninstalled checkout
import apex.pyprof as pyprof  # noqa: E402
from apex.optimizers import FusedAdam  # noqa: E402

pyprof.init()


class LeNet5(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = torch.nn.Conv2d(1, 6, 5)
        self.conv2 = torch.nn.Conv2d(6, 16, 5)
        self.fc1 = torch.nn.Linear(16 * 5 * 5, 120)
        self.fc2 = torch.nn.Linear(120, 84)
        self.fc3 = torch.nn.Linear(84, 10)

    def forward(self, x):
        with pyprof.layer("features"):
            x = F.max_pool2d(F.relu(self.conv1(x)), (2, 2))
            x = F.max_pool2d(F.relu(self.conv2(x)), 2)
        with pyprof.layer("classifier"):
            x = x.flatten(1)
            x = F.relu(self.fc1(x))
            x = F.relu(self.fc2(x))
            return self.fc3(x)


def scaled_gelu(x, s):
    return F.gelu(x) * s


class Custom:
    scaled_gelu = staticmethod(scaled_gelu)


pyprof.wrap(Custom, "scaled_gelu")


def main():
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    net = LeNet5().to(dev)
    opt = FusedAdam(net.parameters(), lr=1e-3)
    x = torch.randn(256, 1, 32, 32, device=dev)
    y = torch.randint(0, 10, (256,), device=dev)
    for _ in range(3):
        opt.zero_grad()
        out = Custom.scaled_gelu(net(x), 0.5)
        loss = F.cross_entropy(out, y)
        loss.backward()
        opt.step()
    if dev == "cuda":
        torch.cuda.synchronize()
    print("loss", float(loss))


if __name__ == "__main__":
    main()
