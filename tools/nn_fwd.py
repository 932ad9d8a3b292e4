"""Run the leaf-eval forward a few times (for rocprofv3 kernel tracing)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "harmonies-alphazero_amd"))
import torch
from hzamd.net import HarmoniesNet
torch.backends.cudnn.benchmark = True
dev = "cuda:0"
torch.manual_seed(0)
net = HarmoniesNet().to(dev).eval()
cl = len(sys.argv) > 1 and sys.argv[1] == "cl"
folded = len(sys.argv) > 1 and sys.argv[1] == "folded"
B = 4096
board = (torch.rand(B, 38, 5, 7, device=dev) > 0.8).float()
glob = torch.rand(B, 42, device=dev)
if cl:
    net = net.to(memory_format=torch.channels_last)
    board = board.to(memory_format=torch.channels_last)
if folded:
    from hzamd.infer import FoldedNet
    net = FoldedNet(net)
with torch.no_grad():
    for _ in range(8):
        net(board, glob)
torch.cuda.synchronize()
print("done")
