"""Which kernel torch's fill_ launches on ROCm (run under rocprofv3 --kernel-trace): fills of a 2 GiB float tensor
with 0.0 and with 1.5, and the same bytes as uint8 / int64."""
import torch
x = torch.empty(1 << 29, dtype=torch.float32, device=0)
for v in (0.0, 1.5):
    x.fill_(v)
x.view(torch.uint8).fill_(3)
x.view(torch.int64).fill_(7)
x.zero_()
torch.cuda.synchronize()
print('ok')
