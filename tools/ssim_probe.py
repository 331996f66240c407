"""Diagnostic: time nic_ms_ssim on a 64 x 256^2 batch (run under rocprofv3 --kernel-trace
--stats for the per-kernel split)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from neural_network_image_compression_amd.codec import Codec  # noqa: E402

c = Codec(0)
g = torch.Generator().manual_seed(0)
a = torch.randint(0, 256, (64, 256, 256, 3), generator=g, dtype=torch.uint8).cuda()
b = torch.randint(0, 256, (64, 256, 256, 3), generator=g, dtype=torch.uint8).cuda()
for _ in range(30):
    c.ms_ssim(a, b)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    c.ms_ssim(a, b)
e1.record()
torch.cuda.synchronize()
print(f"ms_ssim 64x256^2: {e0.elapsed_time(e1) / 20:.4f} ms")
