"""Diagnostic (not the product): encode a few fixed synthetic batches (config 2, odd sizes, a
wide image for the k3 pair's strips, a kodak-size image) and save the u8 latents and fp32
pre-quant latents, so two library builds can be compared bit for bit:
    python tools/enc_dump_check.py out_a.npz;  NIC_LIB=other/libnic.so python tools/enc_dump_check.py out_b.npz"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from neural_network_image_compression_amd import weights as W  # noqa: E402
from neural_network_image_compression_amd.codec import Codec  # noqa: E402

c = Codec(0)
c.set_weights(W.seeded_weights(0))
g = torch.Generator().manual_seed(5)
out = {}
for i, (n, h, w) in enumerate(((64, 256, 256), (3, 37, 53), (2, 64, 2400), (1, 512, 768))):
    x = torch.randint(0, 256, (n, h, w, 3), generator=g, dtype=torch.uint8).cuda()
    z, f = c.encode(x, prequant=True)
    out[f"z{i}"] = z.cpu().numpy()
    out[f"f{i}"] = f.cpu().numpy()
np.savez(sys.argv[1], **out)
