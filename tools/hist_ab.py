"""A/B of the histogram-entropy kernel variants (NIC_HIST, see launch_hist) on real 4K latents.

    python tools/hist_ab.py [frames] [variants, comma-separated; d = library default]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from neural_network_image_compression_amd import weights as W  # noqa: E402
from neural_network_image_compression_amd.codec import Codec  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 8
c = Codec(0)
c.set_weights(W.seeded_weights(0))
g = torch.Generator().manual_seed(0)
x = torch.randint(0, 256, (F, 2160, 3840, 3), generator=g, dtype=torch.uint8).cuda()
z = c.encode(x)
torch.cuda.synchronize()
ref = None
for v in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["d", "big", "small"]):
    if v == "d":  # the library default
        os.environ.pop("NIC_HIST", None)
    else:
        os.environ["NIC_HIST"] = v
    for _ in range(3):
        bits, cnt = c.entropy(z, counts=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        c.entropy(z)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    cn = cnt.cpu()
    ok = ref is None or bool(torch.equal(cn, ref))
    ref = cn if ref is None else ref
    print(f"NIC_HIST={v:3s} {ms * 1e3:7.1f} us  {z.numel() / (ms * 1e-3) / 1e9:7.1f} GB/s  counts_equal={ok}", flush=True)
# latent value distribution (how skewed the bins are: same-address LDS atomics serialise)
cn = ref.double()
for pl in range(3):
    p = cn[pl] / cn[pl].sum()
    top = torch.topk(p, 4)
    print(f"plane {pl}: top bins {top.indices.tolist()} share {[round(v, 3) for v in top.values.tolist()]}")
# streaming reference: a torch int32 sum over the same bytes
zi = z.view(-1).view(torch.int32)
for _ in range(3):
    zi.sum()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    zi.sum()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
print(f"torch int32 sum: {ms * 1e3:7.1f} us  {z.numel() / (ms * 1e-3) / 1e9:7.1f} GB/s")
