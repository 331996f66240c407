"""Per-step device time of the config-2 step (encode + decode) from a cold start: HIP events
around each of the first N steps, to separate one-time costs from the clock ramp.
usage: python tools/step_ramp.py [N]"""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from neural_network_image_compression_amd import weights as W  # noqa: E402
from neural_network_image_compression_amd.codec import Codec  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
c = Codec(0)
c.set_weights(W.seeded_weights(0))
c.reserve(64, 256, 256)
x = torch.randint(0, 256, (64, 256, 256, 3), generator=torch.Generator().manual_seed(1000), dtype=torch.uint8).cuda()
z = torch.empty((64, 32, 32, 96), dtype=torch.uint8, device="cuda")
r = torch.empty_like(x)
torch.cuda.synchronize()
time.sleep(0.5)  # idle, as between the driver's setup and its warmup
ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
ev[0].record()
for i in range(n):
    c.encode(x, out=z)
    c.decode(z, out=r)
    ev[i + 1].record()
torch.cuda.synchronize()
ms = [round(ev[i].elapsed_time(ev[i + 1]), 3) for i in range(n)]
print(json.dumps({"per_step_ms": ms}))
