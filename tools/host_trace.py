"""Host-array surface under rocprofv3 --sys-trace: a few Encoder()(numpy) -> Decoder()(numpy)
round trips of the config-2 batch after warm-up (tools/host_timeline.py reads the trace).
usage: rocprofv3 --sys-trace -d gpurun_out/<tag> -o ht -- python3 tools/host_trace.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from neural_network_image_compression_amd import weights as W  # noqa: E402
from neural_network_image_compression_amd.codec import Codec, Decoder, Encoder  # noqa: E402

c = Codec(0)
c.set_weights(W.seeded_weights(0))
c.reserve(64, 256, 256)
x = np.random.default_rng(0).integers(0, 256, (64, 256, 256, 3), dtype=np.uint8)
enc, dec = Encoder(codec=c), Decoder(codec=c)
for _ in range(5):
    dec(enc(x))
torch.cuda.synchronize()
t = []
for _ in range(5):
    t0 = time.perf_counter()
    dec(enc(x))
    t.append((time.perf_counter() - t0) * 1e3)
print("roundtrip ms", [round(v, 3) for v in t], flush=True)
c.close()
