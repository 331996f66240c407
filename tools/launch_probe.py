"""Diagnostic: is the config-2 step launch-bound?  Times K eager steps (host issue time and
device time) and the same step captured once into a hipGraph (torch.cuda.CUDAGraph) and
replayed K times.  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from neural_network_image_compression_amd import weights as W  # noqa: E402
from neural_network_image_compression_amd._lib import latent_shape  # noqa: E402
from neural_network_image_compression_amd.codec import Codec  # noqa: E402

K = int(os.environ.get("K", "20"))
B, H = 64, 256
codec = Codec(0)
codec.set_weights(W.seeded_weights(0))
codec.reserve(B, H, H)
x = torch.randint(0, 256, (B, H, H, 3), generator=torch.Generator().manual_seed(1000), dtype=torch.uint8).cuda()
h8, w8 = latent_shape(H, H)
z = torch.empty((B, h8, w8, 96), dtype=torch.uint8, device="cuda")
r = torch.empty((B, H, H, 3), dtype=torch.uint8, device="cuda")


def step():
    codec.encode(x, out=z)
    codec.decode(z, out=r)


for _ in range(3):
    step()
torch.cuda.synchronize()
ref = r.clone()
t0 = time.perf_counter()
for _ in range(K):
    step()
t_issue = time.perf_counter() - t0
torch.cuda.synchronize()
t_eager = time.perf_counter() - t0

s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    step()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    step()
g.replay()
torch.cuda.synchronize()
same = bool(torch.equal(r, ref))
t0 = time.perf_counter()
for _ in range(K):
    g.replay()
torch.cuda.synchronize()
t_graph = time.perf_counter() - t0
print(json.dumps({"steps": K, "eager_ms": round(t_eager / K * 1e3, 4), "eager_issue_ms": round(t_issue / K * 1e3, 4),
                  "graph_ms": round(t_graph / K * 1e3, 4), "graph_matches_eager": same,
                  "eager_mps": round(B * H * H / 1e6 / (t_eager / K), 1),
                  "graph_mps": round(B * H * H / 1e6 / (t_graph / K), 1)}), flush=True)

# batch split over L contexts / streams: kernels of one lane fill the other lane's
# inter-kernel gaps and tails
res = {}
for L in (2, 3, 4):
    cs = [codec] + [Codec(0) for _ in range(L - 1)]
    for c in cs[1:]:
        c.set_weights(W.seeded_weights(0))
    bounds = [B * i // L for i in range(L + 1)]
    for i, c in enumerate(cs):
        c.reserve(bounds[i + 1] - bounds[i], H, H)
    ss = [torch.cuda.Stream() for _ in range(L)]

    def lstep():
        cur = torch.cuda.current_stream()
        for i in range(L):
            ss[i].wait_stream(cur)
            with torch.cuda.stream(ss[i]):
                a, b = bounds[i], bounds[i + 1]
                cs[i].encode(x[a:b], out=z[a:b])
                cs[i].decode(z[a:b], out=r[a:b])
        for i in range(L):
            cur.wait_stream(ss[i])

    for _ in range(3):
        lstep()
    torch.cuda.synchronize()
    ok = bool(torch.equal(r, ref))
    t0 = time.perf_counter()
    for _ in range(K):
        lstep()
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    res[f"lanes{L}"] = {"ms": round(t / K * 1e3, 4), "mps": round(B * H * H / 1e6 / (t / K), 1), "matches": ok}
print(json.dumps(res), flush=True)
