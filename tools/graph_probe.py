"""Does replaying the config-2 step (nic_encode + nic_decode, every launch of the device path) as
one captured HIP graph shorten it?  Direct calls vs torch.cuda.CUDAGraph replay of the same step
on the same context, alternating rounds, outputs compared byte for byte.

    python tools/graph_probe.py [--steps 50] [--rounds 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import torch

    from bench import bench_weights
    from neural_network_image_compression_amd._lib import latent_shape
    from neural_network_image_compression_amd.codec import Codec

    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    B, H, W = 64, 256, 256
    codec = Codec(0)
    codec.set_weights(bench_weights("spread"))
    codec.reserve(B, H, W)
    g = torch.Generator().manual_seed(1000)
    x = torch.randint(0, 256, (B, H, W, 3), generator=g, dtype=torch.uint8).to(dev)
    h8, w8 = latent_shape(H, W)
    z = torch.empty((B, h8, w8, 96), dtype=torch.uint8, device=dev)
    r = torch.empty((B, 8 * h8, 8 * w8, 3), dtype=torch.uint8, device=dev)

    def step():
        codec.encode(x, out=z)
        codec.decode(z, out=r)

    for _ in range(20):
        step()
    torch.cuda.synchronize()
    z_ref, r_ref = z.clone(), r.clone()

    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()  # warm the side stream
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(graph):
        step()
    torch.cuda.synchronize()
    z.zero_()
    r.zero_()
    graph.replay()
    torch.cuda.synchronize()
    same = bool(torch.equal(z, z_ref) and torch.equal(r, r_ref))

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.steps * 1e3

    res = {"direct_ms": [], "graph_ms": []}
    for _ in range(args.rounds):
        res["direct_ms"].append(round(timed(step), 4))
        res["graph_ms"].append(round(timed(graph.replay), 4))
    res["outputs_identical"] = same
    res["mp_per_s_direct"] = round(B * H * W / 1e6 / (min(res["direct_ms"]) / 1e3), 1)
    res["mp_per_s_graph"] = round(B * H * W / 1e6 / (min(res["graph_ms"]) / 1e3), 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
