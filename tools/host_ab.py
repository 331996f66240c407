"""Host-array surface A/B (diagnostic, not the product): Decoder()(Encoder()(numpy)) of the
config-2 batch against the device-resident pass, in one process, after a warm-up long enough
for the clocks to settle; medians over many repetitions (the per-call times are noisy).
usage: python tools/host_ab.py [--chunks 4] [--reps 40]  (library switches via environment)"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="4")
    ap.add_argument("--reps", type=int, default=40)
    args = ap.parse_args()
    import numpy as np
    import torch

    from neural_network_image_compression_amd import weights as W
    from neural_network_image_compression_amd.codec import Codec, Decoder, Encoder

    c = Codec(0)
    c.set_weights(W.seeded_weights(0))
    c.reserve(64, 256, 256)
    x = torch.randint(0, 256, (64, 256, 256, 3), generator=torch.Generator().manual_seed(1000), dtype=torch.uint8)
    xh, xd = x.numpy(), x.cuda()
    enc, dec = Encoder(codec=c), Decoder(codec=c)

    def med(f):
        for _ in range(10):
            f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            f()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return round(float(np.median(ts)) * 1e3, 3)

    res = {"device_ms": med(lambda: c.decode(c.encode(xd)))}
    zd = c.encode(xd)
    res["dev_enc_4x16_ms"] = med(lambda: [c.encode(xd[k:k + 16]) for k in range(0, 64, 16)])
    res["dev_dec_4x16_ms"] = med(lambda: [c.decode(zd[k:k + 16]) for k in range(0, 64, 16)])
    z = enc(xh)
    for k in (int(v) for v in args.chunks.split(",")):
        enc.host_chunks = dec.host_chunks = k
        res[f"enc_ms_c{k}"] = med(lambda: enc(xh))
        res[f"dec_ms_c{k}"] = med(lambda: dec(z))
        res[f"host_ms_c{k}"] = med(lambda: dec(enc(xh)))
    res["device_ms_after"] = med(lambda: c.decode(c.encode(xd)))
    res["env"] = {k: v for k, v in os.environ.items() if k.startswith("NIC_")}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
