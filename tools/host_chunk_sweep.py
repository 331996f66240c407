"""Host-array surface (Encoder()(numpy) -> Decoder()(numpy), nic_encode_host /
nic_decode_host) against the number of pipeline chunks per call, beside the device-resident
pass.  usage: python tools/host_chunk_sweep.py [--chunks 2,3,4,5,6,8]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="2,3,4,5,6,8")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch

    from neural_network_image_compression_amd import weights as W
    from neural_network_image_compression_amd.codec import Codec, Decoder, Encoder

    c = Codec(0)
    c.set_weights(W.seeded_weights(0))
    c.reserve(64, 256, 256)
    x = torch.randint(0, 256, (64, 256, 256, 3), generator=torch.Generator().manual_seed(1000), dtype=torch.uint8)
    xh, xd = x.numpy(), x.cuda()
    enc, dec = Encoder(codec=c), Decoder(codec=c)

    def t(f):
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            f()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.reps * 1e3

    res = {"device_ms": round(t(lambda: c.decode(c.encode(xd))), 3)}
    for k in (int(v) for v in args.chunks.split(",")):
        enc.host_chunks = dec.host_chunks = k
        res[f"host_ms_chunks{k}"] = round(t(lambda: dec(enc(xh))), 3)
    res["device_mp_s"] = round(64 * 65536 / 1e3 / res["device_ms"], 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
