"""Inter-kernel gaps of the config-2 passes without a profiler: a diagnostic build
(-DNIC_DIAG_KTIME, libnic_ktime.so via NIC_LIB) records each kernel's first-wave start and
last-wave exit on the 100 MHz device clock; one encode or decode call per reading.

    NIC_LIB=$PWD/neural_network_image_compression_amd/libnic_ktime.so python tools/ktime_probe.py
"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SLOTS = ["colour_split", "conv12", "k3_pair", "conv8", "fp32_chain", "dconv1", "dconv7", "gather"]
ENC = [0, 1, 2, 3, 4]
DEC = [5, 2, 6, 7, 4]


def main():
    import torch

    from bench import bench_weights
    from neural_network_image_compression_amd import _lib
    from neural_network_image_compression_amd._lib import latent_shape
    from neural_network_image_compression_amd.codec import Codec

    L = _lib.lib()
    f = L.nic_diag_ktime
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    f.restype = ctypes.c_int
    buf = (ctypes.c_ulonglong * 32)()

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
    for _ in range(30):
        codec.encode(x, out=z)
        codec.decode(z, out=r)
    torch.cuda.synchronize()

    def reading(call, order):
        assert f(None, 1) == 0
        call()
        torch.cuda.synchronize()
        assert f(buf, 0) == 0
        t = [(buf[2 * k], buf[2 * k + 1]) for k in range(16)]
        dur = [(t[k][1] - t[k][0]) * 10 for k in order]  # ns
        gaps = [(t[b][0] - t[a][1]) * 10 for a, b in zip(order, order[1:])]
        return dur, gaps

    out = {}
    for name, call, order in (("encode", lambda: codec.encode(x, out=z), ENC),
                              ("decode", lambda: codec.decode(z, out=r), DEC)):
        durs, gaps = [], []
        for _ in range(15):
            # keep the clock up between readings: a full step before each
            codec.encode(x, out=z)
            codec.decode(z, out=r)
            d, gp = reading(call, order)
            durs.append(d)
            gaps.append(gp)
        out[name] = {
            "kernels": [SLOTS[k] for k in order],
            "duration_us_median": [round(statistics.median(c) / 1e3, 2) for c in zip(*durs)],
            "gap_us_median": [round(statistics.median(c) / 1e3, 2) for c in zip(*gaps)],
        }
        out[name]["gap_us_total"] = round(sum(out[name]["gap_us_median"]), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
