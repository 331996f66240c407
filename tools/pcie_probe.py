"""Host-path (PCIe-inclusive) timing probe of the NumPy surface: device pass, staged/direct
H2D, pinned results, host copy rates.  usage: python tools/pcie_probe.py"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time, numpy as np, torch, json
from neural_network_image_compression_amd import weights as W
from neural_network_image_compression_amd.codec import Codec, Encoder, Decoder
c = Codec(0); c.set_weights(W.seeded_weights(0)); c.reserve(64, 256, 256)
x = torch.randint(0, 256, (64, 256, 256, 3), dtype=torch.uint8)
xh = x.numpy(); xd = x.cuda()
enc, dec = Encoder(codec=c), Decoder(codec=c)
def t(f, reps=10):
    f(); torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(reps): f()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / reps * 1e3
res = {}
res["device_ms"] = t(lambda: c.decode(c.encode(xd)))
zd = c.encode(xd)
res["dev_enc_ms"] = t(lambda: c.encode(xd))
res["dev_dec_ms"] = t(lambda: c.decode(zd))
res["dev_enc_4x16_ms"] = t(lambda: [c.encode(xd[k:k + 16]) for k in range(0, 64, 16)])
res["dev_dec_4x16_ms"] = t(lambda: [c.decode(zd[k:k + 16]) for k in range(0, 64, 16)])
xs = np.zeros((1, 8, 8, 3), np.uint8)
res["enc_np_tiny_ms"] = t(lambda: enc(xs))
res["enc_np_ms"] = t(lambda: enc(xh))
z = enc(xh)
res["dec_np_pinned_ms"] = t(lambda: dec(z))
zp = z.copy()
res["dec_np_page_ms"] = t(lambda: dec(zp))
res["roundtrip_ms"] = t(lambda: dec(enc(xh)))
enc.host_chunks = dec.host_chunks = 1
res["enc_np_ch1_ms"] = t(lambda: enc(xh))
res["dec_np_ch1_ms"] = t(lambda: dec(z))
xpin = c._host_out(xh.shape); xpin[:] = xh
for ch in (1, 2, 3, 4, 5, 6, 8):
    enc.host_chunks = dec.host_chunks = ch
    res[f"ch{ch}"] = {"enc_page": t(lambda: enc(xh)), "enc_pin": t(lambda: enc(xpin)),
                      "dec_page": t(lambda: dec(zp)), "dec_pin": t(lambda: dec(z)),
                      "roundtrip": t(lambda: dec(enc(xh)))}
enc.host_chunks = dec.host_chunks = 4
st = torch.empty(xh.size, dtype=torch.uint8, pin_memory=True).numpy()
res["memcpy_1thr_ms"] = t(lambda: np.copyto(st, xh.reshape(-1)))
pin = torch.from_numpy(st)
res["h2d_12MB_ms"] = t(lambda: xd.view(-1).copy_(pin, non_blocking=True))
res["d2h_12MB_ms"] = t(lambda: pin.copy_(xd.view(-1), non_blocking=True))
res["mp_per_batch"] = 64 * 256 * 256 / 1e6
r3 = lambda v: round(v, 3) if isinstance(v, float) else ({k: r3(u) for k, u in v.items()} if isinstance(v, dict) else v)
print(json.dumps(r3(res)))
