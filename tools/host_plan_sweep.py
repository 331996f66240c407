"""Host-array surface (Encoder()(numpy) -> Decoder()(numpy), config-2 batch) per chunk plan and
staging-copy thread count, each setting in a fresh process (the switches are read at library
load): chunks and
NIC_HOST_COPY_THREADS.  Prints one JSON line per setting; usage: python tools/host_plan_sweep.py [n settings]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, time, json, numpy as np, torch
sys.path.insert(0, %r)
from neural_network_image_compression_amd import weights as W
from neural_network_image_compression_amd.codec import Codec, Encoder, Decoder
c = Codec(0); c.set_weights(W.seeded_weights(0)); c.reserve(64, 256, 256)
x = torch.randint(0, 256, (64, 256, 256, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(1000))
xh = x.numpy(); xd = x.cuda()
enc, dec = Encoder(codec=c), Decoder(codec=c)
enc.host_chunks = dec.host_chunks = int(sys.argv[1])
def t(f, reps=40):
    for _ in range(5): f()
    torch.cuda.synchronize(); best = []
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(reps): f()
        torch.cuda.synchronize(); best.append((time.perf_counter() - t0) / reps * 1e3)
    return min(best)
dev = t(lambda: c.decode(c.encode(xd)))
z = enc(xh)
r = {"device_ms": dev, "enc_page_ms": t(lambda: enc(xh)), "dec_pin_ms": t(lambda: dec(z)),
     "roundtrip_ms": t(lambda: dec(enc(xh)))}
r["ratio"] = r["device_ms"] / r["roundtrip_ms"]
print(json.dumps({k: round(v, 4) for k, v in r.items()}))
''' % ROOT

SETTINGS = [("3", {}), ("3", {"NIC_HOST_COPY_THREADS": "0"}), ("3", {"NIC_HOST_COPY_THREADS": "7"}), ("4", {}),
            ("2", {}), ("5", {})]
for chunks, env in SETTINGS[:int(sys.argv[1]) if len(sys.argv) > 1 else None]:
    e = dict(os.environ, **env)
    out = subprocess.run([sys.executable, "-c", CHILD, chunks], env=e, capture_output=True, text=True, timeout=240)
    line = out.stdout.strip().splitlines()[-1] if out.returncode == 0 and out.stdout.strip() else None
    print(json.dumps({"chunks": int(chunks), "env": env, "result": json.loads(line) if line else out.stderr[-500:]}),
          flush=True)
