"""Child-process run of the chained re-run's barrier-timeout path (the timeout must
be reported, once, and leave the ctx usable).  NIC_DIAG_BARRIER=skip makes the last block of
fp32_chain_kernel never arrive at its grid barriers and cuts the bounded wait to ~1 ms, so a
tripped pass's exact-fp32 re-run times out.  Run by
test_gpu_parity.py::test_chain_barrier_timeout_reported; prints TIMEOUT-OK."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (HIP runtime before libnic.so)

from conftest import load_case  # noqa: E402
from neural_network_image_compression_amd import _lib  # noqa: E402
from neural_network_image_compression_amd import weights as W  # noqa: E402
from neural_network_image_compression_amd.codec import Codec, Encoder  # noqa: E402
from test_gpu_parity import range_scaled_weights  # noqa: E402


def expect_ehip(fn):
    try:
        fn()
    except _lib.NicError as e:
        assert e.code == _lib.NIC_EHIP, e
        assert "timed out" in str(e), e
        return
    raise AssertionError("no NIC_EHIP raised")


def main():
    assert os.environ.get("NIC_DIAG_BARRIER") == "skip"
    g = load_case("kodim21_256")
    x = torch.from_numpy(g["x"]).cuda()
    c = Codec(0)
    c.set_weights(range_scaled_weights(W.seeded_weights(0, init="spread")))
    # two tripped passes before anyone looks: the first chain times out, the second exits at
    # its entry (the sticky flag), neither hangs the queue
    c.encode(x)
    c.encode(x)
    torch.cuda.synchronize()
    expect_ehip(c.range_trips)  # reported once ...
    n = c.range_trips()         # ... then cleared
    assert n >= 1, n
    # the ERROR policy's synchronising check reports a timeout left by a FALLBACK pass
    c.encode(x)
    c.set_range_policy("error")
    expect_ehip(lambda: c.encode(x))
    c.set_range_policy("fallback")
    c.range_trips()
    # the host-array surface (it synchronises) reports its own chain's timeout
    enc = Encoder(codec=c)
    expect_ehip(lambda: enc(g["x"]))
    c.range_trips()
    # in-range weights never reach the chain: a clean pass on the same process
    ok = Codec(0)
    ok.set_weights(W.seeded_weights(0, init="spread"))
    z = ok.encode(x).cpu().numpy()
    assert ok.range_trips() == 0
    assert np.abs(z.astype(int) - g["latent"].astype(int)).max() <= 1
    print("TIMEOUT-OK")


if __name__ == "__main__":
    main()
