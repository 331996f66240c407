"""Child-process parity check of the alternative f16x3 kernel form: NIC_K3P=0 runs the k3 residual
layers (conv3 / conv4, dconv5 / dconv6) as two weight-stationary launches instead of the fused
pair.  The switch is read once when libnic.so loads, so it cannot be toggled inside the pytest
process.  Run by tests/test_gpu_parity.py::test_alternative_kernels_parity; applies the same
contract as the golden encode/decode tests there and prints ALT-OK."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402  (HIP runtime before libnic.so)

from conftest import load_case  # noqa: E402
from neural_network_image_compression_amd import weights as W  # noqa: E402
from neural_network_image_compression_amd.codec import Codec  # noqa: E402
from oracle import nic_oracle as O  # noqa: E402
from test_gpu_parity import PREQUANT_ATOL, check_codes, check_recon  # noqa: E402


def main():
    assert os.environ.get("NIC_K3P") == "0"
    c = Codec(0, precision="f16x3")
    c.set_weights(W.seeded_weights(0, init="spread"))
    for case in ("kodim21_256", "imagenet4", "odd37x53"):
        g = load_case(case)
        z, f = c.encode(torch.from_numpy(g["x"]).cuda(), prequant=True)
        z, f = z.cpu().numpy(), f.cpu().numpy()
        assert np.abs(f - g["prequant"]).max() <= PREQUANT_ATOL, case
        check_codes(z, g["latent"], g["prequant"])
        r = c.decode(torch.from_numpy(g["latent"]).cuda()).cpu().numpy()
        check_recon(r, g["recon"])
        np.testing.assert_array_equal(O.quantise_u8(f), z)
    c.set_timing(True)
    c.decode(c.encode(torch.from_numpy(load_case("imagenet4")["x"]).cuda()))
    assert c.layer_times()["conv3"][1] == 1  # conv3 ran as its own launch (not fused)
    dump = os.environ.get("NIC_ALT_DUMP")
    if dump:  # reconstructions for a bit-exact comparison in the parent process
        np.savez(dump, **{k: v.cpu().numpy() for k, v in alt_cases(c).items()})
    print("ALT-OK")


def alt_cases(c):
    """Outputs compared bit for bit across kernel variants: decodes of the golden latents, of
    random latents whose dconv7 grid has partial 8x8 tiles (odd sizes) and of a 3-image 256^2
    batch; encodes (codes and fp32 pre-quant latent) of the golden inputs."""
    out = {}
    for case in ("kodim21_256", "imagenet4", "odd37x53"):
        g = load_case(case)
        out[case] = c.decode(torch.from_numpy(g["latent"]).cuda())
        out[case + "_z"], out[case + "_f"] = c.encode(torch.from_numpy(g["x"]).cuda(), prequant=True)
    rng = np.random.default_rng(77)
    for i, (h8, w8) in enumerate(((5, 7), (9, 3), (32, 32), (8, 300))):
        z = rng.integers(0, 256, (3 if w8 < 100 else 1, h8, w8, 96), dtype=np.uint8)
        out[f"rand{i}"] = c.decode(torch.from_numpy(z).cuda())
    # a 64 x 2400 image: its 600-column k3 planes run the fused residual pair in 62-column strips
    x = rng.integers(0, 256, (1, 64, 2400, 3), dtype=np.uint8)
    out["wide_z"], out["wide_f"] = c.encode(torch.from_numpy(x).cuda(), prequant=True)
    torch.cuda.synchronize()
    return out


if __name__ == "__main__":
    main()
