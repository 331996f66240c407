"""Child-process run of the f16 range-guard contract (tests/test_gpu_parity.py
range_guard_contract) under a load-time switch: NIC_CHAIN=0 (the gated exact-fp32 re-run as
one launch per layer) or NIC_DIAG_CHAIN=N (the chained re-run on N blocks per CU, block 0
started late: no co-residency).  Run by
test_gpu_parity.py::test_f16_range_guard_rerun_variants; prints RANGE-OK."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402,F401  (HIP runtime before libnic.so)

from conftest import load_case  # noqa: E402
from neural_network_image_compression_amd import weights as W  # noqa: E402
from test_gpu_parity import range_guard_contract  # noqa: E402


def main():
    assert os.environ.get("NIC_CHAIN") == "0" or os.environ.get("NIC_DIAG_CHAIN")
    range_guard_contract(load_case, W.seeded_weights(0, init="spread"))
    print("RANGE-OK")


if __name__ == "__main__":
    main()
