import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libnic.so")


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def load_case(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as d:
        return {k: d[k] for k in d.files}


@pytest.fixture(scope="session")
def golden():
    return load_case


@pytest.fixture(scope="session")
def weights_spread():
    from neural_network_image_compression_amd import weights as W
    return W.seeded_weights(0, init="spread")


@pytest.fixture(scope="session")
def weights_glorot():
    from neural_network_image_compression_amd import weights as W
    return W.seeded_weights(0, init="glorot")


TRAINED_COEFS = ("0.01", "0.02", "0.03")


def trained_weights(coef="0.01"):
    """A codec trained for 30 epochs on the reference's 19,000 patches with entropy_loss_coef
    `coef` (tools/train_rd.py, TF encode_png target, seed 0, round 4), committed under
    tests/golden/trained."""
    from neural_network_image_compression_amd import weights as W
    pre = os.path.join(GOLDEN, "trained", f"coef{coef}_")
    w = W.load(pre + "encoder", "encoder")
    w.update(W.load(pre + "decoder", "decoder"))
    return w


@pytest.fixture(scope="session")
def weights_trained():
    return trained_weights("0.01")


@pytest.fixture(scope="session")
def weights_by_init(weights_spread, weights_glorot, weights_trained):
    """Every committed weight set by the manifest's "init" name."""
    out = {"spread": weights_spread, "glorot": weights_glorot, "trained_coef0.01": weights_trained}
    for c in TRAINED_COEFS[1:]:
        out[f"trained_coef{c}"] = trained_weights(c)
    return out
