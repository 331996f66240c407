"""Training side path (training.py, restating tf2_0/src/training.py:25-172 on PyTorch
autograd): its forward pass and SSIM against the oracle, one optimisation step on CPU, and
(on the GPU) trained weights flowing through the reference's checkpoint format into the HIP
codec."""
import numpy as np
import pytest
import torch

from oracle import nic_oracle as O
from neural_network_image_compression_amd import training as T
from neural_network_image_compression_amd import weights as W


def _smooth(n, h, w, seed):
    rng = np.random.default_rng(seed)
    a = np.cumsum(np.cumsum(rng.integers(-2, 3, (n, h, w, 3)), axis=1), axis=2).astype(np.float64)
    a -= a.min(axis=(1, 2, 3), keepdims=True)
    a *= 255.0 / np.maximum(a.max(axis=(1, 2, 3), keepdims=True), 1)
    return a.astype(np.uint8)


def test_ssim_matches_oracle():
    rng = np.random.default_rng(0)
    x = rng.random((2, 40, 37, 1))
    y = np.clip(x + 0.1 * rng.standard_normal(x.shape), 0, 1)
    ref, _ = O._ssim_per_channel(x, y)
    got = T.ssim(torch.from_numpy(x).permute(0, 3, 1, 2), torch.from_numpy(y).permute(0, 3, 1, 2))
    np.testing.assert_allclose(got.numpy(), ref.mean(axis=1), atol=1e-10)


def test_forward_matches_oracle():
    w = W.seeded_weights(0)
    x = _smooth(2, 48, 40, 1)
    p = {k: torch.from_numpy(v) for k, v in w.items()}
    planes = T.colour_planes(torch.from_numpy(x).float() / 255)
    enc = lambda m, t: T.base_encoder({k[len(m) + 1:]: v for k, v in p.items() if k.startswith(m + "/")}, t)  # noqa
    z = torch.cat([enc("encoderY", planes[0]), enc("encoderCbCr", planes[1]), enc("encoderCbCr", planes[2])], 1)
    np.testing.assert_allclose(z.permute(0, 2, 3, 1).numpy(), O.encode_f32(w, x), atol=2e-5)
    zu = O.encode(w, x)
    zn = torch.from_numpy(zu).float().permute(0, 3, 1, 2) / 255
    dec = {k[len("decoderY") + 1:]: v for k, v in p.items() if k.startswith("decoderY/")}
    r = T.base_decoder(dec, zn[:, :32])
    ref = O.base_decoder(O._model_params(w, "decoderY"), zu[..., :32].astype(np.float32) / np.float32(255))
    np.testing.assert_allclose(r.permute(0, 2, 3, 1).numpy(), ref, atol=2e-5)


def test_train_step_cpu(tmp_path):
    tr = T.Training(device="cpu", seed=0, checkpoint_dir=str(tmp_path) + "/")
    before = tr.weights()
    log = tr(_smooth(4, 64, 64, 2), None, max_epochs=1, batch_size=2, entropy_loss_coef=0.01, verbose=False)
    assert len(log) == 2
    for m in log:
        assert all(np.isfinite(m["ssim"])) and all(np.isfinite(m["bpp"])) and np.isfinite(m["entropy_loss"])
        assert all(b > 0 for b in m["bpp"])
    after = tr.weights()
    changed = [k for k in before if not np.array_equal(before[k], after[k])]
    assert {k.split("/")[0] for k in changed} == set(W.MODEL_NAMES)
    tr._save()
    back = W.load(str(tmp_path / "encoder"), "encoder")
    for k, v in back.items():
        np.testing.assert_array_equal(v, after[k])


def test_epoch_samples_cpu(tmp_path):
    """An epoch of `epoch_samples` images over reshuffled passes of a smaller subset (the
    reference's epoch length over its full set); the coefficient schedule steps per epoch."""
    tr = T.Training(device="cpu", seed=0, checkpoint_dir=str(tmp_path) + "/")
    log = tr(_smooth(3, 32, 32, 4), None, max_epochs=2, batch_size=2, entropy_loss_coef=0.01, verbose=False,
             epoch_samples=5)
    assert len(log) == 6  # ceil(5 / 2) steps per epoch
    assert [m["epoch"] for m in log] == [0, 0, 0, 1, 1, 1]


@pytest.mark.gpu
def test_trained_weights_into_hip_codec(tmp_path):
    """GPU training steps -> TF checkpoint (training.py:167-172) -> Encoder.load -> HIP encode
    equals the oracle with the trained weights."""
    from neural_network_image_compression_amd.codec import Encoder
    tr = T.Training(device="cuda", seed=1, checkpoint_dir=str(tmp_path) + "/")
    tr(_smooth(4, 128, 128, 3), None, max_epochs=2, batch_size=2, entropy_loss_coef=0.01, verbose=False)
    tr._save()
    enc = Encoder(0)
    enc.load(str(tmp_path / "encoder"))
    x = _smooth(1, 64, 72, 4)
    z, f = enc.codec.encode(torch.from_numpy(x).cuda(), prequant=True)
    np.testing.assert_allclose(f.cpu().numpy(), O.encode_f32(tr.weights(), x), atol=2e-5)


def test_adam_matches_keras_update():
    """torch Adam with keras_adam_eps(step) reproduces tf.keras Adam's update rule
    (lr_t = lr sqrt(1-b2^t)/(1-b1^t); theta -= lr_t m / (sqrt(v) + eps)), restated in float64."""
    rng = np.random.default_rng(3)
    theta0 = rng.standard_normal(64)
    grads = [rng.standard_normal(64) * 10.0 ** rng.integers(-9, 1) for _ in range(6)]
    lr, b1, b2, eps = 1e-4, 0.9, 0.999, 1e-7
    th, m, v = theta0.copy(), np.zeros(64), np.zeros(64)
    for t, g in enumerate(grads, 1):
        m = b1 * m + (1 - b1) * g
        v = b2 * v + (1 - b2) * g * g
        th = th - lr * np.sqrt(1 - b2 ** t) / (1 - b1 ** t) * m / (np.sqrt(v) + eps)
    p = torch.tensor(theta0, dtype=torch.float64, requires_grad=True)
    opt = torch.optim.Adam([p], lr=lr, betas=(b1, b2), eps=eps)
    for t, g in enumerate(grads, 1):
        p.grad = torch.tensor(g)
        opt.param_groups[0]["eps"] = T.keras_adam_eps(t)
        opt.step()
    np.testing.assert_allclose(p.detach().numpy(), th, rtol=0, atol=1e-15)
