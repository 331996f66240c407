"""GPU quality metrics (csrc/nic_quality.hip, through the C-ABI) against the oracle.

Contract:
  * MS-SSIM (tf.image.ssim_multiscale, tf2_0/tests/calc_ssim.py:13): |GPU - oracle| <=
    MSSSIM_ATOL per image, and the per-scale mean SSIM / cs terms within TERM_ATOL.  The
    GPU filters in fp32 (separable Gaussian, shifted by -0.5) and reduces in fp64; the
    oracle is float64 throughout.  Parity vs TensorFlow itself is unpinned (no TF here).
  * squared error: bit-exact (integer), PSNR equal to the oracle's to 1e-9 dB.
"""
import os

import numpy as np
import pytest

from oracle import nic_oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

MSSSIM_ATOL = 2e-6
TERM_ATOL = 2e-6


@pytest.fixture(scope="module")
def codec():
    from neural_network_image_compression_amd.codec import Codec
    return Codec(0)


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _pairs():
    rng = np.random.default_rng(11)
    x = rng.integers(0, 256, (2, 256, 256, 3), dtype=np.uint8)
    noisy = np.clip(x.astype(int) + rng.integers(-20, 21, x.shape), 0, 255).astype(np.uint8)
    smooth = np.cumsum(rng.integers(-3, 4, (1, 177, 203, 3)), axis=2)
    smooth = np.clip(smooth - smooth.min() + 40, 0, 255).astype(np.uint8)
    smooth2 = np.clip(smooth.astype(int) + rng.integers(-6, 7, smooth.shape), 0, 255).astype(np.uint8)
    indep = rng.integers(0, 256, (1, 180, 176, 3), dtype=np.uint8)
    small = rng.integers(0, 256, (2, 161, 161, 3), dtype=np.uint8)  # smallest size TF accepts
    return {
        "smallest_161x161": (small, np.clip(small.astype(int) + rng.integers(-30, 31, small.shape), 0, 255
                                            ).astype(np.uint8)),
        "noise_vs_noisy": (x, noisy),
        "odd_177x203": (smooth, smooth2),
        "independent_noise": (indep, rng.integers(0, 256, indep.shape, dtype=np.uint8)),
        "identical": (x[:1], x[:1]),
    }


@pytest.mark.parametrize("case", ["noise_vs_noisy", "odd_177x203", "independent_noise", "identical",
                                  "smallest_161x161"])
def test_ms_ssim_vs_oracle(case, codec):
    a, b = _pairs()[case]
    got, terms = codec.ms_ssim(_dev(a), _dev(b), per_scale=True)
    got, terms = got.cpu().numpy(), terms.cpu().numpy()
    ref_terms = O.ms_ssim_terms(a, b)
    ref = O.ms_ssim(a, b)
    print(f"{case}: ms_ssim gpu {got} oracle {ref} max|d| {np.abs(got - ref).max():.2e} "
          f"terms max|d| {np.abs(terms - ref_terms).max():.2e}")
    np.testing.assert_allclose(terms, ref_terms, rtol=0, atol=TERM_ATOL)
    np.testing.assert_allclose(got, ref, rtol=0, atol=MSSSIM_ATOL)
    if case == "identical":
        np.testing.assert_allclose(got, 1.0, atol=1e-6)


def test_ms_ssim_codec_recon(codec, golden):
    """The reference's use: original vs decoded image (kodim21 crop, golden recon)."""
    g = golden("kodim21_256")
    got = codec.ms_ssim(_dev(g["x"]), _dev(g["recon"])).cpu().numpy()
    ref = O.ms_ssim(g["x"], g["recon"])
    np.testing.assert_allclose(got, ref, rtol=0, atol=MSSSIM_ATOL)


def test_ms_ssim_errors(codec):
    a = _dev(np.zeros((1, 160, 200, 3), np.uint8))  # scale 4 would be 10 px: below the 11-px window
    with pytest.raises(ValueError):
        codec.ms_ssim(a, a)
    b = _dev(np.zeros((1, 200, 200, 3), np.uint8))
    with pytest.raises(ValueError):
        codec.ms_ssim(b, _dev(np.zeros((1, 200, 201, 3), np.uint8)))
    assert codec.ms_ssim(_dev(np.zeros((0, 200, 200, 3), np.uint8)), _dev(np.zeros((0, 200, 200, 3), np.uint8))).numel() == 0


@pytest.mark.parametrize("shape", [(3, 64, 64, 3), (4, 5, 7, 3), (1, 1, 1, 3), (2, 256, 256, 3), (5, 33, 2)])
def test_sq_err_exact(shape, codec):
    rng = np.random.default_rng(sum(shape))
    a = rng.integers(0, 256, shape, dtype=np.uint8)
    b = rng.integers(0, 256, shape, dtype=np.uint8)
    ref = ((a.astype(np.int64) - b.astype(np.int64)) ** 2).reshape(shape[0], -1).sum(axis=1)
    np.testing.assert_array_equal(codec.sq_err(_dev(a), _dev(b)).cpu().numpy(), ref)
    if len(shape) == 4:
        assert codec.psnr(_dev(a), _dev(b)) == pytest.approx(O.psnr(a, b), abs=1e-9)
    # unaligned views take the byte path
    a1, b1 = _dev(a.reshape(-1))[1:], _dev(b.reshape(-1))[1:]
    n = shape[0]
    m = (a1.numel() // n) * n
    if m:
        a1, b1 = a1[:m].reshape(n, -1), b1[:m].reshape(n, -1)
        ref1 = ((a.reshape(-1)[1:1 + m].astype(np.int64) - b.reshape(-1)[1:1 + m].astype(np.int64)) ** 2)
        np.testing.assert_array_equal(codec.sq_err(a1, b1).cpu().numpy(), ref1.reshape(n, -1).sum(axis=1))


def test_calc_ssim_driver(tmp_path, codec, golden):
    """calc_ssim.py:19-34 on two directories of PNGs paired by file stem."""
    from PIL import Image

    from neural_network_image_compression_amd.quality import calc_ssim
    g = golden("kodim21_256")
    d1, d2 = tmp_path / "orig", tmp_path / "recon"
    os.makedirs(d1)
    os.makedirs(d2)
    Image.fromarray(g["x"][0]).save(d1 / "kodim21.png")
    Image.fromarray(g["recon"][0]).save(d2 / "kodim21.png")
    Image.fromarray(g["x"][0]).save(d1 / "only_here.png")
    res = calc_ssim(str(d1), str(d2), codec=codec, verbose=False)
    assert set(res) == {"kodim21", "average"}
    assert res["average"] == pytest.approx(float(O.ms_ssim(g["x"], g["recon"])[0]), abs=MSSSIM_ATOL)


def _smooth_images(n, h, w, seed):
    rng = np.random.default_rng(seed)
    a = np.cumsum(np.cumsum(rng.integers(-2, 3, (n, h, w, 3)), axis=1), axis=2).astype(np.float64)
    a -= a.min(axis=(1, 2, 3), keepdims=True)
    a *= 255.0 / np.maximum(a.max(axis=(1, 2, 3), keepdims=True), 1)
    return a.astype(np.uint8)


def test_rd_point_whole_and_tiled(codec, weights_spread):
    """Config-4 harness (rd.py): rate (histogram entropy, PNG of the packed latent) and
    distortion (PSNR, MS-SSIM) of Kodak-sized images, whole and as 256^2 tiles; every figure
    is checked against the oracle's definition applied to the GPU's own latents/recons."""
    from neural_network_image_compression_amd import bitstream
    from neural_network_image_compression_amd.rd import rd_point, tile_patches, untile_patches
    codec.set_weights(weights_spread)
    x = _smooth_images(2, 512, 768, 5)
    for tile in (None, 256):
        res = rd_point(codec, x, tile=tile)
        units = tile_patches(x, tile) if tile else x
        z = codec.encode(_dev(units)).cpu().numpy()
        rec = codec.decode(_dev(z)).cpu().numpy()
        if tile:
            rec = untile_patches(rec, 2, 512, 768)
        H = O.hist_entropy(z).reshape(3, -1)
        sym = (H.astype(np.float64).sum(axis=0) * z.shape[1] * z.shape[2] * 32).reshape(2, -1).sum(axis=1)
        np.testing.assert_allclose(res["bpp_entropy"], sym / (512 * 768), rtol=1e-6)
        packed = O.pack_latent(z)
        sizes = np.array([len(bitstream.png_bytes(p)) for p in packed], np.float64).reshape(2, -1).sum(axis=1)
        np.testing.assert_allclose(res["bpp_png"], 8 * sizes / (512 * 768))
        for i in range(2):
            assert res["psnr_db"][i] == pytest.approx(O.psnr(x[i], rec[i]), abs=1e-9)
        np.testing.assert_allclose(res["ms_ssim"], O.ms_ssim(x, rec), atol=MSSSIM_ATOL)
