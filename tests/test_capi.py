"""CPU-side checks of the C-ABI library: it is built, loads, exports exactly what
include/nic.h declares, and its host-only entry points behave (no GPU calls here)."""
import ctypes
import os

import numpy as np
import pytest

from neural_network_image_compression_amd import _lib
from oracle import nic_oracle as O


def test_library_built_and_loads():
    assert os.path.exists(_lib.LIB_PATH), "run __graft_entry__.build()"
    L = _lib.lib()
    assert L.nic_version() >= 100


def test_exports_every_header_symbol():
    L = _lib.lib()
    syms = _lib.header_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(L, s), f"libnic.so does not export {s}"
    assert set(syms) == set(_lib._SIGNATURES), "ctypes signatures out of sync with nic.h"


def test_ctypes_signatures_match_header_arity():
    # every declaration's parameter count equals its ctypes argtypes (a short list shifts
    # the trailing pointers -- e.g. the stream -- into the wrong registers)
    import re

    text = re.sub(r"/\*.*?\*/", "", open(_lib.HEADER_PATH).read(), flags=re.S)
    for name, params in re.findall(r"\b(nic_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", text):
        params = params.strip()
        n = 0 if params in ("", "void") else params.count(",") + 1
        assert len(_lib._SIGNATURES[name][1]) == n, (name, n, len(_lib._SIGNATURES[name][1]))


def test_exports_are_c_linkage():
    out = os.popen(f"nm -D --defined-only {_lib.LIB_PATH}").read()
    for s in _lib.header_symbols():
        assert f" T {s}\n" in out


@pytest.mark.parametrize("h,w", [(256, 256), (2160, 3840), (37, 53), (1, 1), (8, 9), (512, 768)])
def test_latent_shape_matches_tf_same(h, w):
    hh, ww = h, w
    for _ in range(3):
        hh, ww = O.same_pads(hh, 5, 2)[0], O.same_pads(ww, 5, 2)[0]
    assert _lib.latent_shape(h, w) == (hh, ww)


def test_latent_shape_rejects_bad_sizes():
    with pytest.raises(ValueError):
        _lib.latent_shape(0, 5)


def test_device_constants_match_oracle():
    k, kinv, off = _lib.constants()
    np.testing.assert_array_equal(k, O.YCBCR_KERNEL)
    np.testing.assert_array_equal(kinv, O.YCBCR_INV_KERNEL)
    np.testing.assert_array_equal(off, O.YCBCR_OFF)


def test_null_arguments_are_rejected_without_crashing():
    L = _lib.lib()
    assert L.nic_create(0, None) == _lib.NIC_EINVAL
    assert L.nic_encode(None, None, 1, 8, 8, None, None, None) == _lib.NIC_EINVAL
    assert "NULL" in _lib.last_error()
    assert L.nic_decode(None, None, 1, 1, 1, None, None, None) == _lib.NIC_EINVAL
    assert L.nic_encode_host(None, None, 1, 8, 8, None, 3, None) == _lib.NIC_EINVAL
    assert L.nic_decode_host(None, None, 1, 1, 1, None, 3, None) == _lib.NIC_EINVAL
    assert L.nic_set_weights(None, 0, b"conv1/kernel", None, None, 0) == _lib.NIC_EINVAL
    assert L.nic_pack_latent(None, 1, 1, 1, None, None) == _lib.NIC_EINVAL
    assert L.nic_pack_latent(None, 1, 0, 1, None, None) == _lib.NIC_ESHAPE
    assert L.nic_pack_latent(None, 0, 1, 1, None, None) == _lib.NIC_OK  # empty batch
    assert L.nic_set_timing(None, 1) == _lib.NIC_EINVAL
    assert L.nic_ms_ssim(None, None, None, 1, 256, 256, None, None, None) == _lib.NIC_EINVAL
    assert L.nic_sq_err(None, None, -1, 10, None, None) == _lib.NIC_ESHAPE
    assert L.nic_sq_err(None, None, 2, 10, None, None) == _lib.NIC_EINVAL
    assert L.nic_sq_err(None, None, 0, 10, None, None) == _lib.NIC_OK  # empty batch
    assert L.nic_destroy(None) == _lib.NIC_OK


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = ctypes.c_void_p()
    rc = _lib.lib().nic_create(0, ctypes.byref(h))
    assert rc < 0 and not h.value
    assert _lib.last_error()


def test_training_entry_points_validate_without_a_gpu():
    # argument checks of the training C-ABI (nic_train.hip) run before any HIP call
    import ctypes

    L = _lib.lib()
    b = ctypes.c_int64()
    assert L.nic_conv_gather_work(5, 5, 32, 64, ctypes.byref(b)) == _lib.NIC_OK
    assert b.value == ((25 * 32 + 31) // 32) * 4 * 2 * 64 * 16  # chunks x co tiles x hi/lo x lanes x 16 B
    assert L.nic_conv_gather_work(5, 5, 65, 64, ctypes.byref(b)) == _lib.NIC_ESHAPE  # cin > 64
    assert L.nic_conv_gather_work(5, 5, 32, 64, None) == _lib.NIC_EINVAL
    f = ctypes.c_int64()
    assert L.nic_conv_wgrad_work(4, 32, 32, 3, 3, 64, 64, ctypes.byref(f)) == _lib.NIC_OK
    assert f.value > 0 and f.value % (9 * 64 * 64) == 0  # whole slices of the (tap, a) x b partials
    # shape / enum / NULL checks of the GEMMs themselves
    assert L.nic_conv_gather(None, 1, 8, 8, 0, None, 3, 3, 0, 1, 1, 1, 0, None, None, None, None, 8, 8, 64,
                             None, 0, None) == _lib.NIC_ESHAPE
    assert L.nic_conv_gather(None, 1, 8, 8, 64, None, 3, 3, 2, 1, 1, 1, 0, None, None, None, None, 8, 8, 64,
                             None, 0, None) == _lib.NIC_EINVAL
    assert L.nic_conv_gather(None, 1, 8, 8, 64, None, 3, 3, 0, 1, 1, 1, 0, None, None, None, None, 8, 8, 64,
                             None, 0, None) == _lib.NIC_EINVAL
    assert "NULL" in _lib.last_error()
    assert L.nic_conv_gather(None, 0, 8, 8, 64, None, 3, 3, 0, 1, 1, 1, 0, None, None, None, None, 8, 8, 64,
                             None, 0, None) == _lib.NIC_OK  # empty batch: nothing to do
    assert L.nic_conv_wgrad(None, 1, 8, 8, 64, None, 8, 8, 64, 3, 3, 1, 1, 1, None, None, None, None, 0,
                            None) == _lib.NIC_EINVAL
    assert L.nic_gauss_1d(None, 1, 20, 20, None, 11, 0, 0, None, 20, 9, None) == _lib.NIC_ESHAPE  # 20 - 10 != 9
    assert L.nic_gauss_1d(None, 1, 20, 20, None, 11, 0, 0, None, 20, 10, None) == _lib.NIC_EINVAL
    assert L.nic_absmax_scale(None, -1, None, None, None) == _lib.NIC_ESHAPE
    # the fused-activation gather and the activation / bias gradient (nic_train.hip)
    assert L.nic_conv_gather_act(None, 1, 8, 8, 64, None, 3, 3, 0, 1, 1, 1, 0, None, None, None, None, 8, 8, 64, 2,
                                 None, 0, None) == _lib.NIC_EINVAL  # act not 0 / 1
    assert L.nic_conv_gather_act(None, 0, 8, 8, 64, None, 3, 3, 0, 1, 1, 1, 0, None, None, None, None, 8, 8, 64, 1,
                                 None, 0, None) == _lib.NIC_OK
    assert L.nic_act_bias_grad_work(5000, 64, ctypes.byref(f)) == _lib.NIC_OK and f.value == 20 * 65  # 256-row blocks: 64 sums and a max each
    assert L.nic_act_bias_grad_work(10, 65, ctypes.byref(f)) == _lib.NIC_ESHAPE
    assert L.nic_act_bias_grad(None, None, 10, 64, 1, None, None, None, None, 0, None) == _lib.NIC_EINVAL  # no output
    assert L.nic_act_bias_grad(None, None, 10, 64, 1, None, ctypes.c_void_p(16), None, None, 0, None) == _lib.NIC_EINVAL
    assert L.nic_act_bias_grad(None, None, -1, 64, 0, None, None, None, None, 0, None) == _lib.NIC_ESHAPE
    assert L.nic_ssim_map_work(3, 5000, ctypes.byref(f)) == _lib.NIC_OK and f.value == 3 * 5  # 1,024-pixel blocks
    assert L.nic_ssim_map(None, None, None, None, 3, 0, 1e-4, 9e-4, None, None, 0, None) == _lib.NIC_ESHAPE
    assert L.nic_ssim_map(None, None, None, None, 3, 100, 1e-4, 9e-4, None, None, 0, None) == _lib.NIC_EINVAL
    assert L.nic_ssim_map_grad(None, None, None, None, None, 0, 100, 1e-4, 9e-4, None, None, None, None,
                               None) == _lib.NIC_OK  # no planes
