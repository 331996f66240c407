"""ctypes binding of the in-tree C-ABI library ``libnic.so`` (include/nic.h).

The product path has no CPU fallback: if the library is missing or a call fails, this
module raises.  ``torch`` is imported before the library is loaded so that the process
holds a single HIP runtime (torch's bundled ``libamdhip64.so.7`` satisfies the library's
``DT_NEEDED`` by SONAME), which makes torch streams and device pointers valid here.
"""
from __future__ import annotations

import ctypes
import os
import re
import threading
from typing import List, Optional

HERE = os.path.dirname(os.path.abspath(__file__))
# NIC_LIB: load another build of the same C-ABI (A/B comparisons of kernel variants)
LIB_PATH = os.environ.get("NIC_LIB") or os.path.join(HERE, "libnic.so")
HEADER_PATH = os.path.join(os.path.dirname(HERE), "include", "nic.h")

LAYER_NAMES = ("conv1", "conv2", "conv3", "conv4", "conv8", "dconv1", "dconv5", "dconv6", "dconv7", "dconv8")

PRECISION_FP32 = 0
PRECISION_F16X3 = 1
PRECISIONS = {"fp32": PRECISION_FP32, "f16x3": PRECISION_F16X3}

NIC_OK = 0
NIC_EINVAL = -1
NIC_ESHAPE = -2
NIC_ENOWEIGHTS = -3
NIC_EHIP = -4
NIC_ENOMEM = -5
NIC_ERANGE = -6

RANGE_POLICIES = {"fallback": 0, "error": 1}  # nic.h NIC_RANGE_FALLBACK / NIC_RANGE_ERROR

_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_f32p = ctypes.POINTER(ctypes.c_float)
c_vp = ctypes.c_void_p

_SIGNATURES = {
    "nic_version": (ctypes.c_int, []),
    "nic_constants": (ctypes.c_int, [c_vp, c_vp, c_vp]),
    "nic_last_error": (ctypes.c_char_p, []),
    "nic_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(c_vp)]),
    "nic_destroy": (ctypes.c_int, [c_vp]),
    "nic_set_weights": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_char_p, c_vp, ctypes.POINTER(ctypes.c_int64),
                                       ctypes.c_int]),
    "nic_weights_ready": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "nic_reserve": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "nic_latent_shape": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                        ctypes.POINTER(ctypes.c_int)]),
    "nic_encode": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_vp]),
    "nic_decode": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_vp]),
    "nic_encode_host": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_vp, ctypes.c_int, c_vp]),
    "nic_decode_host": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_vp, ctypes.c_int, c_vp]),
    "nic_entropy_hist": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_vp]),
    "nic_encode_entropy": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_vp,
                                          c_vp]),
    "nic_encode_entropy_fold": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.POINTER(ctypes.c_int)]),
    "nic_set_precision": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "nic_get_precision": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_int)]),
    "nic_set_range_policy": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "nic_range_trips": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_int64)]),
    "nic_png_sizes": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_vp, ctypes.c_int]),
    "nic_png_bound": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_vp]),
    "nic_png_encode": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_vp,
                                      ctypes.c_int64, c_vp, ctypes.c_int]),
    "nic_rerun_launch_info": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                             ctypes.POINTER(ctypes.c_int)]),
    "nic_set_timing": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "nic_layer_times": (ctypes.c_int, [c_vp, c_vp, c_vp]),
    "nic_ms_ssim": (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_vp]),
    "nic_sq_err": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, ctypes.c_int64, c_vp, c_vp]),
    "nic_pack_latent": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_vp, c_vp]),
    "nic_unpack_latent": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_vp, c_vp]),
    # training side path (nic_train.hip)
    "nic_conv_gather_work": (ctypes.c_int, [ctypes.c_int] * 4 + [ctypes.POINTER(ctypes.c_int64)]),
    "nic_conv_gather": (ctypes.c_int, [c_vp] + [ctypes.c_int] * 4 + [c_vp] + [ctypes.c_int] * 7 + [c_vp] * 4
                        + [ctypes.c_int] * 3 + [c_vp, ctypes.c_int64, c_vp]),
    "nic_conv_gather_act": (ctypes.c_int, [c_vp] + [ctypes.c_int] * 4 + [c_vp] + [ctypes.c_int] * 7 + [c_vp] * 4
                            + [ctypes.c_int] * 4 + [c_vp, ctypes.c_int64, c_vp]),
    "nic_act_bias_grad_work": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]),
    "nic_act_bias_grad": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_vp,
                                         c_vp, ctypes.c_int64, c_vp]),
    "nic_conv_wgrad_work": (ctypes.c_int, [ctypes.c_int] * 7 + [ctypes.POINTER(ctypes.c_int64)]),
    "nic_conv_wgrad": (ctypes.c_int, [c_vp] + [ctypes.c_int] * 4 + [c_vp] + [ctypes.c_int] * 8 + [c_vp] * 4
                       + [ctypes.c_int64, c_vp]),
    "nic_absmax_scale": (ctypes.c_int, [c_vp, ctypes.c_int64, c_vp, c_vp, c_vp]),
    "nic_gauss_1d": (ctypes.c_int, [c_vp] + [ctypes.c_int] * 3 + [c_vp] + [ctypes.c_int] * 3 + [c_vp]
                     + [ctypes.c_int] * 2 + [c_vp]),
    "nic_ssim_map_work": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
    "nic_ssim_map": (ctypes.c_int, [c_vp] * 4 + [ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_float]
                     + [c_vp, c_vp, ctypes.c_int64, c_vp]),
    "nic_ssim_map_grad": (ctypes.c_int, [c_vp] * 5 + [ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_float]
                          + [c_vp] * 5),
    "nic_adam_keras": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int64] + [ctypes.c_float] * 4 + [c_vp]),
}


class NicError(RuntimeError):
    """A C-ABI call returned a negative status."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def header_symbols(path: str = HEADER_PATH) -> List[str]:
    """Function names declared in include/nic.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nic_[a-z0-9_]+)\s*\(", text)))


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is not built: run `make -C {os.path.join(HERE, 'csrc')}` "
                "or __graft_entry__.build(); there is no CPU fallback")
        import torch  # noqa: F401  (one HIP runtime per process, see module doc)

        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    return (lib().nic_last_error() or b"").decode(errors="replace")


def check(code: int, what: str = "") -> None:
    if code != NIC_OK:
        msg = last_error()
        if code in (NIC_EINVAL, NIC_ESHAPE):
            raise ValueError(f"{what}: [{code}] {msg}")
        raise NicError(code, f"{what}: {msg}" if what else msg)


def latent_shape(h: int, w: int):
    a, b = ctypes.c_int(), ctypes.c_int()
    check(lib().nic_latent_shape(h, w, ctypes.byref(a), ctypes.byref(b)), "nic_latent_shape")
    return a.value, b.value


def constants():
    import numpy as np

    k = np.zeros(9, np.float32)
    ki = np.zeros(9, np.float32)
    off = np.zeros(3, np.float32)
    check(lib().nic_constants(k.ctypes.data, ki.ctypes.data, off.ctypes.data), "nic_constants")
    return k.reshape(3, 3), ki.reshape(3, 3), off
