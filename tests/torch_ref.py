"""Independent PyTorch-CPU restatement of the TF2 codec, used only to cross-check the
NumPy oracle (two restatements written differently must agree).

Differences in construction from oracle/nic_oracle.py: convolutions via F.conv2d with an
explicit asymmetric F.pad, transposed convolutions via F.conv_transpose2d + crop.
"""
import numpy as np
import torch
import torch.nn.functional as F


def same_pad(n, k, s):
    out = -(-n // s)
    pad = max((out - 1) * s + k - n, 0)
    return pad // 2, pad - pad // 2


def conv(x, kernel_hwio, bias, stride):
    # x: (N,C,H,W) float64 torch
    k = torch.from_numpy(kernel_hwio).double().permute(3, 2, 0, 1)  # (Cout,Cin,kh,kw)
    t, b = same_pad(x.shape[2], kernel_hwio.shape[0], stride)
    l, r = same_pad(x.shape[3], kernel_hwio.shape[1], stride)
    y = F.conv2d(F.pad(x, (l, r, t, b)), k, stride=stride)
    y = y.float()  # round the conv sum to fp32, then BiasAdd in fp32
    y = y + torch.from_numpy(bias).view(1, -1, 1, 1)
    return torch.maximum(y * np.float32(0.2), y)


def tconv(x, kernel_hwoi, bias, stride):
    k = torch.from_numpy(kernel_hwoi).double().permute(3, 2, 0, 1)  # (Cin,Cout,kh,kw)
    n = x.shape[2] * stride, x.shape[3] * stride
    pt, _ = same_pad(n[0], kernel_hwoi.shape[0], stride)
    pl, _ = same_pad(n[1], kernel_hwoi.shape[1], stride)
    full = F.conv_transpose2d(x, k, stride=stride)
    full = F.pad(full, (0, max(0, pl + n[1] - full.shape[3]), 0, max(0, pt + n[0] - full.shape[2])))
    y = full[:, :, pt:pt + n[0], pl:pl + n[1]].float()
    y = y + torch.from_numpy(bias).view(1, -1, 1, 1)
    return torch.maximum(y * np.float32(0.2), y)


def encoder(p, x):
    x = conv(x, p["conv1/kernel"], p["conv1/bias"], 2).double()
    x = conv(x, p["conv2/kernel"], p["conv2/bias"], 2)
    res = x
    x = conv(x.double(), p["conv3/kernel"], p["conv3/bias"], 1)
    x = conv(x.double(), p["conv4/kernel"], p["conv4/bias"], 1)
    x = x + res
    x = conv(x.double(), p["conv8/kernel"], p["conv8/bias"], 2)
    return x.clamp(0, 1)


def decoder(p, x):
    x = tconv(x, p["dconv1/kernel"], p["dconv1/bias"], 2)
    res = x
    x = tconv(x.double(), p["dconv5/kernel"], p["dconv5/bias"], 1)
    x = tconv(x.double(), p["dconv6/kernel"], p["dconv6/bias"], 1)
    x = x + res
    x = tconv(x.double(), p["dconv7/kernel"], p["dconv7/bias"], 2)
    x = tconv(x.double(), p["dconv8/kernel"], p["dconv8/bias"], 2)
    return x.clamp(0, 1)


def params(weights, model):
    pre = model + "/"
    return {k[len(pre):]: v for k, v in weights.items() if k.startswith(pre)}


def encode_f32(weights, x_u8):
    """(N,H,W,3) u8 -> (N,h,w,96) fp32, colour transform done in fp32 torch ops."""
    k = np.array([[0.299, 0.587, 0.114], [-0.16874, -0.33126, 0.5], [0.5, -0.41869, -0.08131]], np.float32)
    xf = torch.from_numpy(x_u8).float() / 255.0
    r, g, b = xf[..., 0], xf[..., 1], xf[..., 2]
    planes = []
    for i, off in enumerate((0.0, 0.5, 0.5)):
        v = ((r * float(k[i, 0]) + g * float(k[i, 1])) + b * float(k[i, 2])) + off
        planes.append(v[:, None].double())
    outs = [encoder(params(weights, "encoderY"), planes[0]),
            encoder(params(weights, "encoderCbCr"), planes[1]),
            encoder(params(weights, "encoderCbCr"), planes[2])]
    return torch.cat(outs, dim=1).permute(0, 2, 3, 1).numpy()


def decode_planes(weights, z_u8):
    zn = torch.from_numpy(z_u8).float() / 255.0
    zn = zn.permute(0, 3, 1, 2).double()
    return [decoder(params(weights, "decoderY"), zn[:, 0:32]),
            decoder(params(weights, "decoderCbCr"), zn[:, 32:64]),
            decoder(params(weights, "decoderCbCr"), zn[:, 64:96])]
