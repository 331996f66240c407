"""HIP training convolutions (csrc/nic_train.hip via train_hip) against float64 references.

Every convolution shape of the Training step (tf2_0/src/training.py:74-151): the encoder's
Conv2Ds (encoder.py:10-17), the decoder's Conv2DTransposes (decoder.py:10-17) and the
Entropynet's Conv2Ds (training.py:25-42) -- forward, input gradient, kernel gradient and
bias gradient -- are compared with the torch restatement of training.py evaluated in float64
on the CPU.  Split-f16x3 arithmetic is fp32-class: max |error| <= 2e-5 x max |reference|
per tensor (the fp32 rounding of the float64 result alone is ~6e-8)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from neural_network_image_compression_amd import training as T  # noqa: E402

pytestmark = pytest.mark.gpu

TOL = 2e-5

# (kind, cin, cout, k, stride, (h, w)) -- Keras layer shapes of the step
SHAPES = [
    ("conv", 1, 32, 5, 2, (34, 41)),   # conv1 (odd size: SAME pads differ per side)
    ("conv", 32, 64, 5, 2, (17, 21)),  # conv2
    ("conv", 64, 64, 3, 1, (12, 9)),   # conv3 / conv4 / Entropynet conv2, conv3
    ("conv", 64, 32, 5, 2, (9, 12)),   # conv8
    ("conv", 32, 64, 5, 2, (8, 8)),    # Entropynet conv1 on a latent
    ("tconv", 32, 64, 5, 2, (5, 7)),   # dconv1
    ("tconv", 64, 64, 3, 1, (10, 9)),  # dconv5 / dconv6
    ("tconv", 64, 64, 5, 2, (9, 8)),   # dconv7
    ("tconv", 64, 1, 5, 2, (11, 10)),  # dconv8
]


def _rel_err(a, ref):
    a = a.detach().double().cpu()
    ref = ref.detach().double().cpu()
    return float((a - ref).abs().max() / ref.abs().max().clamp_min(1e-300))


def _run(kind, cin, cout, k, stride, hw, n=3, gscale=1.0, seed=0, act=False):
    from neural_network_image_compression_amd import train_hip

    g = torch.Generator().manual_seed(seed)
    h, w = hw
    x = torch.randn((n, h, w, cin), generator=g)
    kshape = (k, k, cin, cout) if kind == "conv" else (k, k, cout, cin)
    kern = torch.randn(kshape, generator=g) * (1.0 / np.sqrt(k * k * cin))
    bias = torch.randn((cout,), generator=g) * 0.1
    # HIP, NHWC, activation fused in the epilogue when act
    xd, kd, bd = (t.cuda().requires_grad_() for t in (x, kern, bias))
    fn = train_hip._fns()[0 if kind == "conv" else 1]
    y = fn.apply(xd, kd, bd, stride, act)
    gy = torch.randn(y.shape, generator=g) * gscale
    y.backward(gy.cuda())
    # float64 reference, NCHW torch restatement of training.py
    xr, kr, br = (t.double().requires_grad_() for t in (x, kern, bias))
    xn = xr.permute(0, 3, 1, 2)
    if kind == "conv":
        yr = T.conv_same(xn, kr, br, stride, act=False)
    else:
        import torch.nn.functional as F

        # tconv_same applies leaky; undo by comparing the pre-activation: rebuild it here
        n_out = (xn.shape[2] * stride, xn.shape[3] * stride)
        pt, _ = T.same_pad(n_out[0], k, stride)
        pl, _ = T.same_pad(n_out[1], k, stride)
        full = F.conv_transpose2d(xn, kr.permute(3, 2, 0, 1), stride=stride)
        full = F.pad(full, (0, max(0, pl + n_out[1] - full.shape[3]), 0, max(0, pt + n_out[0] - full.shape[2])))
        yr = full[:, :, pt:pt + n_out[0], pl:pl + n_out[1]] + br.view(1, -1, 1, 1)
    if act:
        import torch.nn.functional as F

        yr = F.leaky_relu(yr, 0.2)
    yr = yr.permute(0, 2, 3, 1)
    yr.backward(gy.double())
    return (y, xd.grad, kd.grad, bd.grad), (yr, xr.grad, kr.grad, br.grad)


@pytest.mark.parametrize("kind,cin,cout,k,stride,hw", SHAPES)
def test_conv_forward_and_gradients_match_float64(kind, cin, cout, k, stride, hw):
    hip, ref = _run(kind, cin, cout, k, stride, hw)
    for name, a, r in zip(("y", "dx", "dkernel", "dbias"), hip, ref):
        assert a.shape == r.shape, name
        assert _rel_err(a, r) <= TOL, (name, _rel_err(a, r))


@pytest.mark.parametrize("kind,cin,cout,k,stride,hw", [SHAPES[0], SHAPES[2], SHAPES[5], SHAPES[8]])
def test_fused_activation_and_bias_gradient_match_float64(kind, cin, cout, k, stride, hw):
    # leaky_relu(0.2) in the gather epilogue (nic_conv_gather_act) and its gradient with the
    # bias gradient in one pass (nic_act_bias_grad)
    hip, ref = _run(kind, cin, cout, k, stride, hw, act=True, seed=2)
    for name, a, r in zip(("y", "dx", "dkernel", "dbias"), hip, ref):
        assert a.shape == r.shape, name
        assert _rel_err(a, r) <= TOL, (name, _rel_err(a, r))


def test_fused_activation_is_torch_leaky_bit_for_bit():
    # forward: the fused epilogue equals F.leaky_relu of the unfused output bit for bit; backward:
    # dx and dkernel equal those through torch's leaky_relu backward bit for bit (same dz), the
    # bias gradient is the same sum in a fixed (different) order
    import torch.nn.functional as F

    from neural_network_image_compression_amd import train_hip

    g = torch.Generator().manual_seed(9)
    x = torch.randn((2, 13, 11, 32), generator=g).cuda()
    kern = (torch.randn((5, 5, 32, 64), generator=g) * 0.05).cuda()
    bias = (torch.randn((64,), generator=g) * 0.1).cuda()
    gy = torch.randn((2, 7, 6, 64), generator=g).cuda()
    fn = train_hip._fns()[0]
    grads = []
    for fused in (True, False):
        xd, kd, bd = (t.clone().requires_grad_() for t in (x, kern, bias))
        y = fn.apply(xd, kd, bd, 2, True) if fused else F.leaky_relu(fn.apply(xd, kd, bd, 2, False), 0.2)
        y.backward(gy)
        grads.append((y.detach(), xd.grad, kd.grad, bd.grad))
    (y1, dx1, dk1, db1), (y0, dx0, dk0, db0) = grads
    assert torch.equal(y1, y0) and torch.equal(dx1, dx0) and torch.equal(dk1, dk0)
    assert torch.allclose(db1, db0, rtol=1e-5, atol=1e-5)
    # deterministic
    xd, kd, bd = (t.clone().requires_grad_() for t in (x, kern, bias))
    fn.apply(xd, kd, bd, 2, True).backward(gy)
    assert torch.equal(bd.grad, db1)


def test_act_bias_grad_edges():
    # nic_act_bias_grad: the vector (16-B) and scalar paths (a buffer offset by one float takes
    # the scalar one) give the same dz and scale bit for bit and the same bias sums (in another
    # order); one column; an empty tensor (db = 0, scale = 1)
    from neural_network_image_compression_amd import train_hip

    g = torch.Generator().manual_seed(13)
    for cols in (64, 32, 1):
        y = torch.randn((3, 17, 9, cols), generator=g).cuda()
        dy = torch.randn((3, 17, 9, cols), generator=g).cuda()
        dz, db, sdz = train_hip.act_bias_grad(y, dy, 1)
        ref = dy * torch.where(y > 0, torch.ones_like(y), torch.full_like(y, 0.2))
        assert torch.equal(dz, ref)
        assert torch.allclose(db, ref.sum(dim=(0, 1, 2)), rtol=1e-5, atol=1e-5)
        assert torch.equal(sdz, train_hip.scale(ref))
        by, bdy = torch.empty(y.numel() + 1, device="cuda"), torch.empty(dy.numel() + 1, device="cuda")
        by[1:].copy_(y.flatten())
        bdy[1:].copy_(dy.flatten())
        dz2, db2, sdz2 = train_hip.act_bias_grad(by[1:].view(y.shape), bdy[1:].view(dy.shape), 1)
        assert torch.equal(dz2, dz) and torch.equal(sdz2, sdz)
        assert torch.allclose(db2, db, rtol=1e-5, atol=1e-5)
    e = torch.empty((0, 4, 4, 64), device="cuda")
    dz, db, sdz = train_hip.act_bias_grad(e, e, 1)
    assert dz.numel() == 0 and torch.equal(db, torch.zeros(64, device="cuda")) and float(sdz) == 1.0


@pytest.mark.parametrize("gscale", [1e-9, 1e6])
def test_operand_scales_keep_tiny_and_large_gradients(gscale):
    # power-of-two operand scales: a 1e-9 gradient (below f16's smallest subnormal) and a
    # 1e6 one (past f16's max) keep fp32-class accuracy
    hip, ref = _run("conv", 64, 64, 3, 1, (9, 10), gscale=gscale, seed=3)
    for name, a, r in zip(("dx", "dkernel", "dbias"), hip[1:], ref[1:]):
        assert _rel_err(a, r) <= TOL, (name, gscale, _rel_err(a, r))


def test_batch_of_128x128_patches_encoder_decoder_shapes():
    # the training batch geometry (64 x 128^2 patches would be slow in float64 on the CPU;
    # 2 patches cover every grid size of the step)
    for kind, cin, cout, k, s, hw in [("conv", 1, 32, 5, 2, (128, 128)), ("tconv", 64, 64, 5, 2, (32, 32))]:
        hip, ref = _run(kind, cin, cout, k, s, hw, n=2)
        for name, a, r in zip(("y", "dx", "dkernel", "dbias"), hip, ref):
            assert _rel_err(a, r) <= TOL, (kind, name, _rel_err(a, r))


def test_wgrad_is_deterministic():
    from neural_network_image_compression_amd import train_hip

    g = torch.Generator().manual_seed(5)
    x = torch.randn((4, 32, 32, 64), generator=g).cuda()
    dy = torch.randn((4, 32, 32, 64), generator=g).cuda()
    a = train_hip.wgrad(x, dy, 3, 3, 1, (1, 1))
    b = train_hip.wgrad(x, dy, 3, 3, 1, (1, 1))
    assert torch.equal(a, b)


def test_hip_training_step_matches_torch_backend(tmp_path):
    # one step's losses and parameter gradients: HIP convolutions (NHWC) vs PyTorch autograd
    # (MIOpen, NCHW), same weights, data, flips and noise
    from neural_network_image_compression_amd import weights as W

    w0 = W.seeded_weights(0, init="glorot")
    g = torch.Generator().manual_seed(7)
    imgs = torch.randint(0, 256, (4, 64, 64, 3), generator=g, dtype=torch.uint8)
    out = {}
    for be in ("hip", "torch"):
        tr = T.Training(device="cuda", weights=w0, seed=0, checkpoint_dir=str(tmp_path) + "/", backend=be)
        f = tr.losses(imgs, 0.01, flip=True)
        gy = torch.autograd.grad(f["loss0"], tr._variables("Y"), retain_graph=True)
        gc = torch.autograd.grad(f["loss1"], tr._variables("CbCr"), retain_graph=True)
        ge = torch.autograd.grad(f["entropy_loss"], tr.entropy_model.parameters())
        out[be] = (f, gy, gc, ge)
    fh, ft = out["hip"][0], out["torch"][0]
    for key in ("loss0", "loss1", "ssim0"):
        a, b = float(fh[key].detach()), float(ft[key].detach())
        assert abs(a - b) <= 1e-4 * max(1.0, abs(b)), key
    assert torch.allclose(fh["aprox"], ft["aprox"], rtol=1e-3, atol=1e-4)
    for part in (1, 2):  # codec gradients (the entropy net's target may differ by a code flip)
        for a, b in zip(out["hip"][part], out["torch"][part]):
            assert _rel_err(a, b) <= 2e-3, _rel_err(a, b)


def test_ssim_gaussian_on_hip_matches_float64():
    # the SSIM loss's separable Gaussian (VALID, one channel) and its input gradient
    g = torch.Generator().manual_seed(11)
    x = torch.rand((3, 1, 40, 37), generator=g)
    y = (x + 0.05 * torch.randn(x.shape, generator=g)).clamp(0, 1)
    xd, yd = x.cuda().requires_grad_(), y.cuda()
    s_hip = T.ssim(xd, yd, hip=True)
    s_hip.sum().backward()
    xr = x.double().requires_grad_()
    s_ref = T.ssim(xr, y.double())
    s_ref.sum().backward()
    assert _rel_err(s_hip, s_ref) <= TOL
    assert _rel_err(xd.grad, xr.grad) <= 1e-4


def test_ssim_map_fused_matches_float64_both_inputs():
    # the map's arithmetic and per-plane mean in one HIP pass (nic_ssim_map) and its backward
    # (nic_ssim_map_grad), weighted per plane, gradients to both images, a training-size plane
    g = torch.Generator().manual_seed(12)
    x = torch.rand((4, 1, 128, 128), generator=g)
    y = (x + 0.1 * torch.randn(x.shape, generator=g)).clamp(0, 1)
    wts = torch.tensor([1.0, -0.5, 2.0, 0.25])
    xd, yd = x.cuda().requires_grad_(), y.cuda().requires_grad_()
    s_hip = T.ssim(xd, yd, hip=True)
    (s_hip * wts.cuda()).sum().backward()
    xr, yr = x.double().requires_grad_(), y.double().requires_grad_()
    s_ref = T.ssim(xr, yr)
    (s_ref * wts.double()).sum().backward()
    assert _rel_err(s_hip, s_ref) <= TOL
    assert _rel_err(xd.grad, xr.grad) <= 1e-4 and _rel_err(yd.grad, yr.grad) <= 1e-4
    # deterministic
    xd2 = x.cuda().requires_grad_()
    s2 = T.ssim(xd2, yd.detach(), hip=True)
    assert torch.equal(s2, s_hip.detach())


def test_strided_operands_and_scale():
    """A strided view (not contiguous) gives the same scale and the same convolution as its
    contiguous copy: the C-ABI reads data_ptr() / numel() of a contiguous tensor only."""
    from neural_network_image_compression_amd import train_hip

    g = torch.Generator().manual_seed(5)
    base = torch.randn((3, 9, 12, 64), generator=g).cuda()
    base[:, :, :, 0] *= 1e3  # the max sits where a flat read of the view would miss it
    view = base.permute(0, 2, 1, 3)  # (3, 12, 9, 64), strided
    assert not view.is_contiguous()
    assert torch.equal(train_hip.scale(view), train_hip.scale(view.contiguous()))
    kern = (torch.randn((3, 3, 64, 64), generator=g) * 0.05).cuda()
    y_view = train_hip.conv_same(view, kern, None, 1, act=False)
    y_copy = train_hip.conv_same(view.contiguous(), kern, None, 1, act=False)
    assert torch.equal(y_view, y_copy)
    with pytest.raises(TypeError):  # a host operand never reaches the C-ABI
        train_hip.gather(view.contiguous(), kern.cpu(), 0, 1, (1, 1), 0, (12, 9), 64)


def _np_keras_adam(var, m, v, g, step, lr=1e-4, b1=0.9, b2=0.999, eps=1e-7):
    """TF's ApplyAdam (tf.keras Adam, training.py:149) restated in NumPy fp32, op by op:
    m += (g - m)(1 - b1); v += (g g - v)(1 - b2); var -= (m alpha) / (sqrt(v) + eps)."""
    from neural_network_image_compression_amd.train_hip import keras_adam_alpha

    f = np.float32
    alpha = f(keras_adam_alpha(step, lr, b1, b2))
    b1c, b2c = f(1) - f(b1), f(1) - f(b2)
    m = m + (g - m) * b1c
    v = v + (g * g - v) * b2c
    var = var - (m * alpha) / (np.sqrt(v) + f(eps))
    return var, m, v


def test_keras_adam_on_hip_matches_tf_formula_bit_exact():
    # the optimiser step of the HIP training backend (nic_adam_keras, one launch over every
    # tensor) against the fp32 NumPy restatement of TF's ApplyAdam: bit-identical over 3 steps,
    # tensor sizes around the 1,024-element block boundary; and within fp32 rounding of
    # torch.optim.Adam with Keras' epsilon-hat (training.keras_adam_eps)
    from neural_network_image_compression_amd.train_hip import KerasAdam

    rng = np.random.default_rng(5)
    sizes = [(5, 5, 32, 64), (64,), (1023,), (1025,), (1,), (3, 3, 64, 64)]
    host = [rng.standard_normal(s).astype(np.float32) for s in sizes]
    params = [torch.from_numpy(h.copy()).cuda() for h in host]
    ref = [torch.from_numpy(h.copy()).cuda().requires_grad_() for h in host]
    opt = KerasAdam(params)
    topt = torch.optim.Adam(ref, lr=1e-4, betas=(0.9, 0.999), eps=1e-7)
    var = [h.copy() for h in host]
    m = [np.zeros_like(h) for h in host]
    v = [np.zeros_like(h) for h in host]
    for step in range(1, 4):
        grads = [rng.standard_normal(s).astype(np.float32) * np.float32(10.0 ** -step) for s in sizes]
        opt.step([torch.from_numpy(g).cuda() for g in grads])
        for i, g in enumerate(grads):
            var[i], m[i], v[i] = _np_keras_adam(var[i], m[i], v[i], g, step)
            ref[i].grad = torch.from_numpy(g).cuda()
        for group in topt.param_groups:
            group["eps"] = T.keras_adam_eps(step)
        topt.step()
        torch.cuda.synchronize()
        for i in range(len(sizes)):
            np.testing.assert_array_equal(params[i].cpu().numpy(), var[i], err_msg=f"var {i} step {step}")
            np.testing.assert_array_equal(opt.m[i].cpu().numpy(), m[i])
            np.testing.assert_array_equal(opt.v[i].cpu().numpy(), v[i])
            d = (params[i] - ref[i].detach()).abs().max().item()
            assert d <= 1e-6 * max(1.0, ref[i].detach().abs().max().item()), (i, step, d)


def test_keras_adam_rebound_param_and_long_record():
    # (1) a parameter rebound after construction (p.data = new storage) is followed
    # -- the update lands in the new tensor, the old one is untouched; (2) a table record longer
    # than the max_n that sized the grid is still updated whole (the kernel strides over n)
    import ctypes

    from neural_network_image_compression_amd import _lib
    from neural_network_image_compression_amd.train_hip import KerasAdam

    rng = np.random.default_rng(9)
    h = rng.standard_normal(3000).astype(np.float32)
    p = torch.from_numpy(h.copy()).cuda()
    opt = KerasAdam([p])
    old = p.data
    p.data = torch.from_numpy(h.copy() + 1).cuda()  # rebound: new storage, same shape
    g = rng.standard_normal(3000).astype(np.float32)
    opt.step([torch.from_numpy(g).cuda()])
    torch.cuda.synchronize()
    var, _, _ = _np_keras_adam(h + np.float32(1), np.zeros_like(h), np.zeros_like(h), g, 1)
    np.testing.assert_array_equal(p.cpu().numpy(), var)
    np.testing.assert_array_equal(old.cpu().numpy(), h)
    # raw C-ABI: one record of n = 5000 launched with max_n = 1000 (grid of one block column)
    n = 5000
    v0 = rng.standard_normal(n).astype(np.float32)
    gv = rng.standard_normal(n).astype(np.float32)
    var_t, m_t, v_t = torch.from_numpy(v0.copy()).cuda(), torch.zeros(n).cuda(), torch.zeros(n).cuda()
    g_t = torch.from_numpy(gv).cuda()
    tab = torch.tensor([[var_t.data_ptr(), m_t.data_ptr(), v_t.data_ptr(), g_t.data_ptr(), n]],
                       dtype=torch.int64).cuda()
    from neural_network_image_compression_amd.train_hip import keras_adam_alpha
    alpha = keras_adam_alpha(1, 1e-4, 0.9, 0.999)
    L = _lib.lib()
    _lib.check(L.nic_adam_keras(tab.data_ptr(), 1, 1000, ctypes.c_float(alpha), ctypes.c_float(0.9),
                                ctypes.c_float(0.999), ctypes.c_float(1e-7), None), "nic_adam_keras")
    torch.cuda.synchronize()
    ref, _, _ = _np_keras_adam(v0, np.zeros(n, np.float32), np.zeros(n, np.float32), gv, 1)
    np.testing.assert_array_equal(var_t.cpu().numpy(), ref)
