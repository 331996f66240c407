#!/usr/bin/env python
"""Benchmark of the codec hot path: BASELINE.json's metric, Megapixels/s encode+decode.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 64] [--size 256]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU, RCCL)

A step = nic_encode + nic_decode of one batch of `--batch` synthetic u8 256x256x3 images
already resident in HBM (BASELINE config 2 at N=1; config 3's 8 x 64 sharding at N=8:
weak scaling, each rank owns its own 64 images, no data-path collective).  Weights are
the seeded 'spread' init (random-init weights of the architecture; the trained codecs under
tests/golden/trained are parity fixtures, not the timed workload), generated on rank 0 and
broadcast over RCCL once at setup.

Rank 0 prints ONE JSON line with the driver's keys plus:
  roofline     -- dominant kernel: algorithmic FLOP per launch / its mean launch time,
                  measured with hipEvents on the launch stream over a timed pass;
  layers       -- the same per layer;
  cpu_baseline -- the PyTorch-CPU (oneDNN) restatement of tf2_0 on this process's host
                  cores (TF itself is not installable), bounded sample, rank 0 at N=1 only;
                  the NumPy oracle's rate beside it as `numpy_oracle`;
  parity       -- PSNR of one benchmarked image's reconstruction vs the oracle.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Megapixels/sec encode+decode"
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense f16/bf16 MFMA peak
# f16x3 issues 3 f16 MFMAs per algorithmic fp32 MAC: its peak in algorithmic FLOP/s
F16X3_PEAK_TFLOPS = F16_MFMA_PEAK_TFLOPS / 3
HBM_PEAK_GBS = 8000.0


def layer_geometry(h: int, w: int):
    """Per-plane (FLOP, name) of every layer for an h x w input (2 x MAC)."""
    def same(n):
        return -(-n // 2)
    h1, w1 = same(h), same(w)
    h2, w2 = same(h1), same(w1)
    h8, w8 = same(h2), same(w2)
    g = {
        "conv1": 2 * h1 * w1 * 1 * 32 * 25,
        "conv2": 2 * h2 * w2 * 32 * 64 * 25,
        "conv3": 2 * h2 * w2 * 64 * 64 * 9,
        "conv4": 2 * h2 * w2 * 64 * 64 * 9,
        "conv8": 2 * h8 * w8 * 64 * 32 * 25,
        "dconv1": 2 * h8 * w8 * 32 * 64 * 25,
        "dconv5": 2 * (2 * h8) * (2 * w8) * 64 * 64 * 9,
        "dconv6": 2 * (2 * h8) * (2 * w8) * 64 * 64 * 9,
        "dconv7": 2 * (2 * h8) * (2 * w8) * 64 * 64 * 25,
        "dconv8": 2 * (4 * h8) * (4 * w8) * 64 * 1 * 25,
    }
    return g


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:  # pragma: no cover
        pass
    return "unknown"


def _host_threads() -> int:
    """Host cores this process may use: the box's CPU share (OMP_NUM_THREADS is set to it on
    the GPU box; os.cpu_count() there reports the whole machine)."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except AttributeError:  # pragma: no cover
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return min(n, int(omp)) if omp.isdigit() and int(omp) > 0 else n


def cpu_baseline_numpy(weights, size: int, seconds: float):
    """NumPy oracle (fp32 BLAS accumulation) on synthetic images of the same workload until
    `seconds` of CPU work have run (at least one image)."""
    from oracle import nic_oracle as O

    try:
        from threadpoolctl import threadpool_info
        cores = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:  # pragma: no cover
        cores = os.cpu_count() or 1
    rng = np.random.default_rng(1)
    n, t0 = 0, time.perf_counter()
    while True:
        x = rng.integers(0, 256, (1, size, size, 3), dtype=np.uint8)
        O.decode(weights, O.encode(weights, x, acc=np.float32), acc=np.float32)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(n * size * size / 1e6 / el, 4), "unit": "MP/s", "cores": int(cores),
            "sample": f"{n} synthetic {size}x{size}x3 images, oracle/nic_oracle.py fp32 BLAS, {el:.1f} s"}


def cpu_baseline(weights, size: int, seconds: float, batch: int = 4):
    """SURVEY §8d's CPU baseline: the PyTorch-CPU (oneDNN) restatement of tf2_0's
    Encoder()(x) -> Decoder()(z) (training.base_encoder / base_decoder with TF-SAME padding,
    fp32) on all host cores of this process, batches of 4 images (the reference's directory
    batch, utils.py:53-62), for `seconds` of CPU work.  Not TF2 itself (not installable)."""
    import torch

    from neural_network_image_compression_amd import training as T
    from neural_network_image_compression_amd import weights as Wm

    threads = _host_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    params = {m: {k.split("/", 1)[1]: torch.from_numpy(np.ascontiguousarray(v)) for k, v in weights.items()
                  if k.startswith(m + "/")} for m in Wm.MODEL_ID}
    inv = torch.from_numpy(np.linalg.inv(np.array(T.YCBCR, np.float64)).astype(np.float32))
    off = torch.tensor(T.YCBCR_OFF, dtype=torch.float32)
    rng = np.random.default_rng(1)

    def one_batch():
        x = torch.from_numpy(rng.integers(0, 256, (batch, size, size, 3), dtype=np.uint8))
        y, cb, cr = T.colour_planes(x.float() / 255.0)  # encoder.py:39-41
        zy = T.base_encoder(params["encoderY"], y)
        zc = T.base_encoder(params["encoderCbCr"], torch.cat([cb, cr]))
        z = torch.round(torch.cat([zy, zc[:batch], zc[batch:]], 1) * 255).to(torch.uint8)  # encoder.py:45-47
        zn = z.float() / 255.0  # decoder.py:40-41
        dy = T.base_decoder(params["decoderY"], zn[:, :32])
        dc = T.base_decoder(params["decoderCbCr"], torch.cat([zn[:, 32:64], zn[:, 64:]]))
        planes = torch.cat([dy, dc[:batch], dc[batch:]], 1).permute(0, 2, 3, 1) - off  # decoder.py:45-46
        rgb = (planes @ inv.t()).clamp(0, 1)
        return torch.round(rgb * 255).to(torch.uint8)

    try:
        with torch.inference_mode():
            one_batch()  # oneDNN primitive creation outside the timed sample
            n, t0 = 0, time.perf_counter()
            while True:
                one_batch()
                n += batch
                el = time.perf_counter() - t0
                if el >= seconds:
                    break
    finally:
        torch.set_num_threads(prev)
    return {"value": round(n * size * size / 1e6 / el, 4), "unit": "MP/s", "cores": threads, "kind": "port",
            "cpu": _cpu_model(),
            "sample": f"{n} synthetic {size}x{size}x3 images in batches of {batch}, encode+decode, PyTorch-CPU "
                      f"(oneDNN) restatement of tf2_0 (training.base_encoder/base_decoder, TF-SAME, fp32): "
                      f"CPU restatement of tf2_0, not TF2 (not installable), {el:.1f} s"}


def power_probe(device, weights, x, z, r, dom_layers, flop, steps, peak):
    """The dominant kernel's rate with every weight zero (a second codec on the same GPU, same
    kernels, same launch shapes): the MFMA operands are then all zero and the chip holds a
    higher clock.  Same cycles, different clock -- the gap between `frac` and this figure is
    the data-dependent MFMA power the split-f16 pass draws (DVFS), not scheduling."""
    import torch

    from neural_network_image_compression_amd.codec import Codec

    zw = {k: np.zeros_like(v) for k, v in weights.items()}
    c = Codec(device)
    c.set_weights(zw)
    c.reserve(*x.shape[:3])
    for _ in range(10):
        c.encode(x, out=z)
        c.decode(z, out=r)
    c.set_timing(True)
    for _ in range(steps):
        c.encode(x, out=z)
        c.decode(z, out=r)
    lt = c.layer_times()
    c.set_timing(False)
    torch.cuda.synchronize()
    c.close()  # release the second context now (not from a finaliser at interpreter exit)
    ms = sum(lt[k][0] for k in dom_layers)  # the dominant kernel's launches (layers timed as it)
    n = sum(lt[k][1] for k in dom_layers)
    avg = ms / max(n, 1)
    tf = flop / (avg * 1e-3) / 1e12
    per_layer = {k: round(v[0] / v[1], 4) for k, v in lt.items() if v[1] > 0}
    return {"zero_operand_avg_ms": round(avg, 4), "zero_operand_tflops": round(tf, 2),
            "zero_operand_frac": round(tf / peak, 4), "zero_operand_layer_ms": per_layer,
            "note": "same kernels with all-zero weights (zero MFMA operands): the chip clocks higher "
                    "(DVFS); frac below this is the power limit of random-data split-f16 MFMAs"}


def parity_sample(codec, x0, weights):
    """PSNR of the GPU reconstruction of one benchmarked image vs the oracle's (fp64 acc)."""
    import torch

    from oracle import nic_oracle as O

    xh = x0.cpu().numpy()
    z = codec.encode(x0)
    r = codec.decode(z).cpu().numpy()
    torch.cuda.synchronize()
    r_ref = O.decode(weights, O.encode(weights, xh))
    out = {"psnr_gpu_vs_oracle_db": round(O.psnr(r, r_ref), 2),
           "psnr_x_gpu_db": round(O.psnr(xh, r), 4), "psnr_x_oracle_db": round(O.psnr(xh, r_ref), 4)}
    if min(xh.shape[1:3]) >= 161:
        # MS-SSIM (calc_ssim.py:13) of the GPU reconstruction by the GPU metric, and of the
        # oracle's reconstruction by the oracle's metric
        out["msssim_x_gpu"] = round(float(codec.ms_ssim(x0, torch.from_numpy(r).to(x0.device)).item()), 6)
        out["msssim_x_oracle"] = round(float(O.ms_ssim(xh, r_ref)[0]), 6)
    return out


def host_box_rates(xh, enc, dec, reps):
    """What the host-array surface depends on besides the device: the CPUs this
    process may run on, single-thread pageable -> pinned memcpy of the batch, pinned H2D / D2H
    copies of it, and the encode / decode calls' own medians -- so boxes can be compared."""
    import torch
    nbytes = xh.nbytes
    pin = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    pin_np = pin.numpy()
    src = xh.reshape(-1)
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")

    def best(fn, n=7):
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return min(ts)

    def h2d():
        dev.copy_(pin, non_blocking=True)
        torch.cuda.synchronize()

    def d2h():
        pin.copy_(dev, non_blocking=True)
        torch.cuda.synchronize()

    t_cp = best(lambda: np.copyto(pin_np, src))
    t_h2d, t_d2h = best(h2d), best(d2h)
    te, td = [], []
    z = None
    for _ in range(reps):
        t0 = time.perf_counter()
        z = enc(xh)
        t1 = time.perf_counter()
        dec(z)
        te.append(t1 - t0)
        td.append(time.perf_counter() - t1)
    return {"cpus_allowed": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count(),
            "pageable_to_pinned_gbps": round(nbytes / t_cp / 1e9, 1),
            "h2d_pinned_gbps": round(nbytes / t_h2d / 1e9, 1), "d2h_pinned_gbps": round(nbytes / t_d2h / 1e9, 1),
            "bytes": int(nbytes), "encode_call_ms_median": round(float(np.median(te)) * 1e3, 3),
            "decode_call_ms_median": round(float(np.median(td)) * 1e3, 3)}


def bench_weights(kind: str):
    """The timed workload's weights: the seeded 'spread' init (default), or the committed
    round-4 trained codec (entropy_loss_coef 0.01) for the informational operand comparison."""
    from neural_network_image_compression_amd import weights as Wm
    if kind == "seeded":
        return Wm.seeded_weights(0)
    pre = os.path.join(ROOT, "tests", "golden", "trained", "coef0.01_")
    w = Wm.load(pre + "encoder", "encoder")
    w.update(Wm.load(pre + "decoder", "decoder"))
    return w


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """`python bench.py --gpus N` outside a launcher: start N ranks as the driver does
    (torch.distributed.run, one process per GPU, rendezvous on 127.0.0.1) as a CHILD process
    and return its exit code.  Runs before anything touches the GPU (no exec from a process
    that initialised HIP)."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on this image
    return subprocess.run(cmd, env=env).returncode


def world_from_env(gpus):
    """(world, rank, local_rank) of this process.  `--gpus` and the launcher's WORLD_SIZE must
    agree: a mismatch is an error, never a silent 1-GPU run."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if gpus is not None and gpus != world:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world} ranks were launched "
                         f"(run `python bench.py --gpus {gpus}` without a launcher, or "
                         f"torch.distributed.run --nproc-per-node {gpus})")
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def launch_check(world: int, rank: int) -> None:
    """--launch-check: the ranks and process group of a `--gpus N` run without the codec (the
    CPU test of the launcher; gloo).  Rank 0 prints one JSON line with n_gpus = world."""
    import torch
    import torch.distributed as dist

    if world > 1:
        # gloo by default: the probe tensor is a host tensor (RCCL would need it on
        # cuda:LOCAL_RANK); NIC_BENCH_BACKEND=nccl moves it to the rank's GPU
        backend = os.environ.get("NIC_BENCH_BACKEND", "gloo")
        dist.init_process_group(backend)
        t = torch.tensor([1.0])
        if backend == "nccl":
            t = t.to(f"cuda:{int(os.environ.get('LOCAL_RANK', '0'))}")
        dist.all_reduce(t)
        ranks = int(t.item())
        dist.destroy_process_group()
    else:
        ranks = 1
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "ranks_joined": ranks,
                          "parallelism": f"dp{world}"}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one GPU each); without a launcher, N > 1 starts N ranks under "
                         "torch.distributed.run; under a launcher it must equal WORLD_SIZE")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks and the process group only (no GPU work) and print n_gpus")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10,
                    help="untimed steps first: kernel durations settle over the first ~15 steps (clocks)")
    ap.add_argument("--batch", type=int, default=None, help="images (frames) per GPU per step")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--workload", default="config2", choices=["config2", "kodak", "4k"],
                    help="config2: 64 x 256^2 encode+decode (BASELINE headline); kodak: 768x512 "
                         "whole images encode+decode (config 4 shape); 4k: 3840x2160 frames, "
                         "encode + per-plane histogram entropy (config 5)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--weights", default="seeded", choices=["seeded", "trained"],
                    help="trained: the round-4 codec (entropy_loss_coef 0.01, tests/golden/trained) -- "
                         "informational: the MFMA operands set the power-limited clock")
    ap.add_argument("--images", default="random", choices=["random", "natural"],
                    help="natural (config2 only): random 256x256 crops of kodim21 (tests/golden) -- informational")
    ap.add_argument("--precision", default="f16x3", choices=["f16x3", "fp32"],
                    help="arithmetic of the Cin>=32 convolutions (see include/nic.h)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-power-probe", action="store_true")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the host-array (PCIe-inclusive) surface: its chunked launches would mix "
                         "smaller grids into a profiler's per-kernel averages")
    ap.add_argument("--no-quality", action="store_true", help="skip the MS-SSIM / PSNR timing")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="per-layer HBM bytes per launch from the rocprofv3 PMC pass")
    args = ap.parse_args()
    if args.gpus is not None and args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world, rank, local = world_from_env(args.gpus)
    if args.launch_check:
        launch_check(world, rank)
        return

    import torch
    import torch.distributed as dist

    from neural_network_image_compression_amd import weights as W
    from neural_network_image_compression_amd.codec import Codec

    backend = os.environ.get("NIC_BENCH_BACKEND", "nccl")  # "nccl" is RCCL on ROCm
    ndev = torch.cuda.device_count()  # does not initialise the GPU on this image
    if world > 1 and backend == "nccl" and world > ndev:
        raise SystemExit(f"bench.py: {world} RCCL ranks need {world} GPUs, {ndev} visible "
                         "(NIC_BENCH_BACKEND=gloo shares one GPU between ranks for tests)")
    # one process per GPU; ranks beyond the visible GPUs share them round-robin (the 1-GPU
    # test box runs the world > 1 path this way, with NIC_BENCH_BACKEND=gloo)
    dev_idx = local % max(1, ndev)
    torch.cuda.set_device(dev_idx)
    device = torch.device(f"cuda:{dev_idx}")
    coll_dev = device if backend == "nccl" else torch.device("cpu")  # gloo: host tensors
    if world > 1:
        dist.init_process_group(backend, device_id=device if backend == "nccl" else None)
        from neural_network_image_compression_amd.parallel import broadcast_weights
        weights = broadcast_weights(bench_weights(args.weights) if rank == 0 else None, dist)  # RCCL, once
    else:
        weights = bench_weights(args.weights)

    if args.workload == "config2":
        B, H, W = args.batch or 64, args.size, args.size
    elif args.workload == "kodak":
        B, H, W = args.batch or 24, 512, 768
    else:
        B, H, W = args.batch or 8, 2160, 3840
    S = args.size
    codec = Codec(dev_idx, precision=args.precision)
    codec.set_weights(weights)
    codec.reserve(B, H, W)
    g = torch.Generator().manual_seed(1000 + rank)
    if args.images == "natural" and args.workload == "config2" and H <= 512 and W <= 768:
        # SURVEY 8(d) config 2's natural-image variant: random crops of kodim21
        k = torch.from_numpy(np.load(os.path.join(ROOT, "tests", "golden", "kodim21_full.npz"))["x"][0])
        ys = torch.randint(0, 512 - H + 1, (B,), generator=g).tolist()
        xs = torch.randint(0, 768 - W + 1, (B,), generator=g).tolist()
        x = torch.stack([k[y:y + H, c:c + W] for y, c in zip(ys, xs)]).contiguous().to(device)
    else:
        x = torch.randint(0, 256, (B, H, W, 3), generator=g, dtype=torch.uint8).to(device)
    from neural_network_image_compression_amd._lib import latent_shape
    h8, w8 = latent_shape(H, W)
    z = torch.empty((B, h8, w8, 96), dtype=torch.uint8, device=device)
    r = torch.empty((B, 8 * h8, 8 * w8, 3), dtype=torch.uint8, device=device)

    # config 5: the histogram counted in conv8's epilogue (nic_encode_entropy, default) or the
    # two-call form (NIC_BENCH_HIST=sep: nic_encode, then nic_entropy_hist re-reading the latent)
    hist_fold = os.environ.get("NIC_BENCH_HIST", "fold") != "sep"
    if args.workload == "4k" and hist_fold:
        def step():
            codec.encode_entropy(x, out=z)
    elif args.workload == "4k":
        def step():
            codec.encode(x, out=z)
            codec.entropy(z)
    else:
        def step():
            codec.encode(x, out=z)
            codec.decode(z, out=r)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # headline: K steps, barrier + sync on both sides, max over ranks
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    # per-layer device time: hipEvents around every launch on the launch stream
    codec.set_timing(True)
    barrier()
    for _ in range(args.steps):
        step()
    lt = codec.layer_times()
    codec.set_timing(False)
    torch.cuda.synchronize()
    ent_ms = None
    if args.workload == "4k":
        # histogram entropy: torch events on the current stream (the one nic_entropy_hist runs on)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            codec.entropy(z)
        e1.record()
        torch.cuda.synchronize()
        ent_ms = e0.elapsed_time(e1) / args.steps
    host_path = None
    if args.workload in ("config2", "kodak") and rank == 0 and not args.no_host_path:
        # the reference's own surface with host arrays: Encoder()(numpy) -> Decoder()(numpy)
        # (H2D of the u8 images, D2H + H2D of the latents, D2H of the recons: 9 B/pixel of
        # PCIe traffic around the device pass) -- reported beside `value`, never as it
        from neural_network_image_compression_amd.codec import Decoder, Encoder
        enc, dec = Encoder(codec=codec), Decoder(codec=codec)
        xh = x.cpu().numpy()
        for _ in range(3):  # pinned staging allocated, clocks settled
            dec(enc(xh))
        reps = max(10, args.steps)
        t0 = time.perf_counter()
        for _ in range(reps):
            dec(enc(xh))
        hp = (time.perf_counter() - t0) / reps
        host_path = {"mp_per_s": round(B * H * W / 1e6 / hp, 1), "ms_per_batch": round(hp * 1e3, 3),
                     "box": host_box_rates(xh, enc, dec, reps),
                     "path": "Encoder()(numpy) -> Decoder()(numpy) via nic_encode_host / nic_decode_host: "
                             f"{Encoder.host_chunks} ramped chunks per call, H2D / device pass / D2H on three "
                             "HIP streams; pageable input staged through pinned memory, results returned "
                             "in page-locked arrays (the decoder DMAs the encoder's result directly)"}
    quality = None
    if args.workload in ("config2", "kodak") and min(H, W) >= 161 and not args.no_quality:
        # device MS-SSIM (nic_ms_ssim) and PSNR (nic_sq_err) of the batch's reconstruction;
        # outside the encode+decode metric, timed with torch events on the current stream
        rec = codec.decode(codec.encode(x))
        codec.ms_ssim(x, rec)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            ms = codec.ms_ssim(x, rec)
        e1.record()
        torch.cuda.synchronize()
        q_ms = e0.elapsed_time(e1) / args.steps
        nbytes = 2 * B * H * W * 3  # both u8 images read once at scale 0
        quality = {"ms_ssim_mean": round(float(ms.mean().item()), 6), "psnr_db": round(codec.psnr(x, rec), 4),
                   "ms_ssim_ms": round(q_ms, 4), "ms_ssim_mp_per_s": round(B * H * W / 1e6 / (q_ms * 1e-3), 1),
                   "ms_ssim_gbps_scale0": round(nbytes / (q_ms * 1e-3) / 1e9, 1),
                   "kernels": "ssim_tile_kernel x5 scales + ssim_pool_kernel x4 + msssim_combine_kernel"}

    coll = None
    if world > 1:
        # config 3's exchange, outside the timed steps: the shards' u8 latents
        # (and recons) gathered to rank 0 over RCCL in global order (parallel.gather_rows)
        from neural_network_image_compression_amd.parallel import gather_rows
        outs = [z] if args.workload == "4k" else [z, r]
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in outs:
            gather_rows(t.to(coll_dev), world * B, dist, dst=0)
        torch.cuda.synchronize()
        barrier()
        coll = {"gather_ms": round((time.perf_counter() - t0) * 1e3, 3),
                "gathered_bytes": int(world * B * sum(t[0].numel() for t in outs)),
                "op": "gather to rank 0 of padded shards (RCCL) of the u8 latents" +
                      ("" if args.workload == "4k" else " and recons") + ", once after the timed steps"}
    if rank != 0:
        barrier()
        torch.cuda.synchronize()
        codec.close()
        if world > 1:
            dist.destroy_process_group()
        return

    P = 3 * B
    geo = layer_geometry(H, W)
    layers = {}
    conv1_fused = lt["conv1"][1] == 0 and lt["conv2"][1] > 0  # f16x3: conv1 runs inside conv2's kernel
    # f16x3: dconv8's MACs run inside dconv7's kernel (the per-pixel tap projections); the
    # dconv8 launch is then an HBM-bound gather (csrc/nic_capi.hip decode_pass)
    d78_fused = args.precision == "f16x3"
    moved = {"conv2": "conv1" if conv1_fused else None, "dconv7": "dconv8" if d78_fused else None}
    # the fused k3 residual pairs (planes up to 64 columns): one launch each, timed as conv4 / dconv6
    k3_fused = {"conv4": "conv3", "dconv6": "dconv5"}
    for b, a_ in k3_fused.items():
        if lt[a_][1] == 0 and lt[b][1] > 0:
            moved[b] = a_
    flops = {}
    for name, (ms, n) in lt.items():
        if n == 0:
            continue
        avg = ms / max(n, 1)
        if name == "dconv8" and d78_fused:
            # reads 25 fp32 projections per dconv7 output pixel, writes 3 B per output pixel
            nbytes = P * (4 * h8) * (4 * w8) * 25 * 4 + B * (8 * h8) * (8 * w8) * 3
            flops[name] = 0
            layers[name] = {"avg_ms": round(avg, 4), "gbytes_per_launch": round(nbytes / 1e9, 3),
                            "gbps": round(nbytes / (avg * 1e-3) / 1e9, 1) if avg > 0 else None,
                            "hbm_frac": round(nbytes / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if avg > 0 else None,
                            "fused": "gather of dconv7's tap projections + inverse colour + quantiser"}
            continue
        extra = moved.get(name)
        flop = flops[name] = (geo[name] + (geo[extra] if extra else 0)) * P
        layers[name] = {"avg_ms": round(avg, 4), "gflop_per_launch": round(flop / 1e9, 3),
                        "tflops": round(flop / (avg * 1e-3) / 1e12, 2) if avg > 0 else None}
        if name == "conv2" and conv1_fused:
            layers[name]["fused"] = "conv1 (colour transform + conv1 computed into conv2's LDS halo)"
        if name == "dconv7" and d78_fused:
            layers[name]["fused"] = "dconv8's MACs (25 tap projections per output pixel, split-f16 MFMA)"
        if moved.get(name) in ("conv3", "dconv5"):
            layers[name]["fused"] = f"{moved[name]} -> {name} -> + residual (one launch, row-streamed through LDS)"
    if ent_ms is not None:
        nbytes = B * h8 * w8 * 96 + 3 * B * 4  # u8 latent read once + 3 floats per image
        ent = {"avg_ms": round(ent_ms, 4), "gbytes_per_launch": round(nbytes / 1e9, 4),
               "gbps": round(nbytes / (ent_ms * 1e-3) / 1e9, 1),
               "hbm_frac": round(nbytes / (ent_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
               "kernels": "latent_hist_kernel (per-block partial counts) + hist_entropy_kernel (reduce + entropy)"}
        if hist_fold:  # not in the step: the codes are counted in conv8's epilogue
            ent = {"in_step": "folded into conv8 (per-block LDS counts of the codes it quantises) + "
                              "hist_fold_kernel (partials -> counts, bits)",
                   "standalone_two_call_form": ent}
        layers["entropy"] = ent
    # the dominant kernel = the one with the most device time per step.  The encoder's and the
    # decoder's fused k3 residual pairs are launches of one kernel (conv_k3pair_kernel, equal FLOP),
    # so they count together ("k3_pair": FLOP per launch / the mean of their launch times).
    kern = {}  # kernel -> (time per step, [layers])
    for k in layers:
        if "tflops" not in layers[k]:
            continue
        kk = "k3_pair" if moved.get(k) in ("conv3", "dconv5") else k
        t, ls = kern.get(kk, (0.0, []))
        kern[kk] = (t + layers[k]["avg_ms"], ls + [k])
    dom = max(kern, key=lambda k: kern[k][0])
    dom_layers = kern[dom][1]
    dom_ms = sum(layers[k]["avg_ms"] for k in dom_layers) / len(dom_layers)
    dom_flop = flops[dom_layers[0]]
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("batch") == B and tj.get("size") == S and H == W == S:
                traffic = tj["layers"].get(dom, {}).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    achieved = round(dom_flop / (dom_ms * 1e-3) / 1e12, 2)
    peak = F16X3_PEAK_TFLOPS if args.precision == "f16x3" else FP32_MFMA_PEAK_TFLOPS
    roofline = {"bound": "mfma", "kernel": dom, "layers": dom_layers, "achieved": achieved, "peak": round(peak, 1),
                "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic,
                "flop_per_launch": dom_flop, "avg_launch_ms": round(dom_ms, 4),
                "share_of_step": round(kern[dom][0] / (el / args.steps * 1e3), 4),
                "peak_basis": ("dense f16 MFMA 2.5 PFLOP/s / 3 passes (algorithmic fp32 FLOP)"
                               if args.precision == "f16x3" else "dense fp32 MFMA 157.3 TFLOP/s")}
    if dom == "k3_pair":  # the direct 9-tap pair issues exactly the algorithmic products
        roofline["k3_form"] = "direct 9-tap"
        roofline["issued_tflops"] = round(dom_flop / (dom_ms * 1e-3) / 1e12, 2)
        roofline["issued_frac"] = round(dom_flop / (dom_ms * 1e-3) / 1e12 / peak, 4)
    others = sorted((k for k in kern if k != dom), key=lambda k: -kern[k][0])
    if others:  # the next kernel by device time, for continuity with earlier lines (dconv7)
        k2 = others[0]
        l2 = kern[k2][1]
        ms2 = sum(layers[k]["avg_ms"] for k in l2) / len(l2)
        roofline["next_kernel"] = {"kernel": k2, "avg_launch_ms": round(ms2, 4),
                                   "achieved": round(flops[l2[0]] / (ms2 * 1e-3) / 1e12, 2),
                                   "frac": round(flops[l2[0]] / (ms2 * 1e-3) / 1e12 / peak, 4)}
    enc_only = args.workload == "4k"
    total_flop = sum(v for k, v in geo.items() if not (enc_only and k.startswith("dconv"))) * P
    ms_step = el / args.steps * 1e3
    value = world * B * H * W * args.steps / 1e6 / el
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "MP/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32" if args.precision == "fp32" else "fp32 (split-f16x3 MFMA)",
        "data": "synthetic" if args.images == "random" or args.workload != "config2" else "kodim21 crops",
        "config": {"workload": {"config2": f"config2: {B}x{H}x{W}x3 u8 synthetic per GPU, encode+decode",
                                "kodak": f"config4 shape: {B}x{H}x{W}x3 whole images per GPU, encode+decode",
                                "4k": f"config5: {B}x{H}x{W}x3 frames per GPU, encode + histogram entropy"
                                }[args.workload] + " (torch seed 1000+rank)",
                   "global_batch": world * B, "image": [H, W, 3], "parallelism": f"dp{world}",
                   "weights": "seeded spread init (random-init weights of the architecture)" if args.weights == "seeded"
                   else "trained codec, entropy_loss_coef 0.01 (tests/golden/trained)"},
        "step_tflops": round(total_flop / (ms_step * 1e-3) / 1e12, 2),
        "step_frac_peak": round(total_flop / (ms_step * 1e-3) / 1e12 / peak, 4),
        "roofline": roofline, "layers": layers,
    }
    if quality is not None:
        out["quality"] = quality
    if coll is not None:
        out["collectives"] = coll
    if host_path is not None:
        out["pcie_inclusive"] = host_path
    if args.workload == "4k":
        out["metric"] = "Megapixels/sec encode + entropy (4K frames)"
        out["frames_per_s"] = round(world * B * args.steps / el, 2)
    if world == 1 and not args.no_cpu_baseline and args.workload == "config2":
        out["cpu_baseline"] = cpu_baseline(weights, S, args.cpu_seconds)
        out["cpu_baseline"]["numpy_oracle"] = cpu_baseline_numpy(weights, S, args.cpu_seconds / 2)
    if not args.no_parity and args.workload == "config2":
        out["parity"] = parity_sample(codec, x[:1], weights)
    if not args.no_power_probe and args.workload == "config2" and args.precision == "f16x3":
        out["roofline"]["power_probe"] = power_probe(dev_idx, weights, x, z, r, dom_layers, dom_flop, args.steps, peak)
    print(json.dumps(out), flush=True)
    barrier()
    torch.cuda.synchronize()
    codec.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
