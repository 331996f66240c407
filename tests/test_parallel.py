"""Multi-process (world_size 2, gloo, CPU) tests of the patch-parallel plumbing.

The device codec needs a GPU, so each rank runs the CPU oracle on its shard in its place:
what is tested here is the sharding, the weight broadcast and the latent gather that
bench.py / parallel.py run over RCCL on the GPU box."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from neural_network_image_compression_amd.parallel import shard_range


@pytest.mark.parametrize("n,world", [(512, 8), (10, 4), (3, 4), (0, 2), (7, 1)])
def test_shard_range_partitions(n, world):
    seen = []
    for r in range(world):
        lo, hi = shard_range(n, world, r)
        assert 0 <= lo <= hi <= n
        seen += list(range(lo, hi))
    assert seen == list(range(n))
    sizes = [np.subtract(*shard_range(n, world, r)[::-1]) for r in range(world)]
    assert max(sizes) - min(sizes) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_total, out_dir):
    import torch
    import torch.distributed as dist

    from neural_network_image_compression_amd import weights as W
    from neural_network_image_compression_amd.parallel import broadcast_weights, gather_rows, shard_range
    from oracle import nic_oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = broadcast_weights(W.seeded_weights(0) if rank == 0 else None, dist)
        digest = W.digest(w)
        rng = np.random.default_rng(42)
        x = rng.integers(0, 256, (n_total, 16, 24, 3), dtype=np.uint8)  # every rank builds the same batch
        lo, hi = shard_range(n_total, world, rank)
        z_local = torch.from_numpy(O.encode(w, x[lo:hi]))
        z_all = gather_rows(z_local, n_total, dist, dst=0)
        # per-image entropy rows (n_local, 3), gathered on every rank
        bits_local = torch.from_numpy(O.hist_entropy(z_local.numpy()).reshape(3, hi - lo).T.copy())
        bits_all = gather_rows(bits_local, n_total, dist, dst=None)
        np.save(os.path.join(out_dir, f"bits{rank}.npy"), bits_all.numpy())
        if rank == 0:
            np.save(os.path.join(out_dir, "z_all.npy"), z_all.numpy())
            with open(os.path.join(out_dir, "digest.txt"), "w") as f:
                f.write(digest)
        else:
            assert z_all is None
            with open(os.path.join(out_dir, f"digest{rank}.txt"), "w") as f:
                f.write(digest)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [5, 4])
def test_two_rank_broadcast_and_gather(tmp_path, n_total):
    from neural_network_image_compression_amd import weights as W
    from oracle import nic_oracle as O

    world = 2
    mp.spawn(_worker, args=(world, _free_port(), n_total, str(tmp_path)), nprocs=world, join=True)
    w = W.seeded_weights(0)
    assert open(tmp_path / "digest.txt").read() == W.digest(w)
    assert open(tmp_path / "digest1.txt").read() == W.digest(w)
    rng = np.random.default_rng(42)
    x = rng.integers(0, 256, (n_total, 16, 24, 3), dtype=np.uint8)
    z = O.encode(w, x)
    np.testing.assert_array_equal(np.load(tmp_path / "z_all.npy"), z)
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"bits{r}.npy"), O.hist_entropy(z).reshape(3, n_total).T)


class _OracleCodec:
    """Stand-in for codec.Codec on a CPU rank (test infrastructure: the oracle computes what
    the HIP codec would), with the same encode / decode / entropy tensor interface."""

    def __init__(self, w):
        self.w = w

    def encode(self, x):
        import torch
        from oracle import nic_oracle as O
        return torch.from_numpy(O.encode(self.w, x.numpy()))

    def decode(self, z):
        import torch
        from oracle import nic_oracle as O
        return torch.from_numpy(O.decode(self.w, z.numpy()))

    def entropy(self, z):
        import torch
        from oracle import nic_oracle as O
        return torch.from_numpy(O.hist_entropy(z.numpy()).ravel())


def _sharded_worker(rank, world, port, n_total, out_dir):
    import torch
    import torch.distributed as dist

    from neural_network_image_compression_amd import weights as W
    from neural_network_image_compression_amd.parallel import broadcast_weights, run_sharded, shard_range

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = broadcast_weights(W.seeded_weights(0) if rank == 0 else None, dist)
        x = np.random.default_rng(7).integers(0, 256, (n_total, 16, 24, 3), dtype=np.uint8)
        lo, hi = shard_range(n_total, world, rank)
        z, r, b = run_sharded(_OracleCodec(w), torch.from_numpy(x[lo:hi]), n_total, dist, dst=0)
        if rank == 0:
            np.savez(os.path.join(out_dir, "sharded.npz"), z=z.numpy(), r=r.numpy(), b=b.numpy())
        else:
            assert z is None and r is None and b is None
    finally:
        dist.destroy_process_group()


def test_run_sharded_config3_plumbing(tmp_path):
    """Config 3 on 2 gloo ranks with a ragged split: encode -> decode -> entropy per shard,
    latents / recons / per-image entropy rows gathered to rank 0 in global order."""
    from neural_network_image_compression_amd import weights as W
    from oracle import nic_oracle as O

    n_total = 5
    mp.spawn(_sharded_worker, args=(2, _free_port(), n_total, str(tmp_path)), nprocs=2, join=True)
    w = W.seeded_weights(0)
    x = np.random.default_rng(7).integers(0, 256, (n_total, 16, 24, 3), dtype=np.uint8)
    got = np.load(tmp_path / "sharded.npz")
    z = O.encode(w, x)
    np.testing.assert_array_equal(got["z"], z)
    np.testing.assert_array_equal(got["r"], O.decode(w, z))
    np.testing.assert_array_equal(got["b"], O.hist_entropy(z).reshape(3, n_total).T)
