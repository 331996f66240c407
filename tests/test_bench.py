"""bench.py keeps the driver's contract: one JSON line with the required keys (a short
run on the GPU; the CPU test only checks the CLI)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_cli_parses():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0 and "--warmup" in out.stdout and "--gpus" in out.stdout


def _bench(args, env_extra=None, timeout=300):
    env = dict(os.environ, NIC_BENCH_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    for k in [k for k, v in env.items() if v == ""]:
        env.pop(k)  # "" in env_extra: unset
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, cwd=ROOT, env=env)


def test_bench_gpus_flag_spawns_ranks():
    # `python bench.py --gpus 2` with no launcher starts 2 ranks (torch.distributed.run as a
    # child process); --launch-check stops after the process group (gloo, no GPU work)
    # (NIC_BENCH_BACKEND unset: the launch check's process group defaults to gloo)
    out = _bench(["--gpus", "2", "--launch-check"], env_extra={"NIC_BENCH_BACKEND": ""}, timeout=240)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_joined"] == 2 and d["parallelism"] == "dp2"


def test_bench_gpus_flag_mismatch_fails():
    # under a launcher, --gpus must equal WORLD_SIZE: never a silent 1-GPU line
    out = _bench(["--gpus", "2", "--launch-check"], env_extra={"WORLD_SIZE": "1", "RANK": "0"})
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]


@pytest.mark.gpu
def test_bench_gpus2_without_launcher():
    # the world-2 codec path started by `--gpus 2` alone (both ranks share the box's one GPU
    # over gloo): rank 0's single line reports n_gpus 2 and the gathered bytes of both shards
    out = _bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "4", "--no-power-probe",
                  "--no-host-path", "--no-quality"])
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 8 and d["value"] > 0
    assert d["collectives"]["gathered_bytes"] == 8 * (32 * 32 * 96 + 256 * 256 * 3)


@pytest.mark.gpu
def test_bench_json_line():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
                          "--batch", "4", "--cpu-seconds", "1"], capture_output=True, text=True, timeout=300,
                         cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["value"] > 0
    r = d["roofline"]
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(r) and 0 < r["frac"] < 1
    assert {"value", "unit", "cores", "kind", "sample"} <= set(d["cpu_baseline"])
    assert d["parity"]["psnr_gpu_vs_oracle_db"] >= 50


@pytest.mark.gpu
def test_bench_world2_path_under_torchrun():
    # bench.py's world > 1 path exactly as the driver launches it (torch.distributed.run, one
    # process per rank): weight broadcast, MAX-over-ranks timing, the config-3 gather to rank 0,
    # rank 0's single JSON line.  The GPU box has one GPU, so both ranks share it and the
    # process group is gloo (NIC_BENCH_BACKEND; RCCL refuses two ranks on one device)
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, NIC_BENCH_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--batch", "4", "--no-power-probe", "--no-host-path", "--no-quality"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 8 and d["config"]["parallelism"] == "dp2"
    assert d["value"] > 0 and d["scaling"] == "weak"
    c = d["collectives"]
    assert c["gathered_bytes"] == 8 * (32 * 32 * 96 + 256 * 256 * 3)  # latents + recons of both shards
