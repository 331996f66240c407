"""Config 3's multi-GPU path on the device: RCCL process group, weight broadcast, sharded
encode -> decode -> entropy and the gathers, with the real HIP codec (one rank: the GPU box
has one GPU).  Runs in a child process so the RCCL communicator does not outlive the test."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_run_sharded_over_rccl_world1():
    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "nccl_sharded_check.py")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = subprocess.run([sys.executable, script], env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0 and "NCCL-OK" in out.stdout, out.stdout[-2000:] + out.stderr[-3000:]
