"""bench.py's multi-rank path on the one GPU of the test box (verdict r03 item 5).

Two fresh rank processes (torch.distributed.run, gloo: RCCL refuses two ranks on one device) run
bench.py's world-2 branch end to end: server keys broadcast from rank 0, TAE_MEM_DEVICE contexts built
from the received device buffers, counter blocks sharded by rank (main.rs:108-115, 148-152), the round key
broadcast, max-over-ranks timing and the min-over-ranks correctness gate.  Rank 0's JSON line must report
two GPUs' worth of blocks and `correct: true`.  The ranks are children of this process (never an exec
of a GPU-initialised process)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_world2_gloo_on_one_gpu():
    env = dict(os.environ, TAE_BENCH_BACKEND="gloo", OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "8"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
           "--blocks-per-gpu", "4", "--rounds", "1", "--key-schedule", "plain"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]  # rank 0 alone prints
    rec = json.loads(lines[0])
    assert rec["correct"] is True
    assert rec["n_gpus"] == 2
    assert rec["config"]["global_blocks"] == 8
    assert rec["value"] > 0 and rec["ms_per_step"] > 0


def test_bench_rccl_world1():
    """The RCCL path itself (verdict r04 item 4): one fresh rank under torch.distributed.run takes bench.py's
    torch.distributed branch at world size 1 with the nccl backend (= RCCL on ROCm): communicator init on
    the device, D.broadcast_u64 of the whole server key set (KSK, BSK, PFPKSK: 672 MB) as device int64
    tensors, a TAE_MEM_DEVICE context built from them, the round-key broadcast, and max_over_ranks /
    min_over_ranks on device tensors; the decrypted blocks must equal AES (reference sharding:
    main.rs:105-115, 141-159)."""
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "8"))
    env.pop("TAE_BENCH_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--force-dist", "--steps", "1", "--warmup", "0",
           "--blocks-per-gpu", "4", "--rounds", "1", "--key-schedule", "plain", "--cpu-baseline", "off",
           "--single-block", "off", "--model8-leg", "off", "--host-buffers", "off"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    rec = json.loads(lines[0])
    assert rec["correct"] is True and rec["n_gpus"] == 1
    d = rec["dist"]
    assert d["backend"] == "nccl" and d["world"] == 1, d
    assert d["server_key_bytes"] > 600_000_000 and d["key_tensors_on"].startswith("cuda"), d
