"""bench.py's own rank launcher (the driver runs `python bench.py --gpus N`):
N > 1 without torchrun spawns N rank processes and rank 0 prints one line
with n_gpus = N; under torchrun WORLD_SIZE must equal --gpus.  The CPU tests
use --dry-run (control plane only: gloo barriers and the max-over-ranks
timing, no GPU); the GPU test rehearses two real ranks on the one GPU."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def _line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_n_ranks(n):
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-run", "--steps", "4", "--warmup", "1"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-2000:]
    line = _line(p.stdout)
    assert line["n_gpus"] == n and line["ranks_reporting"] == n and line["steps"] == 4


def test_world_size_must_match_gpus():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], cwd=ROOT,
                       env=_env(WORLD_SIZE="3", RANK="0"), capture_output=True, text=True, timeout=60)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr
    p = subprocess.run([sys.executable, BENCH, "--gpus", "0", "--dry-run"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=60)
    assert p.returncode != 0


def test_torchrun_ranks():
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
                        "--nproc-per-node", "2", BENCH, "--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-2000:]
    line = _line(p.stdout)
    assert line["n_gpus"] == 2 and line["ranks_reporting"] == 2


_SMALL = ["--entities", "100000", "--steps", "3", "--warmup", "2", "--no-config5", "--no-cpu-baseline",
          "--profile-stages", "0", "--client-msgs", "0", "--e2e-steps", "0"]


@pytest.mark.gpu
def test_launcher_two_ranks_on_one_gpu():
    """Two real ranks (independent spaces, weak) plus the decomposed-world leg
    over gloo, both on device 0 (RCCL needs one GPU per rank)."""
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--device", "0", "--comm", "gloo", "--mode", "spaces"]
                       + _SMALL, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    line = _line(p.stdout)
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["value"] > 0
    assert line["c3world"]["n_gpus"] == 2 and line["c3world"]["value"] > 0


@pytest.mark.gpu
def test_bench_loopback_world_line():
    """--comm loopback: the default N > 1 headline (the 1M space decomposed
    into N strips, strong) with its N ranks as threads of one process on the
    one GPU, every step through gw_step -> gw_world_step over the loopback
    transport (the RCCL path's call sequence); also the world headline of two
    gloo rank processes with the weak spaces leg beside it."""
    p = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--device", "0", "--comm", "loopback"] + _SMALL
                       + ["--profile-stages", "1"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    line = _line(p.stdout)
    assert line["ranks"] == 3 and line["comm"] == "loopback" and line["scaling"] == "strong"
    assert line["value"] > 0 and line["events_per_sec"] > 0 and line["roofline"]["frac"] > 0
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--device", "0", "--comm", "gloo"] + _SMALL,
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    line = _line(p.stdout)
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and line["value"] > 0
    assert line["spaces"]["scaling"] == "weak" and line["spaces"]["value"] > 0
