"""bench.py's multi-GPU plumbing on the CPU (gloo dry run): `--gpus N` without WORLD_SIZE starts N ranks under
torch.distributed.run as a child process, every rank joins, the MAX over ranks reaches rank 0, and exactly one JSON
line comes out; a WORLD_SIZE that disagrees with --gpus is refused (--gpus was parsed and ignored)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, env=env, capture_output=True, text=True,
                          timeout=timeout)


def json_lines(out):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


@pytest.mark.parametrize("n", [2, 3])
def test_spawn_n_ranks_one_line(n):
    r = run(["--gpus", str(n), "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert d["n_gpus"] == n and d["ranks_reported"] == n and d["dry_run"] is True
    assert d["max_over_ranks"] == float(n)  # rank r contributes 1 + r: the MAX over all ranks reached rank 0


def test_strong_scaling_flag():
    r = run(["--gpus", "2", "--dry-run", "--scaling", "strong"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert json_lines(r.stdout)[0]["scaling"] == "strong"


def test_world_size_must_match_gpus():
    r = run(["--gpus", "2", "--dry-run"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE" in r.stderr


@pytest.mark.gpu
def test_two_ranks_on_one_gpu():
    """The N > 1 path end to end on real kernels (a one-GPU box: both ranks on cuda:0, gloo collectives): each rank
    classifies its own resident batches, its parity sample is green, the MAX-over-ranks line counts both ranks'
    packets, and the verdict gather runs.  RCCL itself is the driver's multi-GPU run."""
    r = run(["--gpus", "2", "--shared-gpu", "--n", "262144", "--steps", "8", "--warmup", "2", "--configs", "",
             "--no-cpu-baseline", "--no-host-inclusive"], timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert d["n_gpus"] == 2 and d["ranks_reported"] == 2 and d["shared_gpu_rehearsal"] is True
    assert d["config"]["global_batch"] == 2 * 262144 and d["parity_sample_ok"] is True
    assert d["value"] > 0 and "error" not in d["gather"], d.get("gather")


def test_spawn_forwards_packets_option():
    """`--n` (packets per GPU) reaches the ranks: torch.distributed.run's parser would read it as an ambiguous
    abbreviation of its own options, so the spawn forwards it as `--packets`."""
    r = run(["--gpus", "2", "--dry-run", "--n", "4096"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert json_lines(r.stdout)[0]["ranks_reported"] == 2
