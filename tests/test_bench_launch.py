"""bench.py's multi-rank launcher (the driver's `bench.py --gpus N`): without a
torchrun environment it starts N fresh rank processes itself (127.0.0.1
rendezvous), rank 0 prints ONE line with n_gpus == N, and a world size that
does not match --gpus exits non-zero.  CPU: the --dry-run plumbing under gloo;
GPU: the real HIP training step with 2 ranks sharing one device (gloo)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env,
                       cwd=REPO)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, lines


def test_launcher_dry_run_two_ranks():
    p, lines = _run(["--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1", "--dry-run-numel", "4096"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["world_size"] == 2 and line["backend"] == "gloo"
    assert len(line["per_rank_ms_per_step"]) == 2
    assert line["ms_per_step"] >= max(line["per_rank_ms_per_step"]) - 1e-6


def test_launcher_single_rank_dry_run():
    p, lines = _run(["--dry-run", "--steps", "2", "--warmup", "0"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert json.loads(lines[0])["n_gpus"] == 1


def test_world_mismatch_exits_nonzero():
    p, lines = _run(["--gpus", "2", "--dry-run", "--steps", "1"], env_extra={"WORLD_SIZE": "1", "RANK": "0"})
    assert p.returncode != 0 and not lines
    assert "!= --gpus 2" in p.stderr


@pytest.mark.gpu
def test_bench_two_ranks_on_one_gpu():
    """The real train step (HIP path, GradBuckets all-reduce) with 2 self-launched
    ranks sharing the device through gloo: one line, n_gpus == 2, per-rank times
    and the exposed all-reduce wait of both ranks."""
    p, lines = _run(["--gpus", "2", "--steps", "2", "--warmup", "1", "--unrolls", "2", "--frames", "4", "--ny", "32",
                     "--nx", "32", "--no-secondary", "--no-configs", "--no-cpu-baseline", "--no-all-branches"],
                    env_extra={"DLCS_DIST_BACKEND": "gloo"}, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["world_size"] == 2 and line["backend"] == "gloo"
    assert len(line["per_rank_ms_per_step"]) == 2
    assert len(line["allreduce"]["exposed_allreduce_ms_per_step"]) == 2
    assert line["value"] > 0 and line["loss"] == line["loss"]
