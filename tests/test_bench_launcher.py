"""bench.py's multi-rank launcher (CPU, gloo): `--gpus N` without WORLD_SIZE
starts N ranks through torch.distributed.run, a WORLD_SIZE that disagrees with
--gpus is refused, and ablation switches stop the run before any line."""
import json
import os
import subprocess
import sys

from conftest import REPO

BENCH = os.path.join(REPO, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra)
    return env


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_launcher_starts_two_ranks_over_gloo():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "0"],
                       env=_env(RSK_BENCH_TEST_TAG="x"), capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout      # rank 0 alone prints
    line = lines[0]
    assert line["dry_run"] and line["n_gpus"] == 2 and line["rccl_world"] == 2
    assert sorted(line["ranks"]) == [0, 1]
    assert len(set(line["pids"])) == 2 and os.getpid() not in line["pids"]   # two fresh child processes
    assert line["scenario_shards"] == [[0, 4096], [4096, 8192]]
    assert line["steps"] == 3
    assert line["env"] == {"RSK_BENCH_TEST_TAG": "x"}


def test_single_rank_runs_in_process():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--dry-run", "--steps", "2"],
                       env=_env(), capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    (line,) = _json_lines(p.stdout)
    assert line["n_gpus"] == 1 and line["rccl_world"] == 1 and line["pids"] == [line["pids"][0]]
    assert "launching" not in p.stderr


def test_world_size_mismatch_fails_loudly():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dry-run"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=240)
    assert p.returncode != 0
    assert "WORLD_SIZE=2" in p.stderr and not _json_lines(p.stdout)


def test_ablation_switch_refused():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--dry-run"],
                       env=_env(RSK_ABLATE_TILE="2"), capture_output=True, text=True, timeout=240)
    assert p.returncode != 0 and "ablation" in p.stderr and not _json_lines(p.stdout)
