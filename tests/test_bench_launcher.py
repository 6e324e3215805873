"""bench.py --gpus N without an external launcher.

The driver's scaling run may call `python bench.py --gpus N` directly.  bench.py must then start N
ranks itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as torch.distributed.run sets them) from a
parent that never touches the GPU, and rank 0 must print ONE line with n_gpus == N; a WORLD_SIZE
that disagrees with --gpus must fail.  --dry-run 1 runs the same launcher and gloo control plane
with no GPU.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(kw)
    return env


def _json_lines(out):
    return [json.loads(x) for x in out.splitlines() if x.startswith("{")]


def test_launcher_spawns_ranks_and_merges_one_line():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "1", "--steps", "3", "--warmup", "1"],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout  # rank 0 only
    assert len(p.stdout.strip().splitlines()) == 1, p.stdout  # nothing else: gloo's messages go to stderr
    line = lines[0]
    assert line["n_gpus"] == 2 and line["dry_run"] is True
    ranks = sorted(line["ranks"], key=lambda r: r["rank"])
    assert [r["rank"] for r in ranks] == [0, 1]
    assert [r["local_rank"] for r in ranks] == [0, 1]
    assert all(r["world_size"] == 2 for r in ranks)
    assert all(r["master_addr"] == "127.0.0.1" for r in ranks)
    assert len({r["master_port"] for r in ranks}) == 1 and ranks[0]["master_port"]
    assert len({r["pid"] for r in ranks}) == 2  # two processes, neither the launcher
    assert len(line["per_rank_ms_per_step"]) == 2
    assert line["ms_per_step"] == max(line["per_rank_ms_per_step"])


def test_world_size_mismatch_refused():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dry-run", "1"],
                       env=_env(RANK="0", LOCAL_RANK="0", WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                                MASTER_PORT="29999"),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0
    assert not _json_lines(p.stdout)
    assert "refusing" in p.stderr


def test_failing_rank_fails_the_launch():
    # a rank that dies makes the launcher stop the others and exit non-zero with no line
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "2"],
                       env=_env(), capture_output=True, text=True, timeout=120)
    assert p.returncode == 3
    assert not _json_lines(p.stdout)
    assert "rank 1 exited" in p.stderr


def test_single_gpu_dry_run_is_world_of_one():
    p = subprocess.run([sys.executable, BENCH, "--dry-run", "1"], env=_env(), capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr
    (line,) = _json_lines(p.stdout)
    assert line["n_gpus"] == 1 and len(line["ranks"]) == 1


def test_torchrun_launch_stdout_is_the_line():
    # the driver's N > 1 command: torch.distributed.run merges every rank's stdout; the gloo
    # control plane's "[Gloo] Rank r is connected ..." messages must not land there
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29561", BENCH, "--gpus", "2",
                        "--dry-run", "1", "--steps", "3", "--warmup", "1"],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    out = p.stdout.strip().splitlines()
    assert len(out) == 1, p.stdout
    line = json.loads(out[0])
    assert line["n_gpus"] == 2 and sorted(r["rank"] for r in line["ranks"]) == [0, 1]
