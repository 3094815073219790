"""CPU: `python bench.py --gpus N` starts its own N ranks when no launcher did (--gpus was parsed but
never used, so a plain --gpus 8 run reported n_gpus 1).  The dist-check leg exercises only the plumbing (env
of every rank, one gloo all_gather); the training legs use the same path with nccl (RCCL) on the GPUs."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["MPLC_DIST_BACKEND"] = "gloo"
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_gpus_flag_spawns_ranks():
    r = _run(["--gpus", "3", "--leg", "dist-check"])
    assert r.returncode == 0, r.stderr
    # exactly one JSON line, from rank 0 (gloo itself prints a "[Gloo] Rank 0 is connected" line)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 3
    assert line["ranks"] == [[0, 0], [1, 1], [2, 2]]  # RANK and LOCAL_RANK (= the GPU index) per child
    assert line["master"][0] == "127.0.0.1"


def test_single_gpu_runs_in_process():
    r = _run(["--leg", "dist-check"])
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1


def test_launcher_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--leg", "dist-check"], extra_env={"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
