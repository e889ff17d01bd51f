"""bench.py's rank launch logic (--gpus N must launch N ranks).

plan_ranks decides, before anything touches a GPU, whether this process is
one rank, must start N rank processes, or must refuse; the subprocess checks
run the real script on this GPU-less host, where every multi-GPU request
without --rehearse is refused."""

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import plan_ranks  # noqa: E402


def test_single_gpu_runs_in_process():
    assert plan_ranks(1, {}, 1, False) == ("run", None)
    assert plan_ranks(1, {}, 0, False) == ("run", None)  # fails later, loudly, without a GPU


def test_spawns_one_rank_per_gpu():
    assert plan_ranks(8, {}, 8, False) == ("spawn", 8)
    assert plan_ranks(2, {}, 8, False) == ("spawn", 2)


def test_refuses_too_few_gpus_unless_rehearsal():
    mode, why = plan_ranks(4, {}, 1, False)
    assert mode == "refuse" and "1 GPU(s) visible" in why
    assert plan_ranks(4, {}, 1, True) == ("spawn", 4)


def test_launcher_world_size_must_match():
    assert plan_ranks(8, {"WORLD_SIZE": "8"}, 8, False) == ("run", None)
    mode, why = plan_ranks(8, {"WORLD_SIZE": "4"}, 8, False)
    assert mode == "refuse" and "disagree" in why
    assert plan_ranks(0, {}, 8, False)[0] == "refuse"


@pytest.mark.parametrize("argv,env,msg", [
    (["--gpus", "2"], {}, "GPU(s) visible"),
    (["--gpus", "2"], {"WORLD_SIZE": "3"}, "disagree"),
])
def test_script_refuses(argv, env, msg):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    e["HIP_VISIBLE_DEVICES"] = ""  # no device here anyway; never one in this test
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + argv, env=e,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, r.stderr[-2000:]
    assert msg in r.stderr
