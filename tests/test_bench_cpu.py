"""bench.py --gpus N without a launcher: it either starts N ranks
(torch.distributed.run, one child process) or fails -- it never times one process and reports
n_gpus = N."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(extra_env):
    env = dict(os.environ, DFU_DIST_BACKEND="gloo", **extra_env)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps",
                        "1", "--warmup", "0", "--no-cpu-baseline", "--no-parity"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, [json.loads(ln) for ln in lines]


def test_gpus2_without_enough_devices_fails():
    import torch
    if torch.cuda.device_count() >= 2:
        return  # a real 2-GPU node: the launch path runs instead (driver's SCALE runs)
    p, lines = _run({})
    assert p.returncode == 2, p.stderr[-2000:]
    assert "needs 2 GPUs" in p.stderr
    assert not lines  # no line at all, least of all an n_gpus 2 one


def test_gpus2_rehearsal_launches_two_ranks():
    """DFU_SHARE_DEVICE=1 (the one-GPU gloo rehearsal): the parent launches 2 ranks; without a
    GPU they fail, and the failure is the exit status -- never a one-process line."""
    p, lines = _run({"DFU_SHARE_DEVICE": "1"})
    assert "[bench] launching 2 ranks" in p.stderr
    for ln in lines:  # (on a GPU box the ranks run: every line reports the 2 ranks it ran)
        assert ln["n_gpus"] == 2 and ln["config"]["dist"]["ranks"] == 2
    if not lines:
        assert p.returncode != 0
