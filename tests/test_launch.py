"""``--gpus N`` launcher (asr_rescoring_amd/launch.py) on CPU: N fresh rank processes with the
torchrun rendezvous variables, gloo world 2, exactly rank 0's line relayed, failures propagated."""
import io
import json
import os
import sys
import textwrap

import pytest

from asr_rescoring_amd import launch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = textwrap.dedent("""
    import json, os, sys
    import torch, torch.distributed as dist
    env = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE",
                                          "MASTER_ADDR", "MASTER_PORT")}
    dist.init_process_group("gloo")
    t = torch.tensor([float(dist.get_rank() + 1)])
    dist.all_reduce(t)
    if dist.get_rank() == 0:
        print(json.dumps({"env": env, "sum": float(t.item()), "argv": sys.argv[1:]}))
    else:
        print("rank", dist.get_rank(), "stdout line")      # must not reach the parent's stdout
    dist.barrier()
    dist.destroy_process_group()
""")

FAILING = textwrap.dedent("""
    import os, sys, time
    import torch.distributed as dist
    if os.environ["RANK"] == "1":
        sys.exit(3)
    dist.init_process_group("gloo")     # rank 0 waits for a peer that never comes
    time.sleep(600)
""")


def test_need_spawn_rules():
    assert launch.need_spawn(2, env={})
    assert not launch.need_spawn(1, env={})
    assert not launch.need_spawn(8, env={"WORLD_SIZE": "8"})     # torchrun already set the ranks


def test_rank_env():
    e = launch.rank_env(1, 4, 1234, base={"X": "y"})
    assert e["X"] == "y" and e["RANK"] == "1" and e["LOCAL_RANK"] == "1" and e["WORLD_SIZE"] == "4"
    assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "1234"


def test_spawn_world2_gloo_one_line(tmp_path):
    w = tmp_path / "worker.py"
    w.write_text(WORKER)
    out = io.StringIO()
    rc = launch.spawn_ranks(2, ["--flag", "v"], script=str(w), stdout=out)
    assert rc == 0
    lines = [ln for ln in out.getvalue().splitlines() if ln.strip()]
    assert len(lines) == 1, lines
    rec = json.loads(lines[0])
    assert rec["sum"] == 3.0                        # both ranks took part in the collective
    assert rec["env"]["RANK"] == "0" and rec["env"]["LOCAL_RANK"] == "0"
    assert rec["env"]["WORLD_SIZE"] == "2" and rec["env"]["MASTER_ADDR"] == "127.0.0.1"
    assert rec["argv"] == ["--flag", "v"]


def test_spawn_failure_terminates_peers(tmp_path):
    w = tmp_path / "failing.py"
    w.write_text(FAILING)
    rc = launch.spawn_ranks(2, [], script=str(w), stdout=io.StringIO(), grace_s=10)
    assert rc == 3


def test_bench_gpus_n_spawns_before_any_gpu_call(monkeypatch):
    """bench.py --gpus 2 with no WORLD_SIZE hands off to the launcher (same argv, bench.py itself)
    before touching the GPU, and exits with the launcher's status."""
    sys.path.insert(0, REPO)
    import bench
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(launch, "spawn_ranks", lambda n, argv, script=None, **k: calls.append((n, list(argv), script)) or 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "1"])
    import torch
    monkeypatch.setattr(torch.cuda, "set_device", lambda *a: pytest.fail("GPU call before the hand-off"))
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    assert calls == [(2, ["--gpus", "2", "--steps", "1"], os.path.abspath(bench.__file__))]
