"""`python bench.py --gpus N` without a launcher: the parent starts N ranks
itself (bench.launch_ranks) with the torch.distributed.run environment, before any GPU call,
never execs, relays rank 0's line and exits non-zero when a rank fails.

CPU tests: the launcher on a probe script that rendezvouses over gloo with the environment
it was given (env://, exactly what bench.dist_setup does) and prints one line from rank 0;
a failing rank ends the job promptly with its exit code; bench.py itself with --gpus 2 and
no GPU fails loudly instead of hanging. The GPU test runs bench.py --gpus 2 on one MI355X
(two gloo ranks sharing the card) and checks the one strong-scaling line it prints."""
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

PROBE = textwrap.dedent("""
    import json, os, sys, time
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if os.environ.get("PROBE_FAIL_RANK") == str(rank):
        sys.exit(3)
    if os.environ.get("PROBE_HANG_RANK") == str(rank):
        time.sleep(600)
    dist.init_process_group("gloo")            # env:// from MASTER_ADDR / MASTER_PORT / RANK / WORLD_SIZE
    t = torch.tensor([rank + 1.0])
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"rank": rank, "world": world, "sum": t.item(), "argv": sys.argv[1:],
                          "local": os.environ["LOCAL_RANK"], "addr": os.environ["MASTER_ADDR"]}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
""")


@pytest.fixture
def probe(tmp_path):
    p = tmp_path / "probe.py"
    p.write_text(PROBE)
    return str(p)


def _launch(probe, n, env, argv=("--gpus", "3")):
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.launch_ranks(%d, %r, script=%r, grace_s=5.0))" % (REPO, n, list(argv), probe))
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240,
                          env={k: v for k, v in dict(os.environ, **env).items()
                               if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})


def test_launch_ranks_starts_a_world_and_relays_rank0_line(probe):
    r = _launch(probe, 3, {})
    assert r.returncode == 0, r.stderr
    # (gloo's own "[Gloo] Rank r is connected" messages go to each rank's stdout: bench.py moves
    # them to stderr itself, reserve_line_stdout; the probe does not)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1                        # rank 0's line only
    d = json.loads(lines[0])
    assert d["world"] == 3 and d["sum"] == 6.0 and d["local"] == "0" and d["addr"] == "127.0.0.1"
    assert d["argv"] == ["--gpus", "3"]           # the ranks get the parent's arguments


def test_a_failing_rank_fails_the_job_promptly(probe):
    t0 = time.time()
    r = _launch(probe, 2, {"PROBE_FAIL_RANK": "1"})
    assert r.returncode == 3
    assert time.time() - t0 < 120                 # rank 0, blocked in the rendezvous, was stopped
    assert "rank 1 exited with 3" in r.stderr


def test_a_hung_rank_is_killed_after_another_fails(probe):
    r = _launch(probe, 3, {"PROBE_FAIL_RANK": "2", "PROBE_HANG_RANK": "1"})
    assert r.returncode == 3


def test_bench_gpus2_without_launcher_and_gpu_fails_loudly():
    """No GPU here: both ranks fail at their first GPU call; the parent reports it and
    exits non-zero (no hang, no line)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = env.get("HIP_VISIBLE_DEVICES", "")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--no-extra"], capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    if r.returncode == 0:
        pytest.skip("a GPU is visible: covered by the gpu test")
    assert not r.stdout.strip()
    assert "[launch] rank" in r.stderr


@pytest.mark.gpu
def test_bench_gpus2_without_launcher_prints_one_strong_line(tmp_path):
    """Two ranks on one MI355X (gloo; each rank's own HIP tracer), started by bench.py itself:
    one JSON line, strong scaling, gathered results equal to rank 0's single-GPU trace, the
    schedule label read back from the library. A small strong-scaling frame keeps it short."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--no-extra",
           "--steps", "5", "--warmup", "2", "--strong-steps", "5", "--strong-scene", "sponza",
           "--strong-size", "320x240x4", "--detail-out", str(tmp_path / "detail.json"),
           "--bvh-cache", str(tmp_path / "cache")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=420, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and line["value"] > 0
    st = line["strong_scaling"]
    assert st["gathered_equals_single_gpu"] is True
    assert line["config"]["schedule"] and line["config"]["schedule"] == st["schedule_name"]
