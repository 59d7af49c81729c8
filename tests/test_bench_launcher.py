"""bench.py's multi-GPU launcher (CPU): `python bench.py --gpus N` without torchrun starts N rank processes
itself, before the parent touches a GPU, and fails when fewer than N GPUs are visible.  The workers here are
a stub that joins a gloo group and reports its rank and shard offset (the bench's env partition); the real
ranks run the same `launch_workers` with bench.py as the script."""

import json
import os
import subprocess
import sys
import textwrap

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

STUB = textwrap.dedent("""
    import json, os, sys
    sys.path.insert(0, {repo!r})
    import torch, torch.distributed as dist
    import bench
    assert bench.launch_mode(int(sys.argv[sys.argv.index("--gpus") + 1]), os.environ) == "rank"
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = torch.tensor([rank, int(os.environ["LOCAL_RANK"]), bench.shard_offset(rank, 4096)])
    got = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(got, mine)
    if rank == 0:
        print(json.dumps({{"world": world, "rows": [g.tolist() for g in got]}}), flush=True)
    dist.destroy_process_group()
""")


def test_launch_mode():
    assert bench.launch_mode(1, {}) == "single"  # --gpus 1: this process, no launcher (output unchanged)
    assert bench.launch_mode(2, {}) == "spawn"
    assert bench.launch_mode(8, {"WORLD_SIZE": "8"}) == "rank"  # torchrun's (or the launcher's) ranks
    assert bench.launch_mode(1, {"WORLD_SIZE": "4"}) == "rank"  # torchrun without --gpus
    with pytest.raises(SystemExit):
        bench.launch_mode(2, {"WORLD_SIZE": "4"})
    with pytest.raises(SystemExit):
        bench.launch_mode(0, {})


def test_launch_workers_two_ranks_gloo(tmp_path):
    stub = tmp_path / "stub_worker.py"
    stub.write_text(STUB.format(repo=REPO))
    out = tmp_path / "out.txt"
    with open(out, "w") as f:
        rc = bench.launch_workers(2, ["--gpus", "2"], script=str(stub), check_devices=False, stdout=f, timeout=120)
    assert rc == 0
    lines = [json.loads(x) for x in out.read_text().splitlines() if x.startswith("{")]
    assert len(lines) == 1, "only rank 0 prints"
    assert lines[0]["world"] == 2
    rows = sorted(lines[0]["rows"])
    assert rows == [[0, 0, 0], [1, 1, 4096]], rows  # two distinct ranks, one GPU each, offsets rank * n


def test_launch_workers_failing_rank_fails_the_job(tmp_path):
    stub = tmp_path / "bad_worker.py"
    stub.write_text("import os, sys, time\n"
                    "if os.environ['RANK'] == '1': sys.exit(3)\n"
                    "time.sleep(60)\n")
    rc = bench.launch_workers(2, [], script=str(stub), check_devices=False, stdout=subprocess.DEVNULL, timeout=120)
    assert rc == 3  # rank 1's status; rank 0 was stopped rather than waited out


def test_gpus_beyond_visible_devices_fail_before_any_rank_starts():
    """this container has no GPU: --gpus 2 must exit non-zero without a silent one-rank line"""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, cwd=REPO,
                       env=dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""))
    assert r.returncode != 0
    assert r.stdout.strip() == "", r.stdout
    assert "needs 2 GPUs" in r.stderr


def test_launcher_stdout_passthrough_unbuffered(tmp_path):
    """a rank's stdout reaches the launcher's (the one JSON line of rank 0)"""
    stub = tmp_path / "echo_worker.py"
    stub.write_text("import os\nprint('rank', os.environ['RANK'], os.environ['MASTER_ADDR'])\n")
    buf = tmp_path / "o.txt"
    with open(buf, "w") as f:
        assert bench.launch_workers(2, [], script=str(stub), check_devices=False, stdout=f, timeout=60) == 0
    got = sorted(buf.read_text().split("\n")[:-1])
    assert got == ["rank 0 127.0.0.1", "rank 1 127.0.0.1"]

