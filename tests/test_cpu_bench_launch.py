"""bench.py's rank launcher (`python bench.py --gpus N` without torchrun, VERDICT r03
missing #1): N child processes get the torchrun environment (RANK, LOCAL_RANK,
WORLD_SIZE, MASTER_*), rendezvous over gloo on 127.0.0.1, and a failing rank ends the
job with its exit code instead of leaving the others hanging."""
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHILD = textwrap.dedent("""
    import os, sys, torch, torch.distributed as dist
    dist.init_process_group("gloo")
    r, w = dist.get_rank(), dist.get_world_size()
    assert r == int(os.environ["LOCAL_RANK"]) and w == int(sys.argv[1])
    t = torch.tensor([float(r + 1)])
    dist.all_reduce(t)
    if sys.argv[2] == "fail" and r == 1:
        sys.exit(7)
    if sys.argv[2] == "fail":
        dist.barrier()  # rank 1 never arrives: the launcher must end this rank
    if r == 0:
        print("n_gpus", w, "sum", int(t))
    dist.destroy_process_group()
""")


def _run(tmp_path, n, mode):
    child = tmp_path / "child.py"
    child.write_text(CHILD)
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.spawn_ranks(%d, %r, [%r, %r]))" % (ROOT, n, str(child), str(n), mode))
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                          env={k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE")})


def test_spawn_ranks_world2(tmp_path):
    r = _run(tmp_path, 2, "ok")
    assert r.returncode == 0, r.stderr
    assert "n_gpus 2 sum 3" in r.stdout


def test_spawn_ranks_world4(tmp_path):
    r = _run(tmp_path, 4, "ok")
    assert r.returncode == 0, r.stderr
    assert "n_gpus 4 sum 10" in r.stdout


def test_spawn_ranks_failing_rank_ends_job(tmp_path):
    r = _run(tmp_path, 2, "fail")
    assert r.returncode == 7


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
