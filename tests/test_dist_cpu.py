"""N>1 path of bench.py on the CPU (gloo, world_size 2): the replica plumbing -- rank setup,
per-rank camera pose (C5: main pose + rotateRight(45 deg * rank)), barrier and max-over-ranks
timing.  No data-path collective exists to test (replicas only)."""
import os
import socket

import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    w, r, local, pg = bench.dist_setup()
    u = bench.camera_for_rank(1920, 1080, r).uniforms()
    bench.barrier(pg)
    mx = bench.max_over_ranks(pg, 1.0 + r)
    sm = bench.sum_over_ranks(pg, 1.0)
    q.put((r, w, local, mx, sm, list(u.view)))
    pg.destroy_process_group()


def test_two_rank_replicas():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, w0, l0, m0, s0, v0), (r1, w1, l1, m1, s1, v1) = res
    assert (r0, r1) == (0, 1) and w0 == w1 == 2 and (l0, l1) == (0, 1)
    assert m0 == m1 == 2.0 and s0 == s1 == 2.0   # max / sum over ranks
    assert v0 != v1                               # each rank renders its own view


def test_single_rank_defaults(monkeypatch):
    import bench
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    w, r, local, pg = bench.dist_setup()
    assert (w, r, local, pg) == (1, 0, 0, None)
    assert bench.max_over_ranks(None, 3.5) == 3.5


def test_gpus_flag_spawns_ranks():
    """`bench.py --gpus N` with no launcher environment starts N rank processes itself (the
    parent makes no GPU call); rank 0 prints one line with every rank's view (dry run: the
    plumbing only, no GPU)"""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "3", "--dry-run"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1, r.stdout  # the JSON line alone (gloo's connection lines go to stderr)
    d = json.loads(lines[0])
    assert d["dry_run"] and d["n_gpus"] == 3 and d["max_over_ranks"] == 3.0
    assert [x["rank"] for x in d["ranks"]] == [0, 1, 2] and [x["view"] for x in d["ranks"]] == [0, 1, 2]
    assert len({tuple(x["view_matrix"]) for x in d["ranks"]}) == 3  # each rank its own pose


def test_torchrun_launch_prints_one_line():
    """the driver's N > 1 launch: `torch.distributed.run --nproc-per-node N bench.py --gpus N`
    (dry run); stdout is rank 0's JSON line and nothing else"""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and [x["view"] for x in d["ranks"]] == [0, 1]


def test_failing_rank_ends_the_spawn():
    """a rank that fails makes `bench.py --gpus N` exit non-zero (the others are ended)"""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    env["GS_BENCH_DRYRUN_FAIL_RANK"] = "1"  # rank 1 exits before the rendezvous; rank 0 would wait
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 3
