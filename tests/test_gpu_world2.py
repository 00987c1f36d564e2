"""World > 1 on real HIP shards (one-GPU box): two rank processes on GPU 0,
torch.distributed over gloo (RCCL refuses two ranks on one device; the
8-GPU node runs the same code over RCCL).  Covers what the CPU gloo tests
cannot: ShardedIndexFlat with libvsearch shards — raw per-shard 2k-1 lists
(the paged search past k = 32, k up to 300), the all-gather and vs_merge_topk over two
parts on the GPU, removals/appends across shards, a search on a stream other than torch's
current one (tests/gpu_world_worker.py)
— and bench.py's own N = 2 paths: the row-sharded search with its live
exact check, and C4's split-and-gather of the writer's rows to rank 0
(graph_refresher/main.py:339-389).

The ranks are separate processes started before either touches HIP (as
bench.py's launch_ranks does), each with a time limit of its own."""

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(argv, world, timeout, extra_env=None):
    port = _port()
    procs = []
    for r in range(world):
        env = {k: v for k, v in os.environ.items()
               if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(world),
                    "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port)})
        env.update(extra_env or {})
        procs.append(subprocess.Popen(["timeout", "-k", "10", str(timeout), sys.executable, "-u"]
                                      + argv, env=env, cwd=ROOT, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate() for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, (p.returncode, o[-2000:], e[-4000:])
    lines = [l for l in outs[0][0].splitlines() if l.startswith("{")]
    assert len(lines) == 1, outs[0][0][-2000:]
    return json.loads(lines[0])


def test_sharded_world2_real_shards_match_oracle():
    res = _run_ranks([os.path.join(ROOT, "tests", "gpu_world_worker.py")], 2, 100)
    bad = [k for k, v in res.items() if not v]
    assert not bad, bad
    assert len(res) == 2 * (1 + 1 + 14 + 1 + 3 + 3 + 1)


_BENCH_ENV = {"VS_BENCH_BACKEND": "gloo", "VS_BENCH_DEVICE": "0"}


def test_bench_world2_knn_on_one_gpu():
    """bench.py's row-sharded C2-shaped step at N = 2 (reduced corpus): the
    merged lists pass the live fp32-engine check with no id beyond the tie
    tolerance, and rank 0 reports the world the collective saw."""
    res = _run_ranks([os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "c2",
                      "--ntotal", "200000", "--batch", "1024", "--steps", "2", "--warmup", "1",
                      "--batch1-steps", "0", "--wide-k-steps", "2", "--no-cpu-baseline"],
                     2, 100, _BENCH_ENV)
    assert res["n_gpus"] == 2 and res["ranks_seen"] == 2
    assert res["result_sane"] is True
    ec = res["filter_verify"]["exact_check"]
    assert ec["queries"] == 256 and ec["rows_beyond_tie_tolerance"] == 0
    assert res["wide_k"] and all(w["result_sane"] is True for w in res["wide_k"])


def test_bench_world2_selfjoin_split_and_gather():
    """C4 at N = 2 (reduced): each rank self-joins its block of students over
    the replicated corpus; the rows are gathered to rank 0 (the writer)."""
    res = _run_ranks([os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "c4",
                      "--ntotal", "60000", "--steps", "2", "--warmup", "1"], 2, 100, _BENCH_ENV)
    assert res["n_gpus"] == 2 and res["result_sane"] is True
    assert res["writer"]["rows_gathered_on_rank0"] == 60000
    assert res["writer"]["edges_total"] == 60000 * 50
    ec = res["filter_verify"]["exact_check"]
    assert ec["rows_beyond_tie_tolerance"] == 0
