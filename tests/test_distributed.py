"""N>1 path of bench.py on CPU: world_size-2 gloo over 127.0.0.1.

The path shards (independent QP instances): every rank draws its own shard of the batch, solves
it with no data-path collective, and the only exchanges are the barrier and the MAX over ranks
of the wall time (gloo, host tensors).  The test runs bench.run -- the very control flow the
driver launches with torch.distributed.run -- with the library's CPU QP path as the backend
(--backend cpu); on a GPU box the same flow drives the HIP kernels."""
import json
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from conftest import REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, argv):
    import sys
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS="2")
    import bench
    out = bench.run(bench.parse_args(argv))
    goals = [[30, 1.5, 0, 0], [29.9, -1.5, 0, 0], [30, 1.5, 0, 0]]
    X, env, offsets = bench.sample_shard(rank, 240, goals)
    q.put((rank, out, X[:3].copy(), env.tolist(), offsets.tolist()))


def _run_world(world, argv):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, argv)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=400) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_bench_two_rank_flow_gloo():
    argv = ["--gpus", "2", "--steps", "2", "--warmup", "1", "--backend", "cpu", "--per-gpu", "240", "--cpu-threads", "2",
            "--cpu-sample", "96"]
    (r0, out0, x0, e0, o0), (r1, out1, x1, e1, o1) = _run_world(2, argv)
    assert out1 is None and out0 is not None            # rank 0 alone reports
    json.dumps(out0)                                    # one JSON-serialisable line
    assert out0["n_gpus"] == 2 and out0["steps"] == 2 and out0["warmup"] == 1 and out0["scaling"] == "weak"
    assert out0["config"]["global_batch"] == 480 and out0["config"]["per_gpu_batch"] == 240
    # value = instances of all ranks / max-over-ranks wall time
    assert abs(out0["value"] - 480 * 2 / (out0["ms_per_step"] * 2e-3)) <= 1e-3 * out0["value"]
    ss = out0["status_split"]
    assert sum(ss.values()) == 240 and ss["max_iter"] == 0 and ss["numerical"] == 0 and ss["optimal"] > 100
    # the CPU baseline and the iteration reference come from the oracle on rank 0 at any world size
    cb = out0["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["single_thread"]["value"] > 0 and cb["cpu_model"]
    assert cb["product_cpu_path"]["value"] > 0
    assert not np.allclose(x0, x1)                      # independent shards
    assert e0 == sorted(e0) and e1 == sorted(e1)        # grouped by environment
    assert o0[-1] == 240 and o1[-1] == 240


def test_bench_single_rank_config4_flow_on_cpu():
    """The OutputFB workload (observer + QP) through the same flow, one rank."""
    import bench
    out = bench.run(bench.parse_args(["--steps", "1", "--warmup", "0", "--backend", "cpu", "--workload", "config4",
                                      "--per-gpu", "96", "--cpu-threads", "2", "--cpu-sample", "48"]))
    assert out["config"]["workload"].startswith("config4") and out["config"]["step"].startswith("observer")
    assert sum(out["status_split"].values()) == 96 and out["status_split"]["optimal"] > 10


def _plain_env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    return env


def test_bench_starts_its_own_ranks_from_a_plain_shell():
    """`python bench.py --gpus 2` without a launcher: the script starts two ranks itself and relays
    rank 0's line, so the line's n_gpus is the number of ranks that ran."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "cpu", "--steps", "1",
                        "--warmup", "0", "--per-gpu", "120", "--cpu-threads", "2", "--no-cpu"],
                       env=_plain_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 240 and out["config"]["parallelism"].startswith("shard2")


def test_bench_refuses_a_world_size_that_differs_from_gpus():
    """A launcher that starts one rank while the command line says --gpus 2 (or the reverse) must not
    produce a line."""
    import subprocess
    import sys
    env = _plain_env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "cpu", "--steps", "1",
                        "--warmup", "0", "--per-gpu", "60", "--no-cpu"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and r.stdout.strip() == "" and "WORLD_SIZE" in r.stderr
