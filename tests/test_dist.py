"""World-size-2 gloo test of the multi-process path on CPU: source sharding per rank, barrier and the
max/sum reductions bench.py uses.  The per-rank engine here is the oracle (CPU); on the GPU box the
same harness drives libhgx."""
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = textwrap.dedent("""
    import json, os, sys
    sys.path[:0] = [{root!r}, {oracle!r}]
    import numpy as np
    from hypergraphdb_amd import dist as hdist, synth
    from oracle_ctypes import OracleGraph
    ctx = hdist.init_from_env("gloo")
    g = synth.config2(scale=0.0005, n_sources=32)
    seeds = hdist.rank_sources(g, 32, ctx.rank)
    orc = OracleGraph(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
    counts, trav = orc.bfs_many(seeds, 3, 4, nthreads=1)
    ctx.barrier()
    tot = ctx.sum(float(trav.sum()))
    mx = ctx.max(float(ctx.rank + 1))
    out = dict(rank=ctx.rank, seeds=seeds.tolist(), trav=float(trav.sum()), tot=tot, mx=mx)
    with open(os.path.join({tmp!r}, f"rank{{ctx.rank}}.json"), "w") as f:
        json.dump(out, f)
    ctx.close()
""")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gloo_sharding(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT, oracle=os.path.join(ROOT, "oracle"), tmp=str(tmp_path)))
    port = free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env))
    for p in procs:
        assert p.wait(timeout=300) == 0
    import json
    res = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(2)]
    # disjoint source draws per rank (weak scaling), same totals seen by both ranks
    assert res[0]["seeds"] != res[1]["seeds"]
    assert res[0]["tot"] == res[1]["tot"] == res[0]["trav"] + res[1]["trav"]
    assert res[0]["mx"] == res[1]["mx"] == 2.0
    # rank 0's batch is the config's own source draw
    sys.path[:0] = [ROOT]
    from hypergraphdb_amd import synth
    g = synth.config2(scale=0.0005, n_sources=32)
    assert res[0]["seeds"] == g["seeds"].tolist()


def test_bench_launches_its_ranks():
    """`bench.py --gpus N` starts N ranks itself (one process per GPU) when not run under
    torch.distributed.run; --dry-run joins the group without touching a GPU."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["ranks_joined"] == 2
    # under a launcher, a world size that disagrees with --gpus is an error, not a silent 1-GPU run
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"],
                       env=dict(env, WORLD_SIZE="3", RANK="0"), capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr
