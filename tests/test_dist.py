"""Multi-rank path of bench.py on CPU (gloo, world_size 2): each rank evaluates its own shard, the only
cross-rank traffic is the barrier and the max/sum of timings and pair counts (no data-path collective)."""
import os
import socket
import sys

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bench
    import cases
    from kyverno_amd import engine as E
    from kyverno_amd import synth
    r, w, local, pg = bench.dist_setup(world)
    data, nsl = synth.corpus_ndjson(300, seed=bench.SEED + r, workers=1)
    rs = E.Ruleset(cases.best_practices())
    b = E.Batch(rs, data, nsl)
    res = E.evaluate(rs, b, backend="cpu")  # explicit CPU instantiation: no GPU in this container
    bench.barrier(pg)
    pairs = bench.all_sum(pg, len(rs.rules) * b.n)
    tmax = bench.all_max(pg, float(r + 1))
    applicable = bench.all_sum(pg, res.counts["pass"] + res.counts["fail"])
    q.put((r, pairs, tmax, applicable, res.counts["pass"] + res.counts["fail"], len(rs.rules) * b.n))
    pg.destroy_process_group()


def test_two_rank_shards():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(i, 2, port, q)) for i in range(2)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    (r0, pairs0, t0, app0, mine0, n0), (r1, pairs1, t1, app1, mine1, n1) = out
    assert pairs0 == pairs1 == n0 + n1
    assert t0 == t1 == 2.0
    assert app0 == app1 == mine0 + mine1
