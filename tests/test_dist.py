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


def _rank_gather(rank, world, port, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import torch.distributed as dist
    import cases
    from kyverno_amd import engine as E
    from kyverno_amd import scan as SC
    from kyverno_amd import synth
    dist.init_process_group("gloo", rank=rank, world_size=world)
    docs, nsl = synth.mixed(701, seed=77, edge=True)
    cut = 350
    mine = docs[:cut] if rank == 0 else docs[cut:]
    rs = E.Ruleset(cases.best_practices() + cases.quirk_policies())
    res = E.evaluate(rs, E.Batch(rs, mine, nsl), backend="cpu")
    full, offs = SC.gather_verdicts(res.status)
    fails = SC.gather_failures(res.failures(), offs[rank])
    tot = SC.reduce_summary(np.array([[res.counts["fail"]]], dtype=np.int64))
    q.put((rank, full, offs, fails, int(tot[0, 0])))
    dist.destroy_process_group()


def test_two_rank_verdict_and_failure_gather():
    """SURVEY §8(e) collectives on gloo (world_size 2, uneven shards): the gathered verdict matrix and failing-path
    records equal a single-process evaluation of the whole corpus"""
    import numpy as np
    sys.path.insert(0, ROOT)
    import cases
    from kyverno_amd import engine as E
    from kyverno_amd import synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_gather, args=(i, 2, port, q)) for i in range(2)]
    for p in ps:
        p.start()
    out = sorted((q.get(timeout=240) for _ in ps), key=lambda x: x[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    docs, nsl = synth.mixed(701, seed=77, edge=True)
    rs = E.Ruleset(cases.best_practices() + cases.quirk_policies())
    ref = E.evaluate(rs, E.Batch(rs, docs, nsl), backend="cpu")
    for rank, full, offs, fails, tot in out:
        assert offs == [0, 350]
        assert np.array_equal(full, ref.status)
        assert tot == ref.counts["fail"]
        rf = ref.failures()
        want = sorted(zip(rf["res"].tolist(), rf["rule"].tolist(), rf["alt"].tolist(), rf["path_template"].tolist(),
                          map(tuple, rf["idx"].tolist())))
        got = sorted((int(r[0]), int(r[1]), int(r[2]), int(r[3]), tuple(int(x) for x in r[4:8])) for r in fails)
        assert got == want and len(got) > 50


def test_bench_spawns_ranks_for_gpus_flag():
    """`bench.py --gpus 2` without a launcher starts its own two ranks before any GPU call; with no GPU here both
    ranks fail in the device evaluation, which the parent must report through its exit code"""
    import subprocess
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--resources", "200",
                        "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-e2e"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert r.stderr.count("rank 0:") >= 1 and r.stderr.count("rank 1:") >= 1, r.stderr[-2000:]
    assert "no HIP device" in r.stderr


def _rank_device(rank, world, port, q):
    """one rank of `bench.py --gpus 2`: its evaluations must name its own LOCAL_RANK device ordinal in kyv_eval_opts
    (the library's kyv_eval is replaced by a recorder here: no GPU in this container)"""
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bench
    import cases
    from kyverno_amd import _lib as K
    from kyverno_amd import engine as E
    from kyverno_amd import synth
    r, w, local, pg = bench.dist_setup(world)
    rs = E.Ruleset(cases.best_practices()[:2])
    b = E.Batch(rs, synth.mixed(20, seed=r)[0])
    seen = []
    L = K.lib()

    def fake_eval(rsh, bh, opts, out):
        o = opts._obj  # the EvalOpts behind ctypes.byref
        seen.append((o.backend, o.device))
        return 7  # an error code: nothing to evaluate without a GPU

    real = L.kyv_eval
    L.kyv_eval = fake_eval
    try:
        E.evaluate(rs, b, backend="gpu", device=local)
    except K.KyvError:
        pass
    finally:
        L.kyv_eval = real
    q.put((rank, local, seen))
    pg.destroy_process_group()


def test_ranks_evaluate_on_their_local_rank_device():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_device, args=(i, 2, port, q)) for i in range(2)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    from kyverno_amd import _lib as K
    for rank, local, seen in out:
        assert local == rank
        assert seen == [(K.BACKEND_GPU, rank)]
