"""Multi-GPU assembly from device-resident results: gather_verdicts_device / gather_failures_device
all-gather over RCCL what kyv_batch_export_status / kyv_batch_export_failures write straight from the batch's resident
verdicts and failing-path records into torch device tensors. On the one-GPU box the group is a world_size-1 RCCL
group; the wire format, the input-order permutation and the offsets are checked against the host copies of the same
evaluation. (Ranks > 1 run only on the driver's 8-GPU node; the gloo tests in test_dist.py cover the host gathers.)"""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys
import torch  # before the library: one HIP runtime shared with torch / RCCL (kyverno_amd/_lib.py)
import torch.distributed as dist
sys.path.insert(0, os.environ["ROOT"]); sys.path.insert(0, os.path.join(os.environ["ROOT"], "tests"))
import numpy as np
import cases
from kyverno_amd import engine as E, scan as SC, synth
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
docs, nsl = synth.mixed(3001, seed=91, edge=True)
rs = E.Ruleset(cases.best_practices() + cases.quirk_policies())
b = E.Batch(rs, docs, nsl)
res = E.evaluate(rs, b, backend="gpu", device=0)
full, offs = SC.gather_verdicts_device(b, device="cuda:0")
assert offs == [0], offs
assert full.shape == res.status.shape, (full.shape, res.status.shape)
assert np.array_equal(full, np.asarray(res.status) & 7)
t, _ = SC.gather_verdicts_device(b, device="cuda:0", tensor=True)
assert t.is_cuda and t.dtype == torch.uint8
rows = SC.gather_failures_device(b, 1000, device="cuda:0")
f = res.failures()
want = sorted(zip((f["res"].astype(np.int64) + 1000).tolist(), f["rule"].tolist(), f["alt"].tolist(),
                  f["path_template"].tolist(), map(tuple, f["idx"].tolist())))
# rows come back in (resource, rule, alternative) order, as the host-array gather returns them
got = [(int(r[0]), int(r[1]), int(r[2]), int(r[3]), tuple(int(x) for x in r[4:8])) for r in rows]
assert got == want and len(got) > 100, (len(got), len(want))
dist.destroy_process_group()
print("gather ok", full.shape, len(got))
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_device_resident_gather_rccl():
    env = dict(os.environ, ROOT=ROOT, KYV_TORCH_FIRST="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "gather ok" in r.stdout


NATIVE = r"""
import os, sys
sys.path.insert(0, os.environ["ROOT"]); sys.path.insert(0, os.path.join(os.environ["ROOT"], "tests"))
import numpy as np
import cases
from kyverno_amd import engine as E, scan as SC, synth
docs, nsl = synth.mixed(3001, seed=92, edge=True)
# rows that do not fit 16 bytes travel as side entries: a failing path through container index >= 255
wide = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "wide", "namespace": "default"},
        "spec": {"containers": [{"name": "c%d" % i, "image": "nginx:1.%d" % i} for i in range(300)]}}
wide["spec"]["containers"][290]["image"] = "nginx:latest"
docs.insert(17, wide)
rs = E.Ruleset(cases.best_practices() + cases.quirk_policies())
b = E.Batch(rs, docs, nsl)
comm = SC.Comm(SC.Comm.unique_id(), 1, 0, 0)
# before any evaluation of the batch: every collective returns an error (flag exchange) instead of hanging
for call in (lambda: comm.reduce_counts(b), lambda: comm.gather_report(b, 1000, root=0)):
    try:
        call()
        raise AssertionError("a gather without resident results succeeded")
    except SC.K.KyvError as e:
        assert "rank 0" in str(e), str(e)
res = E.evaluate(rs, b, backend="gpu", device=0)
st = comm.gather(b, 1000)
st = comm.gather(b, 1000)  # a second gather reuses the communicator's buffers
assert st["status_ms"] > 0 and st["status_bytes_per_rank"] == len(rs.rules) * ((b.n + 1) // 2), st
packed = comm.status_of(0)
assert np.array_equal(packed, SC.pack_status(np.asarray(res.status))), "gathered verdicts differ"
rows = comm.failures_of(0)
f = res.failures()
want = sorted(zip((f["res"].astype(np.int64) + 1000).tolist(), f["rule"].tolist(), f["alt"].tolist(),
                  f["path_template"].tolist(), map(tuple, f["idx"].tolist())))
got = sorted((int(r[0]), int(r[1]), int(r[2]), int(r[3]), tuple(int(x) for x in r[4:8])) for r in rows)
assert got == want and len(got) > 100 and st["failure_rows_total"] == len(got), (len(got), len(want), st)
# report assembly to one consumer rank: 16-byte rows on the wire, expanded on the root to the same rows
st2 = comm.gather_report(b, 1000, root=0)
assert np.array_equal(comm.status_of(0)[:packed.size], packed), "reported verdicts differ"
got2 = sorted((int(r[0]), int(r[1]), int(r[2]), int(r[3]), tuple(int(x) for x in r[4:8])) for r in comm.failures_of(0))
assert got2 == want and st2["failure_rows_total"] == len(want), (len(got2), st2)
assert any(r[0] == 1000 + 17 and max(r[4]) >= 255 and max(r[4]) != 0xFFFF for r in got2), "no side-entry row"
# the per-rule tallies summed over ranks (one rank here): the evaluation's own counts
tot = comm.reduce_counts(b)
assert np.array_equal(tot, np.asarray(res.rule_counts)), "reduced tallies differ"
# a rule-sliced evaluation keeps every slice's failing-path rows resident (no copy-back), in the rows of the
# copy-back evaluation of the same batch
os.environ["KYV_SLICE_MB"] = "1"
rs2 = E.Ruleset(cases.best_practices() + cases.quirk_policies())
b2 = E.Batch(rs2, docs, nsl)
ref = E.evaluate(rs2, b2, backend="gpu", device=0)
f2 = ref.failures()
want2 = sorted(zip((f2["res"].astype(np.int64) + 1000).tolist(), f2["rule"].tolist(), f2["alt"].tolist(),
                   f2["path_template"].tolist(), map(tuple, f2["idx"].tolist())))
assert sorted(want2) == sorted(want), "sliced evaluation rows differ from the one-slice evaluation"
comm.gather_report(b2, 1000, root=0)  # rows of the copy-back evaluation (host copy of its slices)
got3 = sorted((int(r[0]), int(r[1]), int(r[2]), int(r[3]), tuple(int(x) for x in r[4:8])) for r in comm.failures_of(0))
assert got3 == want2, (len(got3), len(want2))
E.evaluate(rs2, b2, backend="gpu", device=0, copy_back=False)  # resident rows
comm.gather_report(b2, 1000, root=0)
got4 = sorted((int(r[0]), int(r[1]), int(r[2]), int(r[3]), tuple(int(x) for x in r[4:8])) for r in comm.failures_of(0))
assert got4 == want2, (len(got4), len(want2))
comm.close()
print("native gather ok", packed.size, len(got), st, st2)
"""


@pytest.mark.gpu
def test_native_rccl_gather():
    """the library's own RCCL communicator (kyv_comm_*): no torch in the process; a one-rank group on this box"""
    env = dict(os.environ, ROOT=ROOT)
    r = subprocess.run([sys.executable, "-c", NATIVE], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "native gather ok" in r.stdout
