"""Batched background scan: report results and summaries for a batch of resources.

The reference reconciles one resource at a time (pkg/controllers/report/background/controller.go:250-361): for
each background policy `scanner.ScanResource` builds a JSON context and calls `engine.Validate`
(pkg/controllers/report/utils/scanner.go:60-110); every EngineResponse becomes report rows
(`EngineResponseToReportResults`, pkg/utils/report/results.go:84-124) and the report carries `CalculateSummary`
(results.go:38-54). Here a whole batch goes through one `kyv_eval`; the per-policy summary is assembled from the
device's per-rule verdict totals (`kyv_results_rule_counts`), so rows are only materialised on request.

Multi-GPU: each rank scans its own contiguous shard; the collectives only assemble results, over the
process group (RCCL with the "nccl" backend on device tensors, gloo on CPU):
  reduce_summary   all-reduce (sum) of the per-policy summaries;
  gather_verdicts  all-gather of every rank's verdict matrix, two pairs per byte (status values are 3-bit);
  gather_failures  count-then-gather of the compacted failing-path records.

With a GPU evaluation the collectives read the rank's device-resident results (gather_verdicts_device /
gather_failures_device: the library writes the wire form straight into a torch device tensor on the current stream,
kyv_batch_export_status / kyv_batch_export_failures), so the verdicts never pass through host memory on the way to
RCCL. Load torch before the library in such a process (KYV_TORCH_FIRST=1, see _lib.py).

Pairs outside the device subset (KYV_ST_FALLBACK, PANIC, ND) are listed by `fallback_pairs()`: the Go shim
evaluates exactly those with the reference engine; they are counted as `cpu_fallback`, not in pass/fail/....
"""
import ctypes

import numpy as np

from . import _lib as K
from . import engine as E

SUMMARY_FIELDS = ("pass", "fail", "warn", "error", "skip", "cpu_fallback")


def policy_key(pol):
    """cache.MetaNamespaceKeyFunc: "<namespace>/<name>" for namespaced policies, "<name>" otherwise"""
    md = pol.get("metadata") or {}
    ns = md.get("namespace") or ""
    return ns + "/" + md.get("name", "") if ns else md.get("name", "")


class BackgroundScan:
    """Background scan over batches: policies compiled once (background: false policies are not scanned)."""

    def __init__(self, policies, backend="gpu", device=0):
        self.policies = [p for p in policies if isinstance(p, dict) and p.get("kind") in ("ClusterPolicy", "Policy")
                         and (p.get("spec") or {}).get("background", True) is not False]
        self.ruleset = E.Ruleset(self.policies, background=True)
        self.backend, self.device = backend, device
        self.meta = []
        # keyed like the policy cache (namespace, name): namespaced Policies may share a name across namespaces
        by_key = {((p.get("metadata") or {}).get("namespace") or "" if p.get("kind") == "Policy" else "",
                   (p.get("metadata") or {}).get("name")): p for p in self.policies}
        for pm in self.ruleset.policies:
            pol = by_key.get((pm["namespace"], pm["name"])) or {}
            ann = (pol.get("metadata") or {}).get("annotations") or {}
            sev = ann.get("policies.kyverno.io/severity", "")
            self.meta.append({
                "key": policy_key(pol) if pol else pm["name"],
                "scored": ann.get("policies.kyverno.io/scored") != "false",
                "category": ann.get("policies.kyverno.io/category", ""),
                "severity": sev if sev in ("high", "medium", "low") else "",
                "apply_one": pm["apply_one"], "first_rule": pm["first_rule"], "nrules": pm["nrules"],
            })

    def scan(self, resources, ns_labels=None):
        batch = E.Batch(self.ruleset, resources, ns_labels)
        res = E.evaluate(self.ruleset, batch, backend=self.backend, device=self.device)
        return ScanReport(self, batch, res)


class ScanReport:
    def __init__(self, scan, batch, res):
        self.scan, self.batch, self.res = scan, batch, res

    def summary_matrix(self):
        """int64 [policies, 6]: SUMMARY_FIELDS per policy over the batch (CalculateSummary of its report rows)."""
        out = np.zeros((len(self.scan.meta), len(SUMMARY_FIELDS)), dtype=np.int64)
        rc, st = self.res.rule_counts, self.res.status
        for pi, m in enumerate(self.scan.meta):
            ks = range(m["first_rule"], m["first_rule"] + m["nrules"])
            fail_col = 1 if m["scored"] else 2  # fail on an unscored policy is reported as warn (results.go:117-119)
            if not m["apply_one"]:
                for k in ks:
                    c = rc[k]
                    out[pi, 0] += c[K.ST_PASS]
                    out[pi, fail_col] += c[K.ST_FAIL]
                    out[pi, 3] += c[K.ST_ERROR]
                    out[pi, 4] += c[K.ST_SKIP]
                    out[pi, 5] += c[K.ST_FALLBACK] + c[K.ST_PANIC] + c[K.ST_ND]
                continue
            # applyRules: One (validation.go:176-178): rules after the first applied (pass / fail) one give no
            # response; after a CPU-fallback rule the truncation point is the CPU engine's to decide
            active = np.ones(st.shape[1], dtype=bool)
            for k in ks:
                s = st[k]
                m_ = active & (s != K.ST_NONE)
                out[pi, 0] += int(np.count_nonzero(m_ & (s == K.ST_PASS)))
                out[pi, fail_col] += int(np.count_nonzero(m_ & (s == K.ST_FAIL)))
                out[pi, 3] += int(np.count_nonzero(m_ & (s == K.ST_ERROR)))
                out[pi, 4] += int(np.count_nonzero(m_ & (s == K.ST_SKIP)))
                cpu = m_ & ((s == K.ST_FALLBACK) | (s == K.ST_PANIC) | (s == K.ST_ND))
                out[pi, 5] += int(np.count_nonzero(cpu))
                active &= ~((s == K.ST_PASS) | (s == K.ST_FAIL) | cpu)
        return out

    def summary(self):
        mat = self.summary_matrix()
        return {m["key"]: dict(zip(SUMMARY_FIELDS, map(int, mat[i]))) for i, m in enumerate(self.scan.meta)}

    def results(self, i):
        """report rows (EngineResponseToReportResults) of resource i over every scanned policy"""
        rows = []
        st = self.res.status
        rules = self.scan.ruleset.rules
        for m in self.scan.meta:
            applied = 0
            for k in range(m["first_rule"], m["first_rule"] + m["nrules"]):
                s = int(st[k, i])
                if s == K.ST_NONE:
                    continue
                if s in (K.ST_FALLBACK, K.ST_PANIC, K.ST_ND):
                    rows.append({"policy": m["key"], "rule": rules[k]["name"], "result": None, "cpu_fallback": True})
                    if m["apply_one"]:
                        break
                    continue
                result = {K.ST_PASS: "pass", K.ST_FAIL: "fail", K.ST_ERROR: "error", K.ST_SKIP: "skip"}[s]
                if result == "fail" and not m["scored"]:
                    result = "warn"
                row = {"source": "kyverno", "policy": m["key"], "rule": rules[k]["name"], "result": result,
                       "message": self.res.message(i, k), "scored": m["scored"], "category": m["category"],
                       "severity": m["severity"]}
                if rules[k]["kind"] == "podSecurity":
                    row["pss_mask"] = self.res.pss_mask(i, k)
                    # results.go:102-116: properties of the failed PodSecurity checks (IDs sorted, one per failing
                    # check version, joined with ","); None when the library cannot render the checks (exclusions
                    # in Go-map order): the CPU engine builds that row
                    chk = self.res.pss_checks(i, k)
                    if chk is None:
                        row["properties"] = None
                    else:
                        controls = sorted(c["id"] for c in chk["checks"] if not c["allowed"])
                        if controls:
                            row["properties"] = {"standard": chk["level"], "version": chk["version"],
                                                 "controls": ",".join(controls)}
                rows.append(row)
                if s in (K.ST_PASS, K.ST_FAIL):
                    applied += 1
                if m["apply_one"] and applied > 0:
                    break
        return rows

    def fallback_pairs(self):
        """(resource index, policy key, rule name) of every pair the CPU engine must evaluate"""
        st = self.res.status
        out = []
        rule_pol = {}
        for m in self.scan.meta:
            for k in range(m["first_rule"], m["first_rule"] + m["nrules"]):
                rule_pol[k] = m["key"]
        ks, rs = np.nonzero((st == K.ST_FALLBACK) | (st == K.ST_PANIC) | (st == K.ST_ND))
        for k, r in zip(ks.tolist(), rs.tolist()):
            out.append((r, rule_pol.get(k), self.scan.ruleset.rules[k]["name"]))
        return sorted(out)


def reduce_summary(matrix, group=None, device=None):
    """Sum per-policy summaries over the ranks of a torch.distributed group (RCCL all-reduce on GPU tensors with the
    "nccl" backend; gloo on CPU). Every rank must pass the matrix of the same BackgroundScan policies."""
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(matrix, dtype=np.int64))
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t.cpu().numpy()


def _all_gather_var(t, group, dist, torch):
    """all-gather of a tensor whose dim 0 differs per rank: sizes first, then equal-size (padded) tensors"""
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    world = dist.get_world_size(group)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(x.item()) for x in sizes]
    m = max(sizes) if sizes else 0
    pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return [p[:k] for p, k in zip(parts, sizes)], sizes


def gather_verdicts(status, group=None, device=None):
    """All-gather the verdict matrices of every rank's shard: status is this rank's uint8
    [rules, n_rank] (rule-major KYV_ST_* bytes, low 3 bits used); on the wire two pairs share a byte. Returns
    (uint8 [rules, sum n_rank] in rank order, list of each rank's first global resource index)."""
    import torch
    import torch.distributed as dist
    st = torch.from_numpy(np.ascontiguousarray(np.asarray(status) & 7, dtype=np.uint8))
    if device is not None:
        st = st.to(device)
    nr, n = st.shape
    n2 = n + (n & 1)
    buf = torch.zeros((nr, n2), dtype=torch.uint8, device=st.device)
    buf[:, :n] = st
    packed = (buf[:, 0::2] | (buf[:, 1::2] << 4)).t().contiguous()  # [n2 / 2, rules]: ranks differ in dim 0
    parts, sizes = _all_gather_var(packed, group, dist, torch)
    cols, offs, at = [], [], 0
    for p, k in zip(parts, sizes):
        q = p.t()
        full = torch.stack((q & 15, q >> 4), dim=2).reshape(nr, 2 * k)
        cols.append(full)
    counts = torch.tensor([n], dtype=torch.int64, device=st.device)
    world = dist.get_world_size(group)
    ns = [torch.zeros_like(counts) for _ in range(world)]
    dist.all_gather(ns, counts, group=group)
    out = []
    for c, k in zip(cols, ns):
        k = int(k.item())
        out.append(c[:, :k])
        offs.append(at)
        at += k
    return torch.cat(out, dim=1).cpu().numpy(), offs


def _sort_rows(t):
    """failing-path rows in (global resource, rule, alternative) order: the device export writes them in compaction
    order (kind-major by rule and walk chunk), the host path in input order; both gathers return this one order"""
    import torch
    for col in (2, 1, 0):
        t = t[torch.sort(t[:, col], stable=True).indices]
    return t


def gather_failures(failures, res_offset, group=None, device=None):
    """Count-then-gather of the compacted failing-path records (engine.Results.failures()) of every rank: int64 rows
    (global resource index, rule, anyPattern alternative, path template, idx0..3) sorted by (resource, rule,
    alternative). Resolved metadata
    keys are batch-local dictionary ids and stay with the owning rank (which formats those paths)."""
    import torch
    import torch.distributed as dist
    f = np.asarray(failures)
    rows = np.zeros((len(f), 8), dtype=np.int64)
    if len(f):
        rows[:, 0] = f["res"].astype(np.int64) + int(res_offset)
        rows[:, 1] = f["rule"]
        rows[:, 2] = f["alt"]
        rows[:, 3] = f["path_template"]
        rows[:, 4:8] = f["idx"]
    t = torch.from_numpy(rows)
    if device is not None:
        t = t.to(device)
    parts, _ = _all_gather_var(t, group, dist, torch)
    return _sort_rows(torch.cat(parts, dim=0)).cpu().numpy()


def _export_target(device):
    import torch
    dev = torch.device(device if device is not None else "cuda")
    if dev.type != "cuda":
        raise ValueError("device-resident gather needs a GPU device, got %s" % dev)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    return torch.device("cuda", idx), idx, torch.cuda.current_stream(idx).cuda_stream


def _export_check(n):
    if n < 0:
        raise K.KyvError(K.lib().kyv_last_error().decode(errors="replace"))
    return n


def gather_verdicts_device(batch, group=None, device=None, tensor=False):
    """gather_verdicts over the verdicts the batch's last GPU evaluation left on `device` (its kyv_eval device
    ordinal, normally LOCAL_RANK): the library packs them (two per byte, rule-major) into a device tensor, the ranks
    all-gather those (RCCL), and the full matrix is unpacked on the device. Returns (uint8 [rules, sum n_rank] in rank
    order -- a device tensor with tensor=True, else numpy --, list of each rank's first global resource index)."""
    import torch
    import torch.distributed as dist
    dev, idx, stream = _export_target(device)
    L = K.lib()
    total = _export_check(L.kyv_batch_export_status(batch.h, idx, None, 0, None))
    buf = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    _export_check(L.kyv_batch_export_status(batch.h, idx, ctypes.c_void_p(buf.data_ptr()), buf.numel(),
                                            ctypes.c_void_p(stream)))
    nr = len(batch.ruleset.rules)
    parts, _ = _all_gather_var(buf[:total], group, dist, torch)
    counts = torch.tensor([batch.n], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(counts) for _ in range(dist.get_world_size(group))]
    dist.all_gather(ns, counts, group=group)
    cols, offs, at = [], [], 0
    for p, k in zip(parts, ns):
        k = int(k.item())
        h = (k + 1) // 2
        q = p.view(nr, h)
        cols.append(torch.stack((q & 15, q >> 4), dim=2).reshape(nr, 2 * h)[:, :k])
        offs.append(at)
        at += k
    full = torch.cat(cols, dim=1) if cols else torch.zeros((nr, 0), dtype=torch.uint8, device=dev)
    return (full if tensor else full.cpu().numpy()), offs


def local_verdicts_device(batch, device=None, ncols=None):
    """The verdicts the batch's last GPU evaluation left on `device`, without a collective: packed on the device by
    the library (kyv_batch_export_status, input order), the first `ncols` resources unpacked there and copied to the
    host -> uint8 [rules, ncols]. bench.py checks the timed evaluation's own verdicts against the oracle this way."""
    import torch
    dev, idx, stream = _export_target(device)
    L = K.lib()
    total = _export_check(L.kyv_batch_export_status(batch.h, idx, None, 0, None))
    buf = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    _export_check(L.kyv_batch_export_status(batch.h, idx, ctypes.c_void_p(buf.data_ptr()), buf.numel(),
                                            ctypes.c_void_p(stream)))
    nr = len(batch.ruleset.rules)
    n = batch.n if ncols is None else min(int(ncols), batch.n)
    h = (batch.n + 1) // 2
    q = buf[: nr * h].view(nr, h)[:, : (n + 1) // 2]
    out = torch.stack((q & 15, q >> 4), dim=2).reshape(nr, -1)[:, :n]
    return out.cpu().numpy()


def gather_failures_device(batch, res_offset, group=None, device=None, tensor=False):
    """gather_failures over the failing-path records resident on `device`: int64 rows (global resource index, rule,
    alternative, path template, idx0..3) written by the library into a device tensor, then all-gathered (RCCL).
    A rule-sliced evaluation keeps no resident records (the library says so): use gather_failures there."""
    import torch
    import torch.distributed as dist
    dev, idx, stream = _export_target(device)
    L = K.lib()
    n = _export_check(L.kyv_batch_export_failures(batch.h, idx, int(res_offset), None, 0, None))
    t = torch.empty((max(n, 1), 8), dtype=torch.int64, device=dev)
    _export_check(L.kyv_batch_export_failures(batch.h, idx, int(res_offset), ctypes.c_void_p(t.data_ptr()), n,
                                              ctypes.c_void_p(stream)))
    parts, _ = _all_gather_var(t[:n], group, dist, torch)
    full = _sort_rows(torch.cat(parts, dim=0))
    return full if tensor else full.cpu().numpy()


class Comm:
    """The library's own RCCL communicator (kyv_comm_*, include/kyvgpu.h): report assembly of a one-process-per-GPU
    scan with no framework on the device path. Rank 0 draws the id (`Comm.unique_id()`), the caller hands it to the
    other ranks out of band (bench.py: a gloo broadcast), and every rank builds `Comm(id, nranks, rank, device)`.
    `gather(batch, res_offset)` all-gathers the device-resident results of the batch's last GPU evaluation (packed
    verdicts, failing-path rows) into communicator-owned device buffers and returns their HIP-event times."""

    def __init__(self, uid, nranks, rank, device):
        import ctypes
        L = K.lib()
        self._h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(bytes(uid), len(uid))
        K.check(L.kyv_comm_init(buf, len(uid), int(nranks), int(rank), int(device), ctypes.byref(self._h)))
        self.nranks, self.rank, self.device = int(nranks), int(rank), int(device)

    @staticmethod
    def unique_id():
        import ctypes
        buf = ctypes.create_string_buffer(128)
        K.check(K.lib().kyv_comm_unique_id(buf, 128))
        return bytes(buf.raw[:128])

    def gather(self, batch, res_offset=0):
        import ctypes
        st = K.GatherStats()
        K.check(K.lib().kyv_comm_gather_results(self._h, batch.h, int(res_offset), ctypes.byref(st)))
        return {"status_ms": st.status_ms, "failures_ms": st.failures_ms,
                "status_bytes_per_rank": int(st.status_bytes_per_rank),
                "failure_rows_per_rank_max": int(st.failure_rows_per_rank_max),
                "failure_rows_total": int(st.failure_rows_total)}

    def gather_report(self, batch, res_offset=0, root=0):
        """report assembly to one consumer rank (kyv_comm_gather_report): every rank's packed verdicts and its
        failing-path rows (16 B each on the wire) sent to `root` at exact sizes; status_of / failures_of then work on
        the root only"""
        import ctypes
        st = K.GatherStats()
        K.check(K.lib().kyv_comm_gather_report(self._h, batch.h, int(res_offset), int(root), ctypes.byref(st)))
        return {"status_ms": st.status_ms, "failures_ms": st.failures_ms,
                "status_bytes_per_rank": int(st.status_bytes_per_rank),
                "failure_rows_per_rank_max": int(st.failure_rows_per_rank_max),
                "failure_rows_total": int(st.failure_rows_total)}

    def reduce_counts(self, batch):
        """cluster-wide per-rule verdict tallies of the batch's last evaluation (kyv_comm_reduce_counts: one
        ncclAllReduce of the device-resident tallies): int64 [rules, 8]; a collective, every rank calls it"""
        L = K.lib()
        # the size query never fails (0 when this rank has no results); the collective call is made in every case, so
        # a rank without results fails together with its peers instead of leaving them in the all-reduce
        n = max(0, L.kyv_comm_reduce_counts(self._h, batch.h, None, 0))
        out = np.zeros(max(n, 1), dtype=np.int64)
        got = L.kyv_comm_reduce_counts(self._h, batch.h, out.ctypes.data, n)
        if got < 0 or got != n:
            raise K.KyvError(L.kyv_last_error().decode())
        return out[:n].reshape(-1, 8)

    def status_of(self, q):
        """rank q's packed verdicts from the last gather (kyv_batch_export_status layout, padded)"""
        L = K.lib()
        n = L.kyv_comm_gathered_status(self._h, int(q), None, 0)
        out = np.empty(max(n, 0), dtype=np.uint8)
        if n > 0 and L.kyv_comm_gathered_status(self._h, int(q), out.ctypes.data, n) != n:
            raise K.KyvError(K.lib().kyv_last_error().decode())
        return out

    def failures_of(self, q):
        """rank q's failing-path rows from the last gather: int64 [rows, 8]"""
        L = K.lib()
        n = L.kyv_comm_gathered_failures(self._h, int(q), None, 0)
        out = np.empty((max(n, 0), 8), dtype=np.int64)
        if n > 0 and L.kyv_comm_gathered_failures(self._h, int(q), out.ctypes.data, n) != n:
            raise K.KyvError(K.lib().kyv_last_error().decode())
        return out

    def close(self):
        if self._h:
            K.lib().kyv_comm_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pack_status(status):
    """host packing of input-order verdict bytes [rules][n] into the kyv_batch_export_status layout (low nibble =
    even resource) -- the checker of a gathered segment"""
    st = np.asarray(status, dtype=np.uint8) & 7
    rules, n = st.shape
    half = (n + 1) // 2
    out = np.zeros((rules, half), dtype=np.uint8)
    out[:, :] = st[:, 0::2]
    if n > 1:
        out[:, :n // 2] |= (st[:, 1::2] << 4).astype(np.uint8)
    return out.reshape(-1)
