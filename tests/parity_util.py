"""Shared parity harness: evaluate (resource x rule) pairs through libkyvgpu and compare with the oracle.

The oracle (oracle/, CPU restatement of the reference) is used here only as the checker.
"""
import json

from kyverno_amd import _lib as K
from kyverno_amd import engine as E
from oracle import oracle as O

ORACLE_STATUS = {"pass": K.ST_PASS, "fail": K.ST_FAIL, "skip": K.ST_SKIP, "error": K.ST_ERROR, "panic": K.ST_PANIC}


def oracle_pairs(policies, resources, ns_labels):
    """-> dict (policy name, rule name, resource index) -> oracle rule result (matched pairs only)."""
    out = {}
    for ri, res in enumerate(resources):
        ns = (res.get("metadata") or {}).get("namespace") if isinstance(res.get("metadata"), dict) else None
        nsl = ns_labels.get(ns) if (ns_labels and isinstance(ns, str)) else None
        pr = O.validate(policies, json.dumps(res), nsl if nsl is not None else {})
        for p in pr:
            for rr in p["rules"]:
                out[(p["policy"], rr["name"], ri)] = rr
    return out


def compare(policies, resources, ns_labels=None, backend="gpu", check_messages=True, max_report=20, jit=None):
    """Returns a stats dict; raises AssertionError on verdict/path/message mismatches."""
    rs = E.Ruleset(policies)
    b = E.Batch(rs, resources, ns_labels)
    res = E.evaluate(rs, b, backend=backend, **({} if backend != "gpu" else {"jit": jit}))
    ora = oracle_pairs(policies, resources, ns_labels or {})
    st = res.status
    stats = {"pairs": 0, "matched": 0, "compared": 0, "fallback": 0, "nd": 0, "messages": 0, "unsupported": 0}
    bad = []
    for k, rule in enumerate(rs.rules):
        pol = rs.policies[rule["policy"]]["name"]
        for ri in range(len(resources)):
            stats["pairs"] += 1
            s = int(st[k, ri])
            o = ora.get((pol, rule["name"], ri))
            if s == K.ST_NONE:
                if o is not None:
                    bad.append(("matched by oracle only", pol, rule["name"], ri, o["status"]))
                continue
            stats["matched"] += 1
            if o is None:
                if s not in (K.ST_FALLBACK,):
                    bad.append(("matched by device only", pol, rule["name"], ri, K.STATUS_NAMES[s]))
                continue
            if s == K.ST_FALLBACK or o["status"] == "unsupported":
                stats["fallback"] += 1
                if o["status"] == "unsupported" and s != K.ST_FALLBACK:
                    bad.append(("oracle unsupported, device verdict", pol, rule["name"], ri, K.STATUS_NAMES[s]))
                continue
            if s == K.ST_ND or o.get("nondeterministic"):
                # Go-map-order dependent: both sides must say so (a device that wrongly returns ND is a mismatch)
                if s == K.ST_ND and o.get("nondeterministic"):
                    stats["nd"] += 1
                else:
                    bad.append(("nondeterministic on one side", pol, rule["name"], ri, K.STATUS_NAMES[s],
                                o["status"], bool(o.get("nondeterministic"))))
                continue
            stats["compared"] += 1
            want = ORACLE_STATUS.get(o["status"])
            if want != s:
                bad.append(("status", pol, rule["name"], ri, K.STATUS_NAMES[s], o["status"], o["message"][:160]))
                continue
            if s == K.ST_FAIL and rule["kind"] == "pattern":
                p = res.path(ri, k)
                if p != o["path"]:
                    bad.append(("path", pol, rule["name"], ri, p, o["path"]))
            if check_messages:
                m = res.message(ri, k)
                if m is not None:
                    stats["messages"] += 1
                    if m != o["message"] and not o.get("message_unpinned"):
                        bad.append(("message", pol, rule["name"], ri, m[:200], o["message"][:200]))
    stats["bad"] = bad[:max_report]
    stats["nbad"] = len(bad)
    stats["counts"] = res.counts
    return stats, res


# oracle matrix code -> device status
_MATRIX_TO_DEVICE = {0: K.ST_NONE, 1: K.ST_PASS, 2: K.ST_FAIL, 3: K.ST_SKIP, 4: K.ST_ERROR, 5: K.ST_PANIC,
                     6: K.ST_FALLBACK, 7: K.ST_ND}


def compare_matrix(policies, resources, ns_labels=None, backend="gpu", jit=None, threads=8, texts=True):
    """Parity at scale: every (resource, rule) verdict of the device vs the oracle's verdict matrix
    (oracle.validate_matrix) and, with texts, the failing path and message of every FAIL pair (compare_fail_texts).
    resources: list of dicts, or NDJSON bytes (one resource per line). Nondeterministic pairs are excluded from the
    count only when BOTH sides say ND (one-sided ND is a mismatch). Returns (stats, results); stats["nbad"] counts
    mismatching pairs and texts."""
    import numpy as np
    rs = E.Ruleset(policies)
    b = E.Batch(rs, resources, ns_labels)
    res = E.evaluate(rs, b, backend=backend, **({} if backend != "gpu" else {"jit": jit}))
    if isinstance(resources, (bytes, bytearray)):
        lines = [x for x in bytes(resources).split(b"\n") if x.strip()]
        names, m, *tx = O.validate_matrix(policies, b"[" + b",".join(lines) + b"]", ns_labels, threads=threads,
                                          nres=len(lines), texts=("fail",) if texts else ())
        resources = lines
    else:
        names, m, *tx = O.validate_matrix(policies, resources, ns_labels, threads=threads,
                                          texts=("fail",) if texts else ())
    row = {nm: i for i, nm in enumerate(names)}
    lut = np.array([_MATRIX_TO_DEVICE[i] for i in range(8)], dtype=np.uint8)
    st = np.asarray(res.status)
    bad, compared, nd, matched = [], 0, 0, 0
    for k, rule in enumerate(rs.rules):
        key = (rs.policies[rule["policy"]]["name"], rule["name"])
        want = lut[m[row[key]]] if key in row else np.zeros(len(resources), np.uint8)
        got = st[k, : len(resources)]
        # ND (Go-map-order dependent) pairs are excluded only when BOTH sides say ND; one-sided ND is a mismatch
        ndm = (want == K.ST_ND) & (got == K.ST_ND)
        nd += int(ndm.sum())
        diff = np.nonzero(want != got)[0]
        matched += int((got != K.ST_NONE).sum())
        compared += len(resources) - int(ndm.sum())
        for ri in diff[:3]:
            bad.append((key, int(ri), K.STATUS_NAMES[got[ri]], K.STATUS_NAMES[want[ri]]))
    stats = {"pairs": len(rs.rules) * len(resources), "compared": compared, "matched": matched, "nd": nd,
             "nbad": len(bad), "bad": bad[:20], "rules": len(rs.rules)}
    if texts:
        ts = compare_fail_texts(rs, res, names, tx[0], len(resources))
        stats["texts"] = ts
        stats["nbad"] += ts["nbad"]
        stats["bad"] += ts["bad"][:10]
    return stats, res


def compare_status_sample(rs, res, policies, docs, ns_labels, idx, threads=8, texts=True):
    """Parity of the device verdicts `res` (whole batch `docs`) on the resources at positions `idx` against the
    oracle's verdict matrix of those resources alone, with the failing paths / messages of every FAIL pair (texts).
    Returns a stats dict like compare_matrix."""
    import numpy as np
    sub = [docs[i] for i in idx]
    names, m, *tx = O.validate_matrix(policies, sub, ns_labels, threads=threads, texts=("fail",) if texts else ())
    row = {nm: i for i, nm in enumerate(names)}
    lut = np.array([_MATRIX_TO_DEVICE[i] for i in range(8)], dtype=np.uint8)
    st = np.asarray(res.status)[:, np.asarray(idx)]
    bad, compared, nd, matched = [], 0, 0, 0
    for k, rule in enumerate(rs.rules):
        key = (rs.policies[rule["policy"]]["name"], rule["name"])
        want = lut[m[row[key]]] if key in row else np.zeros(len(idx), np.uint8)
        got = st[k]
        ndm = (want == K.ST_ND) & (got == K.ST_ND)  # excluded only when both sides say ND
        nd += int(ndm.sum())
        diff = np.nonzero(want != got)[0]
        matched += int((got != K.ST_NONE).sum())
        compared += len(idx) - int(ndm.sum())
        for ri in diff[:3]:
            bad.append((key, int(idx[ri]), K.STATUS_NAMES[got[ri]], K.STATUS_NAMES[want[ri]]))
    stats = {"pairs": len(rs.rules) * len(idx), "compared": compared, "matched": matched, "nd": nd,
             "nbad": len(bad), "bad": bad[:20], "rules": len(rs.rules)}
    if texts:
        ts = compare_fail_texts(rs, res, names, tx[0], len(idx), idx=idx)
        stats["texts"] = ts
        stats["nbad"] += ts["nbad"]
        stats["bad"] += ts["bad"][:10]
    return stats


def compare_fail_texts(rs, res, names, tx, nres, idx=None):
    """Failing-path and message parity of every FAIL pair: the device's PatternError.Path (single patterns) and
    RuleResponse.Message, rendered in bulk by kyv_results_texts, against the oracle's (validate_matrix(...,
    texts=("fail",))). idx: resource positions of the device batch that the oracle's columns 0..nres-1 stand for
    (default: the first nres). Returns a stats dict; stats["nbad"] counts path + message mismatches."""
    import numpy as np
    row = {nm: i for i, nm in enumerate(names)}
    idx = np.arange(nres) if idx is None else np.asarray(idx)
    st = {"fail_pairs": 0, "paths_compared": 0, "path_mismatches": 0, "messages_compared": 0,
          "message_mismatches": 0, "messages_unrenderable": 0, "oracle_missing": 0, "bad": []}
    status = np.asarray(res.status)
    for k, rule in enumerate(rs.rules):
        key = (rs.policies[rule["policy"]]["name"], rule["name"])
        fails = np.nonzero(status[k, idx] == K.ST_FAIL)[0]
        if not len(fails) or key not in row:
            continue
        r = row[key]
        lo, hi = int(idx[fails[0]]), int(idx[fails[-1]]) + 1
        msgs = res.texts(k, "message", (K.ST_FAIL,), res0=lo, nres=hi - lo)
        paths = res.texts(k, "path", (K.ST_FAIL,), res0=lo, nres=hi - lo) if rule["kind"] == "pattern" else None
        for j in fails.tolist():
            st["fail_pairs"] += 1
            o = tx.get((r, j))
            if o is None:
                st["oracle_missing"] += 1
                if len(st["bad"]) < 20:
                    st["bad"].append(("oracle has no fail text", key, j))
                continue
            opath, omsg, unpinned = o
            d = int(idx[j]) - lo
            if paths is not None:
                st["paths_compared"] += 1
                if paths[d] != opath:
                    st["path_mismatches"] += 1
                    if len(st["bad"]) < 20:
                        st["bad"].append(("path", key, j, paths[d], opath))
            if msgs[d] is None:
                st["messages_unrenderable"] += 1
            elif not unpinned:
                st["messages_compared"] += 1
                if msgs[d] != omsg:
                    st["message_mismatches"] += 1
                    if len(st["bad"]) < 20:
                        st["bad"].append(("message", key, j, msgs[d][:200], omsg[:200]))
    st["nbad"] = st["path_mismatches"] + st["message_mismatches"] + st["oracle_missing"]
    return st
