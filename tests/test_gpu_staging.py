"""The pinned staging ring (kyv_engine.hip Staging: batch uploads and verdict copy-backs go through three pinned 64 MiB
slots) shared by host threads: an upload on one thread (a new batch's first evaluation) while another thread copies
verdicts back must not let either transfer reuse a slot the other's DMA still reads or writes. Every evaluation on both
threads must return exactly the verdicts of the same batch evaluated alone."""
import threading

import numpy as np
import pytest

import cases
from kyverno_amd import engine as E
from kyverno_amd import synth

pytestmark = pytest.mark.gpu


def test_upload_and_copy_back_from_two_threads():
    rs = E.Ruleset(cases.best_practices() + cases.chart_restricted())
    # big enough that both the upload and the copy-back span several ring slots (> 3 x 64 MiB of node rows)
    data_a, nsl = synth.corpus_ndjson(400_000, seed=61)
    data_b, _ = synth.corpus_ndjson(400_000, seed=62)
    a = E.Batch(rs, data_a, nsl)
    ref_a = E.evaluate(rs, a, backend="gpu", copy_back=True).raw.copy()
    ref_b = E.evaluate(rs, E.Batch(rs, data_b, nsl), backend="gpu", copy_back=True).raw.copy()
    errors = []

    def copy_backs():
        try:
            for _ in range(4):
                if not np.array_equal(E.evaluate(rs, a, backend="gpu", copy_back=True).raw, ref_a):
                    errors.append("copy-back of batch A differs")
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(repr(e))

    def uploads():
        try:
            for _ in range(3):
                b = E.Batch(rs, data_b, nsl)  # a fresh batch: its first evaluation uploads it through the ring
                if not np.array_equal(E.evaluate(rs, b, backend="gpu", copy_back=True).raw, ref_b):
                    errors.append("upload + evaluation of batch B differs")
                del b
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=copy_backs), threading.Thread(target=uploads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
