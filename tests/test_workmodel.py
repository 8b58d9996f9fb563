"""Native µBench workmodel reader (csrc/rsk_workmodel.cpp).

CPU-only: the reader is host code inside librsk.so (loading needs no GPU).  It
is checked against ``rsk.workmodel.relation_from_workmodel`` (itself pinned to
the reference's hard-coded relation, main.py:31-52, by
test_host.py::test_workmodel_relation_matches_reference) and against the
synthetic tree it was generated from."""
import json
import os

import numpy as np
import pytest

from conftest import REPO

pytest.importorskip("numpy")


def _lib_or_skip():
    from rsk import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("librsk.so not built")


def _as_sets(names, rp, ci):
    return {n: {names[j] for j in ci[rp[i]:rp[i + 1]]} for i, n in enumerate(names)}


def _check_against_python(wm_obj):
    from rsk import workmodel
    names, rp, ci = workmodel.read_workmodel(json.dumps(wm_obj))
    rel = workmodel.relation_from_workmodel(wm_obj)
    assert names == list(rel)
    assert _as_sets(names, rp, ci) == {k: set(v) for k, v in rel.items()}
    for i in range(len(names)):  # deduplicated, ascending, no self edge
        row = ci[rp[i]:rp[i + 1]]
        assert np.all(np.diff(row) > 0) and i not in row
    return names, rp, ci


def test_workmodelC_relation(wm_golden):
    _lib_or_skip()
    calls = wm_golden["workmodel_calls"]
    wm = {s: {"external_services": [{"seq_len": 100, "services": v}], "workers": 8} for s, v in calls.items()}
    names, rp, ci = _check_against_python(wm)
    ref = wm_golden["relation"]  # the reference's own hard-coded relation
    assert _as_sets(names, rp, ci) == {k: set(v) for k, v in ref.items()}
    assert rp[-1] == 38


def test_edge_cases():
    _lib_or_skip()
    wm = {
        "a": {"external_services": [{"services": ["b", "ghost", "a", "b"]}, {"services": ["c"]}]},
        "x\"q\\u00e9": {"external_services": None, "internal_service": {"deep": [[{"services": ["zz"]}]]}},
        "b": {"external_services": [{"seq_len": 5, "services": None}, {"services": ["ghost2", "a"]}]},
        "c": {},
    }
    names, rp, ci = _check_against_python(wm)
    assert names == ["a", 'x"q\\u00e9', "b", "c", "ghost", "ghost2"]
    # a callee defined after its first mention keeps its definition position
    names, _, _ = _check_against_python({"p": {"external_services": [{"services": ["q", "r"]}]},
                                         "q": {"external_services": [{"services": ["r"]}]}})
    assert names == ["p", "q", "r"]
    _check_against_python({})


def test_unicode_escape_and_duplicate_key():
    _lib_or_skip()
    from rsk import workmodel
    text = '{"s\\u00e9": {"external_services": [{"services": ["t"]}]}, "t": {}, "s\\u00e9": {"external_services": []}}'
    names, rp, ci = workmodel.read_workmodel(text)
    assert names == list(json.loads(text))
    assert rp[-1] == 0  # json.load keeps the last value of a repeated key


@pytest.mark.parametrize("bad", ['{"a": ', '{"a": {"external_services": [}', '[1, 2]', '{"a": {}} x', '{"a" {}}'])
def test_malformed_raises(bad):
    _lib_or_skip()
    from rsk import workmodel
    from rsk._lib import RskError
    with pytest.raises(RskError):
        workmodel.read_workmodel(bad.encode())


def test_synth_workmodel_file_roundtrip(tmp_path):
    _lib_or_skip()
    from rsk import synth, workmodel
    P = 20000
    path = tmp_path / "wm.json"
    workmodel.write_synth_workmodel(str(path), P, seed=3, chunk=777)
    names, rp, ci = workmodel.read_workmodel(str(path))
    assert names == [f"s{i}" for i in range(P)]
    rp2, ci2 = synth.tree_csr(synth.pa_tree_parents(P, np.random.default_rng(3)))
    assert np.array_equal(rp, rp2) and np.array_equal(ci, ci2)
    # the file is valid JSON and the Python restatement agrees
    rel = workmodel.relation_from_workmodel(str(path))
    assert all(set(rel[n]) == {names[j] for j in ci[rp[i]:rp[i + 1]]} for i, n in enumerate(names[:2000]))


def test_missing_file_raises(tmp_path):
    _lib_or_skip()
    from rsk import workmodel
    from rsk._lib import RskError
    with pytest.raises(RskError):
        workmodel.read_workmodel(str(tmp_path / "nope.json"))


def test_malformed_error_names_the_byte_offset():
    _lib_or_skip()
    from rsk import workmodel
    from rsk._lib import RskError
    text = '{"a": {"external_services": [{"services": ["b"'
    with pytest.raises(RskError, match=f"byte offset {len(text)}"):
        workmodel.read_workmodel(text.encode())
