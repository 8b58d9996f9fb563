"""Host C++ under AddressSanitizer + UBSan.

`make -C kubernetes-rescheduling_amd/csrc asan` compiles the librsk sources
that take caller input — the µBench workmodel reader (rsk_workmodel.cpp), the
Kubernetes quantity parser (rsk_snapshot.cpp) and the CAR plan builder
(rsk_plan.cpp) — with g++ -fsanitize=address,undefined -fno-sanitize-recover
into a CPU-only driver (tests/asan/asan_driver.cpp).  The driver reads its
input from exact-length heap buffers (no NUL terminator), so a read past the
end is a report.  Inputs: the workmodelC relation (tests/golden, the
reference's workmodelC.json services, main.py:31-52), truncated and malformed
workmodels, a 20k-service synthetic file, every quantity string of the
reference-generated fixture (unit_convertion.py:1-32) plus malformed ones, and
random relation graphs through the plan builder.  Every run must exit 0 with
no sanitizer report."""
import json
import os
import shutil
import subprocess

import pytest

from conftest import REPO

CSRC = os.path.join(REPO, "kubernetes-rescheduling_amd", "csrc")
EXE = os.path.join(CSRC, "build", "asan", "rsk_asan")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")


@pytest.fixture(scope="module")
def exe():
    subprocess.run(["make", "-s", "-C", CSRC, "asan"], check=True, capture_output=True, timeout=600)
    assert os.path.exists(EXE)
    return EXE


def _run(exe, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=300, env=env)
    report = r.stderr
    assert r.returncode == 0, f"{args}: exit {r.returncode}\n{r.stdout[-2000:]}\n{report[-4000:]}"
    assert "AddressSanitizer" not in report and "runtime error" not in report and "LeakSanitizer" not in report, report
    return r.stdout


def _workmodels(wm_golden):
    calls = wm_golden["workmodel_calls"]
    good = json.dumps({s: {"external_services": [{"seq_len": 100, "services": v}], "workers": 8}
                       for s, v in calls.items()})
    yield "workmodelC", good
    for cut in (1, 2, len(good) // 3, len(good) // 2, len(good) - 1):   # truncated anywhere
        yield f"trunc{cut}", good[:cut]
    yield "escapes", '{"s\\u00e9\\"q": {"external_services": [{"services": ["t\\\\", "\\ud83d\\ude00"]}]}, "t": {}}'
    for k, bad in enumerate(['{"a": ', '{"a": {"external_services": [}', '[1, 2]', '{"a": {}} x', '{"a" {}}', '',
                             '{"a": {"external_services": [{"services": ["b"', '"\\u12', '{"\\', '{' * 5000]):
        yield f"bad{k}", bad


def test_workmodel_reader_clean_under_asan(exe, wm_golden, tmp_path):
    for name, text in _workmodels(wm_golden):
        f = tmp_path / f"{name}.json"
        f.write_text(text, encoding="utf-8")
        out = _run(exe, "wm", str(f))
        if name == "workmodelC":
            assert "pass 0: P=" in out and "pass 1: P=" in out


def test_synthetic_workmodel_clean_under_asan(exe, tmp_path):
    from rsk import workmodel
    f = tmp_path / "synth.json"
    workmodel.write_synth_workmodel(str(f), 20_000, seed=5, chunk=999)
    out = _run(exe, "wm", str(f))
    assert "P=20000" in out


def test_quantity_parser_clean_under_asan(exe, tmp_path):
    g = json.load(open(os.path.join(REPO, "tests", "golden", "quantities.json")))
    extra = ["", "m", "Ki", "1e", "1e309", "-", ".", "1.2.3", "9" * 400, "1Zi", "0x10", "  ", "\t5m", "nan", "inf"]
    for kind in ("cpu", "mem"):
        f = tmp_path / f"{kind}.txt"
        f.write_text("\n".join([s for s, _ in g[kind]] + extra), encoding="utf-8")
        out = _run(exe, "qty", str(f), kind)
        assert f"qty {kind}: status 0" in out


@pytest.mark.parametrize("P,seed", [(300, 1), (3000, 2), (9000, 3)])
def test_plan_builder_clean_under_asan(exe, P, seed):
    out = _run(exe, "plan", str(P), str(seed))
    assert out.count("plan P=") == 12
