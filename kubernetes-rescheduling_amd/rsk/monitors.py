"""The experiment harness's once-per-second monitors as one offline tool
(the harness runs nodemonitor.py and communicationcost.py
each second, auto_full_pipeline_repeat.sh:103,146).

    python -m rsk.monitors DUMP_DIR [--workmodel workmodelC.json] [--csv-dir OUT]

DUMP_DIR holds the API dumps rsk.snapshot reads (nodes.json, node_metrics.json,
pods.json, replicasets.json; see its table).  Prints the CPU-% standard
deviation and the communication cost, and, with ``--csv-dir``, appends them to
``node_std.csv`` / ``communication_cost.csv`` in the reference's format
(nodemonitor.py:59-73, communicationcost.py:52-64: a header on creation, then
``timestamp,value`` rows).  Both metrics run on the GPU through librsk.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
from datetime import datetime


def save_to_csv(value, filename: str, column: str) -> None:
    exists = os.path.isfile(filename)
    with open(filename, "a", newline="") as f:
        w = csv.writer(f)
        if not exists:
            w.writerow(["timestamp", column])
        w.writerow([datetime.now().strftime("%Y-%m-%d %H:%M:%S"), value])


def _load(d: str, name: str, required: bool = True):
    p = os.path.join(d, name)
    if not os.path.exists(p):
        if required:
            raise FileNotFoundError(p)
        return None
    with open(p, "r", encoding="utf-8") as f:
        return json.load(f)


def main(argv=None) -> int:
    from . import snapshot, workmodel

    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("dump_dir")
    ap.add_argument("--workmodel", help="µBench workmodel JSON for the relation (default: relation.json in dump_dir)")
    ap.add_argument("--csv-dir", help="append node_std.csv / communication_cost.csv here")
    a = ap.parse_args(argv)
    nodes, node_metrics = _load(a.dump_dir, "nodes.json"), _load(a.dump_dir, "node_metrics.json")
    pods, rs = _load(a.dump_dir, "pods.json"), _load(a.dump_dir, "replicasets.json", required=False)
    if a.workmodel:
        relation = workmodel.relation_from_workmodel(a.workmodel)
    else:
        relation = _load(a.dump_dir, "relation.json")
    std = snapshot.node_resorce_std(nodes, node_metrics)
    cost = snapshot.communication_cost(pods, relation, rs)
    print(json.dumps({"cpu_std": std, "communication_cost": cost}))
    if a.csv_dir:
        os.makedirs(a.csv_dir, exist_ok=True)
        if std is not None:
            save_to_csv(std, os.path.join(a.csv_dir, "node_std.csv"), "cpu_std")
        if cost != -1:
            save_to_csv(cost, os.path.join(a.csv_dir, "communication_cost.csv"), "cost")
    return 0 if std is not None and cost != -1 else 1


if __name__ == "__main__":
    raise SystemExit(main())
