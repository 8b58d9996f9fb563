#!/usr/bin/env python3
"""Golden fixtures for pick_max_pod's metric-edge cases (delete_replaced_pod.py:41-61),
from the REFERENCE itself (build container only, like make_golden.py):

    python -B tests/golden/make_pick_edges.py [--reference /root/reference]

Writes ``pick_edges.json``: pods (name, node, cpu or None when the pod is absent
from the metrics dict), the hazard node, and what the reference returned — the
picked pod's name, None, or the name of the exception it raised.  Cases: pods
without metrics on the hazard node (the reference's ("0", "0") default meets
``"0" > -1``), pods without metrics elsewhere only, 0-CPU pods (``0 > -1`` holds:
the first one is picked), ties, empty nodes.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from types import SimpleNamespace as NS

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402  (stub path + load_reference)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    ref = make_golden.load_reference(args.reference)
    rng = np.random.default_rng(4242)
    cases = []

    def run(pods, most):
        spods = [NS(metadata=NS(name=n), spec=NS(node_name=node)) for n, node, _ in pods]
        usage = {n: (c, 1) for n, _, c in pods if c is not None}
        try:
            p = ref.D.pick_max_pod(most, spods, usage)
            out = {"picked": None if p is None else p.metadata.name}
        except Exception as e:  # noqa: BLE001 - the reference's own failure is the expected value
            out = {"raises": type(e).__name__}
        cases.append(dict(pods=[list(x) for x in pods], most=most, **out))

    # hand-built corners
    run([["a", "n0", None]], "n0")                                       # only pod lacks metrics
    run([["a", "n0", 5], ["b", "n0", None], ["c", "n0", 9]], "n0")       # missing one in the middle
    run([["a", "n1", None], ["b", "n0", 3]], "n0")                       # missing only on another node
    run([["a", "n0", 0], ["b", "n0", 0]], "n0")                          # 0-CPU pods: first one
    run([["a", "n0", 0], ["b", "n0", 7], ["c", "n0", 7]], "n0")          # ties: first max
    run([["a", "n1", 4]], "n0")                                          # no pod on the node
    run([], "n0")
    # random mixes
    for t in range(60):
        K = int(rng.integers(1, 4))
        pods = []
        for k in range(int(rng.integers(0, 9))):
            node = f"n{int(rng.integers(0, K))}"
            r = rng.random()
            cpu = None if r < 0.15 else (0 if r < 0.3 else int(rng.choice([5, 10, 10, 300])))
            pods.append([f"p{k}", node, cpu])
        run(pods, f"n{int(rng.integers(0, K))}")
    out = os.path.join(HERE, "pick_edges.json")
    with open(out, "w") as f:
        json.dump({"source": "delete_replaced_pod.pick_max_pod (reference, unmodified)", "cases": cases}, f, indent=0)
    print(f"wrote {out}: {len(cases)} cases, {sum('raises' in c for c in cases)} raise")


if __name__ == "__main__":
    main()
