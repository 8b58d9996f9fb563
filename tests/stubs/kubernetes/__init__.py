"""Test-only stand-in for the `kubernetes` Python client (not installed in this image).

It provides exactly the surface the reference modules and our drop-in touch:
``config.load_kube_config`` (no-op), ``client.AppsV1Api`` / ``CoreV1Api`` /
``CustomObjectsApi`` backed by an in-memory :class:`FakeCluster`, ``ApiException``
(also re-exported as ``client.rest.ApiException``), ``ApiClient`` with
``sanitize_for_serialization`` and ``V1*`` placeholders (the reference annotates
with ``client.V1Deployment`` at import time, delete_replaced_pod.py:64).

Every ``create_namespaced_deployment`` call is recorded in ``client.CREATED`` as
``(namespace, deep-copied body)`` so tests can read back the placement decision.
"""
from . import client, config  # noqa: F401
