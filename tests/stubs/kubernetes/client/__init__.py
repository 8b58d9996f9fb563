"""Stub of kubernetes.client backed by an in-memory fake cluster.

Only the calls the reference and the drop-in make are implemented.  The fake
cluster (``FAKE``) is plain data that tests fill in; nothing here talks to a
network.
"""
from __future__ import annotations

import copy
from types import SimpleNamespace

from .rest import ApiException

# (namespace, body) for every create_namespaced_deployment call, in order.
CREATED: list = []
# Optional hook: a callable(namespace, body) that may raise ApiException.
CREATE_HOOK = None


class FakeCluster:
    """In-memory state behind the stub APIs.

    nodes:        list of dicts {name, cpu_capacity: str, mem_capacity: str}
    node_usage:   {name: {'cpu': str, 'memory': str}}
    pods:         list of dicts {name, namespace, node_name, deployment, pod_ip}
    pod_usage:    {namespace: {podname: [{'cpu': str, 'memory': str}, ...]}}
    deployments:  {(namespace, name): dict body}
    """

    def __init__(self):
        self.reset()

    def reset(self):
        self.nodes = []
        self.node_usage = {}
        self.pods = []
        self.pod_usage = {}
        self.deployments = {}
        self.deleted = []


FAKE = FakeCluster()


def reset():
    CREATED.clear()
    FAKE.reset()
    global CREATE_HOOK
    CREATE_HOOK = None


class ApiClient:
    def sanitize_for_serialization(self, obj):
        if obj is None:
            return None
        if isinstance(obj, (str, int, float, bool)):
            return obj
        if isinstance(obj, (list, tuple)):
            return [self.sanitize_for_serialization(o) for o in obj]
        if isinstance(obj, dict):
            return {k: self.sanitize_for_serialization(v) for k, v in obj.items()}
        if isinstance(obj, SimpleNamespace):
            return {k: self.sanitize_for_serialization(v) for k, v in vars(obj).items()}
        return obj


def _ns(**kw):
    return SimpleNamespace(**kw)


def _pod_obj(p):
    owners = [_ns(kind="ReplicaSet", name=f"{p['deployment']}-rs")] if p.get("deployment") else []
    return _ns(
        metadata=_ns(name=p["name"], namespace=p.get("namespace", "default"), owner_references=owners),
        spec=_ns(node_name=p.get("node_name")),
        status=_ns(pod_ip=p.get("pod_ip", "10.0.0.1")),
    )


class CoreV1Api:
    def list_node(self, watch=False):
        items = []
        for n in FAKE.nodes:
            items.append(_ns(metadata=_ns(name=n["name"]),
                             status=_ns(capacity={"cpu": n["cpu_capacity"], "memory": n["mem_capacity"]})))
        return _ns(items=items)

    def list_pod_for_all_namespaces(self, watch=False):
        return _ns(items=[_pod_obj(p) for p in FAKE.pods])


class CustomObjectsApi:
    def list_cluster_custom_object(self, group, version, plural):
        items = [{"metadata": {"name": k}, "usage": dict(v)} for k, v in FAKE.node_usage.items()]
        return {"items": items}

    def list_namespaced_custom_object(self, group, version, namespace, plural):
        items = []
        for podname, containers in FAKE.pod_usage.get(namespace, {}).items():
            items.append({"metadata": {"name": podname},
                          "containers": [{"usage": dict(c)} for c in containers]})
        return {"items": items}


class AppsV1Api:
    def create_namespaced_deployment(self, namespace, body):
        if CREATE_HOOK is not None:
            CREATE_HOOK(namespace, body)
        CREATED.append((namespace, copy.deepcopy(body)))
        return body

    def read_namespaced_replica_set(self, name, namespace):
        dep = name[:-3] if name.endswith("-rs") else name
        return _ns(metadata=_ns(owner_references=[_ns(kind="Deployment", name=dep)]))

    def read_namespaced_deployment(self, name, namespace):
        if (namespace, name) not in FAKE.deployments:
            raise ApiException(404, "Not Found")
        return FAKE.deployments[(namespace, name)]

    def delete_namespaced_deployment(self, name, namespace, body=None):
        FAKE.deployments.pop((namespace, name), None)
        FAKE.deleted.append((namespace, name))
        FAKE.pods[:] = [p for p in FAKE.pods if p.get("deployment") != name]


class _Placeholder:
    def __init__(self, *args, **kwargs):
        self.__dict__.update(kwargs)

    def to_dict(self):
        return dict(self.__dict__)


V1Deployment = V1ObjectMeta = V1DeploymentSpec = V1PodTemplateSpec = _Placeholder
V1PodSpec = V1LabelSelector = V1DeploymentStrategy = V1DeleteOptions = _Placeholder
