"""Stub of kubernetes.config: loading a kubeconfig is a no-op in tests."""


def load_kube_config(*args, **kwargs):
    return None


def load_incluster_config(*args, **kwargs):
    return None
