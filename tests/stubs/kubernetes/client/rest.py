"""Stub of kubernetes.client.rest (delete_replaced_pod.py:3 imports ApiException from here)."""


class ApiException(Exception):
    def __init__(self, status=0, reason=None, body=None):
        super().__init__(f"({status}) {reason}")
        self.status = status
        self.reason = reason
        self.body = body
