"""rsk — MI355X placement scoring for Kubernetes rescheduling (host side).

Modules: ``api`` (array API over librsk.so), ``cluster`` (cluster_monitoring →
arrays), ``workmodel`` (µBench workmodel → relation CSR), ``synth`` (synthetic
clusters), ``dist`` (multi-GPU sharding), ``_lib`` (ctypes binding).
The drop-in ``rescheduling`` module lives one directory up.
"""
__version__ = "0.1.0"
