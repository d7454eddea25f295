"""Model families of the framework: the reference's benchmark workloads (configuration +
synthetic data of the published datasets' shapes) used by bench.py and tools/."""
from .workloads import WORKLOADS, Workload, get

__all__ = ["WORKLOADS", "Workload", "get"]
