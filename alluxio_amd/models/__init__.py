"""Workload-facing integrations (this framework has no neural models of its own: the "models"
it serves are training / inference input pipelines).  ``dataset`` gathers HBM-cached records
into device batches with one kernel launch per batch."""
from .dataset import DeviceBatchLoader, FixedRecordDataset  # noqa: F401
