"""reference scdna_replication_tools/pert_model.py: ``pert_infer_scRT`` (:36-901) with the
reference's constructor, helper methods and ``run_pert_model()`` return tuple; the three
SVI fits and the MAP decode run on the GPU (scdna_replication_tools_amd.pert_model).
Importing it configures root logging as the reference's import does (:25-33)."""
from scdna_replication_tools_amd.pert_model import MapTrace, PivotAxes, configure_reference_logging, pert_infer_scRT  # noqa: F401

configure_reference_logging()

__all__ = ["pert_infer_scRT"]
