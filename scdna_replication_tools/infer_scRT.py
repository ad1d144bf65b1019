"""reference scdna_replication_tools/infer_scRT.py: the ``scRT`` orchestrator (:25-168).

``scRT(cn_s, cn_g1, ...).infer(level='pyro' | 'pert')`` clusters the G1/2 cells when
``clone_col`` is None, computes consensus clone profiles, assigns S-phase cells to
clones and runs ``pert_infer_scRT`` on the GPU (scdna_replication_tools_amd.infer_scRT).
"""
from scdna_replication_tools_amd.cncluster import kmeans_cluster  # noqa: F401
from scdna_replication_tools_amd.infer_scRT import assign_s_to_clones, scRT  # noqa: F401
from scdna_replication_tools.pert_model import pert_infer_scRT  # noqa: F401  (the reference's import: logging set-up)
from scdna_replication_tools.compute_consensus_clone_profiles import compute_consensus_clone_profiles  # noqa: F401

__all__ = ["scRT"]
