"""reference scdna_replication_tools/assign_s_to_clones.py: ``assign_s_to_clones`` (:49-79),
each S-phase cell to the clone profile of highest Pearson r (vectorised per cell)."""
from scdna_replication_tools_amd.infer_scRT import assign_s_to_clones  # noqa: F401

__all__ = ["assign_s_to_clones"]
