"""reference scdna_replication_tools/normalize_by_cell.py: ``compute_cell_corrs`` (:148-180),
the S-cell vs G1-cell Pearson table the correlation-matched CN priors rank (the rest of
that module belongs to the deterministic 'cell' level, outside this build's scope)."""
from scdna_replication_tools_amd.prep import compute_cell_corrs  # noqa: F401

__all__ = ["compute_cell_corrs"]
