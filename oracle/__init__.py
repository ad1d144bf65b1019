"""Test infrastructure: CPU restatement of the reference hot path (see pert_oracle.py).

Never imported by the product package ``scdna_replication_tools_amd``.
"""
