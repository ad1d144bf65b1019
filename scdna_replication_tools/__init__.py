"""Drop-in import path of the reference package (shahcompbio/scdna_replication_tools).

Notebooks and pipelines written against the reference import from here unchanged, e.g.
``from scdna_replication_tools.infer_scRT import scRT`` (inference_tutorial cell 1).  Each
module of this package is the reference module of the same name (file:line cited in
its docstring) and binds the MI355X implementation in ``scdna_replication_tools_amd``:
the PERT fits (steps 1-3, decode) run through libpert_hip.so on the GPU; there is no
CPU fallback.  Modules of the reference outside the PERT hot path (plotting, the
deterministic 'cell' / 'clone' / 'bulk' levels, pseudobulk / T-width / CCC analyses,
the Pyro simulator) are not provided.
"""
