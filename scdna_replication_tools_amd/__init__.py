"""MI355X-native PERT (probabilistic single-cell replication timing) hot path.

Drop-in for the SVI inference path of shahcompbio/scdna_replication_tools:
``pert_model.pert_infer_scRT`` and ``infer_scRT.scRT`` keep the reference's
constructor arguments, return tuple and output columns; the fit itself runs in
hand-written gfx950 HIP kernels (``csrc/``) reached through the C ABI of
``include/pert_hip.h``.
"""
__version__ = "0.1.0"
