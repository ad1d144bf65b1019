"""reference scdna_replication_tools/predict_cycle_phase.py (:23-117): phase calls from the
PERT decode, with the per-cell features batched."""
from scdna_replication_tools_amd.predict_cycle_phase import *  # noqa: F401,F403
from scdna_replication_tools_amd.predict_cycle_phase import predict_cycle_phase  # noqa: F401
