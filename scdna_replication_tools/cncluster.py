"""reference scdna_replication_tools/cncluster.py: ``kmeans_cluster`` (:80-120) -- KMeans + BIC
over the G1/2 profiles, restarts batched on the device -- and ``compute_bic(kmeans, X)``
(:49-77) on a fitted estimator (anything with ``cluster_centers_`` and ``labels_``)."""
import numpy as np

from scdna_replication_tools_amd import cncluster as _c
from scdna_replication_tools_amd.cncluster import kmeans_cluster  # noqa: F401


def compute_bic(kmeans, X):
    """cncluster.py:49-77."""
    return _c.compute_bic(np.asarray(kmeans.cluster_centers_), np.asarray(kmeans.labels_), np.asarray(X))


__all__ = ["kmeans_cluster", "compute_bic"]
