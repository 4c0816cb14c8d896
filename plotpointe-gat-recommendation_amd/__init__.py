"""MI355X-native GAT message passing for the PlotPointe user-item recommender.

Drop-in for the GAT layer of Axionis47/PlotPointe-GAT-Recommendation
(scripts/train_gat_pyg.py:77 GATConv, scripts/train_gat_custom.py:63 SimpleGATLayer).
The directory name is not a Python identifier; import it with
``importlib.import_module("plotpointe-gat-recommendation_amd")`` -- after the first
import it is also registered as ``ppgat_amd``.
"""
import sys as _sys

from . import _lib, data, dist, evaluation, fusion, knn, optim, sampler, torch_ops  # noqa: F401
from .conv import GATConv, SimpleGATLayer  # noqa: F401
from .hip_ops import CSRGraph, csr_build, gat_aggregate, graph_cache  # noqa: F401
from .model import CustomGAT, PyGGAT, bpr_loss  # noqa: F401

_sys.modules.setdefault("ppgat_amd", _sys.modules[__name__])

__all__ = ["GATConv", "SimpleGATLayer", "PyGGAT", "CustomGAT", "bpr_loss", "CSRGraph", "csr_build",
           "gat_aggregate", "graph_cache", "data"]
