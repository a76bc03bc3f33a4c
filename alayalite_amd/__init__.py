"""alayalite_amd: MI355X-native engine for AlayaLite's HNSW search hot path.

Drop-in for the reference package's Index/Client API (``alayalite.Client``, ``alayalite.Index``):
graph search, distance kernels, candidate pool and visited set run as hand-written HIP on gfx950.
"""

from .client import Client
from .index import Index
from .schema import IndexParams
from .utils import calc_gt, calc_gt_device, calc_recall, load_fvecs, load_ivecs

__all__ = ["Client", "Index", "IndexParams", "load_fvecs", "load_ivecs", "calc_recall", "calc_gt", "calc_gt_device"]

__version__ = "0.1.0"
