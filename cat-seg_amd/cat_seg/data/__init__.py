"""Data side of the CAT-Seg eval path: dataset catalogs + the reference's dataset names
(reference cat_seg/data/__init__.py -> datasets/register_*.py, registered on import),
dataset mappers, transforms and the sharded test loader."""
from . import datasets  # noqa: F401  (registers the evaluation datasets)
from .build import InferenceSampler, build_test_loader  # noqa: F401
from .catalog import DatasetCatalog, MetadataCatalog, load_sem_seg  # noqa: F401
from .dataset_mappers import (  # noqa: F401
    CATSegTestDatasetMapper, DETRPanopticDatasetMapper, MaskFormerPanopticDatasetMapper,
    MaskFormerSemanticDatasetMapper, read_image)
