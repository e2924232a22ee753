"""Test-time data loading (detectron2 `build_detection_test_loader` + `InferenceSampler`,
used by the reference through `Trainer.test`, train_net.py:302).

Every rank takes a contiguous slice of the dataset (the first len % world ranks one item
more: `cat_seg.distributed.shard_range`, the InferenceSampler split), maps it with the test
mapper and yields lists of `batch_size` dicts (detectron2 uses 1; CATSeg.forward takes any
number and runs them as one batch on the device).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Union

import torch.distributed as dist
import torch.utils.data as tud

from ..distributed import shard_range
from .catalog import DatasetCatalog
from .dataset_mappers import CATSegTestDatasetMapper


def trivial_batch_collator(batch):
    return batch


class _MapDataset(tud.Dataset):
    def __init__(self, dicts: Sequence[dict], mapper):
        self.dicts, self.mapper = list(dicts), mapper

    def __len__(self):
        return len(self.dicts)

    def __getitem__(self, i):
        return self.mapper(self.dicts[i])


class InferenceSampler(tud.Sampler):
    """This rank's contiguous [begin, end) of range(size), in order."""

    def __init__(self, size: int, rank: Optional[int] = None, world: Optional[int] = None):
        if rank is None or world is None:
            on = dist.is_available() and dist.is_initialized()
            rank, world = (dist.get_rank(), dist.get_world_size()) if on else (0, 1)
        self._range = range(*shard_range(size, rank, world))

    def __iter__(self):
        return iter(self._range)

    def __len__(self):
        return len(self._range)


def build_test_loader(dataset: Union[str, Sequence[dict]], mapper=None, *, cfg=None, batch_size: int = 1,
                      num_workers: int = 0, rank: Optional[int] = None, world: Optional[int] = None):
    """`dataset`: a registered name (DatasetCatalog) or a list of dataset dicts."""
    dicts: List[dict] = DatasetCatalog.get(dataset) if isinstance(dataset, str) else list(dataset)
    mapper = mapper if mapper is not None else CATSegTestDatasetMapper(cfg)
    ds = _MapDataset(dicts, mapper)
    sampler = InferenceSampler(len(ds), rank, world)
    bs = tud.BatchSampler(sampler, batch_size, drop_last=False)
    return tud.DataLoader(ds, batch_sampler=bs, num_workers=num_workers, collate_fn=trivial_batch_collator)
