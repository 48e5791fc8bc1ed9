"""``fluid.dataset`` surface (``DatasetFactory``, dataset classes)."""
from ..data.dataset import (BoxPSDataset, DatasetBase, DatasetFactory, InputTableDataset,  # noqa: F401
                            PadBoxSlotDataset)

InMemoryDataset = PadBoxSlotDataset
