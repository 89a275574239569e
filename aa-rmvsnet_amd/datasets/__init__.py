"""Drop-in ``datasets`` package (reference: datasets/__init__.py, the dataloaders the
drivers select by name: train.py:13, eval.py:9)."""
import importlib


def find_dataset_def(dataset_name):
    """``datasets.<name>.MVSDataset`` (datasets/__init__.py:5-8)."""
    return getattr(importlib.import_module(f"datasets.{dataset_name}"), "MVSDataset")
