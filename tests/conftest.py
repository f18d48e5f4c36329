"""Pytest configuration: import paths, the ``gpu`` marker, and seeding (reference tests/conftest.py:9-15)."""

import random
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "thor-slam_amd", ROOT / "tests"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(autouse=True)
def set_random_seed() -> None:
    random.seed(1337)


def pytest_collection_modifyitems(config, items):
    items.sort(key=lambda x: x.get_closest_marker("slow") is not None)
    gpu_ok = None
    for item in items:
        if item.get_closest_marker("gpu") is None:
            continue
        if gpu_ok is None:
            try:
                import torch

                gpu_ok = bool(torch.cuda.is_available())
            except Exception:
                gpu_ok = False
        if not gpu_ok:
            item.add_marker(pytest.mark.skip(reason="no ROCm GPU visible"))
