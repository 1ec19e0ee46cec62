import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libk3m_hip.so)")
    config.addinivalue_line("markers", "slow: full-size model on the CPU oracle")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
