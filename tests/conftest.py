import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
# In-process ranks on ONE device (tests/test_gpu_dist_ranks.py) each run on their own stream, and
# the direct exchange makes a rank's stream wait on the device for the other ranks' flags: the
# streams must not share a hardware queue (HIP's default is 4 per process; world 8 needs 8). Read
# by the HIP runtime at its initialisation, which no test has triggered yet at this point (the GPU
# box exports 4, so this overrides it; at most 32 are allowed there).
os.environ["GPU_MAX_HW_QUEUES"] = "16"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: larger CPU-oracle cases")
