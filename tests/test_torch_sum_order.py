"""The KL sums of ifit follow torch's CPU float32 summation order (cwq_refmath.h
torch_sum2): its restatement (scripts/torch_sum_order.py) equals torch.sum bit for bit."""
import os
import sys

import pytest

torch = pytest.importorskip("torch")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
import torch_sum_order  # noqa: E402


def test_restated_order_is_torch_sum():
    got = torch_sum_order.check(sizes=(5, 8, 9, 32, 48, 129, 384, 768, 1030), trials=60)
    assert all(v == 1.0 for v in got.values()), got
