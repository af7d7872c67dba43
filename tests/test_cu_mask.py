"""CU-range parsing of the CU-masked stream experiment (ray_amd/ops/cu_mask.py)."""

import pytest

from ray_amd.ops import cu_mask


@pytest.fixture
def cus256(monkeypatch):
    monkeypatch.setattr(cu_mask, "num_cus", lambda device: 256)


def test_last_n(cus256):
    assert cu_mask.cu_range("cuda:0", "64") == list(range(192, 256))


def test_first_n(cus256):
    assert cu_mask.cu_range("cuda:0", "-192") == list(range(0, 192))


def test_explicit_and_clamped(cus256):
    assert cu_mask.cu_range("cuda:0", "10:20") == list(range(10, 20))
    assert cu_mask.cu_range("cuda:0", "250:300") == list(range(250, 256))


def test_empty_range_rejected(cus256):
    with pytest.raises(ValueError):
        cu_mask.cu_range("cuda:0", "300:400")
