"""Offline stand-in for statsmodels (only out-of-scope linear models touch it)."""
from unittest.mock import MagicMock

OLS = GLS = WLS = MagicMock


def __getattr__(name):
    return MagicMock()
