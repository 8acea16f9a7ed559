"""Offline stand-in for scikit-base (fixture generation only; see tests/golden/make_golden.py)."""
