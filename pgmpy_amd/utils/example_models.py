"""get_example_model (mirror of pgmpy/utils/utils.py:16-171) over the bundled BIF files.

The networks used by the benchmarks (alarm, munin, pathfinder) plus asia ship
as data under pgmpy_amd/data/ (copied bnlearn BIF files), so the GPU box needs
no reference checkout and no network access.
"""
import functools
import os

DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")


def available_models():
    return sorted(f[:-7] for f in os.listdir(DATA) if f.endswith(".bif.gz"))


@functools.lru_cache(maxsize=None)
def _reader(model):
    from ..readwrite import BIFReader

    path = os.path.join(DATA, f"{model}.bif.gz")
    if not os.path.exists(path):
        raise ValueError(f"dataset should be one of the options {available_models()}; got {model!r}")
    return BIFReader(path)


def get_example_model(model):
    return _reader(model).get_model()
