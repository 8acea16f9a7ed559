from .BIF import BIFReader

__all__ = ["BIFReader"]
