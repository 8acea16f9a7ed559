from .base import BaseFactor, factor_divide, factor_product, factor_sum_product

__all__ = ["BaseFactor", "factor_product", "factor_sum_product", "factor_divide"]
