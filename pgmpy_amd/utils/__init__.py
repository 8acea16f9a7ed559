from .state_name import StateNameMixin
from .example_models import get_example_model

__all__ = ["StateNameMixin", "get_example_model"]
