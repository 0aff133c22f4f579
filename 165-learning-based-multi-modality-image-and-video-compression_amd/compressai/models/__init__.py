from .google import *  # noqa: F401,F403
from .google import __all__ as _g

__all__ = list(_g)
