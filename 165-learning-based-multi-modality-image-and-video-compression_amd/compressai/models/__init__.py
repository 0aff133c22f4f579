from .google import *  # noqa: F401,F403
from .google import __all__ as _g
from .waseda import Cheng2020Anchor, Cheng2020Attention

__all__ = list(_g) + ["Cheng2020Anchor", "Cheng2020Attention"]
