from .google import *  # noqa: F401,F403
from .google import __all__ as _g
from .master import Guided_compresser, Master_compresser
from .waseda import Cheng2020Anchor, Cheng2020Attention

__all__ = list(_g) + ["Cheng2020Anchor", "Cheng2020Attention", "Guided_compresser", "Master_compresser"]
