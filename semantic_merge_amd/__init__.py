"""MI355X-native op-log composition for semmerge."""
from .ops import Op, Target  # noqa: F401
from .conflict import Conflict  # noqa: F401

__all__ = ["Op", "Target", "Conflict", "compose_oplogs"]


def __getattr__(name):
    # compose_oplogs needs the HIP library; import lazily so schema users do not.
    if name == "compose_oplogs":
        from .compose import compose_oplogs
        return compose_oplogs
    raise AttributeError(name)
