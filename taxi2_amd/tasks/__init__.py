"""GPU-backed TaxI2 tasks: the versusAll / versusReference hot path."""

from .versus_all import VersusAll  # noqa: F401
from .versus_reference import VersusReference  # noqa: F401
