"""GPU-backed TaxI2 tasks: versusAll / versusReference (the hot path) and its callers Decontaminate,
Decontaminate2 and Dereplicate."""

from .versus_all import VersusAll  # noqa: F401
from .versus_reference import VersusReference  # noqa: F401
from .decontaminate import Decontaminate  # noqa: F401
from .decontaminate2 import Decontaminate2  # noqa: F401
from .dereplicate import Dereplicate  # noqa: F401
