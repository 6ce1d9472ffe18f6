"""taxi2_amd -- MI355X-native all-pairs genetic-distance engine behind the TaxI2 API.

Hot path: versusAll / versusReference (SequencePairs -> align -> p / p-gaps / jc / k2p),
computed by hand-written HIP kernels for gfx950 through the C ABI in include/taxi2_mi355x.h.
"""

__version__ = "0.1.0"
