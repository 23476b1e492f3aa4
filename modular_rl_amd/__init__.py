"""modular_rl_amd -- MI355X-native TRPO hot path with the ddlau/modular_rl API surface.

Compute runs in hand-written HIP kernels (libmrl_hip.so, gfx950) behind a C ABI
(include/mrl_hip.h); this package is the Python host layer mirroring the
reference's agent / updater / training-loop interfaces.
"""
__version__ = "0.1.0"
