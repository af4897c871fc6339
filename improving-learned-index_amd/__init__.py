"""MI355X-native DeeperImpact encode-and-retrieve path.

The directory name (improving-learned-index_amd) is not a Python identifier; it is
imported as ``improving_learned_index_amd`` through the shim module of that name at
the repository root.  Compute goes through libdeepimpact_hip.so (include/deepimpact.h);
there is no CPU fallback.
"""
__version__ = "0.1.0"
