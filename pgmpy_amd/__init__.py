"""pgmpy_amd — MI355X-native (gfx950) engine for pgmpy's discrete-factor hot path.

Drop-in mirror of the pgmpy API surface for DiscreteFactor / TabularCPD,
VariableElimination, BeliefPropagation and DiscreteBayesianNetwork.predict /
predict_probability; every factor operation runs in hand-written HIP kernels
(pgmpy_amd/csrc/pgmhip.hip) reached through the C-ABI of include/pgmhip.h.
"""
__version__ = "0.1.0"
