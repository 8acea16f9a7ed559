"""n-ary factor helpers (mirror of pgmpy/factors/base.py:20-163)."""
from abc import abstractmethod
from functools import reduce


class BaseFactor(object):
    def __init__(self, *args, **kwargs):
        pass

    @abstractmethod
    def is_valid_cpd(self):
        pass


def factor_product(*args):
    """Left fold of __mul__ (pgmpy/factors/base.py:20-66)."""
    if not all(isinstance(phi, BaseFactor) for phi in args):
        raise TypeError("Arguments must be factors")
    elif len(set(map(type, args))) != 1:
        raise NotImplementedError("All the args are expected to be instances of the same factor class.")
    if len(args) == 1:
        return args[0].copy()
    return reduce(lambda phi1, phi2: phi1 * phi2, args)


def factor_sum_product(output_vars, factors):
    """sum_{var not in output_vars} prod factors (pgmpy/factors/base.py:69-115).

    The reference runs opt_einsum.contract(..., optimize="greedy"); here the
    greedy pairwise path is planned on the host and each pairwise step is one
    fused product+marginalize kernel (pgmpy_amd.inference.contraction)."""
    from ..inference.contraction import contract_factors
    from .discrete import DiscreteFactor

    state_names = {}
    for phi in factors:
        state_names.update(phi.state_names)
    out = contract_factors([(phi._d(), list(phi.variables)) for phi in factors], list(output_vars))
    return DiscreteFactor(variables=list(output_vars), cardinality=list(out.shape), values=out,
                          state_names={var: state_names[var] for var in output_vars})


def factor_divide(phi1, phi2):
    """phi1 / phi2 (pgmpy/factors/base.py:118-163)."""
    if not isinstance(phi1, BaseFactor) or not isinstance(phi2, BaseFactor):
        raise TypeError("phi1 and phi2 should be factors instances")
    elif type(phi1) != type(phi2):
        raise NotImplementedError("All the args are expected to be instances of the same factor class.")
    return phi1.divide(phi2, inplace=False)
