"""DiscreteFactor with device-resident values (mirror of pgmpy/factors/discrete/DiscreteFactor.py).

Same constructor, attributes and method semantics as the reference class
(DiscreteFactor.py:16-1110): ``variables`` (list), ``cardinality`` (int
array), ``values`` (C-order, ``shape == cardinality``, last variable fastest)
and the state-name maps.  The difference is where ``values`` lives: the
authoritative copy is an fp64 device tensor, and every arithmetic method is a
gfx950 kernel call (pgmpy_amd.engine.contract / gather -> libpgmhip).
Reading ``phi.values`` downloads a host ndarray and makes the host copy
authoritative (so in-place edits of that array are honoured); the next device
operation uploads it again.  There is no numpy arithmetic path: on a machine
without the HIP library or a GPU every operation raises NativeUnavailable.
"""
from itertools import product as _iproduct

import numpy as np

from ... import engine as E
from ...utils.state_name import StateNameMixin
from ..base import BaseFactor


def _is_scalar(x):
    return isinstance(x, (int, float)) and not isinstance(x, bool) or isinstance(x, np.floating)


class DiscreteFactor(BaseFactor, StateNameMixin):
    """Factor over discrete variables (DiscreteFactor.py:16-127)."""

    _version = 0  # bumped whenever the values may change (compiled plans check it)

    def __init__(self, variables, cardinality, values, state_names={}):
        if isinstance(variables, str):
            raise TypeError("Variables: Expected type list or array like, got string")
        values = np.array(values, dtype=np.float64) if not _is_device(values) else values
        if len(cardinality) != len(variables):
            raise ValueError("Number of elements in cardinality must be equal to number of variables")
        size = int(values.numel()) if _is_device(values) else int(values.size)
        if size != np.prod(cardinality):
            raise ValueError(f"Values array must be of size: {np.prod(cardinality)}")
        if len(set(variables)) != len(variables):
            raise ValueError("Variable names cannot be same")
        if not isinstance(state_names, dict):
            raise ValueError(f"state_names must be of type dict. Got {type(state_names)}.")
        self.variables = list(variables)
        self.cardinality = np.array(cardinality, dtype=int)
        shape = tuple(int(c) for c in self.cardinality)
        if _is_device(values):
            self._dev = values.reshape(shape)
            self._host = None
        else:
            self._host = values.reshape(shape)
            self._dev = None
        super(DiscreteFactor, self).store_state_names(variables, cardinality, state_names)

    @classmethod
    def _trusted(cls, variables, cardinality, values, tables):
        """Internal constructor for results the engine built itself (compiled query answers): the
        arguments are already consistent (a host fp64 array of the right size, distinct variables),
        so the constructor's checks and the state tables are skipped — `tables` maps each variable to
        a StateTable the caller keeps; the factor gets its own copies of the three dicts, as __init__
        gives it."""
        self = cls.__new__(cls)
        self.variables = list(variables)
        self.cardinality = np.array(cardinality, dtype=int)
        self._host = values.reshape(tuple(int(c) for c in cardinality))
        self._dev = None
        self.state_names = {v: list(tables[v].names) for v in self.variables}
        self.name_to_no = {v: dict(tables[v].to_no) for v in self.variables}
        self.no_to_name = {v: dict(tables[v].to_name) for v in self.variables}
        return self

    # ------------------------------------------------------------------ storage
    # Two copies may exist: `_dev` (fp64 device tensor) and `_host` (ndarray).  A host array that
    # has been handed to the caller (`values` getter, or an array passed to the setter) may be
    # edited in place at any later time, as the reference's plain ndarray attribute allows; such a
    # factor is "exposed" and its device copy / value token are checked against a CRC of the host
    # bytes, so an edit made long after the read is still seen by the next device op and by every
    # compiled plan that read the factor (pgmpy_amd.inference.plan.PatternPlan.is_current).
    _exposed = False
    _dev_crc = None

    @property
    def values(self):
        if self._host is None:
            self._host = E.to_host(self._dev)
            self._dev_crc = _crc(self._host)
        elif not self._exposed and self._dev is not None:
            self._dev_crc = _crc(self._host)
        if not self._exposed:
            self._exposed = True
            _VALUES_EPOCH[0] += 1
        return self._host

    @values.setter
    def values(self, v):
        self._version += 1
        _VALUES_EPOCH[0] += 1
        if _is_device(v):
            self._dev = v
            self._host = None
            self._exposed = False
        else:
            self._host = np.asarray(v, dtype=np.float64)  # may alias the caller's array: exposed
            self._dev = None
            self._exposed = True

    def _values_readonly(self):
        """Host values for internal readers (plan compilers): a read-only view; the device copy
        stays valid and the version is unchanged."""
        if self._host is None:
            self._host = E.to_host(self._dev)
            if self._exposed:
                self._dev_crc = _crc(self._host)
        v = self._host.view()
        v.flags.writeable = False
        return v

    def _value_token(self):
        """Changes whenever the values may have changed (compiled plans compare it)."""
        if self._exposed and self._host is not None:
            return (self._version, _crc(self._host))
        return (self._version, None)

    def _d(self):
        """Device tensor of the values (uploaded on first use, re-uploaded after a host edit)."""
        if self._dev is not None and self._exposed and self._host is not None:
            crc = _crc(self._host)
            if crc != self._dev_crc:
                self._dev = None
                self._version += 1
                _VALUES_EPOCH[0] += 1
        if self._dev is None:
            h = self._host.reshape(tuple(int(c) for c in self.cardinality))
            self._dev = E.to_device(h)
            if self._exposed:
                self._dev_crc = _crc(self._host)
        return self._dev

    def _set_d(self, t):
        self._version += 1
        _VALUES_EPOCH[0] += 1
        self._dev = t
        self._host = None
        self._exposed = False

    def _meta_copy(self):
        """New factor object with copied metadata and NO values (the caller sets them)."""
        f = self.__class__.__new__(self.__class__)
        f.variables = [*self.variables]
        f.cardinality = np.array(self.cardinality)
        f._host = None
        f._dev = None
        f._exposed = False
        f.state_names = self.state_names.copy()
        f.no_to_name = self.no_to_name.copy()
        f.name_to_no = self.name_to_no.copy()
        for attr in ("variable", "variable_card"):
            if hasattr(self, attr):
                setattr(f, attr, getattr(self, attr))
        return f

    # ------------------------------------------------------------------ metadata
    def scope(self):
        return self.variables

    def get_cardinality(self, variables):
        # DiscreteFactor.py:149-180
        if isinstance(variables, str):
            raise TypeError("variables: Expected type list or array-like, got type str")
        if not all([var in self.variables for var in variables]):
            raise ValueError("Variable not in scope")
        return {var: self.cardinality[self.variables.index(var)] for var in variables}

    def get_value(self, **kwargs):
        # DiscreteFactor.py:182-221
        for variable in kwargs.keys():
            if variable not in self.variables:
                raise ValueError(f"Factor doesn't have the variable: {variable}")
        index = []
        for var in self.variables:
            if var not in kwargs.keys():
                raise ValueError(f"Variable: {var} not found in arguments")
            try:
                index.append(self.name_to_no[var][kwargs[var]])
            except KeyError:
                index.append(kwargs[var])
        return self.values[tuple(index)]

    def set_value(self, value, **kwargs):
        # DiscreteFactor.py:223-266
        if not isinstance(value, (float, int)):
            raise ValueError(f"value must be float. Got: {type(value)}.")
        for variable in kwargs.keys():
            if variable not in self.variables:
                raise ValueError(f"Factor doesn't have the variable: {variable}")
        index = []
        for var in self.variables:
            if var not in kwargs.keys():
                raise ValueError(f"Variable: {var} not found in arguments")
            elif isinstance(kwargs[var], str):
                index.append(self.name_to_no[var][kwargs[var]])
            else:
                index.append(kwargs[var])
        self.values[tuple(index)] = value

    def assignment(self, index):
        # DiscreteFactor.py:268-320 (mixed-radix decode, last variable fastest)
        index = np.array(index)
        max_possible_index = np.prod(self.cardinality) - 1
        if not all(i <= max_possible_index for i in index):
            raise IndexError("Index greater than max possible index")
        assignments = np.zeros((len(index), len(self.scope())), dtype=int)
        rev_card = self.cardinality[::-1]
        for i, card in enumerate(rev_card):
            assignments[:, i] = index % card
            index = index // card
        assignments = np.flip(assignments, axis=(1,))
        return [[(key, self.get_state_names(key, int(val))) for key, val in zip(self.variables, values)]
                for values in assignments]

    def identity_factor(self):
        return DiscreteFactor(self.variables, self.cardinality, np.ones(int(np.prod(self.cardinality))),
                              state_names=self.state_names)

    # ------------------------------------------------------------------ hot-path ops (device)
    def marginalize(self, variables, inplace=True):
        """Sum out `variables` (DiscreteFactor.py:360-411; einsum L408 -> pgm_contract SUM)."""
        if isinstance(variables, str):
            raise TypeError("variables: Expected type list or array-like, got type str")
        phi = self if inplace else self._meta_copy()
        for var in variables:
            if var not in phi.variables:
                raise ValueError(f"{var} not in scope.")
        var_indexes = [self.variables.index(var) for var in variables]
        index_to_keep = sorted(set(range(len(self.variables))) - set(var_indexes))
        old_vars = list(self.variables)
        A = self._d()
        phi.variables = [old_vars[i] for i in index_to_keep]
        phi.cardinality = np.array(self.cardinality)[index_to_keep]
        phi.del_state_names(variables)
        phi._set_d(E.contract(A, old_vars, None, None, phi.variables, reduce="sum", combine="copy"))
        if not inplace:
            return phi

    def maximize(self, variables, inplace=True):
        """Max out `variables` (DiscreteFactor.py:413-483; compat_fns.max L480 -> pgm_contract MAX)."""
        if isinstance(variables, str):
            raise TypeError("variables: Expected type list or array-like, got type str")
        phi = self if inplace else self._meta_copy()
        for var in variables:
            if var not in phi.variables:
                raise ValueError(f"{var} not in scope.")
        var_indexes = [self.variables.index(var) for var in variables]
        index_to_keep = sorted(set(range(len(self.variables))) - set(var_indexes))
        old_vars = list(self.variables)
        A = self._d()
        phi.variables = [old_vars[i] for i in index_to_keep]
        phi.cardinality = np.array(self.cardinality)[index_to_keep]
        phi.del_state_names(variables)
        phi._set_d(E.contract(A, old_vars, None, None, phi.variables, reduce="max", combine="copy"))
        if not inplace:
            return phi

    def normalize(self, inplace=True):
        """values / values.sum() (DiscreteFactor.py:485-533); 0/0 -> NaN is preserved."""
        phi = self if inplace else self._meta_copy()
        A = self._d()
        if inplace:
            E.normalize_(A)
            phi._set_d(A)
        else:
            phi._set_d(E.normalize_(E.copy(A)))
        if not inplace:
            return phi

    def reduce(self, values, inplace=True, show_warnings=True):
        """Fix variables to states (DiscreteFactor.py:535-617; basic indexing L614 -> strided copy)."""
        if isinstance(values, str):
            raise TypeError("values: Expected type list or array-like, got type str")
        if not all([isinstance(state_tuple, tuple) for state_tuple in values]):
            raise TypeError("values: Expected type list of tuples, get type {type}", type(values[0]))
        for var, _ in values:
            if var not in self.variables:
                raise ValueError(f"The variable: {var} is not in the factor")
        phi = self if inplace else self._meta_copy()
        try:
            values = [(var, self.get_state_no(var, state_name)) for var, state_name in values]
        except KeyError:
            if show_warnings:
                import logging

                logging.getLogger("pgmpy").warning(
                    "Found unknown state name. Trying to switch to using all state names as state numbers")
        static = {}
        for var, state in values:
            if isinstance(state, (bool, np.bool_)) or not isinstance(state, (int, np.integer)):
                raise IndexError("only integers, slices (`:`), ellipsis (`...`), numpy.newaxis (`None`) and "
                                 "integer or boolean arrays are valid indices")
            card = int(self.cardinality[self.variables.index(var)])
            s = int(state)
            if s < -card or s >= card:
                raise IndexError(f"index {s} is out of bounds for axis with size {card}")
            static[var] = s % card
        var_index_to_del = [self.variables.index(var) for var, _ in values]
        keep_idx = sorted(set(range(len(self.variables))) - set(var_index_to_del))
        old_vars = list(self.variables)
        A = self._d()
        phi.variables = [old_vars[i] for i in keep_idx]
        phi.cardinality = np.array(self.cardinality)[keep_idx]
        phi.del_state_names([var for var, _ in values])
        phi._set_d(E.gather(A, old_vars, static, phi.variables))
        if not inplace:
            return phi

    def sum(self, phi1, inplace=True):
        """Broadcast add (DiscreteFactor.py:619-715); extra variables of phi1 are appended."""
        phi = self if inplace else self._meta_copy()
        A = self._d()
        if _is_scalar(phi1):
            phi._set_d(E.contract(A, self.variables, E.scalar(phi1), [], self.variables, combine="add"))
        else:
            old_vars = list(self.variables)
            extra_vars = set(phi1.variables) - set(phi.variables)
            if extra_vars:
                phi.variables.extend(extra_vars)
                new_var_card = phi1.get_cardinality(extra_vars)
                phi.cardinality = np.append(phi.cardinality, [new_var_card[var] for var in extra_vars])
                phi.add_state_names(phi1)
            phi._set_d(E.contract(A, old_vars, phi1._d(), phi1.variables, phi.variables, combine="add"))
        if not inplace:
            return phi

    def product(self, phi1, inplace=True):
        """Broadcast multiply over the scope union (DiscreteFactor.py:717-792; einsum L771-777).

        Output variable order is list(set(a) | set(b)) exactly as the reference (L769)."""
        phi = self if inplace else self._meta_copy()
        A = self._d()
        if _is_scalar(phi1):
            phi._set_d(E.contract(A, self.variables, E.scalar(phi1), [], self.variables, combine="mul"))
        else:
            new_variables = list(set(phi.variables).union(phi1.variables))
            B = phi1._d()
            out = E.contract(A, self.variables, B, phi1.variables, new_variables, combine="mul")
            phi_card = {var: card for var, card in zip(self.variables, self.cardinality)}
            phi_card.update({var: card for var, card in zip(phi1.variables, phi1.cardinality)})
            phi.cardinality = np.array([phi_card[var] for var in new_variables])
            phi.variables = new_variables
            phi.add_state_names(phi1)
            phi._set_d(out)
        if not inplace:
            return phi

    def divide(self, phi1, inplace=True):
        """Broadcast divide, scope(phi1) <= scope(self); 0/0 -> 0 (DiscreteFactor.py:794-866)."""
        phi = self if inplace else self._meta_copy()
        if set(phi1.variables) - set(self.variables):
            raise ValueError("Scope of divisor should be a subset of dividend")
        A = self._d()
        phi._set_d(E.contract(A, self.variables, phi1._d(), phi1.variables, self.variables, combine="div"))
        if not inplace:
            return phi

    def sample(self, n, seed=None):
        # DiscreteFactor.py:868-912 (host sampling of a normalized table)
        import pandas as pd

        phi = self.normalize(inplace=False)
        p = phi.values.ravel()
        rng = np.random.default_rng(seed=seed)
        indexes = rng.choice(range(len(p)), size=n, p=p)
        samples = []
        index_to_state = {}
        for index in indexes:
            if index not in index_to_state:
                index_to_state[index] = self.assignment([index])[0]
            samples.append(index_to_state[index])
        return pd.DataFrame([{k: v for k, v in s} for s in samples])

    def copy(self):
        # DiscreteFactor.py:914-953
        f = self._meta_copy()
        if self._dev is not None:
            f._dev = E.copy(self._dev)
        else:
            f._host = np.array(self._host)
        return f

    def is_valid_cpd(self):
        """Do the values sum to 1 over the first variable (DiscreteFactor.py:955-965)?  The
        reference calls self.to_factor(), which only TabularCPD defines; a DiscreteFactor is
        already a factor, so its own marginal is used."""
        col_sums = self.marginalize(self.scope()[:1], inplace=False)._values_readonly()
        return bool(np.allclose(np.asarray(col_sums).flatten(), np.ones(int(np.prod(self.cardinality[:0:-1]))),
                                atol=0.01))

    # ------------------------------------------------------------------ printing
    def __str__(self):
        return self._str(phi_or_p="phi", tablefmt="grid")

    def _str(self, phi_or_p="phi", tablefmt="grid", print_state_names=True):
        from tabulate import tabulate

        string_header = list(map(str, self.scope()))
        string_header.append(f"{phi_or_p}({','.join(string_header)})")
        flat = self.values.ravel()
        table = []
        for vi, prob in enumerate(_iproduct(*[range(c) for c in self.cardinality])):
            if self.state_names and print_state_names:
                row = [f"{self.variables[i]}({self.state_names[self.variables[i]][prob[i]]})"
                       for i in range(len(self.variables))]
            else:
                row = [f"{self.variables[i]}_{prob[i]}" for i in range(len(self.variables))]
            row.append(flat[vi])
            table.append(row)
        return tabulate(table, headers=string_header, tablefmt=tablefmt, floatfmt=".4f")

    def __repr__(self):
        var_card = ", ".join([f"{var}:{card}" for var, card in zip(self.variables, self.cardinality)])
        return f"<DiscreteFactor representing phi({var_card}) at {hex(id(self))}>"

    # ------------------------------------------------------------------ operators
    def __mul__(self, other):
        return self.product(other, inplace=False)

    def __rmul__(self, other):
        return self.__mul__(other)

    def __add__(self, other):
        return self.sum(other, inplace=False)

    def __radd__(self, other):
        return self.__add__(other)

    def __truediv__(self, other):
        return self.divide(other, inplace=False)

    __div__ = __truediv__

    def __eq__(self, other, atol=1e-08):
        """Order-invariant, state-name-aware allclose (DiscreteFactor.py:1033-1084)."""
        if not (isinstance(self, DiscreteFactor) and isinstance(other, DiscreteFactor)):
            return False
        if set(self.scope()) != set(other.scope()):
            return False
        ovals = np.asarray(other._values_readonly())
        perm = [other.variables.index(v) for v in self.variables]
        ovals = ovals.transpose(perm) if ovals.ndim else ovals
        ocard = np.array(other.cardinality)[perm] if len(perm) else np.array(other.cardinality)
        for axis, var in enumerate(self.variables):
            if set(self.state_names[var]) != set(other.state_names[var]):
                return False
            elif self.state_names[var] != other.state_names[var]:
                ref_index = [other.state_names[var].index(s) for s in self.state_names[var]]
                sl = [slice(None)] * len(self.variables)
                sl[axis] = ref_index
                ovals = ovals[tuple(sl)]
        svals = np.asarray(self._values_readonly())
        if ovals.shape != svals.shape:
            return False
        if not np.allclose(ovals, svals, atol=atol):
            return False
        if not all(self.cardinality == ocard):
            return False
        return True

    def __ne__(self, other):
        return not self.__eq__(other)

    def __hash__(self):
        # DiscreteFactor.py:1089-1110 (axes sorted by variable hash)
        variable_hashes = [hash(v) for v in self.variables]
        order = sorted(range(len(variable_hashes)), key=lambda i: variable_hashes[i])
        vals = np.asarray(self._values_readonly())
        vals = vals.transpose(order) if order else vals
        card = np.array(self.cardinality)[order] if order else np.array(self.cardinality)
        return hash(str(sorted(variable_hashes)) + str(hash(np.ascontiguousarray(vals).tobytes()))
                    + str(hash(np.ascontiguousarray(card).tobytes())) + str(hash(frozenset(self.state_names))))


# bumped whenever any factor's values may change without a CRC check seeing it: a values setter
# call, a device replacement, or a host array handed out for the first time (values_epoch())
_VALUES_EPOCH = [0]


def values_epoch():
    return _VALUES_EPOCH[0]


def _crc(a):
    import zlib

    return zlib.crc32(memoryview(np.ascontiguousarray(a)).cast("B"))


def _is_device(x):
    try:
        import torch
    except ImportError:  # pragma: no cover
        return False
    return isinstance(x, torch.Tensor)
