"""State names: per-variable tables mapping state name <-> state number.

Behaviour follows pgmpy/utils/state_name.py (StateNameMixin, L8-145): the same public
attributes (``state_names``, ``name_to_no``, ``no_to_name``), the same lookup fallbacks
and the same error types/messages.  The structure is this package's own: every
variable's states live in one :class:`StateTable`, which also produces the uint8 code
lookup tables the batched evidence encoder (pgmpy_amd.inference.batch) needs, and the
merge policy of ``add_state_names`` is a single decision function.
"""

MISSING_CODE = 255  # uint8 code of an unobserved cell (pgmpy_amd._native.PGM_EV_MISSING)


class StateTable:
    """States of one variable: ordered names, name -> number, number -> name."""

    __slots__ = ("names", "to_no", "to_name")

    def __init__(self, names):
        self.names = list(names)
        self.to_no = {s: i for i, s in enumerate(self.names)}
        self.to_name = dict(enumerate(self.names))

    @classmethod
    def numbered(cls, card):
        t = cls(range(int(card)))
        t.to_name = t.to_no  # identity maps (the reference shares one dict here too)
        return t

    def textual(self):
        """True if any state is a non-numeric string: such names win a merge (state_name.py:102-113)."""
        return any(isinstance(s, str) and not s.isdigit() for s in self.names)

    def code_lut(self, values):
        """int64 state numbers of the objects in `values` (-1 where unknown): used by the evidence
        encoder to turn category lists / unique cell values into uint8 codes."""
        import numpy as np

        get = self.to_no.get
        return np.fromiter((get(v, -1) if _hashable(v) else -1 for v in values), dtype=np.int64, count=len(values))


def _hashable(v):
    try:
        hash(v)
        return True
    except TypeError:
        return False


def _validate(state_names):
    for var, names in state_names.items():
        if not isinstance(names, (list, tuple)):
            raise ValueError("The state names must be for the form: {variable: list_of_states}")
        if len(set(names)) != len(names):
            raise ValueError(f"Repeated statenames for variable: {var}")


def _merge_decision(var, mine, theirs):
    """How add_state_names treats a variable both factors know: "same", "keep" (ours is textual,
    theirs numeric), "take" (theirs textual, ours numeric), or a ValueError (both of one kind)."""
    if mine == theirs:
        return "same"
    ours_text = StateTable(mine).textual()
    theirs_text = StateTable(theirs).textual()
    if ours_text != theirs_text:
        return "keep" if ours_text else "take"
    raise ValueError(
        f"State name conflict detected for variable '{var}'.\n"
        f"First factor has states: {mine}\n"
        f"Second factor has states: {theirs}\n"
        f"When the same variable appears in multiple factors, "
        f"the state names must be identical. Please ensure consistent "
        f"state naming across your model.")


class StateNameMixin:
    """Mixin for factors/CPDs: stores one StateTable per variable and exposes the reference's dicts."""

    def store_state_names(self, variables, cardinality, state_names):
        if state_names:
            _validate(state_names)
            tables = {var: StateTable(names) for var, names in state_names.items()}
            self.state_names = state_names.copy()
        else:
            tables = {var: StateTable.numbered(cardinality[i]) for i, var in enumerate(variables)}
            self.state_names = {var: t.names for var, t in tables.items()}
        self.name_to_no = {var: t.to_no for var, t in tables.items()}
        self.no_to_name = {var: t.to_name for var, t in tables.items()}

    def state_table(self, var):
        """The StateTable of `var` (built from the public dicts, so edits to them are seen)."""
        t = StateTable.__new__(StateTable)
        t.names = list(self.state_names[var])
        t.to_no = self.name_to_no[var]
        t.to_name = self.no_to_name[var]
        return t

    def get_state_names(self, var, state_no):
        return self.no_to_name[var][state_no] if self.state_names else state_no

    def get_state_no(self, var, state_name):
        if not self.state_names:
            return state_name
        table = self.name_to_no[var]
        if state_name in table:
            return table[state_name]
        raise KeyError(f"state: {state_name} is an unknown for variable: {var}."
                       f" It must be one of {list(table.keys())}")

    def add_state_names(self, phi1):
        for var, theirs in phi1.state_names.items():
            decision = _merge_decision(var, self.state_names[var], theirs) if var in self.state_names else "take"
            if decision != "take":
                continue
            self.state_names[var] = theirs
            for attr in ("name_to_no", "no_to_name"):
                src = getattr(phi1, attr)
                if var in src:
                    getattr(self, attr)[var] = src[var]

    def del_state_names(self, var_list):
        for var in var_list:
            for attr in ("state_names", "name_to_no", "no_to_name"):
                del getattr(self, attr)[var]
