"""State-name <-> state-number maps (restates pgmpy/utils/state_name.py:1-145).

Host-side bookkeeping only; evidence state names are turned into uint8 codes
here before anything reaches the device.
"""


class StateNameMixin:
    def store_state_names(self, variables, cardinality, state_names):
        # state_name.py:8-60
        if state_names:
            for key, value in state_names.items():
                if not isinstance(value, (list, tuple)):
                    raise ValueError("The state names must be for the form: {variable: list_of_states}")
                elif not len(set(value)) == len(value):
                    raise ValueError(f"Repeated statenames for variable: {key}")
            self.state_names = state_names.copy()
            self.name_to_no = {}
            self.no_to_name = {}
            for key in self.state_names:
                self.name_to_no[key] = {name: no for no, name in enumerate(self.state_names[key])}
                self.no_to_name[key] = {no: name for no, name in enumerate(self.state_names[key])}
        else:
            self.state_names = {var: list(range(int(cardinality[i]))) for i, var in enumerate(variables)}
            self.name_to_no = {var: {i: i for i in range(int(cardinality[idx]))} for idx, var in enumerate(variables)}
            self.no_to_name = self.name_to_no.copy()

    def get_state_names(self, var, state_no):
        # state_name.py:62-69
        if self.state_names:
            return self.no_to_name[var][state_no]
        return state_no

    def get_state_no(self, var, state_name):
        # state_name.py:71-84
        if self.state_names:
            try:
                return self.name_to_no[var][state_name]
            except KeyError:
                raise KeyError(
                    f"state: {state_name} is an unknown for variable: {var}."
                    f" It must be one of {list(self.name_to_no[var].keys())}"
                )
        return state_name

    def add_state_names(self, phi1):
        # state_name.py:86-136 (string names win over numeric ones; other conflicts raise)
        for var in phi1.state_names:
            if var in self.state_names:
                if self.state_names[var] != phi1.state_names[var]:
                    self_str = any(isinstance(s, str) and not s.isdigit() for s in self.state_names[var])
                    phi1_str = any(isinstance(s, str) and not s.isdigit() for s in phi1.state_names[var])
                    if self_str and not phi1_str:
                        continue
                    elif not self_str and phi1_str:
                        self.state_names[var] = phi1.state_names[var]
                        if var in phi1.name_to_no:
                            self.name_to_no[var] = phi1.name_to_no[var]
                        if var in phi1.no_to_name:
                            self.no_to_name[var] = phi1.no_to_name[var]
                    else:
                        raise ValueError(
                            f"State name conflict detected for variable '{var}'.\n"
                            f"First factor has states: {self.state_names[var]}\n"
                            f"Second factor has states: {phi1.state_names[var]}\n"
                            "When the same variable appears in multiple factors, the state names must be identical."
                        )
            else:
                self.state_names[var] = phi1.state_names[var]
                if var in phi1.name_to_no:
                    self.name_to_no[var] = phi1.name_to_no[var]
                if var in phi1.no_to_name:
                    self.no_to_name[var] = phi1.no_to_name[var]

    def del_state_names(self, var_list):
        # state_name.py:138-145
        for var in var_list:
            del self.state_names[var]
            del self.name_to_no[var]
            del self.no_to_name[var]
