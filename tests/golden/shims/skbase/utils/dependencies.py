"""Offline stand-in for skbase.utils.dependencies._check_soft_dependencies.

Only used when importing the read-only reference to generate golden fixtures.
"""
import importlib.util


def _check_soft_dependencies(*packages, severity="error", msg=None, **kwargs):
    names = []
    for p in packages:
        if isinstance(p, (list, tuple)):
            names.extend(p)
        else:
            names.append(p)
    ok = True
    for p in names:
        mod = str(p).split(">")[0].split("<")[0].split("=")[0].split("!")[0].strip()
        if importlib.util.find_spec(mod) is None:
            ok = False
            break
    if not ok and severity == "error":
        raise ModuleNotFoundError(msg or f"missing soft dependency among {names}")
    return ok
