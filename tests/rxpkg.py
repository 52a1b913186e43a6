"""Import helper: the package directory name is not a Python identifier, load it by path."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd")


def _load(name, path):
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, path, submodule_search_locations=None)
    m = importlib.util.module_from_spec(spec)
    sys.modules[name] = m
    spec.loader.exec_module(m)
    return m


rx = _load("rxsu2", os.path.join(PKG_DIR, "__init__.py"))
meshgen = _load("rxsu2_meshgen", os.path.join(PKG_DIR, "meshgen.py"))
synth = _load("rxsu2_synth", os.path.join(PKG_DIR, "synth.py"))
