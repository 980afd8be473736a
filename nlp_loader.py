"""Load the package directory `neighborhood-link-prediction-openmp_amd/` as module `nlp_amd`
(the directory name is not a Python identifier)."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "neighborhood-link-prediction-openmp_amd")


def load():
    if "nlp_amd" in sys.modules:
        return sys.modules["nlp_amd"]
    spec = importlib.util.spec_from_file_location("nlp_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["nlp_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_sub(name):
    load()
    return importlib.import_module("nlp_amd." + name)
