"""Registers the package directory ``adipose_tissue-unet_amd/`` (a name that is not a valid Python
identifier) as the importable package ``adipose_amd``."""
import importlib.util
import os
import sys

PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "adipose_tissue-unet_amd")


def load():
    mod = sys.modules.get("adipose_amd")
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        "adipose_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["adipose_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


load()
