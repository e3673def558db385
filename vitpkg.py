"""Import helper for the `vit.rs_amd/` package (its directory name is not a Python identifier).

    from vitpkg import vit      # the vit.rs_amd package, registered as `vit_rs_amd`
"""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "vit.rs_amd")


def load():
    if "vit_rs_amd" in sys.modules:
        return sys.modules["vit_rs_amd"]
    spec = importlib.util.spec_from_file_location(
        "vit_rs_amd", os.path.join(_DIR, "__init__.py"), submodule_search_locations=[_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["vit_rs_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


vit = load()
