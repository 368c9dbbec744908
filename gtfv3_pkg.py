"""Import helper for the `geosongpu-ci_amd/` package.

The package directory name contains a hyphen (it is named after the reference
repository), so it cannot be imported with a plain `import`.  `load()` registers
it under the importable alias `geosongpu_ci_amd`.
"""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "geosongpu-ci_amd")
ALIAS = "geosongpu_ci_amd"


def load():
    if ALIAS in sys.modules:
        return sys.modules[ALIAS]
    spec = importlib.util.spec_from_file_location(
        ALIAS, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR]
    )
    mod = importlib.util.module_from_spec(spec)
    sys.modules[ALIAS] = mod
    spec.loader.exec_module(mod)
    return mod
